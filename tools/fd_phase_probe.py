"""Probe: the FD Jacobian share of one LevMarqMPI rank in columns mode (its cost-balanced tiles,
all m rows) on one GPU, as one launch vs one launch per tile (the phased launch order that lets
each tile's m-slice exchange start while the next tile computes).  m = 16384, n = 2048.
Prints one JSON line: per (P, rank) the single-launch kernel time and the per-tile kernel times
(HIP events carried by the dispatch, pnol_ctx_timer "fd_jacobian"), medians over reps.

    python tools/fd_phase_probe.py [reps]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    import torch
    from parallelnonlinearoptimizationlibrary_amd import _lib as L, fd_tiles
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective
    m, n = 16384, 2048
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    x = ctx.tensor(np.zeros(n))
    h = ctx.tensor(np.full(n, 1e-7))
    F0 = obj.eval_ckpt(x)
    JT = ctx.empty(n, m)
    lib = L.lib()

    def timed(tiles_list):
        """kernel ms of each call (one call per entry of tiles_list), median over reps"""
        per = []
        for _ in range(reps):
            row = []
            for tl in tiles_list:
                L.check(lib.pnol_ctx_enable_timers(ctx.h, 1), "timers")
                L.check(lib.pnol_ctx_reset_timers(ctx.h), "reset")
                obj.fd_jacobian_tiles(x, h, tl, JT, F0=F0, compute_f0=2)
                ctx.synchronize()
                ms, cnt = C.c_double(), C.c_int()
                L.check(lib.pnol_ctx_timer(ctx.h, b"fd_jacobian", C.byref(ms), C.byref(cnt)), "timer")
                row.append(ms.value)
            per.append(row)
        return [float(v) for v in np.median(np.array(per), axis=0)]

    out = {"m": m, "n": n, "reps": reps}
    full = fd_tiles(n, 1, 0)
    timed([full])   # warm (panels, clocks)
    out["P1_one_launch_ms"] = timed([full])[0]
    for P in (2, 4, 8):
        rows = []
        for r in range(P):
            tl = fd_tiles(n, P, r)
            one = timed([tl])[0]
            by_tile = sorted(tl, key=lambda t: -t[0])        # cheap (late columns) first
            each = timed([[t] for t in by_tile])
            rows.append({"rank": r, "tiles": [t[0] for t in by_tile], "one_launch_ms": one, "per_tile_ms": each,
                         "per_tile_sum_ms": float(sum(each))})
        out[f"P{P}"] = rows
    print(json.dumps(out))


if __name__ == "__main__":
    main()
