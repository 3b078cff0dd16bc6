"""Per-rank LM step model for LevMarqMPI at N = 1/2/4/8 GPUs (cfg 4), measured on ONE
MI355X: each piece of rank r's trip timed on its own, then combined with the transfer volumes of
the exchange steps at an assumed xGMI rate (the 8-GPU run itself is the driver's).

  FD_r(P)   : rank r's cost-balanced FD column tiles (pnol_fd_tiles snake order) for all m rows,
              one tile-list launch (columns mode; the phased per-tile launches add ~6% at P = 8,
              DESIGN 7), max over r
  SYRK(P)   : J^T J over m / P residual rows (a rank's m-slices), with the reduce
  solve     : the persistent tile Cholesky + backward solve at n (replicated on every rank)
  eval      : F(x + sigma) (columns mode: all rows on every rank)
  exchanges : columns mode J slices (P-1)/P^2 * 8mn bytes per rank (all but the last phase hidden
              behind the FD launches), the J^T J node reduce-scatter and the tile allgather
              (~33.5 MB over the ranks), at LINK_GBPS per peer link

    python tools/rank_model.py [--out profiles/r05_rank_model.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LINK_GBPS = 64.0     # assumed effective one-direction rate of one xGMI peer link (GB/s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective
    m, n = args.m, args.n
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    x = ctx.tensor(np.linspace(-0.5, 0.5, n))
    h = ctx.tensor(np.full(n, 1e-7))
    JT = ctx.empty(n, m)
    F0 = ctx.empty(m)

    def timed(fn):
        fn()
        ctx.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2]

    out = {"m": m, "n": n, "link_GBps_assumed": LINK_GBPS, "per_P": {}}
    obj.eval(x)   # F0 for the FD's base point
    for P in (1, 2, 4, 8):
        fd = []
        for r in range(P):
            tiles = L.fd_tiles(n, P, r)
            fd.append(timed(lambda: obj.fd_jacobian_tiles(x, h, tiles, JT, F0, 2)) if tiles else 0.0)   # checkpoints reused, as in the trip
        mp = m // P
        JTs = torch.randn(n, mp, dtype=torch.float64, device=f"cuda:{ctx.device}")
        t_syrk = timed(lambda: ctx.jtj(JTs, 0.01))
        del JTs
        out["per_P"][P] = {"fd_ms_per_rank": fd, "fd_ms_max": max(fd), "syrk_reduce_ms": t_syrk}
    # the replicated pieces at n: solve (Cholesky + backward), F(x + sigma)
    rng = np.random.default_rng(0)
    B = rng.standard_normal((n, n))
    A = ctx.tensor(B @ B.T / n + np.eye(n))
    rhs = ctx.tensor(rng.standard_normal(n))
    t_solve = timed(lambda: ctx.solve_step(A, rhs, x))
    t_eval = timed(lambda: obj.eval(x))
    out["solve_ms"] = t_solve
    out["eval_ms"] = t_eval
    bytes_J = 8.0 * m * n
    for P, d in out["per_P"].items():
        if P == 1:
            exch = 0.0
        else:
            # columns mode: a rank's last phase (one tile's slices to the P-1 other ranks, in
            # parallel over their links) is exposed; the node reduce-scatter + allgather of
            # ~8 n^2 bytes split over P ranks go over P-1 links at once
            last_phase = bytes_J / 16 / P / LINK_GBPS / 1e6          # one 128-column tile's slice share (ms)
            tiles_bytes = 8.0 * n * n
            nodes = tiles_bytes * (P - 1) / P / (P - 1) / LINK_GBPS / 1e6
            gather = tiles_bytes / P / LINK_GBPS / 1e6
            exch = last_phase + nodes + gather
        d["exchange_ms_model"] = exch
        d["step_ms_model"] = d["fd_ms_max"] + d["syrk_reduce_ms"] + exch + t_solve + t_eval
        d["lm_iters_per_s_model"] = 1e3 / d["step_ms_model"]
    s1 = out["per_P"][1]["step_ms_model"]
    for P, d in out["per_P"].items():
        d["speedup_model_vs_1"] = s1 / d["step_ms_model"]
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
