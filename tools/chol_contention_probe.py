"""How the persistent tile Cholesky behaves when several processes share the GPU (the situation of
tests/test_gpu_mpi.py, where 2-8 ranks share the box's one GPU): P child processes each run K LM
trips (pnol_lm_trip_d: FD Jacobian, J^T J partials, the reducing persistent Cholesky, backward
solve) at (m, n) back to back, reading the solve status after every trip (no relaunch: the raw
status the kernel reported).  Per process: trip wall times (median / max) and the nonzero statuses
(kCholTimeout = -7: a dependency wait ran past its spin cap).

    python tools/chol_contention_probe.py --procs 3 --trips 200 --m 1000 --n 700 --out gpurun_out/x.json
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(args):
    import numpy as np
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective
    ctx = Context(0)
    m, n = args.m, args.n
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    h = ctx.tensor(np.full(n, 1e-7))
    JT = ctx.empty(n, m)
    times, bad = [], []
    for k in range(args.trips):
        x = ctx.tensor(np.linspace(-0.5, 0.5 + 1e-3 * k, n))
        t0 = time.perf_counter()
        *_, info = d.lm_trip(x, h, 0.01, JT)
        ctx.synchronize()
        times.append(time.perf_counter() - t0)
        if info != 0:
            bad.append([k, int(info)])
    times.sort()
    print(json.dumps({"pid": os.getpid(), "trips": args.trips, "median_ms": 1e3 * times[len(times) // 2],
                      "max_ms": 1e3 * times[-1], "p99_ms": 1e3 * times[int(0.99 * (len(times) - 1))],
                      "nonzero_status": bad}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=3)
    ap.add_argument("--trips", type=int, default=200)
    ap.add_argument("--m", type=int, default=1000)
    ap.add_argument("--n", type=int, default=700)
    ap.add_argument("--out", default="")
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
    cmd = [sys.executable, os.path.abspath(__file__), "--child", "--trips", str(args.trips), "--m", str(args.m),
           "--n", str(args.n)]
    t0 = time.time()
    procs = [subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE) for _ in range(args.procs)]
    res = []
    for p in procs:
        o, e = p.communicate(timeout=600)
        lines = [l for l in o.decode().splitlines() if l.startswith("{")]
        res.append(json.loads(lines[-1]) if lines else {"rc": p.returncode, "stderr": e.decode()[-2000:]})
    out = {"procs": args.procs, "m": args.m, "n": args.n, "wall_s": time.time() - t0, "per_process": res}
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
