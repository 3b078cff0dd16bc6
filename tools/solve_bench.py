"""Times pnol_solve_d at n (default 2048) for the given methods (wall clock over repeated solves
on cuda:0, synchronised) and prints the relative error vs numpy.
    python tools/solve_bench.py [N] [METHODS...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    methods = [int(a) for a in sys.argv[2:]] or [1, 4]
    from parallelnonlinearoptimizationlibrary_amd.device import Context
    ctx = Context(0)
    rng = np.random.default_rng(n)
    J = rng.standard_normal((2 * n, n))
    A = J.T @ J + np.eye(n)
    b = rng.standard_normal(n)
    x = np.linalg.solve(A, b)
    At, bt = ctx.tensor(A), ctx.tensor(b)
    for m in methods:
        work = [ctx.tensor(A) for _ in range(3)]
        for w in work:
            ctx.solve(w, bt, method=m)
        reps = 20
        mats = [ctx.tensor(A) for _ in range(reps)] if m != 4 else [At] * reps
        ctx.synchronize()
        t0 = time.perf_counter()
        for w in mats:
            sigma, info = ctx.solve(w, bt, method=m)
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / reps
        err = np.linalg.norm(sigma.cpu().numpy() - x) / np.linalg.norm(x)
        print(f"n={n} method={m} info={info} ms={dt * 1e3:.3f} relerr={err:.3e}", flush=True)


if __name__ == "__main__":
    main()
