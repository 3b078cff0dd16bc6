"""Probe: cfg 2 (BFGS, n = 4096, synthetic quadratic) -- the device run against the oracle's
rank-2 run, iteration by iteration (maxIter = 1, 2, ...) and whole: relative X difference,
iteration and evaluation counts.  The numbers the cfg-2 parity test asserts come from here.

    python tools/cfg2_traj_probe.py [n]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(np.max(np.abs(b)), 1e-300))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    import oracle as O
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_bfgs
    O.build()
    ctx = Context(0)
    dd, bb = O.quadratic_data(n)
    P = [1e-4, 0.9, 1e-6, 1, 1000, 1e-6, 1e-3, 200, 1e-9, 1e-6, 0, 0]
    out = {"n": n, "iters": []}
    for k in list(range(1, 9)) + [200]:
        Pk = list(P)
        Pk[7] = k
        X, res = run_bfgs(DeviceObjective(ctx, L.OBJ_QUADRATIC, n, 0, dd, bb), np.zeros(n), Pk)
        Xo, reso, _ = O.bfgs_findmin(O.Obj(O.QUADRATIC, n, 0, dd, bb), np.zeros(n), Pk, rank2=True)
        row = {"maxIter": k, "rel_X": rel(X, Xo), "iters": [int(res.iters), int(reso.iters)],
               "evals": [int(res.evals), int(reso.evals)], "fopt": [res.fopt, reso.fopt]}
        out["iters"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
