"""Writes tests/golden/cfg3_lm_trips.npz: the oracle's LevMarq::findMin (LevenbergMarquardt.cpp:
50-136) at the headline size m = 16384, n = 2048 (cfg 3, the synthetic dense residual
r(x) = A x - y from the splitmix64 stream, seed 0x5EED2018), X / chi^2 / lambda after each of
the first 3 loop trips.

The oracle is the CPU restatement (oracle/pnol_oracle.c); its threaded composition
(oracle/pnol_oracle_par.c) forms every value with the same operations in the same order
(bitwise equal at small sizes: tests/test_oracle_golden.py::test_lm_par_oracle_equals_sequential),
so these are the oracle's bits.  Run in the build container (8 cores: ~2 minutes):

    python tests/golden/make_cfg3_lm_trips.py
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

M, N, TRIPS = 16384, 2048, 3
PARAMS = (0.001, 10.0, 1e-7, TRIPS, 0.0, -1)   # lambda0, lambdaFactor, dXGrad, maxIter, xMinDiff, verbose


def main():
    O.build()
    t0 = time.time()
    o = O.linres(M, N)
    X, res, F0, FOpt, tx, tc, tl = O.lm_findmin_par(o, np.zeros(N), PARAMS, trace_cap=TRIPS,
                                                    threads=os.cpu_count())
    dt = time.time() - t0
    out = os.path.join(HERE, "cfg3_lm_trips.npz")
    np.savez_compressed(out, m=M, n=N, params=np.array(PARAMS, dtype=np.float64), x_trips=tx, chi_trips=tc,
                        lambda_trips=tl, chi0=res.f0, evals=res.evals, iters=res.iters,
                        xstar_rel_err=np.max(np.abs(X - o.xstar)) / np.max(np.abs(o.xstar)))
    print(f"wrote {out}: {len(tc)} trips in {dt:.1f} s; chi0 {res.f0:.6e} chi {list(tc)} lambda {list(tl)} "
          f"evals {res.evals}; |X - x*| / |x*| = {np.max(np.abs(X - o.xstar)) / np.max(np.abs(o.xstar)):.3e}")


if __name__ == "__main__":
    main()
