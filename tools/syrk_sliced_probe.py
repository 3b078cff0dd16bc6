"""The m-sliced J^T J of LevMarqMPI (rows mode) in one process, for PMC passes of the kernel an
N > 1 rank runs: pnol_lm_jacobian_mpi_d writes the sliced JT (8 m-slices of mS rows) and
pnol_lm_normal_mpi_d runs the 64 x 64-tile SYRK (k_syrk_tile<4, 64>, PNOL_SYRK_T64=1) over all
eight slices at m = 16384, n = 2048.  A rank of a P-GPU run launches the same kernel over
8 / P of the slices, so its per-launch bytes are this launch's times (its slices) / 8.
    python tools/syrk_sliced_probe.py [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PNOL_SYRK_T64"] = "1"


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective
    m, n = 16384, 2048
    ctx = Context(0)
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    x = ctx.tensor(np.linspace(-0.5, 0.5, n))
    h = ctx.tensor(np.full(n, 1e-7))
    F0, JTs = d.lm_jacobian_mpi(x, h)
    for _ in range(reps):
        A, r = ctx.lm_normal_mpi(JTs, m, n, 0.37, F0)
    ctx.synchronize()
    print(f"sliced J^T J m={m} n={n}: A[0,0]={float(A[0, 0]):.6e}")


if __name__ == "__main__":
    main()
