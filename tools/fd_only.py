"""Runs the FD Jacobian of the bench workload (linres m=16384, n=2048, all columns) a few
times on cuda:0; a target for rocprofv3 --pmc passes on the FD kernel alone."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parallelnonlinearoptimizationlibrary_amd import _lib as L  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective  # noqa: E402

m, n = 16384, 2048
ctx = Context(0)
obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
x = ctx.tensor(np.linspace(-0.5, 0.5, n))
h = ctx.tensor(np.full(n, 1e-7))
JT = ctx.empty(n, m)
F0 = ctx.empty(m)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    obj.fd_jacobian(x, h, 0, n, JT=JT, F0=F0)
ctx.synchronize()
print("fd_only done")
