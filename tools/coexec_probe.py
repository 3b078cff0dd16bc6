"""Does the VALU-bound FD GEMM co-execute with the MFMA-bound J^T J?  Times each alone and
both launched together on two streams (two contexts), bench workload (m=16384, n=2048)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd import _lib as L  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective  # noqa: E402

m, n = 16384, 2048
c1 = Context(0)
c2 = Context(0)
obj = DeviceObjective.synthetic(c1, L.OBJ_LINRES, n, m)
x = c1.tensor(np.linspace(-0.5, 0.5, n))
h = c1.tensor(np.full(n, 1e-7))
JT = c1.empty(n, m)
F0 = c1.empty(m)
JT2 = torch.randn(n, m, dtype=torch.float64, device="cuda")


def fd():
    obj.fd_jacobian(x, h, 0, n, JT=JT, F0=F0)


def jtj():
    c2.jtj(JT2, 0.01)


def timeit(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for f in (fd, jtj):
    f()
t_fd = timeit(fd)
t_jtj = timeit(jtj)
t_both = timeit(lambda: (fd(), jtj()))
print(f"fd {t_fd:.3f} ms  jtj {t_jtj:.3f} ms  sum {t_fd + t_jtj:.3f}  concurrent {t_both:.3f} ms", flush=True)
