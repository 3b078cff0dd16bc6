"""The scalar FD gradient (term form) at cfg-5 size on its own: pnol_fd_gradient_d on the
synthetic quadratic, n = 16384 by default, back to back.  Run under rocprofv3 --kernel-trace
--stats for the per-kernel split (k_scalar_terms / k_scalar_fd_chain / k_scalar_fd_finish)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from parallelnonlinearoptimizationlibrary_amd import _lib as L  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ctx = Context()
    obj = DeviceObjective.synthetic(ctx, L.OBJ_QUADRATIC, n, 0, bscale=4.0)
    x = torch.rand(n, dtype=torch.float64, device="cuda") - 0.5
    h = torch.full((n,), 1e-6, dtype=torch.float64, device="cuda")
    for _ in range(5):
        obj.fd_gradient(x, h)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        obj.fd_gradient(x, h)
    ctx.synchronize()
    dev_us = (time.perf_counter() - t0) / reps * 1e6
    # the host-pointer entry point (pinned staging, one H2D of x and h, one D2H of g and f0, one sync)
    import ctypes as C
    import numpy as np
    P = C.POINTER(C.c_double)
    xh, hh = x.cpu().numpy().copy(), h.cpu().numpy().copy()
    g, f0 = np.zeros(n), np.zeros(1)
    lib = L.lib()
    for _ in range(5):
        L.check(lib.pnol_fd_gradient(ctx.h, obj.h, xh.ctypes.data_as(P), hh.ctypes.data_as(P), 0, n,
                                     f0.ctypes.data_as(P), g.ctypes.data_as(P)), "fd_gradient")
    t0 = time.perf_counter()
    for _ in range(reps):
        L.check(lib.pnol_fd_gradient(ctx.h, obj.h, xh.ctypes.data_as(P), hh.ctypes.data_as(P), 0, n,
                                     f0.ctypes.data_as(P), g.ctypes.data_as(P)), "fd_gradient")
    host_us = (time.perf_counter() - t0) / reps * 1e6
    print(json.dumps({"n": n, "fd_gradient_us_back_to_back": dev_us, "fd_gradient_host_pointers_us": host_us}))
    obj.close()
    ctx.close()


if __name__ == "__main__":
    main()
