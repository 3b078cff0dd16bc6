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
    print(json.dumps({"n": n, "fd_gradient_us_back_to_back": (time.perf_counter() - t0) / reps * 1e6}))
    obj.close()
    ctx.close()


if __name__ == "__main__":
    main()
