"""Where a BFGS line-search iteration's time goes at cfg 2 (n = 4096, device quadratic):
the host round trip of pnol_dobj_eval_batch with the Wolfe search's two points, against the
eval kernel alone (device points, stream-timed).  Run under rocprofv3 --kernel-trace --stats
for the kernel durations."""
import ctypes as C
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from parallelnonlinearoptimizationlibrary_amd import _lib as L  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = 400
    ctx = Context()
    obj = DeviceObjective.synthetic(ctx, L.OBJ_QUADRATIC, n, 0, bscale=4.0)
    Xs = np.random.default_rng(1).standard_normal(2 * n)
    f = np.zeros(2)
    lib = L.lib()
    P = C.POINTER(C.c_double)
    for _ in range(20):
        L.check(lib.pnol_dobj_eval_batch(ctx.h, obj.h, Xs.ctypes.data_as(P), 2, f.ctypes.data_as(P)), "eval_batch")
    t0 = time.perf_counter()
    for _ in range(reps):
        L.check(lib.pnol_dobj_eval_batch(ctx.h, obj.h, Xs.ctypes.data_as(P), 2, f.ctypes.data_as(P)), "eval_batch")
    host_us = (time.perf_counter() - t0) / reps * 1e6
    x = torch.tensor(Xs[:n], device="cuda")
    out = torch.empty(1, dtype=torch.float64, device="cuda")
    for _ in range(20):
        L.check(lib.pnol_dobj_eval_d(ctx.h, obj.h, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr())), "eval_d")
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        L.check(lib.pnol_dobj_eval_d(ctx.h, obj.h, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr())), "eval_d")
    ctx.synchronize()
    dev_us = (time.perf_counter() - t0) / reps * 1e6
    print(json.dumps({"n": n, "eval_batch_2pts_host_roundtrip_us": host_us,
                      "eval_1pt_device_back_to_back_us": dev_us}))
    obj.close()
    ctx.close()


if __name__ == "__main__":
    main()
