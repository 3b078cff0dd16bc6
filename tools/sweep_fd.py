"""Time the FD Jacobian GEMM variants (PNOL_FD_KERNEL=2..4, argv selects; default all) on the bench workload (linres
m=16384, n=2048, all columns), HIP-event timers on the context stream, one child process per
variant (the selector is read once per process).  Also checks the variants are bitwise equal."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes as C, json, sys, hashlib
sys.path.insert(0, %r)
import numpy as np
from parallelnonlinearoptimizationlibrary_amd import _lib as L
from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective
m, n = 16384, 2048
ctx = Context(0)
obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
x = ctx.tensor(np.linspace(-0.5, 0.5, n)); h = ctx.tensor(np.full(n, 1e-7))
JT = ctx.empty(n, m); F0 = ctx.empty(m)
for _ in range(2):
    obj.fd_jacobian(x, h, 0, n, JT=JT, F0=F0)
ctx.synchronize()
L.check(L.lib().pnol_ctx_enable_timers(ctx.h, 1), "t"); L.check(L.lib().pnol_ctx_reset_timers(ctx.h), "t")
for _ in range(5):
    obj.fd_jacobian(x, h, 0, n, JT=JT, F0=F0)
for _ in range(5):
    obj.eval(x)
ctx.synchronize()
out = {}
for k in ("fd_jacobian", "fd_ckpt", "linres_eval"):
    ms, c = C.c_double(), C.c_int()
    L.lib().pnol_ctx_timer(ctx.h, k.encode(), C.byref(ms), C.byref(c))
    out[k] = ms.value / max(c.value, 1)
out["sha"] = hashlib.sha1(JT.cpu().numpy().tobytes()).hexdigest()
print(json.dumps(out))
""" % ROOT

if __name__ == "__main__":
    shas = set()
    for v in (sys.argv[1:] or ["2", "3", "4"]):
        env = dict(os.environ, PNOL_FD_KERNEL=v)
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-2000:])
            sys.exit(p.returncode)
        r = json.loads(p.stdout.strip().splitlines()[-1])
        shas.add(r["sha"])
        print(v, json.dumps({k: (round(val, 4) if isinstance(val, float) else val) for k, val in r.items()}), flush=True)
    print("bitwise_equal_across_variants", len(shas) == 1)
    sys.exit(0 if len(shas) == 1 else 4)
