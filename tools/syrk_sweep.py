"""Time J^T J (k_syrk_tile + k_syrk_reduce) on the bench shape (m=16384, n=2048, random JT) for
K splits given as "sub:first" arguments (PNOL_SYRK_SUB / PNOL_SYRK_FIRST, read once per
process, so one child per variant).  sub 0 = the default choice."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import ctypes as C, json, sys
sys.path.insert(0, %r)
import numpy as np, torch
from parallelnonlinearoptimizationlibrary_amd import _lib as L
from parallelnonlinearoptimizationlibrary_amd.device import Context
m, n = 16384, 2048
ctx = Context(0)
torch.manual_seed(1234)
JT = torch.randn(n, m, dtype=torch.float64, device="cuda")
for _ in range(2):
    ctx.jtj(JT, 0.25)
ctx.synchronize()
L.check(L.lib().pnol_ctx_enable_timers(ctx.h, 1), "t"); L.check(L.lib().pnol_ctx_reset_timers(ctx.h), "t")
for _ in range(8):
    A = ctx.jtj(JT, 0.25)
ctx.synchronize()
out = {}
for k in ("syrk", "syrk_reduce"):
    ms, c = C.c_double(), C.c_int()
    L.lib().pnol_ctx_timer(ctx.h, k.encode(), C.byref(ms), C.byref(c))
    out[k] = ms.value / max(c.value, 1)
out["tflops"] = m * n * (n + 1) / (out["syrk"] * 1e-3) / 1e12
ref = (JT @ JT.T); ref.diagonal().mul_(1.25)
out["relerr"] = float((A - ref).abs().max() / ref.abs().max())
import hashlib
out["sha"] = hashlib.sha1(A.cpu().numpy().tobytes()).hexdigest()[:12]
print(json.dumps(out))
""" % ROOT

if __name__ == "__main__":
    for v in (sys.argv[1:] or ["0:0", "2:75"]):
        f = v.split(":") + ["0", "0"][len(v.split(":")):]
        env = dict(os.environ, PNOL_SYRK_SUB=f[0], PNOL_SYRK_FIRST=f[1])
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-2000:])
            sys.exit(p.returncode)
        print(v, p.stdout.strip().splitlines()[-1], flush=True)
