"""Streamed LM trip (pnol_lm_trip_stream_d): per-trip wall time and solve status over repeated
trips at one point, against pnol_fd_normal_d + pnol_solve_step_d.  argv: m n trips."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from parallelnonlinearoptimizationlibrary_amd import _lib as L  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective  # noqa: E402

m, n, trips = (int(a) for a in sys.argv[1:4])
lams = [float(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0.37]
ctx = Context(0)
d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
x, h = ctx.tensor(np.linspace(-0.5, 0.5, n)), ctx.tensor(np.full(n, 1e-7))
JT, A, r = ctx.empty(n, m), ctx.empty(n, n), ctx.empty(n)
refs = {}
for lam in lams:
    F0, JT, A, r = d.fd_normal(x, h, lam, JT, A, r)
    s0, _, i0 = ctx.solve_step(A, r, x)
    refs[lam] = (s0.cpu().numpy(), i0)
out = {"m": m, "n": n, "lams": lams, "ref_info": [refs[l][1] for l in lams], "ms": [], "info": [], "equal": []}
JTb = ctx.empty(n, m)
for t in range(trips):
    ctx.synchronize()
    t0 = time.perf_counter()
    lam = lams[t % len(lams)]
    *_, sb, _, ib = d.lm_trip_stream(x, h, lam, JTb)
    out["ms"].append(round((time.perf_counter() - t0) * 1e3, 3))
    out["info"].append(ib)
    out["equal"].append(bool(np.array_equal(sb.cpu().numpy(), refs[lam][0])))
for t in range(trips):   # the two-call trip it replaces, same point
    ctx.synchronize()
    t0 = time.perf_counter()
    F0, JT, A, r = d.fd_normal(x, h, 0.37, JT, A, r)
    ctx.solve_step(A, r, x)
    out.setdefault("ms_two_call", []).append(round((time.perf_counter() - t0) * 1e3, 3))
print(json.dumps(out))
