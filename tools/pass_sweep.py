"""Fused BFGS pass / H.g timing at n = 4096 and 8192 (PASS_SIZES=a,b,..), cold Infinity Cache, one child process per
setting (the tuning variables are read once per process): arguments VAR=value, e.g.
    python tools/pass_sweep.py PNOL_PASS_ROWS=128 PNOL_PASS_ROWS=256 PNOL_GEMV_ROWS=1"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys
sys.path.insert(0, %r)
import bench
from parallelnonlinearoptimizationlibrary_amd.device import Context
ctx = Context(0)
print(json.dumps({n: bench.bench_hg(ctx, n) for n in %r}))
""" % (ROOT, tuple(int(v) for v in os.environ.get("PASS_SIZES", "4096,8192").split(",")))

if __name__ == "__main__":
    for v in sys.argv[1:] or ["PNOL_PASS_ROWS=128", "PNOL_PASS_ROWS=256"]:
        k, _, val = v.partition("=")
        p = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, **{k: val}), capture_output=True,
                           text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-2000:])
            sys.exit(p.returncode)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        print(v, {n: {"hg_us": round(r["hg_us"], 1), "hg_frac": round(r["hg_frac_of_hbm"], 3),
                      "pass_us": round(r["fused_pass_us"], 1), "pass_frac": round(r["fused_pass_frac_of_hbm"], 3)}
                  for n, r in d.items()}, flush=True)
