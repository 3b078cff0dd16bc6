"""Sweep k_gemv_neg rows-per-wave (PNOL_GEMV_ROWS) for p = -D g at n = 8192 / 4096, cold
Infinity Cache (512 MiB fill before each launch), HIP events on the context stream.
Each setting runs in its own child process (the override is read once per process)."""
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
print(json.dumps({n: bench.bench_hg(ctx, n) for n in (8192, 4096)}))
""" % ROOT

if __name__ == "__main__":
    out = {}
    for mode, r in (("0", "2"), ("0", "1"), ("1", "1"), ("1", "2"), ("1", "4"), ("2", "2"), ("2", "4")):
        env = dict(os.environ, PNOL_GEMV_ROWS=r, PNOL_GEMV_MODE=mode)
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-2000:])
            sys.exit(p.returncode)
        res = json.loads(p.stdout.strip().splitlines()[-1])
        r = f"mode{mode}_R{r}"
        out[r] = {n: {k: round(v, 3) if isinstance(v, float) else v for k, v in d.items()
                      if k in ("hg_us", "hg_GBps", "hg_frac_of_hbm", "fused_pass_GBps")} for n, d in res.items()}
        print(r, json.dumps(out[r]), flush=True)
