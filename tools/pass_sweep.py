"""Fused BFGS pass / H.g timing at n = 4096 and 8192 for the row-tile heights given as
arguments (PNOL_PASS_ROWS, read once per process: one child per value), cold Infinity Cache.
    python tools/pass_sweep.py 64 128 256"""
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
print(json.dumps({n: bench.bench_hg(ctx, n) for n in (4096, 8192)}))
""" % ROOT

if __name__ == "__main__":
    for v in sys.argv[1:] or ["128", "256"]:
        p = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, PNOL_PASS_ROWS=v), capture_output=True,
                           text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-2000:])
            sys.exit(p.returncode)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        print(v, {n: (round(r["fused_pass_us"], 1), round(r["fused_pass_frac_of_hbm"], 3)) for n, r in d.items()},
              flush=True)
