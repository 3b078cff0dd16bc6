"""One cfg-5 BFGS_Bnd solve (n = 16384, the bench's synthetic box QP) -- a short command for
rocprofv3 kernel traces of the bounded solver's kernels.  Prints the bench block as JSON."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import bench  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd.device import Context  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
ctx = Context(0)
blk = bench.bench_bfgs_solve(ctx, 2, n, 4.0, bench.CFG5_P, bounds=(np.full(n, -0.5), np.full(n, 0.5)))
print(json.dumps(blk))
