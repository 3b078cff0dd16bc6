"""One small LevMarq solve in a fresh process (smoke()'s size by default): prints the result's
distance to the oracle and the wall time.  argv: m n."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd import _lib as L  # noqa: E402
from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_levmarq  # noqa: E402

m, n = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (512, 96)
ctx = Context(0)
A, xs, y = O.linres_data(m, n)
d = DeviceObjective(ctx, L.OBJ_LINRES, n, m, A, y)
params = (0.001, 10, 1e-7, 3, 0.0, -1)
t0 = time.perf_counter()
X, *_ = run_levmarq(d, np.zeros(n), params)
t1 = time.perf_counter()
Xo, *_ = O.lm_findmin(O.linres(m, n), np.zeros(n), params)
print(f"m={m} n={n} trip={os.environ.get('PNOL_LM_TRIP', '1')} "
      f"err={np.max(np.abs(X - Xo)) / np.max(np.abs(Xo)):.2e} s={t1 - t0:.3f}", flush=True)
