"""bench.py's cpu_baseline building blocks (CPU only): the whole LM trip it times on P threads
computes the reference CPU path's step -- its sigma is bitwise the oracle's LevMarq step
(orc_lm_step, LevenbergMarquardt.cpp:55-83) on the same FD Jacobian -- so the timed trip is
the reference's work, not a shortcut."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_cpu_lm_trip_is_the_reference_step(oracle):
    import bench
    m, n, P = 1024, 130, 3
    A, _, y = oracle.linres_data(m, n)
    objs = [oracle.Obj(oracle.LINRES, n, m, A, y) for _ in range(P)]
    x, h = np.linspace(-0.3, 0.2, n), np.full(n, 1e-7)
    with ThreadPoolExecutor(P) as ex:
        t, sigma = bench.cpu_lm_trip(oracle, objs, x, h, ex, P)
    J = oracle.fd_jacobian(oracle.Obj(oracle.LINRES, n, m, A, y), x, h)
    F = oracle.obj_eval_multi(objs[0], x)
    assert t > 0
    assert np.array_equal(sigma, oracle.lm_step(J, F, 0.001)[3])


def test_cpu_model_reads_proc_cpuinfo():
    import bench
    name, ncpu = bench.cpu_model()
    assert isinstance(name, str) and name and ncpu >= 1
