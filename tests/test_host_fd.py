"""Host-objective FD engine of the C++ drop-in (MultiObjective::gradientApproximation /
gradientApproximationMPI with a C callback objective): no GPU needed, bitwise vs the oracle
(PNOL_Objective.cpp:165-299)."""
import ctypes as C
import os

import numpy as np
import pytest


def _callback_for(oracle, obj):
    def fn(x, n, F, m, user):
        xs = np.ctypeslib.as_array(x, shape=(n,)).copy()
        out = oracle.obj_eval_multi(obj, xs)
        C.memmove(F, out.ctypes.data, 8 * m)
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    return L.HOST_MULTI_FN(fn)


@pytest.mark.parametrize("factory,x0", [("cubic", [0.1] * 4), ("expcurve", [0.1] * 3)])
def test_host_fd_jacobian_bitwise(oracle, factory, x0):
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    obj = getattr(oracle, factory)()
    n, m = len(x0), obj.s.m
    cb = _callback_for(oracle, obj)
    x = np.array(x0); h = np.full(n, 1e-6)
    J = np.zeros((m, n))
    dp = C.POINTER(C.c_double)
    for sharded in (0, 1):   # single process: the MPI form reduces to the serial one
        L.check(L.lib().pnol_host_fd_jacobian(cb, None, x.ctypes.data_as(dp), h.ctypes.data_as(dp), n, m, sharded,
                                              J.ctypes.data_as(dp)), "host fd")
        ref = oracle.fd_jacobian(getattr(oracle, factory)(), x, h)
        assert np.array_equal(J, ref)


@pytest.mark.parametrize("factory,n", [("rosenbrock", 2), ("rosenbrock", 5), ("quadratic", 30), ("goldstein", 2)])
def test_host_fd_hessian_bitwise(oracle, factory, n):
    """Objective::hessianApproximation of the C++ FD engine (PNOL_Objective.cpp:38-85: F, then
    per upper-triangle pair the three points, batched through objEvalBatch) vs the oracle,
    bitwise, with the reference's evaluation count 1 + 3 n (n + 1) / 2."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    obj = {"rosenbrock": lambda: oracle.rosenbrock(n), "quadratic": lambda: oracle.quadratic(n),
           "goldstein": lambda: oracle.Obj(oracle.GOLDSTEIN, 2)}[factory]()
    calls = []

    def fn(x, nn, user):
        calls.append(1)
        return oracle.obj_eval(obj, np.ctypeslib.as_array(x, shape=(nn,)).copy())

    cb = L.HOST_SCALAR_FN(fn)
    rng = np.random.default_rng(n)
    x = rng.uniform(-1.5, 1.5, n); h = np.full(n, 1e-3)
    B = np.zeros((n, n))
    dp = C.POINTER(C.c_double)
    L.check(L.lib().pnol_host_fd_hessian(cb, None, x.ctypes.data_as(dp), h.ctypes.data_as(dp), n,
                                         B.ctypes.data_as(dp)), "host fd hessian")
    assert np.array_equal(B, oracle.fd_hessian(obj, x, h))
    assert len(calls) == 1 + 3 * n * (n + 1) // 2


GA_P = [40, 200, 0.1, 0.3, 0.2, 0.5, 0.01, 0.5, 20, 0]   # setGAParams without graph


@pytest.mark.parametrize("which", [0, 1])
def test_host_ga_bitwise(oracle, which):
    """GeneticAlgorithm / GeneticAlgorithmMPI (one rank) on a host callback objective, each
    generation through objEvalBatch: X, f0, fOpt, generations and evaluations bitwise the
    oracle's restatement (GeneticAlgorithm.cpp:12-297) -- no GPU needed."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    n = 4
    obj = oracle.rosenbrock(n)
    cb = L.HOST_SCALAR_FN(lambda x, nn, user: oracle.obj_eval(obj, np.ctypeslib.as_array(x, shape=(nn,)).copy()))
    lb, ub, x0 = np.full(n, -2.0), np.full(n, 2.0), np.full(n, -1.0)
    X = x0.copy()
    p = np.array(GA_P, dtype=np.float64)
    res = L.Result()
    dp = C.POINTER(C.c_double)
    L.check(L.lib().pnol_host_run_ga(which, cb, None, p.ctypes.data_as(dp), p.size, 12345, X.ctypes.data_as(dp), n,
                                     lb.ctypes.data_as(dp), ub.ctypes.data_as(dp), C.byref(res)), "host ga")
    Xo, reso, st = oracle.ga_findmin(oracle.rosenbrock(n), x0, lb, ub, GA_P[:9], 12345, 0)
    assert st == 0 and np.array_equal(X, Xo)
    assert (res.f0, res.fopt, res.iters, res.evals) == (reso.f0, reso.fopt, reso.iters, reso.evals)


PLATEAU = r'''
import ctypes as C, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from parallelnonlinearoptimizationlibrary_amd import _lib as L
n = 3
x0 = np.full(n, 0.25)
# one better point (x0); every other point ties with the worst -- a penalty-style plateau
cb = L.HOST_SCALAR_FN(lambda x, nn, u: 0.0 if np.array_equal(np.ctypeslib.as_array(x, shape=(nn,)), x0) else 1.0)
lb, ub = np.full(n, -1.0), np.full(n, 1.0)
X = x0.copy()
p = np.array([20, 100, 0.1, 0.3, 0.2, 0.5, 0.01, 0.5, 5, 0], dtype=np.float64)
res = L.Result()
dp = C.POINTER(C.c_double)
L.check(L.lib().pnol_host_run_ga(int(sys.argv[2]), cb, None, p.ctypes.data_as(dp), p.size, 99, X.ctypes.data_as(dp),
                                 n, lb.ctypes.data_as(dp), ub.ctypes.data_as(dp), C.byref(res)), "ga")
assert np.array_equal(X, x0) and res.fopt == 0.0, (X, res.fopt)
print("generations", res.iters, "evals", res.evals)
'''


@pytest.mark.parametrize("which", [0, 1])
def test_host_ga_plateau_terminates(tmp_path, which):
    """A plateau objective (one strictly better member, every other one tied with the worst) gives
    fitness 0 to every member the weighted selection may pick; selection then falls back to
    uniform over members 1..Npop-1 instead of waiting for a draw u == 0 (the reference's loop,
    GeneticAlgorithmMPI.cpp:134-146).  Run in a child with a time limit: a regression hangs."""
    import subprocess
    import sys
    import os
    s = tmp_path / "plateau.py"
    s.write_text(PLATEAU)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, str(s), root, str(which)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-2000:]
    assert b"generations" in r.stdout


def test_recur_simd_matches_scalar_walks(tmp_path):
    """csrc/host/recur_simd.hpp (the bounded solvers' frozen-coordinate scatter / gather, AVX-512
    expand / compress where the host has it) is bitwise the scalar walks it replaces: random
    indicator patterns, tail blocks, all-frozen / all-free words, mismatched reduced lengths."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "recur_simd_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I",
                    os.path.join(root, "parallelnonlinearoptimizationlibrary_amd", "csrc", "host"),
                    os.path.join(root, "tests", "cpp", "recur_simd_check.cpp"), "-o", exe], check=True, timeout=120)
    for scalar in ("0", "1"):   # the AVX-512 paths (where the host has them), then the scalar walks
        env = dict(os.environ)
        env.pop("PNOL_NO_AVX512", None)
        if scalar == "1":
            env["PNOL_NO_AVX512"] = "1"
        r = subprocess.run([exe], capture_output=True, timeout=120, env=env)
        assert r.returncode == 0, (r.stdout + r.stderr).decode()[-2000:]
        assert "fails=0" in r.stdout.decode()
        if scalar == "1":
            assert "avx512=0" in r.stdout.decode()
