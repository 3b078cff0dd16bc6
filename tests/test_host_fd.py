"""Host-objective FD engine of the C++ drop-in (MultiObjective::gradientApproximation /
gradientApproximationMPI with a C callback objective): no GPU needed, bitwise vs the oracle
(PNOL_Objective.cpp:165-299)."""
import ctypes as C

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
