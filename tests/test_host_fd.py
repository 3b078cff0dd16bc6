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
