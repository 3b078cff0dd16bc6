"""ctypes front end of the CPU parity oracle (oracle/pnol_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.  Each wrapper names the reference
function it restates (paths relative to /root/reference/Source).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

SEED = 0x5EED2018

ROSENBROCK, POWER, GOLDSTEIN, BOOTH, QUADRATIC = 0, 1, 2, 3, 4
EXPCURVE, CUBIC, LINRES = 10, 11, 12

_dp = C.POINTER(C.c_double)


class Objective(C.Structure):
    _fields_ = [("kind", C.c_int), ("n", C.c_int), ("m", C.c_int), ("p0", _dp), ("p1", _dp),
                ("power", C.c_double), ("evals", C.c_long)]


class Result(C.Structure):
    _fields_ = [("iters", C.c_int), ("evals", C.c_long), ("f0", C.c_double), ("fopt", C.c_double)]


class BFGSParams(C.Structure):  # BFGS::setParams, BFGS_with_linesearch.hpp:62
    _fields_ = [("c1", C.c_double), ("c2", C.c_double), ("dalpha", C.c_double), ("alphaGuess", C.c_double),
                ("maxIterLineSearch", C.c_int), ("dXGrad", C.c_double), ("dXHess", C.c_double),
                ("maxIter", C.c_double), ("xMinDiff", C.c_double), ("minGrad2Norm", C.c_double),
                ("initHessFD", C.c_int), ("verbose", C.c_int)]


class BFGSMPIParams(C.Structure):  # BFGS_MPI::setParams, BFGS_with_linesearch_MPI.hpp:64
    _fields_ = [("c1", C.c_double), ("c2", C.c_double), ("maxAlphaMult", C.c_double),
                ("alphaGuess", C.c_double), ("maxIterLineSearch", C.c_int), ("dXGrad", C.c_double),
                ("dXHess", C.c_double), ("maxIter", C.c_double), ("xMinDiff", C.c_double),
                ("minGrad2Norm", C.c_double), ("initHessFD", C.c_int), ("verbose", C.c_int)]


class LMParams(C.Structure):  # LevMarq::setParams, LevenbergMarquardt.hpp:41
    _fields_ = [("lambda0", C.c_double), ("lambdaFactor", C.c_double), ("dXGrad", C.c_double),
                ("maxIter", C.c_double), ("xMinDiff", C.c_double), ("verbose", C.c_int)]


class BFGSBndParams(C.Structure):  # BFGS_Bnd::setParams, BFGS_bnd_linesearch.hpp:80
    _fields_ = [("c1", C.c_double), ("c2", C.c_double), ("dalpha", C.c_double), ("alphaGuess", C.c_double),
                ("alphaTol", C.c_double), ("alphaMult", C.c_double), ("maxIterLineSearch", C.c_int),
                ("bndTol", C.c_double), ("dXGrad", C.c_double), ("dXHess", C.c_double),
                ("maxIter", C.c_double), ("xMinDiff", C.c_double), ("minGrad2Norm", C.c_double),
                ("initHessFD", C.c_int), ("verbose", C.c_int)]


class BFGSBndMPIParams(C.Structure):  # BFGSBnd_MPI::setParams, BFGS_with_bnd_linesearch_MPI.hpp:79
    _fields_ = [("c1", C.c_double), ("c2", C.c_double), ("alphaMin", C.c_double), ("maxAlphaMult", C.c_double),
                ("alphaGuess", C.c_double), ("maxIterLineSearch", C.c_int), ("dXGrad", C.c_double),
                ("dXHess", C.c_double), ("maxIter", C.c_double), ("xMinDiff", C.c_double),
                ("minGrad2Norm", C.c_double), ("FStepTolerance", C.c_double), ("initHessFD", C.c_int),
                ("verbose", C.c_int)]


_lib = None
FAST_PATH = os.path.join(HERE, "liboracle_fast.so")


def use_fast():
    """Switch this process to liboracle_fast.so: the same restatement built -O3 -march=x86-64-v3
    (still -ffp-contract=off), for bench.py's timed CPU baseline."""
    global _lib, LIB_PATH
    LIB_PATH = FAST_PATH
    _lib = None
    return lib()


def build() -> str:
    """Compile the oracle with its own Makefile (gcc); returns the library path."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_obj_eval.restype = C.c_double
        _lib.orc_util_dot.restype = C.c_double
        _lib.orc_util_norm2.restype = C.c_double
        _lib.orc_compute_alpha_bnd.restype = C.c_double
        _lib.orc_splitmix_u01.restype = C.c_double
        _lib.orc_splitmix_u01.argtypes = [C.c_ulonglong, C.c_ulonglong]
        _lib.orc_obj_eval_recur.restype = C.c_double
    return _lib


def ptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


class Obj:
    """Owns the numpy buffers behind an orc_objective."""

    def __init__(self, kind, n, m=0, p0=None, p1=None, power=2.0):
        self.p0 = None if p0 is None else np.ascontiguousarray(p0, dtype=np.float64)
        self.p1 = None if p1 is None else np.ascontiguousarray(p1, dtype=np.float64)
        self.s = Objective(kind, n, m, ptr(self.p0) if self.p0 is not None else None,
                           ptr(self.p1) if self.p1 is not None else None, power, 0)

    @property
    def evals(self):
        return self.s.evals

    def ref(self):
        return C.byref(self.s)


# ---- objective factories -------------------------------------------------------------

def rosenbrock(n):
    return Obj(ROSENBROCK, n)


def power(n, p):
    return Obj(POWER, n, power=float(p))


def expcurve(m=100):
    x = np.zeros(m); y = np.zeros(m)
    lib().orc_make_expcurve_data(m, ptr(x), ptr(y))
    return Obj(EXPCURVE, 3, m, x, y)


def cubic(m=100):
    x = np.zeros(m); y = np.zeros(m)
    lib().orc_make_cubic_data(m, ptr(x), ptr(y))
    return Obj(CUBIC, 4, m, x, y)


def quadratic_data(n, seed=SEED, bscale=1.0):
    d = np.zeros(n); b = np.zeros(n)
    lib().orc_make_quadratic(C.c_ulonglong(seed), n, ptr(d), ptr(b))
    return d, b * bscale


def quadratic(n, seed=SEED, bscale=1.0):
    d, b = quadratic_data(n, seed, bscale)
    return Obj(QUADRATIC, n, 0, d, b)


def linres_data(m, n, seed=SEED):
    A = np.zeros((m, n)); xs = np.zeros(n); y = np.zeros(m)
    lib().orc_make_linres(C.c_ulonglong(seed), m, n, ptr(A), ptr(xs), ptr(y))
    return A, xs, y


def linres(m, n, seed=SEED):
    A, xs, y = linres_data(m, n, seed)
    o = Obj(LINRES, n, m, A, y)
    o.xstar = xs
    return o


# ---- restated reference functions ----------------------------------------------------

def obj_eval(o: Obj, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().orc_obj_eval(o.ref(), ptr(x))


def obj_eval_multi(o: Obj, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    F = np.zeros(o.s.m)
    lib().orc_obj_eval_multi(o.ref(), ptr(x), ptr(F))
    return F


def fd_gradient(o: Obj, x, dx):  # Objective::gradientApproximation, PNOL_Objective.cpp:12-34
    x = np.ascontiguousarray(x, dtype=np.float64); dx = np.ascontiguousarray(dx, dtype=np.float64)
    g = np.zeros_like(x)
    lib().orc_fd_gradient(o.ref(), ptr(x), ptr(dx), ptr(g), len(x))
    return g


def fd_gradient_sharded(o: Obj, x, dx, nprocs):  # PNOL_Objective.cpp:88-159
    x = np.ascontiguousarray(x, dtype=np.float64); dx = np.ascontiguousarray(dx, dtype=np.float64)
    g = np.zeros_like(x)
    lib().orc_fd_gradient_sharded(o.ref(), ptr(x), ptr(dx), ptr(g), len(x), nprocs)
    return g


def fd_jacobian(o: Obj, x, dx):  # MultiObjective::gradientApproximation, PNOL_Objective.cpp:165-197
    x = np.ascontiguousarray(x, dtype=np.float64); dx = np.ascontiguousarray(dx, dtype=np.float64)
    J = np.zeros((o.s.m, len(x)))
    lib().orc_fd_jacobian(o.ref(), ptr(x), ptr(dx), ptr(J), len(x), o.s.m)
    return J


def fd_jacobian_sharded(o: Obj, x, dx, nprocs):  # PNOL_Objective.cpp:202-299
    x = np.ascontiguousarray(x, dtype=np.float64); dx = np.ascontiguousarray(dx, dtype=np.float64)
    J = np.zeros((o.s.m, len(x)))
    lib().orc_fd_jacobian_sharded(o.ref(), ptr(x), ptr(dx), ptr(J), len(x), o.s.m, nprocs)
    return J


def fd_hessian(o: Obj, x, dx):  # Objective::hessianApproximation, PNOL_Objective.cpp:38-85
    x = np.ascontiguousarray(x, dtype=np.float64); dx = np.ascontiguousarray(dx, dtype=np.float64)
    B = np.zeros((len(x), len(x)))
    lib().orc_fd_hessian(o.ref(), ptr(x), ptr(dx), ptr(B), len(x))
    return B


def fd_gradient_recur(o: Obj, xr, dxr, const_x, const_ind):  # PNOL_Objective.cpp:337-360
    xr = np.ascontiguousarray(xr, dtype=np.float64); dxr = np.ascontiguousarray(dxr, dtype=np.float64)
    cx = np.ascontiguousarray(const_x, dtype=np.float64)
    ci = np.ascontiguousarray(const_ind, dtype=np.uint8)
    g = np.zeros_like(xr)
    lib().orc_fd_gradient_recur(o.ref(), ptr(xr), ptr(dxr), ptr(g), len(xr), ptr(cx),
                                ci.ctypes.data_as(C.POINTER(C.c_ubyte)), len(cx))
    return g


def matvec(A, x):  # matrixVectorMultiply (utility restatement)
    A = np.ascontiguousarray(A, dtype=np.float64); x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.zeros(A.shape[0])
    lib().orc_util_matvec(ptr(A), ptr(x), ptr(y), A.shape[0], A.shape[1])
    return y


def matmul(A, B):
    A = np.ascontiguousarray(A, dtype=np.float64); B = np.ascontiguousarray(B, dtype=np.float64)
    Cm = np.zeros((A.shape[0], B.shape[1]))
    lib().orc_util_matmul(ptr(A), ptr(B), ptr(Cm), A.shape[0], A.shape[1], B.shape[1])
    return Cm


def lusolve(A, b):
    A = np.ascontiguousarray(A, dtype=np.float64); b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros_like(b)
    lib().orc_util_lusolve(ptr(A), ptr(b), ptr(x), len(b))
    return x


def matinv(A):  # matrixInverse (utility restatement): luSolve per unit column
    A = np.ascontiguousarray(A, dtype=np.float64)
    Ai = np.zeros_like(A)
    lib().orc_util_matinv(ptr(A), ptr(Ai), A.shape[0])
    return Ai


def update_hessian_inv(D, y, s):  # updateHessianInv, BFGS_with_linesearch.cpp:389-432
    D = np.array(D, dtype=np.float64, order="C")
    y = np.ascontiguousarray(y, dtype=np.float64); s = np.ascontiguousarray(s, dtype=np.float64)
    lib().orc_update_hessian_inv(ptr(D), ptr(y), ptr(s), len(y))
    return D


def update_hessian_inv_rank2(D, y, s):
    D = np.array(D, dtype=np.float64, order="C")
    y = np.ascontiguousarray(y, dtype=np.float64); s = np.ascontiguousarray(s, dtype=np.float64)
    lib().orc_update_hessian_inv_rank2(ptr(D), ptr(y), ptr(s), len(y))
    return D


def lm_step(J, F, lam):  # LevenbergMarquardt.cpp:59-83
    J = np.ascontiguousarray(J, dtype=np.float64); F = np.ascontiguousarray(F, dtype=np.float64)
    m, n = J.shape
    JTJ = np.zeros((n, n)); A = np.zeros((n, n)); rhs = np.zeros(n); sigma = np.zeros(n)
    lib().orc_lm_step(ptr(J), ptr(F), C.c_double(lam), m, n, ptr(JTJ), ptr(A), ptr(rhs), ptr(sigma))
    return JTJ, A, rhs, sigma


def bfgs_findmin(o: Obj, x0, params, trace_cap=0, rank2=False):  # BFGS::findMin
    """rank2: updateHessianInv in the O(n^2) rank-2 form (large n)."""
    X = np.array(x0, dtype=np.float64)
    prm = BFGSParams(*params)
    res = Result()
    tr = np.zeros((max(trace_cap, 1), len(X)))
    lib().orc_bfgs_findmin_ex(o.ref(), C.byref(prm), ptr(X), len(X), C.byref(res), ptr(tr), trace_cap, int(rank2))
    return X, res, tr[: min(res.iters, trace_cap)]


def bfgs_mpi_findmin(o: Obj, x0, params, nprocs):  # BFGS_MPI::findMin
    X = np.array(x0, dtype=np.float64)
    prm = BFGSMPIParams(*params)
    res = Result()
    lib().orc_bfgs_mpi_findmin(o.ref(), C.byref(prm), nprocs, ptr(X), len(X), C.byref(res))
    return X, res


def lm_findmin(o: Obj, x0, params, trace_cap=0):  # LevMarq::findMin
    X = np.array(x0, dtype=np.float64)
    m = o.s.m
    F0 = np.zeros(m); FOpt = np.zeros(m)
    prm = LMParams(*params)
    res = Result()
    tr = np.zeros((max(trace_cap, 1), len(X)))
    lib().orc_lm_findmin(o.ref(), C.byref(prm), ptr(X), len(X), ptr(F0), ptr(FOpt), m, C.byref(res),
                         ptr(tr), trace_cap)
    return X, res, F0, FOpt, tr[: min(res.iters + 1, trace_cap)]


_par = None


def lm_findmin_par(o: Obj, x0, params, trace_cap=0, threads=None):
    """LevMarq::findMin as lm_findmin, its FD columns, J^T J tiles and J^T F rows spread over
    OpenMP threads (pnol_oracle_par.c, liboracle_par.so): bitwise lm_findmin's results, plus X,
    chi^2 and lambda after every trip.  Returns (X, res, F0, FOpt, trace_x, trace_chi, trace_lambda)."""
    global _par
    if threads:
        os.environ["OMP_NUM_THREADS"] = str(threads)
    if _par is None:
        path = os.path.join(HERE, "liboracle_par.so")
        if not os.path.exists(path):
            build()
        _par = C.CDLL(path)
    X = np.array(x0, dtype=np.float64)
    m = o.s.m
    F0 = np.zeros(m); FOpt = np.zeros(m)
    prm = LMParams(*params)
    res = Result()
    cap = max(trace_cap, 1)
    tx, tc, tl = np.zeros((cap, len(X))), np.zeros(cap), np.zeros(cap)
    rc = _par.orc_lm_findmin_par(o.ref(), C.byref(prm), ptr(X), len(X), ptr(F0), ptr(FOpt), m, C.byref(res),
                                 ptr(tx), ptr(tc), ptr(tl), trace_cap)
    assert rc == 0
    k = min(res.iters + 1, trace_cap)
    return X, res, F0, FOpt, tx[:k], tc[:k], tl[:k]


def bfgs_bnd_findmin(o: Obj, x0, lb, ub, params):  # BFGS_Bnd::findMinBnd
    X = np.array(x0, dtype=np.float64)
    lb = np.ascontiguousarray(lb, dtype=np.float64); ub = np.ascontiguousarray(ub, dtype=np.float64)
    prm = BFGSBndParams(*params)
    res = Result()
    lib().orc_bfgs_bnd_findmin(o.ref(), C.byref(prm), ptr(X), ptr(lb), ptr(ub), len(X), C.byref(res))
    return X, res


def bfgs_bnd_findmin_ex(o: Obj, x0, lb, ub, params, rank2=False, trace_cap=0):
    """BFGS_Bnd::findMinBnd with the rank-2 update form (rank2) and an F trace; returns
    (X, res, ftrace, max recursion depth)."""
    X = np.array(x0, dtype=np.float64)
    lb = np.ascontiguousarray(lb, dtype=np.float64); ub = np.ascontiguousarray(ub, dtype=np.float64)
    prm = BFGSBndParams(*params)
    res = Result()
    tr = np.zeros(max(trace_cap, 1))
    depth = C.c_int()
    lib().orc_bfgs_bnd_findmin_ex(o.ref(), C.byref(prm), ptr(X), ptr(lb), ptr(ub), len(X), C.byref(res),
                                  int(rank2), ptr(tr), trace_cap, C.byref(depth))
    return X, res, tr[: min(res.iters, trace_cap)], depth.value


def bfgs_bnd_mpi_findmin(o: Obj, x0, lb, ub, params, npool, nprocs=None):  # BFGSBnd_MPI::findMinBnd
    """Returns (X, res, status); status -1 = a NaN/inf pool value (the reference's exit(0))."""
    X = np.array(x0, dtype=np.float64)
    lb = np.ascontiguousarray(lb, dtype=np.float64); ub = np.ascontiguousarray(ub, dtype=np.float64)
    prm = BFGSBndMPIParams(*params)
    res = Result()
    st = lib().orc_bfgs_bnd_mpi_findmin(o.ref(), C.byref(prm), npool, nprocs or npool, ptr(X), ptr(lb), ptr(ub),
                                        len(X), C.byref(res))
    return X, res, st


def bfgs_bnd_mpi_sw_findmin(o: Obj, x0, lb, ub, params, procs):  # BFGS_Bnd_MPI_SW::findMinBnd
    X = np.array(x0, dtype=np.float64)
    lb = np.ascontiguousarray(lb, dtype=np.float64); ub = np.ascontiguousarray(ub, dtype=np.float64)
    prm = BFGSBndParams(*params)
    res = Result()
    lib().orc_bfgs_bnd_mpi_sw_findmin(o.ref(), C.byref(prm), procs, ptr(X), ptr(lb), ptr(ub), len(X), C.byref(res))
    return X, res


def ga_findmin(o: Obj, x0, lb, ub, params, seed, nprocs=0):  # GeneticAlgorithm{,MPI}::findMinBnd
    """params: the first 9 setGAParams values (Npop ... NstaticGenerations); nprocs 0 = serial."""
    X = np.array(x0, dtype=np.float64)
    lb = np.ascontiguousarray(lb, dtype=np.float64); ub = np.ascontiguousarray(ub, dtype=np.float64)
    prm = np.ascontiguousarray(params[:9], dtype=np.float64)
    res = Result()
    st = lib().orc_ga_findmin(o.ref(), ptr(prm), C.c_ulonglong(seed), nprocs, ptr(X), ptr(lb), ptr(ub), len(X),
                              C.byref(res))
    return X, res, st


def check_alpha_pool_bnd(pool, x, lb, ub, p):  # checkAlphaPoolBnd, BFGS_with_bnd_linsearch_MPI.cpp:711-743
    ap = np.array(pool, dtype=np.float64)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (x, lb, ub, p)]
    bnd = C.c_int()
    lib().orc_check_alpha_pool_bnd(C.byref(bnd), ptr(ap), len(ap), *[ptr(a) for a in arrs], len(arrs[0]))
    return bool(bnd.value), ap


def compute_alpha_bnd(x, lb, ub, p):  # computeAlphaBnd, BFGS_with_bnd_linsearch_MPI.cpp:665-708
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (x, lb, ub, p)]
    return lib().orc_compute_alpha_bnd(*[ptr(a) for a in arrs], len(arrs[0]))
