"""Torch-facing wrappers over the C ABI (device buffers are torch float64 CUDA tensors).

PyTorch supplies device memory and the stream (the context runs on torch's current stream,
so launches are ordered with torch ops); every kernel is the library's own HIP code.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def _ptr(t) -> C.c_void_p:
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Context:
    """One GPU (pnol_ctx) bound to torch's current stream on that device."""

    def __init__(self, device: int = 0, use_torch_stream: bool = True):
        import torch
        self.torch = torch
        self.device = device
        h = C.c_void_p()
        L.check(L.lib().pnol_ctx_create(device, C.byref(h)), "pnol_ctx_create")
        self.h = h
        if use_torch_stream:
            # A dedicated torch stream made current: torch ops and this library's launches are
            # ordered on one real stream (the legacy null stream has handle 0, which the C ABI
            # reads as "use the context's own stream").
            with torch.cuda.device(device):
                self.tstream = torch.cuda.Stream(device)
                torch.cuda.set_stream(self.tstream)
                s = self.tstream.cuda_stream
            L.check(L.lib().pnol_ctx_set_stream(self.h, C.c_void_p(s)), "pnol_ctx_set_stream")

    def close(self):
        if self.h:
            L.lib().pnol_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        L.check(L.lib().pnol_ctx_synchronize(self.h), "pnol_ctx_synchronize")

    def stream(self) -> int:
        s = C.c_void_p()
        L.check(L.lib().pnol_ctx_get_stream(self.h, C.byref(s)), "pnol_ctx_get_stream")
        return s.value or 0

    # ---- tensors ------------------------------------------------------------------
    def empty(self, *shape):
        return self.torch.empty(*shape, dtype=self.torch.float64, device=f"cuda:{self.device}")

    def tensor(self, a):
        return self.torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64)).to(f"cuda:{self.device}")

    # ---- kernels ------------------------------------------------------------------
    def hg(self, D, g, p=None):
        """p = -D g (BFGS_with_linesearch.cpp:78-79)."""
        n = g.numel()
        p = self.empty(n) if p is None else p
        L.check(L.lib().pnol_hg_d(self.h, _ptr(D), D.stride(0), _ptr(g), _ptr(p), n), "pnol_hg_d")
        return p

    def gemv_neg(self, A, x, y=None):
        rows, cols = A.shape
        y = self.empty(rows) if y is None else y
        L.check(L.lib().pnol_gemv_neg_d(self.h, _ptr(A), A.stride(0), rows, cols, _ptr(x), _ptr(y)), "pnol_gemv_neg_d")
        return y

    def bfgs_update_exact(self, D, y, s):
        L.check(L.lib().pnol_bfgs_update_exact_d(self.h, _ptr(D), D.stride(0), _ptr(y), _ptr(s), y.numel()),
                "pnol_bfgs_update_exact_d")
        return D

    def bfgs_pass(self, D, y=None, g=None, pending=None, write_back=False):
        """One streaming pass; returns (u, w, v) = (Dc y, Dc^T y, Dc g)."""
        n = D.shape[0]
        u, w, v = self.empty(n), self.empty(n), self.empty(n)
        sp, ap, bp = pending if pending is not None else (None, None, None)
        L.check(L.lib().pnol_bfgs_pass_d(self.h, _ptr(D), D.stride(0), n, _ptr(sp), _ptr(ap), _ptr(bp),
                                         int(write_back), _ptr(y), _ptr(g), _ptr(u), _ptr(w), _ptr(v)),
                "pnol_bfgs_pass_d")
        return u, w, v

    def set_identity(self, D, scale=None):
        L.check(L.lib().pnol_set_identity_d(self.h, _ptr(D), D.stride(0), D.shape[0], _ptr(scale)),
                "pnol_set_identity_d")
        return D

    def jtj(self, JT, lam, A=None, want_diag=False):
        """A = J^T J with A_ii *= (1+lam); JT is n x m (one FD column per row)."""
        n, m = JT.shape
        A = self.empty(n, n) if A is None else A
        diag = self.empty(n) if want_diag else None
        L.check(L.lib().pnol_jtj_d(self.h, _ptr(JT), JT.stride(0), m, n, C.c_double(lam), _ptr(A), A.stride(0),
                                   _ptr(diag)), "pnol_jtj_d")
        return (A, diag) if want_diag else A

    def jtr(self, JT, F, rhs=None):
        n, m = JT.shape
        rhs = self.empty(n) if rhs is None else rhs
        L.check(L.lib().pnol_jtr_d(self.h, _ptr(JT), JT.stride(0), m, n, _ptr(F), _ptr(rhs)), "pnol_jtr_d")
        return rhs

    def lm_normal_mpi(self, JTs, m, n, lam, F, A=None, rhs=None, want_diag=False):
        """LevMarqMPI normal equations from this rank's slices of the m-sliced J^T (layout
        lm_sliced_layout): A = J^T J with A_ii *= (1+lam), rhs = -J^T F, on every rank."""
        A = self.empty(n, n) if A is None else A
        rhs = self.empty(n) if rhs is None else rhs
        diag = self.empty(n) if want_diag else None
        L.check(L.lib().pnol_lm_normal_mpi_d(self.h, _ptr(JTs), m, n, C.c_double(lam), _ptr(F), _ptr(A), A.stride(0),
                                             _ptr(rhs), _ptr(diag)), "pnol_lm_normal_mpi_d")
        return (A, rhs, diag) if want_diag else (A, rhs)

    def lm_normal_solve_mpi(self, JTs, m, n, lam, F, x):
        """pnol_lm_normal_solve_mpi_d: rhs, sigma, x + sigma and the solve status (read back)
        without forming A; lm_normal_unpack_mpi forms A from the same tiles afterwards."""
        rhs, sigma, xnext = self.empty(n), self.empty(n), self.empty(n)
        info = self.torch.zeros(2, dtype=self.torch.int32, device=f"cuda:{self.device}")
        L.check(L.lib().pnol_lm_normal_solve_mpi_d(self.h, _ptr(JTs), m, n, C.c_double(lam), _ptr(F), _ptr(rhs),
                                                   _ptr(sigma), _ptr(info), _ptr(x), _ptr(xnext)),
                "pnol_lm_normal_solve_mpi_d")
        return rhs, sigma, xnext, int(info[0].item())

    def lm_normal_unpack_mpi(self, m, n, lam, A=None):
        A = self.empty(n, n) if A is None else A
        L.check(L.lib().pnol_lm_normal_unpack_mpi_d(self.h, m, n, C.c_double(lam), _ptr(A), A.stride(0)),
                "pnol_lm_normal_unpack_mpi_d")
        return A

    def set_lm_fd_mode(self, mode):
        """LevMarqMPI's FD decomposition on this context: 0 columns (default), 1 rows, -1 env."""
        L.check(L.lib().pnol_lm_set_fd_mode(self.h, int(mode)), "pnol_lm_set_fd_mode")

    def lm_fd_mode(self):
        v = C.c_int()
        L.check(L.lib().pnol_lm_fd_mode(self.h, C.byref(v)), "pnol_lm_fd_mode")
        return v.value

    def solve_step(self, A, rhs, x):
        """The LM loop's solve (pnol_solve_step_d): sigma = A^{-1} rhs by the tile Cholesky (A kept)
        and xnext = x + sigma.  Returns (sigma, xnext, info) -- info read back (synchronises)."""
        n = rhs.numel()
        sigma, xnext = self.empty(n), self.empty(n)
        info = self.torch.zeros(2, dtype=self.torch.int32, device=f"cuda:{self.device}")
        L.check(L.lib().pnol_solve_step_d(self.h, _ptr(A), A.stride(0), _ptr(rhs), _ptr(sigma), n, _ptr(info),
                                          _ptr(x), _ptr(xnext)), "pnol_solve_step_d")
        return sigma, xnext, int(info[0].item())

    def lm_trip_normal(self, m, n, lam, A=None):
        """A = J^T J + Marquardt diagonal from the last LM trip's partials (pnol_lm_trip_normal_d)."""
        A = self.empty(n, n) if A is None else A
        L.check(L.lib().pnol_lm_trip_normal_d(self.h, m, n, C.c_double(lam), _ptr(A), A.stride(0)),
                "pnol_lm_trip_normal_d")
        return A

    def solve(self, A, rhs, method=0):
        """sigma = A^{-1} rhs; A is overwritten.  Returns (sigma, info)."""
        n = rhs.numel()
        sigma = self.empty(n)
        info = C.c_int(0)
        L.check(L.lib().pnol_solve_d(self.h, _ptr(A), A.stride(0), _ptr(rhs), _ptr(sigma), n, method,
                                     C.byref(info)), "pnol_solve_d")
        return sigma, info.value


class DeviceObjective:
    """A pnol_dobj: a built-in objective whose FD batches run on the device."""

    def __init__(self, ctx: Context, kind: int, n: int, m: int = 0, p0=None, p1=None, power: float = 2.0,
                 handle=None):
        self.ctx, self.kind, self.n, self.m = ctx, kind, n, m
        if handle is not None:
            self.h = handle
            return
        a0 = None if p0 is None else np.ascontiguousarray(p0, dtype=np.float64).ravel()
        a1 = None if p1 is None else np.ascontiguousarray(p1, dtype=np.float64).ravel()
        h = C.c_void_p()
        L.check(L.lib().pnol_dobj_create(ctx.h, kind, n, m, _dptr(a0) if a0 is not None else None,
                                         0 if a0 is None else a0.size, _dptr(a1) if a1 is not None else None,
                                         0 if a1 is None else a1.size, C.c_double(power), C.byref(h)),
                "pnol_dobj_create")
        self.h = h

    @classmethod
    def synthetic(cls, ctx: Context, kind: int, n: int, m: int = 0, seed: int = 0x5EED2018, bscale: float = 1.0):
        h = C.c_void_p()
        xs = np.zeros(n)
        L.check(L.lib().pnol_dobj_create_synthetic(ctx.h, kind, n, m, C.c_ulonglong(seed), C.c_double(bscale),
                                                   _dptr(xs), C.byref(h)), "pnol_dobj_create_synthetic")
        o = cls(ctx, kind, n, m, handle=h)
        o.xstar = xs
        return o

    def close(self):
        if getattr(self, "h", None):
            L.lib().pnol_dobj_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def eval(self, x):
        out = self.ctx.empty(self.m if self.m else 1)
        L.check(L.lib().pnol_dobj_eval_d(self.ctx.h, self.h, _ptr(x), _ptr(out)), "pnol_dobj_eval_d")
        return out

    def eval_ckpt(self, x, out=None):
        """F(x), keeping a linear residual's prefix checkpoints of x for a compute_f0=2 FD call."""
        out = self.ctx.empty(self.m if self.m else 1) if out is None else out
        L.check(L.lib().pnol_dobj_eval_ckpt_d(self.ctx.h, self.h, _ptr(x), _ptr(out)), "pnol_dobj_eval_ckpt_d")
        return out

    def fd_gradient(self, x, h, i0=0, cnt=None):
        cnt = self.n - i0 if cnt is None else cnt
        f0, g = self.ctx.empty(1), self.ctx.empty(max(cnt, 1))
        L.check(L.lib().pnol_fd_gradient_d(self.ctx.h, self.h, _ptr(x), _ptr(h), i0, cnt, _ptr(f0), _ptr(g)),
                "pnol_fd_gradient_d")
        return f0, g[:cnt]

    def fd_jacobian(self, x, h, j0=0, cnt=None, JT=None, F0=None, compute_f0=True):
        """JT rows = FD columns j0..j0+cnt; returns (F0, JT)."""
        cnt = self.n - j0 if cnt is None else cnt
        JT = self.ctx.empty(max(cnt, 1), self.m) if JT is None else JT
        F0 = self.ctx.empty(self.m) if F0 is None else F0
        L.check(L.lib().pnol_fd_jacobian_d(self.ctx.h, self.h, _ptr(x), _ptr(h), j0, cnt, _ptr(F0),
                                           int(compute_f0), _ptr(JT), JT.stride(0)), "pnol_fd_jacobian_d")
        return F0, JT


    def fd_jtj(self, x, h, lam, JT, A, F0=None, compute_f0=True, nchunks=4, want_diag=False):
        """Pipelined FD Jacobian (all columns) + A = J^T J with the Marquardt diagonal."""
        F0 = self.ctx.empty(self.m) if F0 is None else F0
        diag = self.ctx.empty(self.n) if want_diag else None
        L.check(L.lib().pnol_fd_jtj_d(self.ctx.h, self.h, _ptr(x), _ptr(h), _ptr(F0), int(compute_f0), _ptr(JT),
                                      JT.stride(0), C.c_double(lam), _ptr(A), A.stride(0), _ptr(diag), nchunks),
                "pnol_fd_jtj_d")
        return (F0, JT, A, diag) if want_diag else (F0, JT, A)

    def fd_normal(self, x, h, lam, JT, A, rhs, F0=None, compute_f0=True):
        """FD Jacobian + A (Marquardt diagonal) + rhs = -J^T F0 in one queue (pnol_fd_normal_d)."""
        F0 = self.ctx.empty(self.m) if F0 is None else F0
        L.check(L.lib().pnol_fd_normal_d(self.ctx.h, self.h, _ptr(x), _ptr(h), _ptr(F0), int(compute_f0), _ptr(JT),
                                         JT.stride(0), C.c_double(lam), _ptr(A), A.stride(0), None, _ptr(rhs)),
                "pnol_fd_normal_d")
        return F0, JT, A, rhs

    def lm_trip(self, x, h, lam, JT, F0=None, compute_f0=True):
        """One LM trip's linear algebra without forming A (pnol_lm_trip_d).
        Returns (F0, JT, rhs, sigma, xnext, info) -- info read back (synchronises)."""
        t = self.ctx.torch
        F0 = self.ctx.empty(self.m) if F0 is None else F0
        rhs, sigma, xnext = self.ctx.empty(self.n), self.ctx.empty(self.n), self.ctx.empty(self.n)
        info = t.zeros(2, dtype=t.int32, device=f"cuda:{self.ctx.device}")
        L.check(L.lib().pnol_lm_trip_d(self.ctx.h, self.h, _ptr(x), _ptr(h), _ptr(F0), int(compute_f0), _ptr(JT),
                                       JT.stride(0), C.c_double(lam), _ptr(rhs), _ptr(sigma), _ptr(info), _ptr(xnext)),
                "pnol_lm_trip_d")
        return F0, JT, rhs, sigma, xnext, int(info[0].item())

    def lm_jacobian_mpi(self, x, h, JTs=None, F0=None, compute_f0=True):
        """The m-sliced J^T this rank's share of the normal equations reads (pnol_lm_jacobian_mpi_d).
        Columns mode (default): this rank's FD tiles for all rows, each tile's m-slices sent to
        the slices' ranks; F0 (when computed) holds all m residuals.  Rows mode
        (Context.set_lm_fd_mode(1)): every FD column on this rank's own m-slices, no exchange;
        F0 then holds only this rank's rows (lm_rank_rows), the other rows read as zero."""
        if JTs is None:
            JTs = self.ctx.empty(lm_sliced_layout(self.m, self.n)[1])
        F0 = self.ctx.torch.zeros(self.m, dtype=self.ctx.torch.float64, device=f"cuda:{self.ctx.device}") \
            if F0 is None else F0
        L.check(L.lib().pnol_lm_jacobian_mpi_d(self.ctx.h, self.h, _ptr(x), _ptr(h), _ptr(F0), int(compute_f0),
                                               _ptr(JTs)), "pnol_lm_jacobian_mpi_d")
        return F0, JTs

    def fd_jacobian_tiles(self, x, h, tiles, JT, F0=None, compute_f0=True):
        """FD rows of the (start, count) tiles into JT (row c = column c); returns (F0, JT)."""
        F0 = self.ctx.empty(self.m) if F0 is None else F0
        k = len(tiles)
        st = (C.c_int * max(k, 1))(*[t[0] for t in tiles])
        ct = (C.c_int * max(k, 1))(*[t[1] for t in tiles])
        L.check(L.lib().pnol_fd_jacobian_tiles_d(self.ctx.h, self.h, _ptr(x), _ptr(h), st, ct, k, _ptr(F0),
                                                 int(compute_f0), _ptr(JT), JT.stride(0)),
                "pnol_fd_jacobian_tiles_d")
        return F0, JT


def lm_rank_rows(m, nranks, rank):
    """Residual rows [r0, r1) held by `rank` of `nranks` (its m-slices; rows mode's F0 rows)."""
    r0, r1 = C.c_int(), C.c_int()
    L.check(L.lib().pnol_lm_rank_rows(m, nranks, rank, C.byref(r0), C.byref(r1)), "pnol_lm_rank_rows")
    return r0.value, r1.value


def lm_sliced_layout(m, n):
    """(slice_rows, number of doubles) of the m-sliced J^T: slice s = rows [s*mS, (s+1)*mS) of J,
    an n x mS row-major block at offset s*n*mS."""
    mS, tot = C.c_int(), C.c_size_t()
    L.check(L.lib().pnol_lm_sliced_layout(m, n, C.byref(mS), C.byref(tot)), "pnol_lm_sliced_layout")
    return mS.value, tot.value


def to_sliced(JT, mS):
    """numpy n x m J^T -> the sliced layout (PNOL_LM_SLICES blocks of n x mS, zero padded)."""
    n, m = JT.shape
    out = np.zeros((L.LM_SLICES, n, mS))
    for s in range(L.LM_SLICES):
        blk = JT[:, s * mS:(s + 1) * mS]
        out[s, :, :blk.shape[1]] = blk
    return out


PROFILE_KEYS = ("iterations", "total_s", "fd_gradient_s", "line_search_s", "update_s", "line_search_points",
                "gradient_calls", "max_recursion_depth")


def run_bfgs(obj: DeviceObjective, x0, params, which=0, host_eval=False, lb=None, ub=None, trace_cap=0,
             profile=None):
    """Run the C++ drop-in BFGS (0), BFGS_MPI (1), BFGS_Bnd (2), BFGSBnd_MPI (3) or
    BFGS_Bnd_MPI_SW (4) on a device objective.  Returns (X, result), plus BFGS_Bnd's F after
    every iteration (numpy array) when trace_cap > 0.  A dict passed as `profile` receives the
    per-phase times and counts (PROFILE_KEYS)."""
    X = np.array(x0, dtype=np.float64)
    p = np.array(params, dtype=np.float64)
    res = L.Result()
    lba = np.ascontiguousarray(lb, dtype=np.float64) if lb is not None else None
    uba = np.ascontiguousarray(ub, dtype=np.float64) if ub is not None else None
    tr = np.zeros(max(trace_cap, 1))
    nt = C.c_int(0)
    prof = np.zeros(8)
    L.check(L.lib().pnol_run_bfgs_ex(which, obj.h, int(host_eval), _dptr(p), p.size, _dptr(X), X.size,
                                     _dptr(lba) if lba is not None else None,
                                     _dptr(uba) if uba is not None else None, C.byref(res),
                                     _dptr(tr) if trace_cap > 0 else None, trace_cap, C.byref(nt),
                                     _dptr(prof) if profile is not None else None), "pnol_run_bfgs")
    if profile is not None:
        profile.update(zip(PROFILE_KEYS, prof.tolist()))
    if trace_cap > 0:
        return X, res, tr[: min(nt.value, trace_cap)]
    return X, res


def run_ga(obj: DeviceObjective, x0, lb, ub, params, seed, which=0, host_eval=False):
    """Run the C++ drop-in GeneticAlgorithm (0) or GeneticAlgorithmMPI (1) on a scalar device
    objective with a fixed selection / mutation stream; params = setGAParams without graph (10
    values).  Returns (X, result); result.iters = generations."""
    X = np.array(x0, dtype=np.float64)
    p = np.array(params, dtype=np.float64)
    lba = np.ascontiguousarray(lb, dtype=np.float64)
    uba = np.ascontiguousarray(ub, dtype=np.float64)
    res = L.Result()
    L.check(L.lib().pnol_run_ga(which, obj.h, int(host_eval), _dptr(p), p.size, seed, _dptr(X), X.size, _dptr(lba),
                                _dptr(uba), C.byref(res)), "pnol_run_ga")
    return X, res


def run_levmarq(obj: DeviceObjective, x0, params, which=0, host_eval=False):
    """Run the C++ drop-in LevMarq (0) or LevMarqMPI (1); returns (X, F0, FOpt, result)."""
    X = np.array(x0, dtype=np.float64)
    p = np.array(params, dtype=np.float64)
    F0, FO = np.zeros(obj.m), np.zeros(obj.m)
    res = L.Result()
    L.check(L.lib().pnol_run_levmarq(which, obj.h, int(host_eval), _dptr(p), _dptr(X), X.size, _dptr(F0), _dptr(FO),
                                     obj.m, C.byref(res)), "pnol_run_levmarq")
    return X, F0, FO, res
