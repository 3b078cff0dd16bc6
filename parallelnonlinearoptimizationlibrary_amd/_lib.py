"""ctypes binding of libpnol_amd.so (the C ABI declared in include/pnol_amd.h).

This is plumbing for tests and bench.py: the product is the HIP library and its C++ drop-in
classes.  Loading fails loudly when the library has not been built; calls that need a GPU
return PNOL_ERR_NODEVICE (raised as PnolError) when no gfx950 device is visible -- there is
no CPU fallback anywhere on this path.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# PNOL_AMD_LIB: an A/B build of the same library (tools/ab_lib.sh); default the in-tree build
LIB_PATH = os.environ.get("PNOL_AMD_LIB") or os.path.join(HERE, "libpnol_amd.so")

PNOL_OK, PNOL_ERR_ARG, PNOL_ERR_HIP, PNOL_ERR_NOMEM, PNOL_ERR_NODEVICE = 0, 1, 2, 3, 4
PNOL_ERR_SINGULAR, PNOL_ERR_COMM, PNOL_ERR_UNSUPPORTED, PNOL_ERR_TIMEOUT = 5, 6, 7, 8
PNOL_SEQ_MAX = 64
LM_SLICES = 8          # PNOL_LM_SLICES: m-slices of the LevMarqMPI J^T J / J^T F summation tree

OBJ_ROSENBROCK, OBJ_POWER, OBJ_QUADRATIC = 0, 1, 4
OBJ_EXPCURVE, OBJ_CUBIC, OBJ_LINRES = 10, 11, 12

_vp = C.c_void_p
_i = C.c_int
_d = C.c_double
_sz = C.c_size_t
_dp = C.POINTER(C.c_double)


class PnolError(RuntimeError):
    def __init__(self, status: int, what: str):
        super().__init__(f"{what}: {status_string(status)} (status {status})")
        self.status = status


class Result(C.Structure):
    _fields_ = [("iters", C.c_int), ("evals", C.c_long), ("f0", C.c_double), ("fopt", C.c_double)]


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, _vp, _vp, _sz, _vp)
HOST_MULTI_FN = C.CFUNCTYPE(None, _dp, C.c_int, _dp, C.c_int, _vp)
HOST_SCALAR_FN = C.CFUNCTYPE(C.c_double, _dp, C.c_int, _vp)

# name -> (restype, argtypes)
_SIGS = {
    "pnol_status_string": (C.c_char_p, [_i]),
    "pnol_version": (_i, []),
    "pnol_device_count": (_i, [C.POINTER(_i)]),
    "pnol_ctx_create": (_i, [_i, C.POINTER(_vp)]),
    "pnol_ctx_destroy": (_i, [_vp]),
    "pnol_ctx_synchronize": (_i, [_vp]),
    "pnol_ctx_get_stream": (_i, [_vp, C.POINTER(_vp)]),
    "pnol_ctx_set_stream": (_i, [_vp, _vp]),
    "pnol_ctx_device": (_i, [_vp, C.POINTER(_i)]),
    "pnol_default_ctx": (_i, [C.POINTER(_vp)]),
    "pnol_ctx_enable_timers": (_i, [_vp, _i]),
    "pnol_ctx_reset_timers": (_i, [_vp]),
    "pnol_ctx_timer": (_i, [_vp, C.c_char_p, C.POINTER(_d), C.POINTER(_i)]),
    "pnol_malloc": (_i, [_vp, _sz, C.POINTER(_vp)]),
    "pnol_free": (_i, [_vp, _vp]),
    "pnol_memcpy_h2d": (_i, [_vp, _vp, _vp, _sz]),
    "pnol_memcpy_d2h": (_i, [_vp, _vp, _vp, _sz]),
    "pnol_host_alloc": (_i, [C.POINTER(_vp), _sz]),
    "pnol_host_free": (_i, [_vp]),
    "pnol_memcpy_d2h_async": (_i, [_vp, _vp, _vp, _sz]),
    "pnol_event_create": (_i, [_vp, C.POINTER(_vp)]),
    "pnol_event_record": (_i, [_vp, _vp]),
    "pnol_event_wait": (_i, [_vp]),
    "pnol_event_destroy": (_i, [_vp]),
    "pnol_hg_d": (_i, [_vp, _vp, _i, _vp, _vp, _i]),
    "pnol_gemv_neg_d": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp]),
    "pnol_bfgs_update_exact_d": (_i, [_vp, _vp, _i, _vp, _vp, _i]),
    "pnol_bfgs_pass_d": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "pnol_set_identity_d": (_i, [_vp, _vp, _i, _i, _vp]),
    "pnol_bfgs_pass_ident_d": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "pnol_bfgs_pass_ident_mpi_d": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "pnol_bfgs_rows": (_i, [_i, _i, _i, C.POINTER(_i), C.POINTER(_i)]),
    "pnol_bfgs_pass_part_tiles": (_i, [_i, _i]),
    "pnol_set_identity_rows_d": (_i, [_vp, _vp, _i, _i, _vp]),
    "pnol_hg_mpi_d": (_i, [_vp, _vp, _i, _vp, _vp, _i]),
    "pnol_bfgs_pass_mpi_d": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "pnol_gather_submatrix_d": (_i, [_vp, _vp, _i, _i, _vp, _i, _vp, _i]),
    "pnol_gather_submatrix_mpi_d": (_i, [_vp, _vp, _i, _i, _vp, _i, _vp, _i]),
    "pnol_jtj_d": (_i, [_vp, _vp, _i, _i, _i, _d, _vp, _i, _vp]),
    "pnol_jtj_mpi_d": (_i, [_vp, _vp, _i, _i, _i, _d, _vp, _i, _vp]),
    "pnol_lm_sliced_layout": (_i, [_i, _i, C.POINTER(_i), C.POINTER(_sz)]),
    "pnol_lm_jacobian_mpi_d": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp]),
    "pnol_lm_eval_mpi_d": (_i, [_vp, _vp, _vp, _vp]),
    "pnol_lm_normal_mpi_d": (_i, [_vp, _vp, _i, _i, _d, _vp, _vp, _i, _vp, _vp]),
    "pnol_lm_normal_solve_mpi_d": (_i, [_vp, _vp, _i, _i, _d, _vp, _vp, _vp, _vp, _vp, _vp]),
    "pnol_lm_normal_unpack_mpi_d": (_i, [_vp, _i, _i, _d, _vp, _i]),
    "pnol_lm_agree_status_d": (_i, [_vp, _vp]),
    "pnol_lm_set_fd_mode": (_i, [_vp, _i]),
    "pnol_lm_fd_mode": (_i, [_vp, C.POINTER(C.c_int)]),
    "pnol_lm_rank_rows": (_i, [_i, _i, _i, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "pnol_jtr_d": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp]),
    "pnol_solve_d": (_i, [_vp, _vp, _i, _vp, _vp, _i, _i, C.POINTER(_i)]),
    "pnol_solve_async_d": (_i, [_vp, _vp, _i, _vp, _vp, _i, _vp]),
    "pnol_solve_step_d": (_i, [_vp, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp]),
    "pnol_matrix_inverse_d": (_i, [_vp, _vp, _i, _i, _vp, _i, C.POINTER(_i)]),
    "pnol_add_d": (_i, [_vp, _vp, _vp, _vp, _i]),
    "pnol_dobj_create": (_i, [_vp, _i, _i, _i, _dp, _sz, _dp, _sz, _d, C.POINTER(_vp)]),
    "pnol_dobj_create_synthetic": (_i, [_vp, _i, _i, _i, C.c_ulonglong, _d, _dp, C.POINTER(_vp)]),
    "pnol_dobj_destroy": (_i, [_vp]),
    "pnol_dobj_info": (_i, [_vp, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i)]),
    "pnol_dobj_eval_d": (_i, [_vp, _vp, _vp, _vp]),
    "pnol_dobj_eval_ckpt_d": (_i, [_vp, _vp, _vp, _vp]),
    "pnol_fd_gradient_d": (_i, [_vp, _vp, _vp, _vp, _i, _i, _vp, _vp]),
    "pnol_fd_gradient": (_i, [_vp, _vp, _dp, _dp, _i, _i, _dp, _dp]),
    "pnol_dobj_eval_batch": (_i, [_vp, _vp, _dp, _i, _dp]),
    "pnol_fd_jacobian_d": (_i, [_vp, _vp, _vp, _vp, _i, _i, _vp, _i, _vp, _i]),
    "pnol_fd_jtj_d": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp, _i, _d, _vp, _i, _vp, _i]),
    "pnol_fd_normal_d": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp, _i, _d, _vp, _i, _vp, _vp]),
    "pnol_lm_trip_d": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp, _i, _d, _vp, _vp, _vp, _vp]),
    "pnol_lm_trip_normal_d": (_i, [_vp, _i, _i, _d, _vp, _i]),
    "pnol_fd_jacobian_tiles_d": (_i, [_vp, _vp, _vp, _vp, C.POINTER(_i), C.POINTER(_i), _i, _vp, _i, _vp, _i]),
    "pnol_comm_unique_id": (_i, [C.c_char_p]),
    "pnol_comm_init_rccl": (_i, [_vp, _i, _i, C.c_char_p]),
    "pnol_comm_init_host": (_i, [_i, _i, ALLGATHER_FN, _vp]),
    "pnol_comm_finalize": (_i, []),
    "pnol_comm_size": (_i, [C.POINTER(_i), C.POINTER(_i)]),
    "pnol_comm_set_launcher_hook": (_i, [_vp]),
    "pnol_comm_bind_launcher": (_i, []),
    "pnol_launcher_world_size": (_i, []),
    "pnol_set_default_device": (_i, [_i]),
    "pnol_comm_allgather_d": (_i, [_vp, _vp, _vp, _sz]),
    "pnol_block_range": (None, [_i, _i, _i, C.POINTER(_i), C.POINTER(_i)]),
    "pnol_fd_tiles": (_i, [_i, _i, _i, C.POINTER(_i), C.POINTER(_i), _i]),
    "pnol_comm_share_fd_rows_d": (_i, [_vp, _vp, _i, _i]),
    "pnol_run_bfgs": (_i, [_i, _vp, _i, _dp, _i, _dp, _i, _dp, _dp, C.POINTER(Result)]),
    "pnol_run_bfgs_ex": (_i, [_i, _vp, _i, _dp, _i, _dp, _i, _dp, _dp, C.POINTER(Result), _dp, _i, C.POINTER(_i),
                              _dp]),
    "pnol_run_levmarq": (_i, [_i, _vp, _i, _dp, _dp, _i, _dp, _dp, _i, C.POINTER(Result)]),
    "pnol_run_levmarq_ex": (_i, [_i, _vp, _i, _dp, _dp, _i, _dp, _dp, _i, C.POINTER(Result), C.POINTER(_i)]),
    "pnol_run_ga": (_i, [_i, _vp, _i, _dp, _i, C.c_ulonglong, _dp, _i, _dp, _dp, C.POINTER(Result)]),
    "pnol_host_fd_hessian": (_i, [HOST_SCALAR_FN, _vp, _dp, _dp, _i, _dp]),
    "pnol_host_fd_jacobian": (_i, [HOST_MULTI_FN, _vp, _dp, _dp, _i, _i, _i, _dp]),
    "pnol_host_run_ga": (_i, [_i, HOST_SCALAR_FN, _vp, _dp, _i, C.c_ulonglong, _dp, _i, _dp, _dp,
                              C.POINTER(Result)]),
}

_lib = None


def declared_symbols():
    """Every entry point include/pnol_amd.h declares (the binding covers all of them)."""
    return sorted(_SIGS)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with __graft_entry__.build() or "
                "`make -C parallelnonlinearoptimizationlibrary_amd/csrc` (hipcc, gfx950). "
                "The HIP path has no CPU fallback.")
        # torch ships its own libamdhip64.so.7; whichever copy is loaded first owns the SONAME
        # for the whole process.  Load torch's first so torch and this library share one HIP
        # runtime (loading /opt/rocm's first leaves torch with "No HIP GPUs are available").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def status_string(status: int) -> str:
    return lib().pnol_status_string(status).decode()


def check(status: int, what: str) -> None:
    if status != PNOL_OK:
        raise PnolError(status, what)


def device_count() -> int:
    c = C.c_int(0)
    check(lib().pnol_device_count(C.byref(c)), "pnol_device_count")
    return c.value


def fd_tiles(ncols: int, nranks: int, rank: int):
    """The cost-balanced FD column tiles of `rank`: [(start, count), ...] (pnol_fd_tiles)."""
    cap = ncols // 1 + 1
    st, ct = (C.c_int * cap)(), (C.c_int * cap)()
    k = lib().pnol_fd_tiles(ncols, nranks, rank, st, ct, cap)
    if k < 0:
        raise PnolError(-k, "pnol_fd_tiles")
    return [(st[i], ct[i]) for i in range(k)]


def block_range(ncols: int, nranks: int, rank: int):
    b, n = C.c_int(), C.c_int()
    lib().pnol_block_range(ncols, nranks, rank, C.byref(b), C.byref(n))
    return b.value, n.value
