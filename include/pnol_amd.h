/*
 * pnol_amd.h -- C ABI of the MI355X-native PNOL hot path (libpnol_amd.so).
 *
 * Plain pointers, sizes and int status codes; no exceptions and no torch/HIP types cross
 * this boundary.  Functions suffixed _d take DEVICE pointers (allocated with pnol_malloc or
 * any hipMalloc'd / torch CUDA buffer on the context's device) and enqueue on the context's
 * stream; call pnol_ctx_synchronize before reading results on the host.  Functions without
 * the suffix take HOST pointers and return after the result is on the host.
 *
 * Each entry point names the reference code it replaces (paths relative to
 * briandaniel/ParallelNonlinearOptimizationLibrary/Source).  The C++ drop-in classes in
 * include/ headers (BFGS, BFGS_MPI, BFGS_Bnd, LevMarq, LevMarqMPI) are built on these.
 */
#ifndef PNOL_AMD_H_
#define PNOL_AMD_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNOL_AMD_VERSION 100 /* 1.0.0 */

enum pnol_status {
    PNOL_OK = 0,
    PNOL_ERR_ARG = 1,        /* bad argument (null pointer, n <= 0, ld < n, misaligned) */
    PNOL_ERR_HIP = 2,        /* a HIP runtime call failed */
    PNOL_ERR_NOMEM = 3,
    PNOL_ERR_NODEVICE = 4,   /* no MI355X (gfx950) visible: the product path has no CPU fallback */
    PNOL_ERR_SINGULAR = 5,   /* zero pivot in the damped solve */
    PNOL_ERR_COMM = 6,       /* collective failed / communicator not initialised */
    PNOL_ERR_UNSUPPORTED = 7,
    PNOL_ERR_TIMEOUT = 8     /* a device dependency wait of the tile Cholesky ran past its cap on
                                every relaunch (a scheduling fault; never mapped to the LU) */
};

typedef struct pnol_ctx pnol_ctx;   /* one GPU: device, stream, workspace, communicator */
typedef struct pnol_dobj pnol_dobj; /* device-resident objective (batched FD evaluation) */

const char* pnol_status_string(int status);
int pnol_version(void);
int pnol_device_count(int* count);              /* gfx950 devices visible to this process */

/* ---- context ---------------------------------------------------------------------- */
int pnol_ctx_create(int device, pnol_ctx** out);
int pnol_ctx_destroy(pnol_ctx* ctx);
int pnol_ctx_synchronize(pnol_ctx* ctx);
int pnol_ctx_get_stream(pnol_ctx* ctx, void** hip_stream);  /* hipStream_t, for interop timing */
int pnol_ctx_set_stream(pnol_ctx* ctx, void* hip_stream);   /* run on a caller-owned stream (NULL: own) */
int pnol_ctx_device(pnol_ctx* ctx, int* device);
/* process default context used by the C++ drop-in classes (device = LOCAL_RANK or 0) */
int pnol_default_ctx(pnol_ctx** out);

/* Per-kernel HIP-event timers on the context's stream (off by default).  Names: "fd_jacobian",
 * "fd_ckpt", "fd_gradient", "linres_eval", "syrk", "syrk_reduce", "jtr", "solve", "hg",
 * "bfgs_pass", "allgather", "exchange_J", "exchange_A".  total_ms sums the recorded launches
 * since the last reset.  on = 2 times only "fd_jacobian", "fd_ckpt", "syrk", "exchange_J",
 * "allgather", "hg" and "bfgs_pass" (fewer event records between launches). */
int pnol_ctx_enable_timers(pnol_ctx* ctx, int on);
/* (also "exchange_J_busy": the columns-mode exchange's span on its own stream; "exchange_J" is
 * then the part of it left after the FD launches end -- the exposed exchange) */
int pnol_ctx_reset_timers(pnol_ctx* ctx);
int pnol_ctx_timer(pnol_ctx* ctx, const char* name, double* total_ms, int* count);

int pnol_malloc(pnol_ctx* ctx, size_t bytes, void** dptr);
int pnol_free(pnol_ctx* ctx, void* dptr);
int pnol_memcpy_h2d(pnol_ctx* ctx, void* dst, const void* src, size_t bytes);  /* synchronous */
/* Pinned host memory, and a device-to-host copy into it queued on the context stream (no
 * wait); completion is observed through an event recorded after it. */
int pnol_host_alloc(void** p, size_t bytes);
int pnol_host_free(void* p);
int pnol_memcpy_d2h_async(pnol_ctx* ctx, void* dst_pinned, const void* src, size_t bytes);
typedef struct pnol_event pnol_event;
int pnol_event_create(pnol_ctx* ctx, pnol_event** ev);
int pnol_event_record(pnol_ctx* ctx, pnol_event* ev);   /* after everything queued so far */
int pnol_event_wait(pnol_event* ev);                    /* host waits (busy-poll) */
int pnol_event_destroy(pnol_event* ev);
int pnol_memcpy_d2h(pnol_ctx* ctx, void* dst, const void* src, size_t bytes);  /* synchronous */

/* ---- BFGS dense inverse Hessian ------------------------------------------------------ */
/* p = -D g.  Replaces matrixVectorMultiply(D, dFdX, p) + negate, BFGS_with_linesearch.cpp:78-79
 * (also BFGS_with_linesearch_MPI.cpp:81-82, BFGS_bnd_linesearch.cpp:142-143).
 * D is n x n row-major with leading dimension ldd (doubles, even, 16-byte aligned base).
 * n <= PNOL_SEQ_MAX uses reference summation order (bitwise equal to the CPU path). */
#define PNOL_SEQ_MAX 64
/* columns per FD point tile (the FD GEMM's point-tile width, the multi-GPU split unit) */
#define PNOL_FD_TILE 128
int pnol_hg_d(pnol_ctx* ctx, const double* D, int ldd, const double* g, double* p, int n);
/* y = -A x for a rows x cols row-major A (the same streaming kernel; also rhs = -J^T F). */
int pnol_gemv_neg_d(pnol_ctx* ctx, const double* A, int lda, int rows, int cols, const double* x, double* y);

/* D <- (I - rho s y^T) D (I - rho y s^T) + rho s s^T, rho = 1/(y.s), in the reference's
 * O(n^3) operation order (updateHessianInv, BFGS_with_linesearch.cpp:389-432).  Bitwise
 * equal to the CPU path; intended for n <= a few hundred. */
int pnol_bfgs_update_exact_d(pnol_ctx* ctx, double* D, int ldd, const double* y, const double* s, int n);

/* One streaming pass over D (16 n^2 bytes when write-back is on, 8 n^2 otherwise):
 *   Dc = D + s_p a_p^T + b_p s_p^T   (pending rank-2 correction; s_p == NULL: none)
 *   if (write_back) D = Dc
 *   u = Dc y, w = Dc^T y, v = Dc g     (any of y/g may be NULL to skip; outputs n doubles)
 * The O(n^2) form of updateHessianInv plus the next H.g: see DESIGN.md "fused BFGS pass". */
int pnol_bfgs_pass_d(pnol_ctx* ctx, double* D, int ldd, int n,
                     const double* s_p, const double* a_p, const double* b_p, int write_back,
                     const double* y, const double* g, double* u, double* w, double* v);
/* pnol_bfgs_pass_d with write_back on a D that is diag(scale) (I when scale == NULL) and is not
 * read: the pending correction (required) is folded into the synthesised diagonal and the result
 * written to D, u/w/v as above -- the first update after a reset (BFGS_bnd_linesearch.cpp:607-616,
 * 647) costs 8 n^2 bytes instead of the 8 n^2 identity write plus the 16 n^2 pass. */
int pnol_bfgs_pass_ident_d(pnol_ctx* ctx, double* D, int ldd, int n, const double* scale, const double* s_p,
                           const double* a_p, const double* b_p, const double* y, const double* g, double* u, double* w,
                           double* v);
/* D = I (BFGS_with_linesearch.cpp:46-56), or diag(scale) when scale != NULL (BFGS_bnd_linesearch.cpp:65-83) */
int pnol_set_identity_d(pnol_ctx* ctx, double* D, int ldd, int n, const double* scale);
/* BFGS D row-sharded over the communicator (the reference keeps a full D per rank,
 * BFGS_with_linesearch_MPI.cpp:31-55): rank r holds rows [begin, begin + count) of D
 * (pnol_bfgs_rows: shards of whole 256-row tiles), stored from Dsh with leading dimension ldd.
 * Every function below is collective; each rank gets the full n-vectors back, bitwise the
 * same as the one-GPU pnol_hg_d / pnol_bfgs_pass_d on the whole D (same per-row order, the
 * column partials of w summed in the same fixed tile order). */
int pnol_bfgs_rows(int n, int nranks, int rank, int* begin, int* count);
/* Row tiles of w = D^T y partials the fused pass's workspace holds for n and nranks ranks:
 * max(the whole-matrix tile count, nranks * the tiles of one pnol_bfgs_rows shard) -- the
 * allgathered layout puts rank r's tiles at r * (tiles per shard).  Shape math only. */
int pnol_bfgs_pass_part_tiles(int n, int nranks);
int pnol_set_identity_rows_d(pnol_ctx* ctx, double* Dsh, int ldd, int n, const double* scale);
int pnol_hg_mpi_d(pnol_ctx* ctx, const double* Dsh, int ldd, const double* g, double* p, int n);
int pnol_bfgs_pass_mpi_d(pnol_ctx* ctx, double* Dsh, int ldd, int n, const double* s_p, const double* a_p,
                         const double* b_p, int write_back, const double* y, const double* g, double* u, double* w,
                         double* v);
/* pnol_bfgs_pass_ident_d on this rank's rows (collective) */
int pnol_bfgs_pass_ident_mpi_d(pnol_ctx* ctx, double* Dsh, int ldd, int n, const double* scale, const double* s_p,
                               const double* a_p, const double* b_p, const double* y, const double* g, double* u,
                               double* w, double* v);
/* Dsub[a][b] = D[idx[a]][idx[b]] for a, b < nsub (idx: device ints, ascending, < n): the
 * free-free block of D handed to the reduced problem, BFGS_with_bnd_linsearch_MPI.cpp:822-843 */
int pnol_gather_submatrix_d(pnol_ctx* ctx, const double* D, int ldd, int n, const int* idx, int nsub,
                            double* Dsub, int lds);
/* The same for a row-sharded D (collective; pnol_bfgs_rows shards of n rows in, of nsub rows
 * out): D = this rank's rows of the source, Dsub = this rank's rows of the block; idx: HOST
 * ints, ascending, < n, the same on every rank.  Each rank gathers the kept columns of its kept
 * rows on the device, and those rows go to their new owners point to point (RCCL; the host
 * backend bounces through host memory) -- D never crosses PCIe whole. */
int pnol_gather_submatrix_mpi_d(pnol_ctx* ctx, const double* D, int ldd, int n, const int* idx, int nsub,
                                double* Dsub, int lds);

/* ---- Levenberg-Marquardt -------------------------------------------------------------- */
/* A = JT JT^T (= J^T J) with A_ii = (1 + lambda) * (J^T J)_ii  (Marquardt scaling).
 * Replaces matrixTranspose + matrixMultiply(JT, J, JTJ) + the diag loop,
 * LevenbergMarquardt.cpp:59-73.  JT is n x m row-major (ld ldjt): column j of J is row j.
 * fp64 MFMA (v_mfma_f64_16x16x4_f64) SYRK on the lower triangle, mirrored; n <= PNOL_SEQ_MAX
 * and m <= 4096 use the reference summation order.  jtj_diag (nullable) receives (J^T J)_ii. */
int pnol_jtj_d(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda,
               double* A, int lda, double* jtj_diag);
/* LevMarqMPI's J^T J (LevenbergMarquardtMPI.cpp:64-78, replicated on every rank in the
 * reference): the 128 x 128 tiles are split over the process communicator's ranks, each rank
 * computes its tile range, one allgather of the packed tiles assembles A on every rank.
 * Bitwise equal to pnol_jtj_d for any rank count; with one rank it is pnol_jtj_d. */
int pnol_jtj_mpi_d(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda,
                   double* A, int lda, double* jtj_diag);
/* LevMarqMPI on the m-sliced Jacobian.  J^T J and J^T F are summed over
 * PNOL_LM_SLICES slices of the m residual rows by one fixed tree, so the rows can be split
 * over up to PNOL_LM_SLICES ranks with bitwise the one-GPU results (pnol_jtj_d / pnol_jtr_d).
 * Layout: slice s is an n x slice_rows row-major block at JTs + s * n * slice_rows (FD column
 * j, residual rows [s slice_rows, (s + 1) slice_rows)); jt_elems = PNOL_LM_SLICES * n * slice_rows. */
#define PNOL_LM_SLICES 8
int pnol_lm_sliced_layout(int m, int n, int* slice_rows, size_t* jt_elems);
/* LevenbergMarquardtMPI.cpp:60 + PNOL_Objective.cpp:202-299 (gradientApproximationMPI's column
 * loop and its MPI_Allreduce), the J^T slices this rank's normal-equation share needs.  Columns
 * mode (the default, the reference's decomposition): this rank's cost-balanced FD tiles
 * (pnol_fd_tiles) for all residual rows, one launch per tile (cheapest first), each tile's
 * m-slices sent to the ranks holding them (RCCL point-to-point on a second stream, gated by an
 * event behind that tile's launch, so all but the last tile's transfer overlap the FD); F0 (when
 * computed) holds all m rows.  Rows mode (pnol_lm_set_fd_mode 1, or PNOL_LM_FD=rows; linear
 * residuals): every FD column evaluated on this rank's own m-slices of residual rows (each row of
 * the residual is its own chain, so these are the same bits) -- no Jacobian exchange; F0 (when
 * computed) then holds only this rank's rows [r0, r1) of pnol_lm_rank_rows, the rest untouched.
 * Linear-residual device objectives; compute_f0 as for pnol_fd_jacobian_tiles_d. */
int pnol_lm_jacobian_mpi_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, double* F0,
                           int compute_f0, double* JTs);
/* LevMarqMPI's FD decomposition on this context: 0 = columns (default), 1 = rows, -1 = read the
 * environment again (PNOL_LM_FD=rows -> 1, else 0).  Every rank must use the same mode (the
 * LevMarqMPI drop-in re-reads the environment once per findMin and checks that all ranks agree);
 * pnol_lm_jacobian_mpi_d and pnol_lm_eval_mpi_d follow it. */
int pnol_lm_set_fd_mode(pnol_ctx* ctx, int mode);
int pnol_lm_fd_mode(pnol_ctx* ctx, int* mode);
/* Residual rows [r0, r1) held by `rank` of `nranks` (<= PNOL_LM_SLICES): its m-slices. */
int pnol_lm_rank_rows(int m, int nranks, int rank, int* r0, int* r1);
/* The LevMarqMPI trial point F(x) (LevenbergMarquardtMPI.cpp:92) with its prefix checkpoints:
 * rows mode: this rank's rows, then every rank's rows to all ranks (point-to-point), so F holds
 * all m residuals everywhere; columns mode (default) or one rank: pnol_dobj_eval_ckpt_d. */
int pnol_lm_eval_mpi_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, double* F);
/* LevenbergMarquardtMPI.cpp:64-80 from this rank's slices of pnol_lm_jacobian_mpi_d: A = J^T J
 * with A_ii = (1 + lambda) (J^T J)_ii and rhs = -(J^T F) on every rank.  Partial tiles of the
 * rank's slices, their tree nodes to each tile's owner (point-to-point), the owners merge, one
 * allgather.  Bitwise pnol_jtj_d + pnol_jtr_d of the row-major J^T for any rank count
 * <= PNOL_LM_SLICES.  n > PNOL_SEQ_MAX or m > 4096. */
int pnol_lm_normal_mpi_d(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F,
                         double* A, int lda, double* rhs, double* jtj_diag);
/* pnol_lm_normal_mpi_d + pnol_solve_step_d without forming A (LevenbergMarquardtMPI.cpp:64-90):
 * the allgathered J^T J tiles (one rank: its split-K partials) go straight into the persistent
 * tile Cholesky's matrix; rhs = -(J^T F), sigma, xnext = x + sigma and *dinfo (device int) are
 * bitwise those of the two calls.  *dinfo != 0: form A with pnol_lm_normal_unpack_mpi_d (same
 * m, n, lambda) and solve with the LU. */
int pnol_lm_normal_solve_mpi_d(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F,
                               double* rhs, double* sigma, int* dinfo, const double* x, double* xnext);
int pnol_lm_normal_unpack_mpi_d(pnol_ctx* ctx, int m, int n, double lambda, double* A, int lda);
/* The trip's solve status agreed over the communicator's ranks, queued on the context stream:
 * dinfo[0] (device int) is this rank's status from pnol_lm_trip_d / pnol_lm_normal_solve_mpi_d /
 * pnol_solve_step_d; dinfo[1] becomes the max over all ranks of its code -- 0 none, 1 a wait of
 * the tile Cholesky ran past its cap (relaunch the Cholesky: pnol_solve_d method 0 does), 2 a
 * non-positive or NaN pivot (the reference-order LU, method 2).  The reference's replicas all run
 * the same luSolve on the same A (LevenbergMarquardtMPI.cpp:88), so they never branch per rank;
 * acting on dinfo[1] keeps every rank on the same branch and the same collectives.  One rank or
 * no communicator: dinfo[1] = the code of dinfo[0]. */
int pnol_lm_agree_status_d(pnol_ctx* ctx, int* dinfo);
/* rhs = -(J^T F), LevenbergMarquardt.cpp:78-80 */
int pnol_jtr_d(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, const double* F, double* rhs);
/* sigma = A^{-1} rhs, replacing luSolve(A, rhs, sigma), LevenbergMarquardt.cpp:83.
 * method 0 = auto (n <= PNOL_SEQ_MAX: reference LU; else the tile Cholesky, LU on a non-positive
 * pivot), 2 = LU with partial pivoting (reference operation order), 4 = lookahead tile Cholesky
 * with diagonal-tile inverses, one launch per panel step, forward solve folded in, 5 = the same
 * factorisation (bitwise) as one persistent launch: one workgroup runs the diagonal chain, the
 * others take the panel / update tiles from an ordered queue (the default of method 0;
 * PNOL_CHOL_PERSIST=0 makes method 0 use 4).  Methods 4 and 5 factor a padded copy and leave A
 * intact.  A Cholesky whose dependency wait ran past its cap is relaunched (method 4 after the
 * first, bitwise the same factorisation), never replaced by the LU; PNOL_ERR_TIMEOUT when the
 * relaunches time out too.  (Methods 1 and 3, the per-panel-launch and tile-DAG Cholesky forms,
 * were removed: PNOL_ERR_UNSUPPORTED.)  info (host, nullable) gets the method family used
 * (1 = Cholesky, 2 = LU) or -1 on a singular matrix. */
int pnol_solve_d(pnol_ctx* ctx, double* A, int lda, const double* rhs, double* sigma, int n,
                 int method, int* info);
/* The method-4 Cholesky solve queued without any host wait: *dinfo (a device int) ends 0 on
 * success, nonzero when a pivot was not positive (sigma is then undefined and the caller
 * falls back to pnol_solve_d with method 2; A is left intact).  Lets the LM loop keep the
 * device busy while the host checks the previous trial point. */
int pnol_solve_async_d(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo);
/* pnol_solve_async_d + pnol_add_d(x, sigma, xnext): the LM trial point X + sigma
 * (LevenbergMarquardt.cpp:83-90) written by the solve's last launch.  xnext is undefined, like
 * sigma, when *dinfo ends nonzero. */
int pnol_solve_step_d(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo,
                      const double* x, double* xnext);
/* Binv = B^{-1} (n x n, row-major, device), bitwise the reference's matrixInverse: luSolve(B, e_c)
 * for every column c (UtilityFunctionLibrary restatement) as ONE partial-pivoting
 * elimination of [B | I] followed by per-column back substitution (the initHessFD inverse,
 * BFGS_with_linesearch.cpp:34-41, BFGS_bnd_linesearch.cpp:55-63).  info (host, nullable): 0, or
 * -1 after a zero pivot (the inverse then holds the inf / NaN the reference would produce). */
int pnol_matrix_inverse_d(pnol_ctx* ctx, const double* B, int ldb, int n, double* Binv, int ldi, int* info);
/* z = x + y (the LM trial point X + sigma on the device: the same IEEE add as the host's) */
int pnol_add_d(pnol_ctx* ctx, const double* x, const double* y, double* z, int n);

/* ---- device objectives and the batched finite-difference engine ---------------------- */
enum pnol_dobj_kind {
    PNOL_OBJ_ROSENBROCK = 0,  /* RosenbrockObject, ExampleObjectives.hpp:79-111 */
    PNOL_OBJ_POWER = 1,       /* PowerObject, :206-234 (power argument) */
    PNOL_OBJ_QUADRATIC = 4,   /* synthetic convex quadratic, p0 = d[n], p1 = b[n] (SURVEY 8(d) cfg 2/5) */
    PNOL_OBJ_EXPCURVE = 10,   /* ExpCurveObjective, :113-154; p0 = xData[m], p1 = yData[m] */
    PNOL_OBJ_CUBIC = 11,      /* CubicObjective, :160-201; p0 = xData[m], p1 = yData[m] */
    PNOL_OBJ_LINRES = 12      /* r = A x - y, p0 = A[m*n] row-major, p1 = y[m] (SURVEY 8(d) cfg 3/4) */
};
/* host_p0/host_p1 are copied to the device (NULL + len 0 when unused). */
int pnol_dobj_create(pnol_ctx* ctx, int kind, int n, int m, const double* host_p0, size_t len0,
                     const double* host_p1, size_t len1, double power, pnol_dobj** out);
/* Generate the synthetic data on the device from the splitmix64 stream (seed);
 * kind PNOL_OBJ_QUADRATIC (bscale scales b) or PNOL_OBJ_LINRES (xstar_out, host, nullable). */
int pnol_dobj_create_synthetic(pnol_ctx* ctx, int kind, int n, int m, unsigned long long seed,
                               double bscale, double* xstar_out, pnol_dobj** out);
int pnol_dobj_destroy(pnol_dobj* obj);
int pnol_dobj_info(pnol_dobj* obj, int* kind, int* n, int* m);
/* f = objEval(x) (scalar kinds, out[0]) or F = objEval(x) (residual kinds, out[0..m)) */
int pnol_dobj_eval_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, double* out);
/* f = objEval(x) as pnol_dobj_eval_d; for a linear residual the base chain's prefix
 * checkpoints of x are kept in the context, so the next pnol_fd_jtj_d / pnol_fd_jacobian_tiles_d
 * on the same (obj, x) with compute_f0 = 2 (F0 = this out) skips its base-chain pass
 * (LevenbergMarquardt.cpp:95 trial point -> :55 Jacobian point after an accepted step). */
int pnol_dobj_eval_ckpt_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, double* out);
/* Forward differences, Objective::gradientApproximation (PNOL_Objective.cpp:12-34):
 * f0 = f(x); g_i = (f(x + h_i e_i) - f0) / h_i for i in [i0, i0 + cnt).  g gets cnt values. */
int pnol_fd_gradient_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, int i0, int cnt,
                       double* f0, double* g);
/* Host-pointer forms (return with the results on the host; context scratch + pinned staging, one
 * upload and one download, no allocation): the per-iteration FD gradient of the C++ classes
 * (PNOL_Objective.cpp:12-34; g gets cnt values, *f0 = f(x)), and a batch of single evaluations
 * (line-search trial points and pool entries, BFGS_with_linesearch.cpp:144-174,
 * BFGS_with_linesearch_MPI.cpp:163-223): out[k] = f(Xs row k) for scalar kinds, out rows
 * k*m .. k*m+m-1 = F(Xs row k) for residual kinds; Xs is npts x n row-major. */
int pnol_fd_gradient(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, int i0, int cnt, double* f0,
                     double* g);
int pnol_dobj_eval_batch(pnol_ctx* ctx, pnol_dobj* obj, const double* Xs, int npts, double* out);
/* MultiObjective::gradientApproximation (PNOL_Objective.cpp:165-197) for columns [j0, j0+cnt):
 * F0 = F(x) (computed here when compute_f0, else read), JT row (j - j0) = (F(x + h_j e_j) - F0)/h_j.
 * compute_f0 = 2 (pnol_fd_jtj_d / pnol_fd_jacobian_tiles_d / pnol_lm_jacobian_mpi_d): F0 was
 * filled by pnol_dobj_eval_ckpt_d(ctx, obj, x, F0); its prefix checkpoints are reused when x's
 * content is still the one they were made at (checked on the device; otherwise F0 and the
 * checkpoints are recomputed, so updating x in place is safe).  compute_f0 = 3: the same without
 * the check -- the caller guarantees x is unchanged (the library's LM loop). */
int pnol_fd_jacobian_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, int j0, int cnt,
                       double* F0, int compute_f0, double* JT, int ldjt);
/* One LevMarq Jacobian + normal matrix, pipelined (LevenbergMarquardt.cpp:55-73): the FD
 * Jacobian of all n columns into JT (as pnol_fd_jacobian_d with j0 = 0) and A = J^T J with
 * A_ii = (1 + lambda) (J^T J)_ii (as pnol_jtj_d).  The FD column chunks run on the context
 * stream and the J^T J tile rows each chunk completes on a second stream, so the VALU-bound
 * FD GEMM and the MFMA-bound J^T J overlap.  Bitwise the same JT and A as the two calls;
 * nchunks <= 1 runs them back to back. */
int pnol_fd_jtj_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, double* F0, int compute_f0,
                  double* JT, int ldjt, double lambda, double* A, int lda, double* jtj_diag, int nchunks);
/* pnol_fd_jtj_d (nchunks = 1) + pnol_jtr_d(JT, F0, rhs) in one queue (LevenbergMarquardt.cpp:55-80):
 * the FD Jacobian, A = J^T J with the Marquardt diagonal, and rhs = -(J^T F0), where F0 = F(x)
 * as computed or reused per compute_f0.  The -J^T F slice tree rides in the J^T J reduce launch.
 * Bitwise the same JT, A and rhs as the separate calls. */
int pnol_fd_normal_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, double* F0, int compute_f0,
                     double* JT, int ldjt, double lambda, double* A, int lda, double* jtj_diag, double* rhs);
/* One LevMarq trip's linear algebra with A never formed (LevenbergMarquardt.cpp:55-90; n > 64,
 * single process): the FD Jacobian into JT (compute_f0 as pnol_fd_jacobian_d), rhs = -(J^T F0),
 * sigma = (J^T J + lambda diag(J^T J))^{-1} rhs by the persistent tile Cholesky -- whose first
 * tasks sum the J^T J split-K partials straight into its own matrix -- and xnext = x + sigma.
 * *dinfo (device int) != 0: a non-positive pivot; form A with pnol_lm_trip_normal_d and solve
 * with the LU (pnol_solve_d method 2).  JT, rhs, sigma, xnext and *dinfo are bitwise those of
 * pnol_fd_normal_d + pnol_solve_step_d. */
int pnol_lm_trip_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, double* F0, int compute_f0,
                   double* JT, int ldjt, double lambda, double* rhs, double* sigma, int* dinfo, double* xnext);
/* A = J^T J + lambda diag(J^T J) from the last pnol_lm_trip_d's partial sums (its m, n, lambda):
 * bitwise pnol_fd_normal_d's A. */
int pnol_lm_trip_normal_d(pnol_ctx* ctx, int m, int n, double lambda, double* A, int lda);
/* The FD Jacobian rows of a tile list (columns [start[t], start[t] + count[t]), count <=
 * PNOL_FD_TILE), column c written to JT + c * ldjt; one base-chain pass for all tiles. */
int pnol_fd_jacobian_tiles_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, const int* start,
                             const int* count, int ntiles, double* F0, int compute_f0, double* JT, int ldjt);

/* ---- communicator (replaces MPI_COMM_WORLD on the FD / pool paths) ------------------- */
/* RCCL over xGMI: one process per GPU.  Exchange the 128-byte id out of band (rank 0 creates). */
int pnol_comm_unique_id(char id[128]);
int pnol_comm_init_rccl(pnol_ctx* ctx, int nranks, int rank, const char id[128]);
/* Host backend (tests / host objectives): the caller supplies the allgather. */
typedef int (*pnol_host_allgather_fn)(const void* send, void* recv, size_t bytes_per_rank, void* user);
int pnol_comm_init_host(int nranks, int rank, pnol_host_allgather_fn fn, void* user);
int pnol_comm_finalize(void);
int pnol_comm_size(int* nranks, int* rank);
/* MPI launcher binding (the reference's *_MPI classes take P and the rank from MPI_COMM_WORLD:
 * LevenbergMarquardtMPI.cpp:16-17, PNOL_Objective.cpp:102-103, BFGS_with_linesearch_MPI.cpp:231-235).
 * The library itself links no MPI.  A program that includes the drop-in headers with <mpi.h>
 * on its include path (the reference header includes it, PNOL_Objective.hpp:20) registers a
 * hook compiled against the program's own MPI (include/pnol_mpi_bind.hpp); the first *_MPI
 * call runs it: P and the rank from MPI_COMM_WORLD, the GPU by node-local rank, and RCCL
 * bootstrapped with the unique id broadcast over MPI (the host backend over MPI_Allgather
 * when node-local ranks outnumber the GPUs).  Hook return: 0 bound (or nothing to bind,
 * P = 1), 1 MPI not initialised yet (asked again on the next *_MPI call), < 0 failure. */
typedef int (*pnol_launcher_hook_fn)(void);
int pnol_comm_set_launcher_hook(pnol_launcher_hook_fn fn);
/* Run the hook if no communicator is bound (what every *_MPI entry point does first).
 * PNOL_ERR_COMM when an MPI launcher's environment (PMI_SIZE, OMPI_COMM_WORLD_SIZE,
 * MV2_COMM_WORLD_SIZE) says the job has more than one rank and still no communicator is
 * bound: a *_MPI class never runs such a job silently as one rank. */
int pnol_comm_bind_launcher(void);
/* The job size an MPI launcher's environment announces (1 without one). */
int pnol_launcher_world_size(void);
/* GPU of the process's default context, when chosen before its first use (the launcher hook
 * picks the node-local rank's GPU); otherwise PNOL_DEVICE, then LOCAL_RANK / MPI_LOCALRANKID /
 * OMPI_COMM_WORLD_LOCAL_RANK modulo the device count, then 0.  PNOL_ERR_ARG once the default
 * context exists on another device. */
int pnol_set_default_device(int device);
/* recv[r * count + i] = send_r[i]  (device buffers on the RCCL backend) */
int pnol_comm_allgather_d(pnol_ctx* ctx, const double* send, double* recv, size_t count);
/* contiguous column block owned by `rank` of `nranks` over `ncols` columns (also the host split) */
void pnol_block_range(int ncols, int nranks, int rank, int* begin, int* count);
/* Cost-balanced FD column tiles of `rank` (LevMarqMPI's Jacobian split, replacing the
 * round-robin owners of PNOL_Objective.cpp:110-121 / 228-240): PNOL_FD_TILE-column tiles
 * dealt in snake order.  Writes up to cap (start, count) pairs; returns the tile count. */
int pnol_fd_tiles(int ncols, int nranks, int rank, int* start, int* count, int cap);
/* Every rank ends with all ncols rows of buf (row c at buf + c * ld) from their pnol_fd_tiles
 * owners: replaces the per-column MPI_Allreduce of PNOL_Objective.cpp:280-288 (RCCL:
 * grouped point-to-point straight into place; host backend: allgather + unpack). */
int pnol_comm_share_fd_rows_d(pnol_ctx* ctx, double* buf, int ld, int ncols);

/* ---- whole-solver drivers: the C++ drop-in classes run on built-in objectives --------- */
/* params arrays follow the classes' setParams order (see the headers in include/). */
typedef struct { int iters; long evals; double f0; double fopt; } pnol_result;
/* which: 0 = BFGS (12 params), 1 = BFGS_MPI (12 params), 2 = BFGS_Bnd (15 params),
 * 3 = BFGSBnd_MPI (14 params [+ pool size, update mode]),
 * 4 = BFGS_Bnd_MPI_SW (15 params [+ Nprocs-equivalent pool size, update mode]) */
int pnol_run_bfgs(int which, pnol_dobj* obj, int host_eval, const double* params, int nparams,
                  double* X, int n, const double* Xlb, const double* Xub, pnol_result* res);
/* pnol_run_bfgs plus diagnostics.  BFGS (0) and BFGS_Bnd (2): res->iters = the iteration count
 * (BFGS_Bnd: totalIter); profile (8 doubles, nullable) = iterations, total seconds, FD-gradient
 * seconds, line-search seconds, D update / direction seconds, line-search points evaluated,
 * gradient calls, deepest boundaryAssessment recursion.  BFGS_Bnd: F after every iteration of
 * any recursion level in ftrace[0 .. min(cap, *ntrace)) (nullable). */
int pnol_run_bfgs_ex(int which, pnol_dobj* obj, int host_eval, const double* params, int nparams, double* X, int n,
                     const double* Xlb, const double* Xub, pnol_result* res, double* ftrace, int trace_cap,
                     int* ntrace, double* profile);
/* which: 0 = GeneticAlgorithm, 1 = GeneticAlgorithmMPI (10 params, the setGAParams order without
 * graph: Npop, maxGenerations, eliteFrac, crossFrac, eliteMutationFrac, mutationSize,
 * eliteMutationSize, initialPopScaling, NstaticGenerations, verbose); seed: the selection /
 * mutation stream (GeneticAlgorithm::setSeed); res->iters = generations.  Each generation's
 * population is one device batch for device objectives (GeneticAlgorithm.cpp:301-310,
 * GeneticAlgorithmMPI.cpp:283-414). */
int pnol_run_ga(int which, pnol_dobj* obj, int host_eval, const double* params, int nparams, unsigned long long seed,
                double* X, int n, const double* Xlb, const double* Xub, pnol_result* res);
/* which: 0 = LevMarq, 1 = LevMarqMPI (6 params). F0/FOpt host arrays of m. */
int pnol_run_levmarq(int which, pnol_dobj* obj, int host_eval, const double* params, double* X, int n,
                     double* F0, double* FOpt, int m, pnol_result* res);
/* pnol_run_levmarq + steps[2] = accepted / rejected loop trips (LevMarq::getAcceptedSteps) */
int pnol_run_levmarq_ex(int which, pnol_dobj* obj, int host_eval, const double* params, double* X, int n,
                        double* F0, double* FOpt, int m, pnol_result* res, int* steps);
/* Host-objective FD through the C++ MultiObjective with a C callback objective
 * (gradientApproximation / gradientApproximationMPI on the active communicator). */
typedef void (*pnol_host_multi_fn)(const double* x, int n, double* F, int m, void* user);
typedef double (*pnol_host_scalar_fn)(const double* x, int n, void* user);
/* Objective::hessianApproximation (PNOL_Objective.cpp:38-85) of a C callback objective through the
 * C++ FD engine (its points handed to objEvalBatch in the reference's order); B n x n row-major. */
int pnol_host_fd_hessian(pnol_host_scalar_fn fn, void* user, const double* x, const double* h, int n, double* B);
int pnol_host_fd_jacobian(pnol_host_multi_fn fn, void* user, const double* x, const double* h, int n, int m,
                          int sharded, double* J_rowmajor);
/* GeneticAlgorithm (which 0) / GeneticAlgorithmMPI (1) findMinBnd (GeneticAlgorithm.cpp:12-297) on a C
 * callback objective, each generation handed to objEvalBatch on the host; params / seed / res as
 * pnol_run_ga.  Needs no device. */
int pnol_host_run_ga(int which, pnol_host_scalar_fn fn, void* user, const double* params, int nparams,
                     unsigned long long seed, double* X, int n, const double* Xlb, const double* Xub,
                     pnol_result* res);

#ifdef __cplusplus
}
#endif
#endif /* PNOL_AMD_H_ */
