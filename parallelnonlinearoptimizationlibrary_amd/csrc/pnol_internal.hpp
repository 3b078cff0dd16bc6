// pnol_internal.hpp -- runtime internals shared by the HIP kernels, the C ABI and the
// C++ drop-in classes.  Not installed; the public surface is include/pnol_amd.h.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdio>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "pnol_amd.h"

namespace pnol {

// Scratch buffers keyed by purpose; grown on demand, never shrunk, freed with the context.
// Allocation happens outside any capturable region (first use of a size), so repeated
// solver iterations allocate nothing.
struct Workspace {
    std::map<std::string, std::pair<void*, size_t>> bufs;
};

}  // namespace pnol

namespace pnol {
// start/stop event pairs per kernel name, resolved lazily (pnol_ctx_timer)
struct Timers {
    int on = 0;   // 0 off, 1 every timer, 2 only the roofline / scaling kernels (hot_timer)
    std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::map<std::string, std::pair<double, int>> done;
    std::vector<hipEvent_t> free_events;   // recycled after resolve (event creation is not free)
};
}  // namespace pnol

struct pnol_ctx {
    int device = 0;
    pnol::Timers timers;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;   // active stream (own or caller-provided)
    int num_cu = 0;
    pnol::Workspace ws;
    void* pinned = nullptr;         // pinned host staging for pnol_memcpy_* (grown on demand)
    size_t pinned_bytes = 0;
    // pnol_fd_gradient's step vector as last uploaded (host copy) and where it went
    std::vector<double> fdg_h_host;
    const double* fdg_h_dev = nullptr;
    // two slots of linear-residual prefix checkpoints ("linres_ckpt0/1"), each tagged with the
    // objective and the device x it was computed at; use = last-use stamp (least recent is reused)
    unsigned long long ckpt_oid[2] = {0, 0};   // pnol_dobj::id (0: untagged)
    const double* ckpt_x[2] = {nullptr, nullptr};
    int ckpt_r0[2] = {0, 0}, ckpt_r1[2] = {0, 0};   // the residual rows the slot's checkpoints cover
    unsigned long ckpt_use[2] = {0, 0};
    unsigned long ckpt_clock = 0;
    int ckpt_last = 0;   // the slot written last
    int* solve_flags = nullptr;     // per-block ready flags of the triangular solves (workspace)
    int solve_epoch = 0;            // value the flags of the current solve are set to
    void* chol_tasks = nullptr;     // uploaded tile-DAG task table (workspace) and its tile count
    int chol_tasks_T = 0;
    int* chol4_flags = nullptr;     // method-4 Cholesky: per-row panel flags + backward-solve flags
    int chol4_cap = 0;              // tile rows the flag buffer holds (2 * cap ints)
    // a persistent Cholesky's dependency wait ran past its cap on this context (the GPU is shared
    // with other processes, so fewer workers are resident than launched): from then on its
    // workers claim in step order (order 0, which drains with any co-residency)
    bool chol_order0 = false;
    // The one-GPU LM trip's results written straight into the host's pinned block by the kernels
    // that form them (set by the LM loop around its launches, null otherwise): sigma by the
    // backward solve, F(x + sigma) and the solve status word by the trial point's evaluation --
    // no copy command behind the trip, whose launch left a ~12 us gap after the evaluation.
    struct TripMirror {
        double* sigma = nullptr;
        double* F = nullptr;
        const int* info_d = nullptr;
        int* info_h = nullptr;
    } trip_mirror;
    // The LM loop's next Jacobian queued behind a gate before the host decides the step (set by
    // lm_prequeue_fd around its launch, null otherwise): k_trip_gate polls the host word hw
    // ({seq, choice}) and passes the choice on in sel (device); the FD launch then takes x0 / F0 /
    // its checkpoints (choice 0: the step rejected), x1 / F01 / the checkpoints of x1 (choice 1:
    // accepted), or returns at once (choice < 0: no further trip).  res: the choice the gate
    // passed on and its seq, for the host's check (pinned).
    struct FdGate {
        const int* hw = nullptr;
        int seq = 0;
        int* sel = nullptr;
        int* res = nullptr;
        const double* x1 = nullptr;
        const double* F01 = nullptr;
        unsigned long long cap = 0;   // ticks of the 100 MHz clock the gate waits at most
    } fd_gate;
    int chol4_epoch = 0;            // last flag value handed out (monotonic; flags reset on regrow)
    hipStream_t aux_stream = nullptr;   // second stream (J^T J rows beside the FD chunks), lazily created
    std::vector<hipEvent_t> aux_events; // chunk-done events between the two streams
    // LevMarqMPI's FD decomposition (fd.hip): -1 = not chosen yet (PNOL_LM_FD at first use),
    // 0 = columns (the reference's: FD column tiles per rank + the m-slice exchange), 1 = rows
    int lm_fd_mode = -1;
    // columns mode's slice exchange (lm_phased_env: 0 one exchange after one FD launch
    // (PNOL_LM_PHASED=0), S >= 1 a phase per tile with the last tile in S column groups
    // (PNOL_LM_SUBPHASES)): read once per LevMarqMPI solve and agreed over the ranks (-1: at first use)
    int lm_phased = -1;
    bool lm_fd_mode_set = false;   // set by pnol_lm_set_fd_mode: the LevMarqMPI drop-in keeps it
    // What the last LM trip without A (launch_fd_normal_solve / launch_lm_normal_solve) left for
    // its A-forming entry points (pnol_lm_trip_normal_d, pnol_lm_normal_unpack_mpi_d): the
    // split-K partials ("syrk_part", kind 1) or the allgathered tiles ("lm_packed", kind 2) of
    // shape (m, n) over nranks ranks.  Every other writer of those buffers clears it.
    struct {
        int kind = 0, m = 0, n = 0, nranks = 0;
    } lm_trip_tiles;
    // columns mode: the m-slice exchange of each FD tile runs on comm_stream, gated by the
    // event recorded behind that tile's FD launch on the context stream
    hipStream_t comm_stream = nullptr;
    std::vector<hipEvent_t> phase_events;
    hipEvent_t comm_done = nullptr;
};

// The tile Cholesky's workspace for order n (chol.hip)
struct CholWs {
    int T = 0, N = 0;
    long ldp = 0;
    double *P = nullptr, *Lm = nullptr, *W = nullptr, *bv = nullptr, *zv = nullptr, *xw = nullptr;
    int *rowflag = nullptr, *bwdflag = nullptr, *pf = nullptr;
    int npf = 0;
    bool gran = false;
};
struct CholRed {   // the LM trip's reducing Cholesky (launch_chol_reducing_*)
    CholWs w;
    int n = 0;
    int* dinfo = nullptr;
};

struct pnol_dobj {
    int kind = 0;
    int n = 0;
    int m = 0;
    double power = 2.0;
    double* p0 = nullptr;     // device data (see pnol_dobj_kind)
    double* p1 = nullptr;
    double* p2 = nullptr;     // derived device data (e.g. pow(xData,3) for the cubic)
    double* at = nullptr;     // LINRES: A in 64-row k-major panels (fd.hip), built on first FD use
    size_t len0 = 0, len1 = 0;
    pnol_ctx* ctx = nullptr;
    int device = 0;           // ctx's device, kept so destroy never reads a context freed before it
    unsigned long long id = pnol_dobj_next_id();   // unique per creation (checkpoint slot tags)
  private:
    static unsigned long long pnol_dobj_next_id() {
        static std::atomic<unsigned long long> next{1};
        return next++;
    }
};

namespace pnol {

#define PNOL_HIP(expr)                                                                       \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "[pnol_amd] HIP error %s at %s:%d: %s\n", hipGetErrorName(e_), \
                         __FILE__, __LINE__, #expr);                                          \
            return PNOL_ERR_HIP;                                                             \
        }                                                                                    \
    } while (0)

#define PNOL_CHECK(expr)             \
    do {                             \
        int s_ = (expr);             \
        if (s_ != PNOL_OK) return s_; \
    } while (0)

// The context's pinned host staging buffer, at least `bytes` (<= 64 MiB; nullptr above that or
// on failure).  One user at a time: callers copy in, copy through the stream and synchronise.
void* pinned_stage(pnol_ctx* ctx, size_t bytes);

// Returns a device scratch buffer of at least `bytes` for `key` (grows, keeps contents undefined).
// fresh (optional): set when the buffer was (re)allocated, i.e. its contents are undefined --
// compare this, not the pointer (hipFree + hipMalloc may return the same address)
int ws_get(pnol_ctx* ctx, const char* key, size_t bytes, void** out, bool* fresh = nullptr);
int ws_get_zeroed(pnol_ctx* ctx, const char* key, size_t bytes, void** out);

// Scoped timer: records a start event now and a stop event at scope exit (when enabled).
class ScopedTimer {
  public:
    ScopedTimer(pnol_ctx* ctx, const char* name, hipStream_t stream = nullptr);
    ~ScopedTimer();
  private:
    pnol_ctx* ctx_;
    const char* name_;
    hipStream_t stream_ = nullptr;
    hipEvent_t a_ = nullptr, b_ = nullptr;
};

// Timer events carried by the kernel dispatch itself (hipExtLaunchKernel start / stop events):
// no extra packets between launches, unlike ScopedTimer's two event records (~5-7 us of
// dispatch gap each).  start() / stop() are nullptr when the timer is off; a sequence of
// launches passes start() to the first and stop() to the last.
class LaunchTimer {
  public:
    LaunchTimer(pnol_ctx* ctx, const char* name);
    ~LaunchTimer();
    hipEvent_t start() const { return a_; }
    hipEvent_t stop() const { return b_; }
  private:
    pnol_ctx* ctx_;
    const char* name_;
    hipEvent_t a_ = nullptr, b_ = nullptr;
};

// Launch-error check after a kernel launch.
inline int launch_check() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        std::fprintf(stderr, "[pnol_amd] kernel launch failed: %s\n", hipGetErrorString(e));
        return PNOL_ERR_HIP;
    }
    return PNOL_OK;
}

// The tile Cholesky's status for a wait that ran past its spin cap (chol.hip): not a numerical
// result -- launch_solve relaunches the factorisation, the LM loop redoes the trip's solve
constexpr int kCholTimeout = -7;
// status codes a solve status maps to, ordered so that the max over ranks is the action every
// rank takes: 0 none, 1 a timed-out wait (relaunch the Cholesky), 2 a non-positive / NaN pivot
// (the reference-order LU)
__host__ __device__ inline int solve_status_code(int info) { return info == 0 ? 0 : info == kCholTimeout ? 1 : 2; }
// dinfo[1] = max over the communicator's ranks of solve_status_code(dinfo[0]) (device ints),
// queued on the context stream (solve.hip)
int launch_status_agree(pnol_ctx* ctx, int* dinfo);

// ---- kernel launchers (defined in kernels/*.hip) ------------------------------------
int launch_gemv_neg(pnol_ctx* ctx, const double* A, int lda, int rows, int cols, const double* x, double* y);
int launch_gemv_neg_seq(pnol_ctx* ctx, const double* A, int lda, int rows, int cols, const double* x, double* y);
// y[(s - s0) * rows + j] = -sum_{k in m-slice s} A_s[j][k] x[s mS + k], s in [s0, s0 + nsl)
// stream: nullptr = the context stream
int launch_gemv_neg_slices(pnol_ctx* ctx, const double* A, int lda, long sstride, int rows, int m, int mS, int s0,
                           int nsl, const double* x, double* y, hipStream_t stream = nullptr);
int launch_bfgs_update_exact(pnol_ctx* ctx, double* D, int ldd, const double* y, const double* s, int n);
int launch_bfgs_pass(pnol_ctx* ctx, double* D, int ldd, int n, const double* s_p, const double* a_p,
                     const double* b_p, int write_back, const double* y, const double* g, double* u, double* w,
                     double* v, int rb = 0, int re = -1, int (*pw_gather)(pnol_ctx*, double*, int, int) = nullptr,
                     int ident_src = 0, const double* id_scale = nullptr);
int launch_set_identity(pnol_ctx* ctx, double* D, int ldd, int n, const double* scale, int rb = 0, int re = -1);
int launch_add(pnol_ctx* ctx, const double* x, const double* y, double* z, int n);
int launch_gather_sub(pnol_ctx* ctx, const double* D, int ldd, int n, const int* idx, int nsub, double* Dsub,
                      int lds);
// Dsub[a][b] = D[ridx[a] - rbase][cidx[b]] (rows of a shard starting at global row rbase)
int launch_gather_rows(pnol_ctx* ctx, const double* D, int ldd, const int* ridx, int nrows, int rbase, const int* cidx,
                       int ncols, double* Dsub, int lds);

// rhs (nullable): also rhs = -J^T F (bitwise launch_jtr), its slice tree in the reduce launch
int launch_jtj(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda, double* A, int lda,
               double* jtj_diag, const double* F = nullptr, double* rhs = nullptr);
// One LM trip's linear algebra without forming A (syrk.hip): FD Jacobian, J^T J split-K
// partials, -J^T F slice partials, then launch_chol_reducing; A only on request from the
// partials of the last trip (the LU fallback)
// fd_queued: the Jacobian at x is already queued (lm_prequeue_fd, released with the decision)
int launch_fd_normal_solve(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, double* F0, int compute_f0,
                           double* JT, int ldjt, double lambda, double* rhs, double* sigma, int* dinfo, double* xnext,
                           bool fd_queued = false);
// The one-GPU LM loop's next FD Jacobian (fd.hip), queued before the host has decided the step:
// k_trip_gate then the FD launch, at x0 (F00 = F(x0)) or x1 (F01) as the host's word hw picks
// ({seq, choice}: 0 -> x0, 1 -> x1, < 0 -> no launch work).  Both points' prefix checkpoints must
// be in the context's slots (PNOL_ERR_UNSUPPORTED otherwise: nothing queued).  sel: a device int;
// res: pinned {choice passed on, seq}.  lm_fd_commit: the checkpoint bookkeeping of the chosen
// point, as its own FD launch would have left it.
int lm_prequeue_fd(pnol_ctx* ctx, pnol_dobj* o, const double* x0, double* F00, const double* x1, double* F01,
                   const double* h, double* JT, int ldjt, const int* hw, int seq, int* sel, int* res,
                   unsigned long long cap);
int lm_fd_commit(pnol_ctx* ctx, pnol_dobj* o, const double* x);
int launch_jtj_from_partials(pnol_ctx* ctx, int m, int n, double lambda, double* A, int lda);
int launch_jtj_sharded(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda, double* A, int lda,
                       double* jtj_diag);
int launch_jtr(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, const double* F, double* rhs);

// Binv = B^{-1} as the reference's matrixInverse (per-column luSolve), bitwise: one elimination
// of [B | I], per-column back substitution; *info_host = -1 on a zero pivot (inf / NaN entries)
int launch_matrix_inverse(pnol_ctx* ctx, const double* B, int ldb, int n, double* Binv, int ldi, int* info_host);
// xnext (nullable): also xnext = xbase + sigma (the LM trial point), written by the final launch
int launch_chol_solve(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo,
                      const double* xbase = nullptr, double* xnext = nullptr);
// variant 0: auto (PNOL_CHOL_PERSIST, default the persistent form), 4: per-step launches,
// 5: one persistent launch for the panel steps (bitwise the same result)
int launch_chol_solve_v(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo,
                        int variant, const double* xbase = nullptr, double* xnext = nullptr);
int launch_solve(pnol_ctx* ctx, double* A, int lda, const double* rhs, double* sigma, int n, int method,
                 int* info);
// The LM trip's damped solve from the J^T J split-K partials (chol.hip): _prep takes the
// workspace (before anything is queued: an allocation may free); _start queues the prep launch
// (progress words, paddings, info) on the context stream; _run queues on `st` the persistent tile
// Cholesky whose first tasks reduce the partials (part: k_syrk_tile's 128 x 128 layout, `sub`
// chunks per m-slice) and the -J^T F slice
// partials jp into its padded matrix and b (rhs gets -J^T F too), then the factorisation, the
// backward solve and xnext = xbase + sigma; bitwise the reduce into A + launch_chol_solve
int launch_chol_reducing_prep(pnol_ctx* ctx, int n, int* dinfo, CholRed& cr);
// preloaded: the matrix and b will be in P / bv before the persistent launch (every version and
// b word starts at 0; launch_chol_preloaded_run), else the reduce tasks store them (words at -1)
// zc / nz: int counters the prep launch also zeroes (k_syrk_red's per-tile partial counts)
int launch_chol_reducing_start(pnol_ctx* ctx, const CholRed& cr, bool preloaded = false, int* zc = nullptr, int nz = 0);
int launch_chol_preloaded_run(pnol_ctx* ctx, hipStream_t st, const CholRed& cr, double* sigma, const double* xbase,
                              double* xnext);
int launch_chol_reducing_run(pnol_ctx* ctx, hipStream_t st, const CholRed& cr, const double* part, int sub,
                             const double* jp, double lambda, double* rhs, double* sigma, const double* xbase,
                             double* xnext);
int launch_chol_reducing_run_packed(pnol_ctx* ctx, hipStream_t st, const CholRed& cr, const double* packed, long slot,
                                    int tpr, const double* rhs, double lambda, double* sigma, const double* xbase,
                                    double* xnext);
// LevMarqMPI's normal equations + solve without forming A (syrk.hip): launch_lm_normal up to the
// allgathered tiles and -J^T F, then the reducing Cholesky reading the tiles; A on request from
// the last call's tiles (the LU fallback)
int launch_lm_normal_solve(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F, double* rhs,
                           double* sigma, int* dinfo, const double* xbase, double* xnext);
int launch_lm_normal_unpack(pnol_ctx* ctx, int m, int n, double lambda, double* A, int lda);

int launch_dobj_eval(pnol_ctx* ctx, pnol_dobj* o, const double* x, double* out);
// rows [r0, r1) only (multiples of 64 but r1 = m; r1 < 0: all): a row-sharded LevMarqMPI rank
int launch_dobj_eval_ckpt(pnol_ctx* ctx, pnol_dobj* o, const double* x, double* out, int r0 = 0, int r1 = -1);
// out[k] = f(Xs row k) (scalar kinds) or out rows = F(Xs row k) (residual kinds), k < npts
int launch_eval_batch(pnol_ctx* ctx, pnol_dobj* o, const double* Xs, int npts, double* out);
// xdev != nullptr: x is a pinned host block, read once by the first kernel and copied to xdev
// (device memory, n doubles) for the rest; f0 / g may be pinned host memory too.  hsrc != nullptr:
// the step vector's new content in pinned host memory, copied to h (device) by the first kernel
int launch_fd_gradient(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, int i0, int cnt,
                       double* f0, double* g, double* xdev = nullptr, const double* hsrc = nullptr);
// ckpt: 1 = run the base-chain pass (F0 when compute_f0, prefix checkpoints), 0 = reuse the
// checkpoints of the previous call at the same x (chunked launches of one Jacobian)
// mS > 0: the sliced J^T layout (row r of J in slice r / mS at JT + (r / mS) * sstride, row
// stride ldjt >= mS); linear residuals on the row-panel kernels only
// after_tile (nullable): one launch per tile in the given order (no sorting), after_tile(t)
// called behind the launch of tile t -- the phased columns-mode exchange (linear residuals)
int launch_fd_jacobian_tiles(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, const int* start,
                             const int* count, int ntiles, double* F0, int compute_f0, double* JT, int jbase,
                             int ldjt, int ckpt = 1, int mS = 0, long sstride = 0, int r0 = 0, int r1 = -1,
                             const std::function<int(int)>* after_tile = nullptr);
// J^T J tiles of tile rows [row_begin, row_end) (128 x 128 tiles, split_k of the whole matrix so
// every tile is summed exactly as by launch_jtj), partials + reduce on `stream`
int launch_jtj_rows(pnol_ctx* ctx, hipStream_t stream, const double* JT, int ldjt, int m, int n, double lambda,
                    double* A, int lda, double* jtj_diag, int row_begin, int row_end);
// FD Jacobian of all columns + A = J^T J (+ Marquardt diagonal), pipelined: FD column chunks on
// the context stream, the J^T J tile rows they complete on a second stream
// rhs (nullable): also rhs = -J^T F0 (pnol_fd_normal_d)
int launch_fd_jtj(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, double* F0, int compute_f0,
                  double* JT, int ldjt, double lambda, double* A, int lda, double* jtj_diag, int nchunks,
                  double* rhs = nullptr);
int launch_fd_jacobian(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, int j0, int cnt,
                       double* F0, int compute_f0, double* JT, int ldjt);
int launch_synthetic_quadratic(pnol_ctx* ctx, unsigned long long seed, int n, double bscale, double* d, double* b);
int launch_synthetic_linres(pnol_ctx* ctx, unsigned long long seed, int m, int n, double* A, double* xstar,
                            double* y);
int launch_fill(pnol_ctx* ctx, double* p, size_t count, double value);

// ---- LM m-slices: J^T J and J^T F are summed over kLmSlices slices of the m
// residual rows by a fixed tree (syrk.hip), so LevMarqMPI can split the rows over up to
// kLmSlices ranks with bitwise the one-GPU A.  Sliced J^T layout: slice s is an n x mS
// row-major block at JTs + s * n * mS (FD column j, rows [s mS, (s + 1) mS) of J).
constexpr int kLmSlices = 8;
// columns mode: each rank's last FD tile is launched and exchanged as this many column groups
// (PNOL_LM_SUBPHASES overrides), so only the last group's m-slices are exposed after the FD
constexpr int kLmSubphases = 1;
inline int lm_slice_rows(int m) { return (((m + kLmSlices - 1) / kLmSlices) + 63) / 64 * 64; }
// rank r of P (<= kLmSlices) holds slices [floor(r 8 / P), floor((r + 1) 8 / P))
inline void lm_rank_slices(int P, int r, int* s0, int* s1) {
    *s0 = r * kLmSlices / P;
    *s1 = (r + 1) * kLmSlices / P;
}
// normal equations from the sliced J^T of this rank's slices (all FD columns): A (+ Marquardt
// diagonal) and rhs = -J^T F on every rank (syrk.hip)
int launch_lm_normal(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F, double* A,
                     int lda, double* rhs, double* jtj_diag);
// the sliced J^T of this rank's m-slices (fd.hip).  Columns mode (default, the reference's
// decomposition): the rank's cost-balanced FD tiles for every row, each tile's m-slices sent to
// the slices' ranks while the next tile computes.  Rows mode (PNOL_LM_FD=rows, linear residuals):
// every FD column on the rank's own residual rows -- no Jacobian exchange.
int launch_lm_jacobian(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, double* F0, int compute_f0,
                       double* JTs);
// LevMarqMPI trial point: F(x) (+ checkpoints) on this rank's rows in rows mode, then every
// rank's rows to all ranks; columns mode: all rows on every rank (fd.hip)
int launch_lm_eval(pnol_ctx* ctx, pnol_dobj* o, const double* x, double* F);
// LevMarqMPI's decomposition on this context: rows mode (1) or columns mode (0); the first call
// reads PNOL_LM_FD ("rows" -> 1, anything else -> 0), later calls keep it.  The LevMarqMPI
// drop-in re-reads the environment once per solve unless pnol_lm_set_fd_mode chose the mode,
// and checks it equal on every rank.
bool lm_rows_mode(pnol_ctx* ctx);
int lm_fd_mode_env();
// host waits bounded while an RCCL communicator is bound (runtime.cpp): PNOL_ERR_COMM after
// ncclCommAbort when an exchange fails or stalls past PNOL_COMM_TIMEOUT_S
int stream_wait(hipStream_t st);
int event_wait(hipEvent_t ev);
int lm_phased_env();   // PNOL_LM_PHASED / PNOL_LM_SUBPHASES (0 unphased, else the last tile's groups)

// Timer events that do not bracket one stream: timer_event records an event on `stream` when
// the timer `name` is on (nullptr otherwise); timer_pair books (a, b) under `name` -- elapsed
// b - a, floored at 0 (a pair across two streams: b may complete before a).
hipEvent_t timer_event(pnol_ctx* ctx, const char* name, hipStream_t stream);
void timer_pair(pnol_ctx* ctx, const char* name, hipEvent_t a, hipEvent_t b);

// Row-tile height of the fused BFGS pass (w = D^T y partials are per row tile): 256 rows when
// that still gives >= 512 workgroups (n >= 8192), else 128 (n = 4096: 256 workgroups instead of
// 128).  A function of n only, so the row-sharded pass sums exactly as the whole-matrix one.
int bfgs_pass_rows(int n);   // blas.hip (PNOL_PASS_ROWS = 64 / 128 / 256 overrides; tuning)

// number of XCDs (8 on MI355X): used only for blockIdx -> tile remaps (speed, never correctness)
constexpr int kNumXcd = 8;

}  // namespace pnol
