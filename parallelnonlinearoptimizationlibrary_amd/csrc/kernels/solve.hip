// solve.hip -- the damped LM solve, sigma = A^{-1} rhs (replaces luSolve, LevenbergMarquardt.cpp:83).
//
// A = J^T J + lambda diag(J^T J) is symmetric positive definite whenever J has full column
// rank, so the fast path is a blocked right-looking Cholesky (nb = 64), one panel per step:
//   k_potrf_diag   factor the 64 x 64 diagonal block (rows in registers, one wave)
//   k_trsm_panel   L21 = A21 L11^{-T}, one row per thread, row held in registers
//   syrk (MODE 1)  A22 -= L21 L21^T on 64 x 64 lower tiles, fp64 MFMA (syrk.hip)
// Method 3 runs the same factorisation as ONE persistent launch (k_chol_dag: POTRF / TRSM /
// UPDATE tile tasks from an atomic work queue, lookahead order, per-tile version flags);
// it is parity-tested but slower today (2.5 vs 1.9 ms at n = 2048: its critical path pays a
// flag hop per task and runs at one wave per SIMD).  Then
//   k_trsv_fwd/bwd forward / backward substitution: a workgroup per 64-row block, blocks
//                  chained by agent-scope ready flags
// A non-positive (or NaN) pivot flips to Gaussian elimination with partial pivoting in the
// reference's operation order (k_lu_*), which is also the method for n <= PNOL_SEQ_MAX so
// the small ExampleObjectives problems are bitwise equal to the CPU path.
#include "../pnol_internal.hpp"

#include <cstdlib>
#include <cstring>
#include <vector>

namespace pnol {
namespace {

constexpr int kNB = 64;
constexpr int kSpinCap = 1 << 24;   // ~1 s of polling: a broken chain ends the kernel, not the GPU
constexpr int kInfoChainTimeout = -7;

// ---- Cholesky ---------------------------------------------------------------------------
// Diagonal block, one wave: lane t holds row t of the 64 x 64 block in registers (fully
// unrolled, static indices).  Step j: the pivot comes from lane j, lane t scales its entry of
// column j, and every lane updates the rest of its row with scalar broadcasts of that column
// (right-looking, no memory round trips inside the factorisation).  Rows and columns
// past nbe are padded with the identity, so the unrolled code has no data-dependent shape.
__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// One right-looking step of the register Cholesky: column J is scaled by the pivot from lane
// J and published through LDS; row t is then updated with 16-byte LDS broadcasts of the
// column (two entries per ds_read_b128), in chunks of 16 columns so that the scheduler does
// not hoist a whole column of loads on top of the 128 registers holding the row.
template <int J>
__device__ __forceinline__ void potrf_step(double (&a)[kNB], double* __restrict__ col, int t, bool& bad) {
    const double piv = readlane_d(a[J], J);
    bad |= !(piv > 0.0);
    const double d = sqrt(piv);
    // a select, not a branch (a divergent branch here splits the scheduling regions and the
    // row spills).  Lanes t < J compute junk from their upper-triangle entries; it only ever
    // reaches upper-triangle entries, which are never written back.
    const double l = (t == J) ? d : a[J] / d;
    a[J] = l;
    col[t] = l;
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the column is in LDS for the wave
    __builtin_amdgcn_wave_barrier();
    constexpr int K0 = (J + 1) & ~1;
#pragma unroll
    for (int k = K0; k < kNB; k += 2) {
        const double2 c = *reinterpret_cast<const double2*>(col + k);
        if (k >= J + 1) a[k] = fma(-l, c.x, a[k]);
        a[k + 1] = fma(-l, c.y, a[k + 1]);
        if ((k & 15) == 14) __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (J + 1 < kNB) potrf_step<J + 1>(a, col, t, bad);
}

// Stage rows [r0, r0 + 64) x columns [c0, c0 + 64) of A into S with all 256 threads: 16
// unconditional loads per thread from clamped addresses are issued back to back (one memory
// latency instead of one per row), then `pick` decides what each entry becomes.
template <class Pick>
__device__ __forceinline__ void stage_block(double (*S)[kNB + 1], const double* __restrict__ A, long lda, int r0,
                                            int c0, int rlast, int clast, Pick pick) {
    const int t = threadIdx.x, c = t & 63, rq = t >> 6;
    double v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = rq + 4 * i;
        v[i] = A[(long)min(r0 + r, rlast) * lda + min(c0 + c, clast)];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = rq + 4 * i;
        S[r][c] = pick(r, c, v[i]);
    }
}

// Factor the diagonal tile at (k0, k0) in place (256 threads: all stage, wave 0 factors in
// registers).  Returns false (uniformly) and sets *info on a non-positive pivot.
__device__ __forceinline__ bool potrf_tile(double* __restrict__ A, long lda, int k0, int nbe, int* info,
                                           double (*S)[kNB + 1], double* __restrict__ col, int* flag_sh) {
    const int t = threadIdx.x;
    stage_block(S, A, lda, k0, k0, k0 + nbe - 1, k0 + nbe - 1, [nbe](int r, int c, double v) {
        return (r < nbe && c < nbe) ? (c <= r ? v : 0.0) : (r == c ? 1.0 : 0.0);
    });
    if (t == 0) *flag_sh = 0;
    __syncthreads();
    if (t < 64) {
        double a[kNB];
#pragma unroll
        for (int k = 0; k < kNB; ++k) a[k] = S[t][k];
        bool bad = false;
        potrf_step<0>(a, col, t, bad);
        if (bad) {
            if (t == 0) {
                *flag_sh = 1;
                atomicExch(info, k0 + 1);
            }
        } else {
#pragma unroll
            for (int k = 0; k < kNB; ++k) S[t][k] = a[k];
        }
    }
    __syncthreads();
    if (*flag_sh) return false;
    const int c = t & 63, rq = t >> 6;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = rq + 4 * i;
        if (r < nbe && c <= r) A[(long)(k0 + r) * lda + k0 + c] = S[r][c];
    }
    return true;
}

// One 64-row block of the panel below a factored diagonal tile: x L11^T = a, one thread per
// row with the row in registers (fully unrolled right-looking substitution, L11 read as LDS
// broadcasts).  All waves stage L11 and the rows (coalesced 512-byte row segments, loads
// batched), wave 0 solves, all waves store.
__device__ __forceinline__ void trsm_tile(double* __restrict__ A, long lda, int n, int k0, int nbe, int rbase,
                                          double (*L)[kNB + 1], double (*X)[kNB + 1]) {
    const int t = threadIdx.x;
    stage_block(L, A, lda, k0, k0, k0 + nbe - 1, k0 + nbe - 1, [nbe](int r, int c, double v) {
        return (r < nbe && c < nbe) ? v : (r == c ? 1.0 : 0.0);
    });
    stage_block(X, A, lda, rbase, k0, n - 1, k0 + nbe - 1, [nbe, rbase, n](int r, int c, double v) {
        return (rbase + r < n && c < nbe) ? v : 0.0;
    });
    __syncthreads();
    if (t < 64) {
        double x[kNB];
#pragma unroll
        for (int j = 0; j < kNB; ++j) x[j] = X[t][j];
#pragma unroll
        for (int j = 0; j < kNB; ++j) {
            x[j] = x[j] / L[j][j];
#pragma unroll
            for (int l = j + 1; l < kNB; ++l) x[l] = fma(-x[j], L[l][j], x[l]);
        }
#pragma unroll
        for (int j = 0; j < kNB; ++j) X[t][j] = x[j];
    }
    __syncthreads();
    const int c = t & 63, rq = t >> 6;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = rq + 4 * i, row = rbase + r;
        if (row < n && c < nbe) A[(long)row * lda + k0 + c] = X[r][c];
    }
}

__global__ __launch_bounds__(256) void k_potrf_diag(double* __restrict__ A, long lda, int k0, int nbe,
                                                    int* __restrict__ info) {
    __shared__ double S[kNB][kNB + 1];
    __shared__ __attribute__((aligned(16))) double col[kNB];
    __shared__ int flag_sh;
    if (*info != 0) return;   // an earlier block already failed
    potrf_tile(A, lda, k0, nbe, info, S, col, &flag_sh);
}

__global__ __launch_bounds__(256) void k_trsm_panel(double* __restrict__ A, long lda, int n, int k0, int nbe,
                                                    const int* __restrict__ info) {
    __shared__ double L[kNB][kNB + 1];
    __shared__ double X[kNB][kNB + 1];
    if (*info != 0) return;
    trsm_tile(A, lda, n, k0, nbe, k0 + nbe + blockIdx.x * kNB, L, X);
}

// ---- Tile-DAG Cholesky: one persistent launch -------------------------------------------
// The factorisation as a DAG of 64 x 64 tile tasks over the lower triangle (T = ceil(n/64)):
//   POTRF(k)      factor tile (k,k)                          needs ver(k,k) >= k
//   TRSM(k,i)     tile (i,k) <- A_ik L_kk^-T, i > k           needs ver(k,k) >= k+1, ver(i,k) >= k
//   UPDATE(k,i,j) tile (i,j) -= L_ik L_jk^T, k < j <= i       needs ver(i,j) >= k,
//                                                             ver(i,k) >= k+1, ver(j,k) >= k+1
// ver(i,j) counts the operations completed on tile (i,j); each task bumps it by one.  Tasks
// are numbered in a topological order with one step of lookahead (the updates of column k+1
// and then POTRF(k+1) / TRSM(k+1,.) come before the rest of step k's updates) and handed out
// by an atomic counter: a workgroup only ever waits on tasks claimed before its own, whose
// owners are running, so the queue drains without assuming co-residency.  Waits are relaxed
// sc1 polls + acquire fences; completion is a release fence by every wave, a workgroup
// barrier and one flag store (MI355X_MICROARCH.md, cross-CU / cross-XCD visibility).
enum { kTaskPotrf = 0, kTaskTrsm = 1, kTaskUpdate = 2 };
constexpr int kUpdPad = 18;                 // LDS row stride of the 16-wide K substages
constexpr int kUpdSub = kNB * kUpdPad;      // doubles per 64 x 16 substage

__device__ __forceinline__ bool wait_ver(const int* v, int target, int* info) {
    int it = 0;
    while (__hip_atomic_load(v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if ((++it & 63) == 0) {
            if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
            if (it > kSpinCap) {
                atomicExch(info, kInfoChainTimeout);
                return false;
            }
        }
    }
    return true;
}

// Stage the 64 x 64 tile (r0.., c0..) into four 64 x 16 K-substages (row stride 18 doubles):
// thread t owns row t >> 2 and the 16 columns of substage t & 3.  Rows >= n read as 0.
template <bool VEC>
__device__ __forceinline__ void stage_upd(double* __restrict__ dst, const double* __restrict__ A, long lda, int n,
                                          int r0, int c0) {
    const int t = threadIdx.x, row = t >> 2, sub = t & 3;
    const int gr = r0 + row;
    const double* src = A + (long)min(gr, n - 1) * lda + c0 + sub * 16;
    double2 v[8];
    if (VEC) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = reinterpret_cast<const double2*>(src)[q];
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = make_double2(src[2 * q], src[2 * q + 1]);
    }
    double* d = dst + sub * kUpdSub + row * kUpdPad;
#pragma unroll
    for (int q = 0; q < 8; ++q)
        reinterpret_cast<double2*>(d)[q] = gr < n ? v[q] : make_double2(0.0, 0.0);
}

// A_ij -= L_ik L_jk^T on fp64 MFMA: 4 waves as 2 x 2, each 32 x 32 (2 x 2 blocks of
// v_mfma_f64_16x16x4_f64), C loaded straight into the accumulator layout (lane l, reg r ->
// row (l >> 4) + 4 r, col l & 15) and the L_ik fragment negated so D = C + (-L_ik) L_jk^T.
// Tile k is never the last (partial) tile, so K = 64 always; rows/cols >= n are skipped.
template <bool VEC>
__device__ __forceinline__ void update_tile(double* __restrict__ A, long lda, int n, int i, int j, int k,
                                            double* __restrict__ P, double* __restrict__ Q) {
    typedef double d4 __attribute__((ext_vector_type(4)));
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wr = wave >> 1, wc = wave & 1;
    stage_upd<VEC>(P, A, lda, n, i * kNB, k * kNB);
    if (i != j) stage_upd<VEC>(Q, A, lda, n, j * kNB, k * kNB);
    const double* Qs = (i != j) ? Q : P;
    const int orow = lane >> 4, ocol = lane & 15;
    d4 acc[2][2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = i * kNB + wr * 32 + mi * 16 + orow + 4 * r;
                const int gj = j * kNB + wc * 32 + ni * 16 + ocol;
                acc[mi][ni][r] = A[(long)min(gi, n - 1) * lda + min(gj, n - 1)];
            }
    __syncthreads();
    const int frow = lane & 15, fk = lane >> 4;
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            double a[2], b[2];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) a[mi] = -P[sub * kUpdSub + (wr * 32 + mi * 16 + frow) * kUpdPad + kk * 4 + fk];
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) b[ni] = Qs[sub * kUpdSub + (wc * 32 + ni * 16 + frow) * kUpdPad + kk * 4 + fk];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
    }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gi = i * kNB + wr * 32 + mi * 16 + orow + 4 * r;
                const int gj = j * kNB + wc * 32 + ni * 16 + ocol;
                if (gi < n && gj < n && (i != j || gj <= gi)) A[(long)gi * lda + gj] = acc[mi][ni][r];
            }
}

template <bool VEC>
__global__ __launch_bounds__(256) void k_chol_dag(double* __restrict__ A, long lda, int n, int T,
                                                  const int4* __restrict__ tasks, int ntasks, int* counter, int* ver,
                                                  int* info, int dbg) {
    __shared__ __attribute__((aligned(16))) double smem[2 * 4 * kUpdSub];   // 73.7 KB, shared by the task kinds
    __shared__ int task_sh, ok_sh, flag_sh;
    const int t = threadIdx.x;
    for (;;) {
        if (t == 0) task_sh = atomicAdd(counter, 1);
        __syncthreads();
        const int g = task_sh;
        if (g >= ntasks) return;
        const int4 tk = tasks[g];   // {kind, k, i, j}
        const int kind = tk.x, k = tk.y, i = tk.z, j = tk.w;
        if (t == 0 && !(dbg & 2)) {
            bool ok;
            if (kind == kTaskPotrf) {
                ok = wait_ver(ver + k * T + k, k, info);
            } else if (kind == kTaskTrsm) {
                ok = wait_ver(ver + k * T + k, k + 1, info) && wait_ver(ver + i * T + k, k, info);
            } else {
                ok = wait_ver(ver + i * T + j, k, info) && wait_ver(ver + i * T + k, k + 1, info) &&
                     wait_ver(ver + j * T + k, k + 1, info);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            ok_sh = ok;
        }
        if (t == 0 && (dbg & 2)) ok_sh = 1;
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (!ok_sh) return;
        int vi = 0, vj = 0;
        if (dbg & 1) {
            vi = kind == kTaskUpdate ? i : (kind == kTaskTrsm ? i : k);
            vj = kind == kTaskUpdate ? j : k;
        } else if (kind == kTaskPotrf) {
            const int k0 = k * kNB, nbe = min(kNB, n - k0);
            auto S = reinterpret_cast<double (*)[kNB + 1]>(smem);
            if (!potrf_tile(A, lda, k0, nbe, info, S, smem + kNB * (kNB + 1), &flag_sh)) return;
            vi = k; vj = k;
        } else if (kind == kTaskTrsm) {
            const int k0 = k * kNB;
            auto L = reinterpret_cast<double (*)[kNB + 1]>(smem);
            auto X = reinterpret_cast<double (*)[kNB + 1]>(smem + kNB * (kNB + 1));
            trsm_tile(A, lda, n, k0, kNB, i * kNB, L, X);
            vi = i; vj = k;
        } else {
            update_tile<VEC>(A, lda, n, i, j, k, smem, smem + 4 * kUpdSub);
            vi = i; vj = j;
        }
        // publish: every wave drains and releases its stores, then one flag store
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (t == 0 && !(dbg & 4)) __hip_atomic_store(ver + vi * T + vj, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// L z = b on one diagonal block, lane i owns b_i; z_J = b_J / L_JJ (reciprocal precomputed by
// each lane for its own row) is broadcast from lane J through scalar registers.
template <int J>
__device__ __forceinline__ void trsv_fwd_step(const double (*T)[65], double& bi, double rd, int lane) {
    const double zj = readlane_d(bi * rd, J);
    bi = (lane == J) ? zj : fma(-T[lane][J], zj, bi);   // T[lane][J] = 0 above the diagonal
    if constexpr (J + 1 < 64) trsv_fwd_step<J + 1>(T, bi, rd, lane);
}

// L^T x = z on one diagonal block, from the last row up.
template <int J>
__device__ __forceinline__ void trsv_bwd_step(const double (*T)[65], double& zi, double rd, int lane) {
    const double xj = readlane_d(zi * rd, J);
    zi = (lane == J) ? xj : fma(-T[J][lane], xj, zi);   // T[J][lane] = 0 right of the diagonal
    if constexpr (J > 0) trsv_bwd_step<J - 1>(T, zi, rd, lane);
}

// ---- Triangular solves: one workgroup per 64-row block, blocks chained by ready flags ----
// Forward (L z = b): workgroup w owns rows [64 w, 64 w + 64).  For each earlier block c it
// prefetches L_wc into registers, waits until z_c is published (flag c == epoch), and
// accumulates L_wc z_c; then it solves its diagonal block (staged in LDS at entry) and
// publishes z_w.  Workgroups only wait on lower blockIdx, so in-order dispatch guarantees
// progress even when the grid is not co-resident.  Backward (L^T x = z) runs the blocks in
// reverse: workgroup b owns block w = nblk - 1 - b and reads the column blocks L_cw, c > w.
// The memory traffic (one read of the lower triangle per direction) is spread over nblk CUs;
// the critical path is one flag hop + one diagonal solve per block.

// 256 threads: stage the lower-triangular diagonal block (identity padding) into T.
__device__ __forceinline__ void stage_diag_256(double (*T)[kNB + 1], const double* __restrict__ L, long lda,
                                               int i0, int nb) {
    stage_block(T, L, lda, i0, i0, i0 + nb - 1, i0 + nb - 1, [nb](int r, int c, double v) {
        return (r < nb && c < nb) ? (c <= r ? v : 0.0) : (r == c ? 1.0 : 0.0);
    });
}

// Wait until *flag == epoch: thread 0 polls with relaxed agent-scope loads (global_load sc1,
// no cache invalidation per poll), then one acquire fence; the workgroup synchronises and
// every thread performs its own acquire fence before reading the data the flag guards
// (MI355X_MICROARCH.md: per-CU L1 and per-XCD L2 are not coherent with other CUs' stores).
// Returns false (uniformly) if the cap was hit.
__device__ __forceinline__ bool wait_flag(const int* flag, int epoch, int* info, int* abort_sh) {
    if (threadIdx.x == 0) {
        int it = 0;
        int ok = 1;
        while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
            __builtin_amdgcn_s_sleep(1);
            if (++it > kSpinCap) {
                ok = 0;
                atomicExch(info, kInfoChainTimeout);   // the host falls back to LU
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        *abort_sh = !ok;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return *abort_sh == 0;
}

__global__ __launch_bounds__(256) void k_trsv_fwd(const double* __restrict__ L, long lda, int n,
                                                  const double* __restrict__ b, double* z, int* flags, int epoch,
                                                  int* info) {
    __shared__ double T[kNB][kNB + 1];
    __shared__ double part[4][kNB];
    __shared__ int abort_sh;
    if (*info != 0) return;
    const int w = blockIdx.x, t = threadIdx.x;
    const int i0 = w * kNB, nb = min(kNB, n - i0);
    stage_diag_256(T, L, lda, i0, nb);
    // thread (r, q): row r of the block, columns q*16 .. q*16+15 of each earlier block
    const int r = t >> 2, q = t & 3;
    const long rowoff = (long)min(i0 + r, n - 1) * lda + q * 16;
    double acc = 0.0;
    double Lv[16], Ln[16];
    if (w > 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) Lv[i] = L[rowoff + i];
    }
    for (int c = 0; c < w; ++c) {
        if (c + 1 < w) {
#pragma unroll
            for (int i = 0; i < 16; ++i) Ln[i] = L[rowoff + (long)(c + 1) * kNB + i];
        }
        if (!wait_flag(flags + c, epoch, info, &abort_sh)) return;
        const double* zc = z + c * kNB + q * 16;   // published, full block (c < w)
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 16; ++i) s = fma(Lv[i], zc[i], s);
        acc += s;
#pragma unroll
        for (int i = 0; i < 16; ++i) Lv[i] = Ln[i];
    }
    part[q][r] = acc;
    __syncthreads();
    if (t < 64) {
        const double sum = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
        double bi = t < nb ? b[i0 + t] - sum : 0.0;
        const double rd = 1.0 / T[t][t];
        trsv_fwd_step<0>(T, bi, rd, t);
        z[i0 + t] = t < nb ? bi : 0.0;   // z has nblk * 64 entries: padded rows are 0
        // release by lane 0: the fence (wait + L2 writeback) is wave-wide and covers the
        // stores of all 64 lanes above
        if (t == 0) __hip_atomic_store(flags + w, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ __launch_bounds__(256) void k_trsv_bwd(const double* __restrict__ L, long lda, int n,
                                                  const double* __restrict__ z, double* xw,
                                                  double* __restrict__ x, int* flags, int epoch, int* info) {
    __shared__ double T[kNB][kNB + 1];
    __shared__ double part[4][kNB];
    __shared__ int abort_sh;
    if (*info != 0) return;
    const int nblk = gridDim.x, bidx = blockIdx.x, t = threadIdx.x;
    const int w = nblk - 1 - bidx;
    const int i0 = w * kNB, nb = min(kNB, n - i0);
    stage_diag_256(T, L, lda, i0, nb);
    // thread (j, q): column j of block w, rows q*16 .. q*16+15 of each later block
    const int j = t & 63, q = t >> 6;
    const int col = min(i0 + j, n - 1);
    double acc = 0.0;
    double Lv[16], Ln[16];
    auto load_blk = [&](double (&dst)[16], int c) {
#pragma unroll
        for (int i = 0; i < 16; ++i) dst[i] = L[(long)min(c * kNB + q * 16 + i, n - 1) * lda + col];
    };
    if (w + 1 < nblk) load_blk(Lv, nblk - 1);
    for (int c = nblk - 1; c > w; --c) {
        if (c - 1 > w) load_blk(Ln, c - 1);
        if (!wait_flag(flags + c, epoch, info, &abort_sh)) return;
        const double* xc = xw + c * kNB + q * 16;   // padded rows of the last block are 0
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 16; ++i) s = fma(Lv[i], xc[i], s);
        acc += s;
#pragma unroll
        for (int i = 0; i < 16; ++i) Lv[i] = Ln[i];
    }
    part[q][j] = acc;
    __syncthreads();
    if (t < 64) {
        const double sum = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
        double zi = t < nb ? z[i0 + t] - sum : 0.0;
        const double rd = 1.0 / T[t][t];
        trsv_bwd_step<63>(T, zi, rd, t);
        xw[i0 + t] = t < nb ? zi : 0.0;
        if (t < nb) x[i0 + t] = zi;
        if (t == 0) __hip_atomic_store(flags + w, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- Gaussian elimination with partial pivoting, reference operation order ------------
// Single workgroup (small n).  M is a working copy (n x n, ld n), b the rhs copy.
__global__ __launch_bounds__(1024) void k_lu_small(double* __restrict__ M, double* __restrict__ b,
                                                   double* __restrict__ f, int n, double* __restrict__ x,
                                                   int* __restrict__ info) {
    __shared__ int piv_sh;
    const int t = threadIdx.x;
    for (int k = 0; k < n; ++k) {
        if (t == 0) {
            int piv = k;
            double best = fabs(M[(long)k * n + k]);
            for (int i = k + 1; i < n; ++i) {
                double v = fabs(M[(long)i * n + k]);
                if (v > best) { best = v; piv = i; }
            }
            piv_sh = piv;
        }
        __syncthreads();
        const int piv = piv_sh;
        if (piv != k) {
            for (int j = t; j < n; j += blockDim.x) {
                double tmp = M[(long)k * n + j];
                M[(long)k * n + j] = M[(long)piv * n + j];
                M[(long)piv * n + j] = tmp;
            }
            if (t == 0) { double tmp = b[k]; b[k] = b[piv]; b[piv] = tmp; }
        }
        __syncthreads();
        const double akk = M[(long)k * n + k];
        for (int i = k + 1 + t; i < n; i += blockDim.x) f[i] = M[(long)i * n + k] / akk;
        __syncthreads();
        const int rows = n - k - 1, cols = n - k;
        for (int e = t; e < rows * cols; e += blockDim.x) {
            int i = k + 1 + e / cols, j = k + e % cols;
            M[(long)i * n + j] = M[(long)i * n + j] - f[i] * M[(long)k * n + j];
        }
        for (int i = k + 1 + t; i < n; i += blockDim.x) b[i] = b[i] - f[i] * b[k];
        __syncthreads();
    }
    if (t == 0) {
        int sing = 0;
        for (int i = n - 1; i >= 0; --i) {
            double s = b[i];
            for (int j = i + 1; j < n; ++j) s = s - M[(long)i * n + j] * x[j];
            double d = M[(long)i * n + i];
            if (d == 0.0) sing = 1;
            x[i] = s / d;
        }
        *info = sing ? -1 : 2;
    }
}

// Multi-launch form for large n (fallback): per column k one pivot/swap/factor kernel and
// one elimination kernel over the trailing block; same per-element operations.
__global__ void k_lu_pivot(double* __restrict__ M, double* __restrict__ b, double* __restrict__ f, int n, int k) {
    __shared__ int piv_sh;
    const int t = threadIdx.x;
    if (t == 0) {
        int piv = k;
        double best = fabs(M[(long)k * n + k]);
        for (int i = k + 1; i < n; ++i) {
            double v = fabs(M[(long)i * n + k]);
            if (v > best) { best = v; piv = i; }
        }
        piv_sh = piv;
    }
    __syncthreads();
    const int piv = piv_sh;
    if (piv != k) {
        for (int j = t; j < n; j += blockDim.x) {
            double tmp = M[(long)k * n + j];
            M[(long)k * n + j] = M[(long)piv * n + j];
            M[(long)piv * n + j] = tmp;
        }
        if (t == 0) { double tmp = b[k]; b[k] = b[piv]; b[piv] = tmp; }
    }
    __syncthreads();
    const double akk = M[(long)k * n + k];
    for (int i = k + 1 + t; i < n; i += blockDim.x) f[i] = M[(long)i * n + k] / akk;
}

__global__ void k_lu_eliminate(double* __restrict__ M, double* __restrict__ b, const double* __restrict__ f,
                               int n, int k) {
    const int rows = n - k - 1, cols = n - k;
    const long total = (long)rows * cols;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        int i = k + 1 + (int)(e / cols), j = k + (int)(e % cols);
        M[(long)i * n + j] = M[(long)i * n + j] - f[i] * M[(long)k * n + j];
    }
    if (blockIdx.x == 0)
        for (int i = k + 1 + threadIdx.x; i < n; i += blockDim.x) b[i] = b[i] - f[i] * b[k];
}

__global__ void k_lu_backsub(const double* __restrict__ M, const double* __restrict__ b, int n,
                             double* __restrict__ x, int* __restrict__ info) {
    if (threadIdx.x != 0) return;
    int sing = 0;
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int j = i + 1; j < n; ++j) s = s - M[(long)i * n + j] * x[j];
        double d = M[(long)i * n + i];
        if (d == 0.0) sing = 1;
        x[i] = s / d;
    }
    *info = sing ? -1 : 2;
}

// ---- matrixInverse: one elimination, n right-hand sides -------------------------------------
// The reference inverts column by column, luSolve(B, e_c): Gaussian elimination
// with partial pivoting on a copy of B, the rhs updated b_i -= f_i b_k with the same f, then back
// substitution.  The pivots and multipliers depend on B alone, so eliminating the augmented
// [B | I] once applies exactly the operations each column's solve applies to its rhs (the rhs
// rows swapped, then b_i - f_i b_k for every k in order), and the back substitution then runs
// per column in the reference's order.  M is n x 2n (row stride ldm >= 2n).
__global__ void k_luinv_pivot(double* __restrict__ M, long ldm, int n, double* __restrict__ f, int k) {
    __shared__ int piv_sh;
    const int t = threadIdx.x;
    if (t == 0) {
        int piv = k;
        double best = fabs(M[(long)k * ldm + k]);
        for (int i = k + 1; i < n; ++i) {
            double v = fabs(M[(long)i * ldm + k]);
            if (v > best) { best = v; piv = i; }
        }
        piv_sh = piv;
    }
    __syncthreads();
    const int piv = piv_sh;
    if (piv != k)
        for (int j = t; j < 2 * n; j += blockDim.x) {   // the row of B and the rhs entries
            double tmp = M[(long)k * ldm + j];
            M[(long)k * ldm + j] = M[(long)piv * ldm + j];
            M[(long)piv * ldm + j] = tmp;
        }
    __syncthreads();
    const double akk = M[(long)k * ldm + k];
    for (int i = k + 1 + t; i < n; i += blockDim.x) f[i] = M[(long)i * ldm + k] / akk;
}

// rows i > k: M[i][j] = M[i][j] - f_i M[k][j] for j in [k, 2n) -- B's columns from k as
// luSolve's elimination, and every rhs column as its b_i = b_i - f_i b_k
__global__ void k_luinv_eliminate(double* __restrict__ M, long ldm, int n, const double* __restrict__ f, int k) {
    const int cols = 2 * n - k;
    const long total = (long)(n - k - 1) * cols;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int i = k + 1 + (int)(e / cols), j = k + (int)(e % cols);
        M[(long)i * ldm + j] = M[(long)i * ldm + j] - f[i] * M[(long)k * ldm + j];
    }
}

// column c of the inverse: x_i = (b_i - sum_{j > i} U_ij x_j) / U_ii, j ascending, i descending;
// one thread per column (the U reads are the same address for the whole wave)
__global__ void k_luinv_backsub(const double* __restrict__ M, long ldm, int n, double* __restrict__ X, long ldx,
                                int* __restrict__ info) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    int sing = 0;
    for (int i = n - 1; i >= 0; --i) {
        const double* Ui = M + (long)i * ldm;
        double s = Ui[n + c];
        for (int j = i + 1; j < n; ++j) s = s - Ui[j] * X[(long)j * ldx + c];
        const double d = Ui[i];
        if (d == 0.0) sing = 1;
        X[(long)i * ldx + c] = s / d;
    }
    if (sing) atomicExch(info, -1);
}

__global__ void k_luinv_load(const double* __restrict__ B, long ldb, int n, double* __restrict__ M, long ldm) {
    const long total = (long)n * 2 * n;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int i = (int)(e / (2 * n)), j = (int)(e % (2 * n));
        M[(long)i * ldm + j] = j < n ? B[(long)i * ldb + j] : (j - n == i ? 1.0 : 0.0);
    }
}

__global__ void k_copy_matrix(const double* __restrict__ A, long lda, double* __restrict__ M, int n) {
    long total = (long)n * n;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x)
        M[e] = A[(e / n) * lda + e % n];
}

__global__ void k_set_int(int* p, int v) { *p = v; }

}  // namespace

static int lu_solve(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo) {
    void *M = nullptr, *b = nullptr, *f = nullptr;
    PNOL_CHECK(ws_get(ctx, "lu_M", sizeof(double) * (size_t)n * n, &M));
    PNOL_CHECK(ws_get(ctx, "lu_b", sizeof(double) * (size_t)n, &b));
    PNOL_CHECK(ws_get(ctx, "lu_f", sizeof(double) * (size_t)n, &f));
    long total = (long)n * n;
    hipLaunchKernelGGL(k_copy_matrix, dim3((int)std::min<long>((total + 255) / 256, 4096)), dim3(256), 0, ctx->stream,
                       A, (long)lda, (double*)M, n);
    PNOL_HIP(hipMemcpyAsync(b, rhs, sizeof(double) * n, hipMemcpyDeviceToDevice, ctx->stream));
    if (n <= 256) {
        hipLaunchKernelGGL(k_lu_small, dim3(1), dim3(1024), 0, ctx->stream, (double*)M, (double*)b, (double*)f, n,
                           sigma, dinfo);
        return launch_check();
    }
    for (int k = 0; k < n; ++k) {
        hipLaunchKernelGGL(k_lu_pivot, dim3(1), dim3(1024), 0, ctx->stream, (double*)M, (double*)b, (double*)f, n, k);
        long work = (long)(n - k - 1) * (n - k);
        int blocks = (int)std::max<long>(1, std::min<long>((work + 255) / 256, 2048));
        hipLaunchKernelGGL(k_lu_eliminate, dim3(blocks), dim3(256), 0, ctx->stream, (double*)M, (double*)b,
                           (const double*)f, n, k);
    }
    hipLaunchKernelGGL(k_lu_backsub, dim3(1), dim3(64), 0, ctx->stream, (const double*)M, (const double*)b, n, sigma,
                       dinfo);
    return launch_check();
}

int launch_matrix_inverse(pnol_ctx* ctx, const double* B, int ldb, int n, double* Binv, int ldi, int* info_host) {
    if (!B || !Binv || n <= 0 || ldb < n || ldi < n) return PNOL_ERR_ARG;
    const long ldm = 2L * n;
    void *M = nullptr, *f = nullptr, *di = nullptr;
    PNOL_CHECK(ws_get(ctx, "luinv_M", sizeof(double) * (size_t)n * ldm, &M));
    PNOL_CHECK(ws_get(ctx, "luinv_f", sizeof(double) * (size_t)n, &f));
    PNOL_CHECK(ws_get(ctx, "luinv_info", sizeof(int) * 4, &di));
    const long total = (long)n * ldm;
    hipLaunchKernelGGL(k_luinv_load, dim3((int)std::min<long>((total + 255) / 256, 4096)), dim3(256), 0, ctx->stream, B,
                       (long)ldb, n, (double*)M, ldm);
    hipLaunchKernelGGL(k_set_int, dim3(1), dim3(1), 0, ctx->stream, (int*)di, 0);
    for (int k = 0; k < n; ++k) {
        hipLaunchKernelGGL(k_luinv_pivot, dim3(1), dim3(1024), 0, ctx->stream, (double*)M, ldm, n, (double*)f, k);
        const long work = (long)(n - k - 1) * (2 * n - k);
        if (work > 0) {
            const int blocks = (int)std::max<long>(1, std::min<long>((work + 255) / 256, 4096));
            hipLaunchKernelGGL(k_luinv_eliminate, dim3(blocks), dim3(256), 0, ctx->stream, (double*)M, ldm, n,
                               (const double*)f, k);
        }
    }
    hipLaunchKernelGGL(k_luinv_backsub, dim3((n + 63) / 64), dim3(64), 0, ctx->stream, (const double*)M, ldm, n, Binv,
                       (long)ldi, (int*)di);
    PNOL_CHECK(launch_check());
    int h = 0;
    PNOL_HIP(hipMemcpyAsync(&h, di, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    PNOL_HIP(hipStreamSynchronize(ctx->stream));
    if (info_host) *info_host = h;
    return PNOL_OK;
}

// Task list of the tile-DAG Cholesky in its lookahead topological order ({kind, k, i, j}).
static std::vector<int4> chol_tasks(int T) {
    std::vector<int4> v;
    v.push_back(make_int4(kTaskPotrf, 0, 0, 0));
    for (int i = 1; i < T; ++i) v.push_back(make_int4(kTaskTrsm, 0, i, 0));
    for (int k = 0; k + 1 < T; ++k) {
        for (int i = k + 1; i < T; ++i) v.push_back(make_int4(kTaskUpdate, k, i, k + 1));
        v.push_back(make_int4(kTaskPotrf, k + 1, k + 1, k + 1));
        for (int i = k + 2; i < T; ++i) v.push_back(make_int4(kTaskTrsm, k + 1, i, 0));
        for (int j = k + 2; j < T; ++j)
            for (int i = j; i < T; ++i) v.push_back(make_int4(kTaskUpdate, k, i, j));
    }
    return v;
}

// Factor A (lower triangle) in one persistent launch; *dinfo != 0 afterwards on failure.
static int chol_factor_dag(pnol_ctx* ctx, double* A, int lda, int n, int* dinfo) {
    const int T = (n + kNB - 1) / kNB;
    const long ntasks = (long)T + (long)T * (T - 1) / 2 + (long)(T - 1) * T * (T + 1) / 6;
    void *tasks_v = nullptr, *ver_v = nullptr;
    PNOL_CHECK(ws_get(ctx, "chol_tasks", sizeof(int4) * (size_t)ntasks, &tasks_v));
    if (tasks_v != ctx->chol_tasks || ctx->chol_tasks_T != T) {
        std::vector<int4> h = chol_tasks(T);
        if ((long)h.size() != ntasks) return PNOL_ERR_ARG;
        PNOL_HIP(hipMemcpyAsync(tasks_v, h.data(), sizeof(int4) * h.size(), hipMemcpyHostToDevice, ctx->stream));
        PNOL_HIP(hipStreamSynchronize(ctx->stream));
        ctx->chol_tasks = tasks_v;
        ctx->chol_tasks_T = T;
    }
    PNOL_CHECK(ws_get(ctx, "chol_ver", sizeof(int) * (size_t)(T * T + 1), &ver_v));
    int* ver = (int*)ver_v;
    PNOL_HIP(hipMemsetAsync(ver, 0, sizeof(int) * (size_t)(T * T + 1), ctx->stream));
    const int grid = (int)std::min<long>(ntasks, 2L * (ctx->num_cu > 0 ? ctx->num_cu : 256));
    const bool vec = (lda % 2) == 0 && (reinterpret_cast<uintptr_t>(A) & 15u) == 0;
    static const int dbg = [] {   // temporary fault-bisection switch
        const char* e = std::getenv("PNOL_DAG_DEBUG");
        return e ? std::atoi(e) : 0;
    }();
    if (dbg & 8) return PNOL_OK;   // skip the launch entirely
    if (vec)
        hipLaunchKernelGGL((k_chol_dag<true>), dim3(grid), dim3(256), 0, ctx->stream, A, (long)lda, n, T,
                           (const int4*)tasks_v, (int)ntasks, ver + T * T, ver, dinfo, dbg);
    else
        hipLaunchKernelGGL((k_chol_dag<false>), dim3(grid), dim3(256), 0, ctx->stream, A, (long)lda, n, T,
                           (const int4*)tasks_v, (int)ntasks, ver + T * T, ver, dinfo, dbg);
    return launch_check();
}

// L L^T sigma = rhs with the factor in the lower triangle of A (two flag-chained launches).
static int chol_trsv(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo) {
    const int nblk = (n + kNB - 1) / kNB;
    void *flags_v = nullptr, *zw = nullptr, *xw = nullptr;
    PNOL_CHECK(ws_get(ctx, "trsv_flags", sizeof(int) * (size_t)(2 * nblk), &flags_v));
    PNOL_CHECK(ws_get(ctx, "trsv_z", sizeof(double) * (size_t)nblk * kNB, &zw));
    PNOL_CHECK(ws_get(ctx, "trsv_x", sizeof(double) * (size_t)nblk * kNB, &xw));
    int* flags = (int*)flags_v;
    if (flags != ctx->solve_flags || ctx->solve_epoch >= (1 << 30)) {
        // fresh (or regrown) flag buffer: flags start below every epoch handed out
        PNOL_HIP(hipMemsetAsync(flags, 0, sizeof(int) * (size_t)(2 * nblk), ctx->stream));
        ctx->solve_flags = flags;
        ctx->solve_epoch = 0;
    }
    const int epoch = ++ctx->solve_epoch;
    hipLaunchKernelGGL(k_trsv_fwd, dim3(nblk), dim3(256), 0, ctx->stream, A, (long)lda, n, rhs, (double*)zw, flags,
                       epoch, dinfo);
    hipLaunchKernelGGL(k_trsv_bwd, dim3(nblk), dim3(256), 0, ctx->stream, A, (long)lda, n, (const double*)zw,
                       (double*)xw, sigma, flags + nblk, epoch, dinfo);
    return launch_check();
}

int launch_solve(pnol_ctx* ctx, double* A, int lda, const double* rhs, double* sigma, int n, int method,
                 int* info) {
    if (!A || !rhs || !sigma || n <= 0 || lda < n) return PNOL_ERR_ARG;
    void* dinfo_v = nullptr;
    PNOL_CHECK(ws_get(ctx, "solve_info", sizeof(int) * 4, &dinfo_v));
    int* dinfo = (int*)dinfo_v;
    int used = 0;
    int variant = method;   // the tile Cholesky's form: 4 per-step launches, 5 persistent
    if (method == 0) {
        method = (n <= PNOL_SEQ_MAX) ? 2 : 4;
        variant = 0;         // the default form (launch_chol_solve_v)
    }
    if (method == 4 || method == 5) {
        // lookahead tile Cholesky with diagonal inverses (chol.hip); A itself is not modified
        PNOL_CHECK(launch_chol_solve_v(ctx, A, lda, rhs, sigma, n, dinfo, variant));
        int hinfo = 0;
        PNOL_HIP(hipMemcpyAsync(&hinfo, dinfo, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        PNOL_HIP(hipStreamSynchronize(ctx->stream));
        if (hinfo == 0) {
            if (info) *info = 1;
            return PNOL_OK;
        }
        method = 2;   // non-positive pivot or a timed-out chain: reference-order LU on A
    }
    const bool multi_launch = method != 3;   // method 3: the tile-DAG launch (experimental)
    if (method == 3) method = 1;
    if (method == 1) {
        // keep a copy of A so a failed factorisation can fall back to LU on the original
        void* Acopy = nullptr;
        PNOL_CHECK(ws_get(ctx, "chol_Acopy", sizeof(double) * (size_t)n * n, &Acopy));
        long total = (long)n * n;
        hipLaunchKernelGGL(k_copy_matrix, dim3((int)std::min<long>((total + 255) / 256, 4096)), dim3(256), 0,
                           ctx->stream, (const double*)A, (long)lda, (double*)Acopy, n);
        hipLaunchKernelGGL(k_set_int, dim3(1), dim3(1), 0, ctx->stream, dinfo, 0);
        if (!multi_launch) PNOL_CHECK(chol_factor_dag(ctx, A, lda, n, dinfo));
        for (int k0 = 0; multi_launch && k0 < n; k0 += kNB) {
            const int nbe = std::min(kNB, n - k0);
            hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(256), 0, ctx->stream, A, (long)lda, k0, nbe, dinfo);
            const int below = n - k0 - nbe;
            if (below > 0) {
                hipLaunchKernelGGL(k_trsm_panel, dim3((below + kNB - 1) / kNB), dim3(256), 0, ctx->stream, A, (long)lda, n,
                                   k0, nbe, (const int*)dinfo);
                PNOL_CHECK(launch_syrk_lower(ctx, A + (long)(k0 + nbe) * lda + k0, lda, below, nbe, -1.0,
                                             A + (long)(k0 + nbe) * lda + k0 + nbe, lda, 1));
            }
        }
        PNOL_CHECK(chol_trsv(ctx, A, lda, rhs, sigma, n, dinfo));
        int hinfo = 0;
        PNOL_HIP(hipMemcpyAsync(&hinfo, dinfo, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        PNOL_HIP(hipStreamSynchronize(ctx->stream));
        if (hinfo == 0) {
            used = 1;
        } else {
            PNOL_CHECK(lu_solve(ctx, (const double*)Acopy, n, rhs, sigma, n, dinfo));
            method = 2;
            used = -2;  // resolved below
        }
    } else {
        PNOL_CHECK(lu_solve(ctx, A, lda, rhs, sigma, n, dinfo));
    }
    if (method == 2) {
        int hinfo = 0;
        PNOL_HIP(hipMemcpyAsync(&hinfo, dinfo, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        PNOL_HIP(hipStreamSynchronize(ctx->stream));
        used = hinfo;
    }
    if (info) *info = used;
    return PNOL_OK;
}

}  // namespace pnol
