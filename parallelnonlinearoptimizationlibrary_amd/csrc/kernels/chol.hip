// chol.hip -- the damped LM solve as a lookahead tile Cholesky with explicit diagonal-tile
// inverses (pnol_solve_d method 4, the default for n > PNOL_SEQ_MAX).  Replaces
// luSolve(A, rhs, sigma), LevenbergMarquardt.cpp:83 / LevenbergMarquardtMPI.cpp:88.
//
// A (n x n, SPD) is copied into a zero-padded T*64 x T*64 workspace P (identity on the padded
// diagonal) and factored by 64 x 64 tiles, one launch per panel step k = -1 .. T-2:
//   diag WG      tile (k+1,k+1): L = A_{k+1,k} W_k^T and A_{k+1,k+1} -= L L^T on fp64 MFMA,
//                then the 64-step Cholesky of the tile (wave 0, rows in registers) with its
//                inverse W_{k+1} = L_{k+1,k+1}^{-1} formed one column step behind (wave 1)
//   panel WGs    L_ik = A_ik W_k^T (TRSM as an MFMA product), published by a per-row flag;
//                they also carry the forward substitution: z_k = W_k b_k, b_i -= L_ik z_k
//   update WGs   A_ij -= L_ik L_jk^T (fp64 MFMA) once rows i and j of the panel are flagged
// The diagonal workgroup recomputes its own L_{k+1,k} instead of waiting for it, so the critical
// path of a step is one workgroup's MFMA + factor + inverse; the trailing update runs beside it.
// A final launch solves L^T x = z by block rows from the bottom up, chained by ready flags, each
// diagonal block applied as the product W_w^T v.
// A non-positive (or NaN) pivot sets *info; the host then solves with Gaussian elimination on
// the untouched A (solve.hip).  Every wait is spin-capped, so a broken chain ends in a fallback.
#include "../pnol_internal.hpp"

#include <algorithm>

namespace pnol {
namespace {

constexpr int NB = 64;
constexpr int kPad = 18;             // LDS row stride of a 64 x 16 K-substage (doubles)
constexpr int kSub = NB * kPad;      // doubles per substage
constexpr int kStage = 4 * kSub;     // one 64 x 64 tile as four substages
constexpr int kSpin = 1 << 24;       // ~1 s of polling
constexpr int kInfoTimeout = -7;
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// 1/sqrt(x) to full double precision: hardware estimate + two Newton steps (r += r (1 - x r^2) / 2)
__device__ __forceinline__ double rsqrt_nr(double x) {
    double r = __builtin_amdgcn_rsq(x);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double e = fma(-x, r * r, 1.0);
        r = fma(0.5 * r, e, r);
    }
    return r;
}

// Stage the 64 x 64 tile at (r0, c0) of P into four 64 x 16 substages (row stride kPad):
// thread t owns row t >> 2 and the 16 columns of substage t & 3 (eight 16-byte loads).
__device__ __forceinline__ void stage_tile(double* __restrict__ dst, const double* __restrict__ P, long ldp, int r0,
                                           int c0) {
    const int t = threadIdx.x, row = t >> 2, sub = t & 3;
    const double2* src = reinterpret_cast<const double2*>(P + (long)(r0 + row) * ldp + c0 + sub * 16);
    double2 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = src[q];
    double2* d = reinterpret_cast<double2*>(dst + sub * kSub + row * kPad);
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = v[q];
}

// acc (this wave's 32 x 32 quadrant (wr, wc)) += sign * X Y^T over the 64-wide K of two staged
// tiles, v_mfma_f64_16x16x4_f64.  Fragment layouts: A/B lane l holds row l & 15, k = l >> 4;
// C/D lane l, register r -> row (l >> 4) + 4 r, column l & 15.
template <bool NEG>
__device__ __forceinline__ void mfma_xyt(d4 (&acc)[2][2], const double* __restrict__ X, const double* __restrict__ Y,
                                         int wr, int wc, int lane) {
    const int frow = lane & 15, fk = lane >> 4;
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            double a[2], b[2];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                a[mi] = X[sub * kSub + (wr * 32 + mi * 16 + frow) * kPad + kk * 4 + fk];
                if (NEG) a[mi] = -a[mi];
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) b[ni] = Y[sub * kSub + (wc * 32 + ni * 16 + frow) * kPad + kk * 4 + fk];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
    }
}

__device__ __forceinline__ int acc_row(int wr, int mi, int lane, int r) { return wr * 32 + mi * 16 + (lane >> 4) + 4 * r; }
__device__ __forceinline__ int acc_col(int wc, int ni, int lane) { return wc * 32 + ni * 16 + (lane & 15); }

__device__ __forceinline__ void acc_zero(d4 (&acc)[2][2]) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};
}

__device__ __forceinline__ void acc_load(d4 (&acc)[2][2], const double* __restrict__ P, long ldp, int r0, int c0,
                                         int wr, int wc, int lane) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[mi][ni][r] = P[(long)(r0 + acc_row(wr, mi, lane, r)) * ldp + c0 + acc_col(wc, ni, lane)];
}

__device__ __forceinline__ void acc_store(const d4 (&acc)[2][2], double* __restrict__ P, long ldp, int r0, int c0,
                                          int wr, int wc, int lane) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                P[(long)(r0 + acc_row(wr, mi, lane, r)) * ldp + c0 + acc_col(wc, ni, lane)] = acc[mi][ni][r];
}

// accumulator -> LDS in the substage layout (the tile as the X operand of the next product)
__device__ __forceinline__ void acc_to_stage(const d4 (&acc)[2][2], double* __restrict__ X, int wr, int wc, int lane) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = acc_row(wr, mi, lane, r), col = acc_col(wc, ni, lane);
                X[(col >> 4) * kSub + row * kPad + (col & 15)] = acc[mi][ni][r];
            }
}

// accumulator -> LDS row-major 64 x 65
__device__ __forceinline__ void acc_to_rows(const d4 (&acc)[2][2], double* __restrict__ S, int wr, int wc, int lane) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) S[acc_row(wr, mi, lane, r) * (NB + 1) + acc_col(wc, ni, lane)] = acc[mi][ni][r];
}

__device__ __forceinline__ bool spin_ge(const int* f, int target, int* info) {
    int it = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if ((++it & 63) == 0) {
            if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
            if (it > kSpin) {
                atomicExch(info, kInfoTimeout);
                return false;
            }
        }
    }
    return true;
}

// ---- the diagonal tile: Cholesky (wave 0) + inverse (wave 1) ------------------------------
// Wave 0, lane t = row t of the tile in registers.  Step J: pivot from lane J, r = 1/sqrt(pivot),
// column J (l_tJ = a_tJ r, diagonal sqrt(pivot), zero above) and r go to LDS, then a rank-1
// update of the rest of the row from broadcast reads of that column.  Every 4 steps a
// workgroup-scope release of `cnt` tells wave 1 that columns < cnt are final.
template <int J>
__device__ __forceinline__ void potrf_step(double (&a)[NB], double* __restrict__ Lc, double* __restrict__ rinv,
                                           int* cnt, int t, bool& bad) {
    const double piv = readlane_d(a[J], J);
    bad |= !(piv > 0.0);
    const double r = rsqrt_nr(piv);
    const double l = (t == J) ? piv * r : (t > J ? a[J] * r : 0.0);
    a[J] = l;
    Lc[J * NB + t] = l;
    rinv[J] = r;   // every lane stores the same value: no divergent branch in the unrolled chain
    if constexpr ((J & 3) == 3) __hip_atomic_store(cnt, J + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): column J is in LDS for the whole wave
    __builtin_amdgcn_wave_barrier();
    constexpr int K0 = (J + 1) & ~1;
#pragma unroll
    for (int k = K0; k < NB; k += 2) {
        const double2 c = *reinterpret_cast<const double2*>(Lc + J * NB + k);
        if (k >= J + 1) a[k] = fma(-l, c.x, a[k]);
        a[k + 1] = fma(-l, c.y, a[k + 1]);
        if ((k & 15) == 14) __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (J + 1 < NB) potrf_step<J + 1>(a, Lc, rinv, cnt, t, bad);
}

// Spin (all lanes, uniform value) until the LDS word *cnt >= target.  The loop is inline asm so
// that the unrolled register-resident chain around it stays one basic block for the scheduler
// (a C++ loop here splits it and the 64-entry column spills).  LDS operations of one wave are
// processed in order, so reads issued after the exit see every LDS write the signalling wave
// made before its store of *cnt.
__device__ __forceinline__ void wait_lds_ge(const int* cnt, int target) {
    const __attribute__((address_space(3))) int* p = (const __attribute__((address_space(3))) int*)cnt;
    int v;
    asm volatile(
        "1:\n\t"
        "ds_read_b32 %0, %1\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_lt_i32 vcc, %0, %2\n\t"
        "s_cbranch_vccz 2f\n\t"
        "s_sleep 0\n\t"
        "s_branch 1b\n\t"
        "2:"
        : "=&v"(v)
        : "v"(p), "v"(target)
        : "vcc", "memory");
}

// Wave 1, lane c = column c of W = L^{-1}, right-looking forward substitution on e_c:
// w_J = y_J / L_JJ, then y_r -= L_rJ w_J for r > J (L_rJ read as a broadcast of column J).
template <int J>
__device__ __forceinline__ void trinv_step(double (&y)[NB], const double* __restrict__ Lc,
                                           const double* __restrict__ rinv, const int* cnt) {
    if constexpr ((J & 3) == 0) wait_lds_ge(cnt, J + 4);
    const double w = y[J] * rinv[J];
    y[J] = w;
    constexpr int K0 = (J + 1) & ~1;
#pragma unroll
    for (int k = K0; k < NB; k += 2) {
        const double2 c = *reinterpret_cast<const double2*>(Lc + J * NB + k);
        if (k >= J + 1) y[k] = fma(-c.x, w, y[k]);
        y[k + 1] = fma(-c.y, w, y[k + 1]);
        if ((k & 15) == 14) __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (J + 1 < NB) trinv_step<J + 1>(y, Lc, rinv, cnt);
}

// S: the updated tile, row-major 64 x 65 (lower triangle meaningful).  Lc: 64 x 64 scratch.
// Writes W_d (row-major, zero above the diagonal) to Wd; sets *info on a bad pivot.
__device__ __forceinline__ void factor_diag(const double* __restrict__ S, double* __restrict__ Lc,
                                            double* __restrict__ rinv, int* cnt, double* __restrict__ Wd, int d,
                                            int* info) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    if (wave == 0) {
        double a[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) a[k] = S[lane * (NB + 1) + k];
        bool bad = false;
        potrf_step<0>(a, Lc, rinv, cnt, lane, bad);
        if (bad && lane == 0) atomicCAS(info, 0, d * NB + 1);
    } else if (wave == 1) {
        double y[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) y[k] = (k == lane) ? 1.0 : 0.0;
        trinv_step<0>(y, Lc, rinv, cnt);
#pragma unroll
        for (int r = 0; r < NB; ++r) Wd[r * NB + lane] = y[r];
    }
}

// ---- one panel step ---------------------------------------------------------------------
// Launch k (-1 <= k <= T-2), R = T-1-k.  blockIdx 0: the diagonal tile k+1; 1..R: panel rows
// i = k+1 .. T-1; then the update tiles (i, j), k+1 <= j <= i, (i, j) != (k+1, k+1), by columns.
// Waits only ever target lower blockIdx (the panel workgroups), and every wait is capped.
__global__ __launch_bounds__(256, 2) void k_chol_step(double* __restrict__ P, long ldp, int T, int k,
                                                   double* __restrict__ W, double* __restrict__ bv,
                                                   double* __restrict__ zv, int* __restrict__ rowflag, int epoch,
                                                   int* __restrict__ info) {
    __shared__ __attribute__((aligned(16))) double smem[2 * kStage];   // 73.7 KB
    __shared__ double rinv[NB];
    __shared__ double zsh[NB];
    __shared__ int cnt;
    __shared__ int ok_sh;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wr = wave >> 1, wc = wave & 1;
    if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    double* X = smem;
    double* Y = smem + kStage;
    const int R = T - 1 - k;
    const int b = blockIdx.x;

    if (b == 0) {   // ---------------- diagonal tile d = k + 1
        const int d = k + 1, d0 = d * NB;
        double* S = Y;   // 64 x 65 rows, overlays the W_k stage once that is consumed
        if (t == 0) cnt = 0;
        if (k >= 0) {
            const int k0 = k * NB;
            stage_tile(X, P, ldp, d0, k0);
            stage_tile(Y, W + (long)k * NB * NB, NB, 0, 0);
            __syncthreads();
            d4 acc[2][2];
            acc_zero(acc);
            mfma_xyt<false>(acc, X, Y, wr, wc, lane);   // L_{d,k} = A_{d,k} W_k^T
            __syncthreads();
            acc_to_stage(acc, X, wr, wc, lane);
            acc_load(acc, P, ldp, d0, d0, wr, wc, lane);
            __syncthreads();
            mfma_xyt<true>(acc, X, X, wr, wc, lane);    // A_dd - L L^T
            acc_to_rows(acc, S, wr, wc, lane);
        } else {
            const int row = t >> 2, c0 = (t & 3) * 16;
#pragma unroll
            for (int q = 0; q < 16; ++q) S[row * (NB + 1) + c0 + q] = P[(long)row * ldp + c0 + q];
        }
        __syncthreads();
        factor_diag(S, X, rinv, &cnt, W + (long)d * NB * NB, d, info);
        return;
    }

    if (b <= R) {   // ---------------- panel row i: L_ik = A_ik W_k^T, forward-solve update
        const int i = k + b, k0 = k * NB, i0 = i * NB;
        stage_tile(X, P, ldp, i0, k0);
        stage_tile(Y, W + (long)k * NB * NB, NB, 0, 0);
        __syncthreads();
        d4 acc[2][2];
        acc_zero(acc);
        mfma_xyt<false>(acc, X, Y, wr, wc, lane);
        acc_store(acc, P, ldp, i0, k0, wr, wc, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                                 // every wave's stores have drained
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(rowflag + i, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // forward substitution carried by the panel: z_k = W_k b_k, b_i -= L_ik z_k
        acc_to_rows(acc, X, wr, wc, lane);   // X is free (the MFMA finished before the barrier)
        if (t < NB) {
            double s = 0.0;
#pragma unroll 16
            for (int j = 0; j < NB; ++j) s = fma(Y[(j >> 4) * kSub + t * kPad + (j & 15)], bv[k0 + j], s);
            zsh[t] = s;
        }
        __syncthreads();
        if (t < NB) {
            double s = 0.0;
#pragma unroll 16
            for (int j = 0; j < NB; ++j) s = fma(X[t * (NB + 1) + j], zsh[j], s);
            bv[i0 + t] -= s;
            if (b == 1) zv[k0 + t] = zsh[t];
        }
        return;
    }

    // ---------------- update tile (i, j)
    int u = b - R - 1 + 1;   // index among the update tiles including (k+1, k+1), which is skipped
    int j = k + 1;
    while (u >= T - j) {
        u -= T - j;
        ++j;
    }
    const int i = j + u;
    if (t == 0) {
        const bool ok = spin_ge(rowflag + i, epoch, info) && spin_ge(rowflag + j, epoch, info);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the L1 invalidate has completed
        ok_sh = ok;
    }
    __syncthreads();
    if (!ok_sh) return;
    const int k0 = k * NB;
    stage_tile(X, P, ldp, i * NB, k0);
    if (i != j) stage_tile(Y, P, ldp, j * NB, k0);
    d4 acc[2][2];
    acc_load(acc, P, ldp, i * NB, j * NB, wr, wc, lane);
    __syncthreads();
    mfma_xyt<true>(acc, X, i != j ? Y : X, wr, wc, lane);
    acc_store(acc, P, ldp, i * NB, j * NB, wr, wc, lane);
}

// ---- backward substitution L^T x = z ------------------------------------------------------
// Workgroup b owns block w = T-1-b.  For c = T-1 .. w+1 it waits for x_c (flag), accumulating
// s_w += L_cw^T x_c with the next L_cw tile prefetched; then x_w = W_w^T (z_w - s_w).
// z_{T-1} = W_{T-1} b_{T-1} is formed here (the factor launches form z_0 .. z_{T-2}).
__global__ __launch_bounds__(256) void k_chol_bwd(const double* __restrict__ P, long ldp, int T, int n,
                                                  const double* __restrict__ W, const double* __restrict__ bv,
                                                  const double* __restrict__ zv, double* xw, double* __restrict__ x,
                                                  int* flags, int epoch, int* info) {
    __shared__ double part[4][NB];
    __shared__ double vsh[NB];
    __shared__ int ok_sh;
    if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    const int t = threadIdx.x, j = t & 63, q = t >> 6;
    const int w = T - 1 - blockIdx.x, w0 = w * NB;
    const double* Ww = W + (long)w * NB * NB;
    double zj = 0.0;
    if (t < NB) {
        if (w == T - 1) {
            double s = 0.0;
#pragma unroll 16
            for (int c = 0; c < NB; ++c) s = fma(Ww[t * NB + c], bv[w0 + c], s);
            zj = s;
        } else {
            zj = zv[w0 + t];
        }
    }
    double acc = 0.0;
    double Lv[16], Ln[16];
    auto load_blk = [&](double (&dst)[16], int c) {
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[r] = P[(long)(c * NB + q * 16 + r) * ldp + w0 + j];
    };
    if (w + 1 < T) load_blk(Lv, T - 1);
    for (int c = T - 1; c > w; --c) {
        if (c - 1 > w) load_blk(Ln, c - 1);
        if (t == 0) {
            const bool ok = spin_ge(flags + c, epoch, info);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ok_sh = ok;
        }
        __syncthreads();
        if (!ok_sh) return;
        const double* xc = xw + c * NB + q * 16;
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) s = fma(Lv[r], xc[r], s);
        acc += s;
#pragma unroll
        for (int r = 0; r < 16; ++r) Lv[r] = Ln[r];
    }
    part[q][j] = acc;
    __syncthreads();
    if (t < NB) vsh[t] = zj - ((part[0][t] + part[1][t]) + (part[2][t] + part[3][t]));
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < 16; ++r) s = fma(Ww[(q * 16 + r) * NB + j], vsh[q * 16 + r], s);
    part[q][j] = s;
    __syncthreads();
    if (t < NB) {
        const double xv = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
        xw[w0 + t] = xv;
        if (w0 + t < n) x[w0 + t] = xv;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(flags + w, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// P = A zero-padded to N x N (identity on the padded diagonal), bv = rhs zero-padded, info = 0
__global__ void k_chol_prep(const double* __restrict__ A, long lda, int n, double* __restrict__ P, long ldp, int N,
                            const double* __restrict__ rhs, double* __restrict__ bv, int* __restrict__ info) {
    const long total = (long)N * N;
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int r = (int)(e / N), c = (int)(e % N);
        P[(long)r * ldp + c] = (r < n && c < n) ? A[(long)r * lda + c] : (r == c ? 1.0 : 0.0);
    }
    if (blockIdx.x == 0) {
        for (int r = threadIdx.x; r < N; r += blockDim.x) bv[r] = r < n ? rhs[r] : 0.0;
        if (threadIdx.x == 0) *info = 0;
    }
}

}  // namespace

// Solve A sigma = rhs (A SPD, untouched) by the lookahead tile Cholesky; *dinfo (device) != 0
// afterwards when a pivot failed or a chain timed out.
int launch_chol_solve(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo) {
    const int T = (n + NB - 1) / NB, N = T * NB;
    const long ldp = N;
    void *P = nullptr, *W = nullptr, *bv = nullptr, *zv = nullptr, *xw = nullptr;
    PNOL_CHECK(ws_get(ctx, "chol4_P", sizeof(double) * (size_t)N * ldp, &P));
    PNOL_CHECK(ws_get(ctx, "chol4_W", sizeof(double) * (size_t)T * NB * NB, &W));
    PNOL_CHECK(ws_get(ctx, "chol4_b", sizeof(double) * (size_t)N, &bv));
    PNOL_CHECK(ws_get(ctx, "chol4_z", sizeof(double) * (size_t)N, &zv));
    PNOL_CHECK(ws_get(ctx, "chol4_x", sizeof(double) * (size_t)N, &xw));
    if (T > ctx->chol4_cap || ctx->chol4_epoch > (1 << 29)) {
        void* f = nullptr;
        const int cap = std::max(T, ctx->chol4_cap);
        PNOL_CHECK(ws_get(ctx, "chol4_flags", sizeof(int) * (size_t)2 * cap, &f));
        PNOL_HIP(hipMemsetAsync(f, 0, sizeof(int) * (size_t)2 * cap, ctx->stream));
        ctx->chol4_flags = (int*)f;
        ctx->chol4_cap = cap;
        ctx->chol4_epoch = 0;
    }
    int* rowflag = ctx->chol4_flags;
    int* bwdflag = ctx->chol4_flags + ctx->chol4_cap;
    const long total = (long)N * N;
    hipLaunchKernelGGL(k_chol_prep, dim3((int)std::min<long>((total + 255) / 256, 4096)), dim3(256), 0, ctx->stream,
                       A, (long)lda, n, (double*)P, ldp, N, rhs, (double*)bv, dinfo);
    for (int k = -1; k <= T - 2; ++k) {
        const int R = T - 1 - k;
        const int grid = k < 0 ? 1 : R + R * (R + 1) / 2;
        const int epoch = ++ctx->chol4_epoch;
        hipLaunchKernelGGL(k_chol_step, dim3(grid), dim3(256), 0, ctx->stream, (double*)P, ldp, T, k, (double*)W,
                           (double*)bv, (double*)zv, rowflag, epoch, dinfo);
    }
    const int epoch = ++ctx->chol4_epoch;
    hipLaunchKernelGGL(k_chol_bwd, dim3(T), dim3(256), 0, ctx->stream, (const double*)P, ldp, T, n, (const double*)W,
                       (const double*)bv, (const double*)zv, (double*)xw, sigma, bwdflag, epoch, dinfo);
    return launch_check();
}

}  // namespace pnol
