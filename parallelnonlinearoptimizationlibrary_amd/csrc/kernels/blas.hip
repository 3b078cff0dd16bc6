// blas.hip -- HBM-streaming fp64 kernels of the BFGS inverse-Hessian path (gfx950).
//
//   k_gemv_neg        p = -D g  (BFGS_with_linesearch.cpp:78-79) and rhs = -J^T F
//                     (LevenbergMarquardt.cpp:78-80): row-major streaming GEMV, 16-B loads,
//                     R rows per wave, one wave reduction per row.  8 bytes/element.
//   k_gemv_neg_seq    the same in the reference's summation order (one thread per row,
//                     sequential from 0.0, no contraction) for n <= PNOL_SEQ_MAX.
//   k_bfgs_exact_*    updateHessianInv (BFGS_with_linesearch.cpp:389-432) in its O(n^3)
//                     operation order, bitwise equal to the CPU path, small n only.
//   k_bfgs_pass       one read(+write) sweep of D: applies a pending rank-2 correction,
//                     optionally writes D back, and accumulates D y, D^T y, D g with
//                     deterministic partial sums.  16 bytes/element with write-back.
//
// All device code is compiled with -ffp-contract=off: every fma here is explicit.
#include "../pnol_internal.hpp"
#include "../pnol_comm.hpp"

#include <cstdlib>

namespace pnol {
namespace {

constexpr int kWave = 64;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
    return v;
}

// ------------------------------------------------------------------------------------
// streaming GEMV: y = -A x, A rows x cols, row-major.
// VEC (lda even, A and x 16-byte aligned): each wave owns R rows and streams them in
// super-chunks of U x 1 KiB per row with 16-byte loads, register double-buffered (the next
// super-chunk is in flight while the current one is reduced).  Each wave starts at a
// different super-chunk (rotation by its global wave index) so the concurrently running
// waves spread over the HBM channels instead of all hitting the same column offset of rows
// that are 2^k bytes apart.  One wave reduction per row at the end.
// ------------------------------------------------------------------------------------
constexpr int kU = 4;

template <int R>
__device__ __forceinline__ void gemv_load(double2 (&a)[R][kU], double2 (&xr)[kU], const double2* const (&arow)[R],
                                          const double2* __restrict__ xv, int base, int lane) {
#pragma unroll
    for (int u = 0; u < kU; ++u) xr[u] = xv[base + u * kWave + lane];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < kU; ++u) a[r][u] = arow[r][base + u * kWave + lane];
}

template <int R>
__device__ __forceinline__ void gemv_fma(const double2 (&a)[R][kU], const double2 (&xr)[kU], double (&acc0)[R],
                                         double (&acc1)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            acc0[r] = fma(a[r][u].x, xr[u].x, acc0[r]);
            acc1[r] = fma(a[r][u].y, xr[u].y, acc1[r]);
        }
}

template <int R>
__global__ __launch_bounds__(256) void k_gemv_neg(const double* __restrict__ A, long lda, int rows, int cols,
                                                  const double* __restrict__ x, double* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int gwave = blockIdx.x * 4 + wave;
    const long row0 = (long)gwave * R;
    if (row0 >= rows) return;

    const double2* __restrict__ xv = reinterpret_cast<const double2*>(x);
    const double2* arow[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        long rr = row0 + r < rows ? row0 + r : rows - 1;   // clamp: loads stay in bounds
        arow[r] = reinterpret_cast<const double2*>(A + rr * lda);
    }
    double acc0[R], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) { acc0[r] = 0.0; acc1[r] = 0.0; }

    const int pairs = cols >> 1;
    constexpr int SC = kU * kWave;                 // pairs per super-chunk
    const int nfull = pairs / SC;
    if (nfull > 0) {
        int sc = gwave % nfull;                    // rotated start
        double2 cur[R][kU], curx[kU];
        gemv_load<R>(cur, curx, arow, xv, sc * SC, lane);
        for (int t = 1; t < nfull; ++t) {
            sc = (sc + 1 == nfull) ? 0 : sc + 1;
            double2 nxt[R][kU], nxtx[kU];
            gemv_load<R>(nxt, nxtx, arow, xv, sc * SC, lane);
            gemv_fma<R>(cur, curx, acc0, acc1);
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int u = 0; u < kU; ++u) cur[r][u] = nxt[r][u];
#pragma unroll
            for (int u = 0; u < kU; ++u) curx[u] = nxtx[u];
        }
        gemv_fma<R>(cur, curx, acc0, acc1);
    }
    for (int c = nfull * SC + lane; c < pairs; c += kWave) {
        double2 xr = xv[c];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            double2 a = arow[r][c];
            acc0[r] = fma(a.x, xr.x, acc0[r]);
            acc1[r] = fma(a.y, xr.y, acc1[r]);
        }
    }
    if ((cols & 1) && lane == 0) {             // odd trailing column
        const double xl = x[cols - 1];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            long rr = row0 + r < rows ? row0 + r : rows - 1;
            acc0[r] = fma(A[rr * lda + cols - 1], xl, acc0[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        double s = wave_sum(acc0[r] + acc1[r]);
        if (lane == 0 && row0 + r < rows) y[row0 + r] = -s;
    }
}

// Workgroup-cooperative variant: a 256-thread workgroup owns R rows and its 4 waves take
// interleaved 4 KiB super-chunks of each row (wave w: chunks w, w+4, ...), so the waves of a
// workgroup stream one contiguous 16 KiB window of a row at a time and the chip keeps ~4x
// fewer concurrent DRAM streams open than with a wave per row.  NT: non-temporal loads
// (D is streamed once; keep it out of L2 / MALL).  Partial sums are combined in a fixed
// order through LDS.
// VEC = false: the same arithmetic with 8-byte loads (rows not 16-byte aligned)
template <int R, bool NT, bool VEC = true>
__device__ __forceinline__ void gemv_neg_wg_body(const double* __restrict__ A, long lda, int rows, int cols,
                                                 const double* __restrict__ x, double* __restrict__ y) {
    __shared__ double part[4][R];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long row0 = (long)blockIdx.x * R;
    const double2* __restrict__ xv = reinterpret_cast<const double2*>(x);
    const double* arow[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        long rr = row0 + r < rows ? row0 + r : rows - 1;
        arow[r] = A + rr * lda;
    }
    double acc0[R], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) { acc0[r] = 0.0; acc1[r] = 0.0; }
    const int pairs = cols >> 1;
    constexpr int SC = kU * kWave;
    const int nfull = pairs / SC;
    auto ld = [&](const double* q) -> double2 {
        if (!VEC) return make_double2(q[0], q[1]);
        const double2* p = reinterpret_cast<const double2*>(q);
        if (NT) {
            double2 v;
            v.x = __builtin_nontemporal_load(&p->x);
            v.y = __builtin_nontemporal_load(&p->y);
            return v;
        }
        return *p;
    };
    int sc = wave;
    if (sc < nfull) {
        double2 cur[R][kU], curx[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) curx[u] = xv[sc * SC + u * kWave + lane];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < kU; ++u) cur[r][u] = ld(arow[r] + 2 * (sc * SC + u * kWave + lane));
        for (sc += 4; sc < nfull; sc += 4) {
            double2 nxt[R][kU], nxtx[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) nxtx[u] = xv[sc * SC + u * kWave + lane];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int u = 0; u < kU; ++u) nxt[r][u] = ld(arow[r] + 2 * (sc * SC + u * kWave + lane));
            gemv_fma<R>(cur, curx, acc0, acc1);
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int u = 0; u < kU; ++u) cur[r][u] = nxt[r][u];
#pragma unroll
            for (int u = 0; u < kU; ++u) curx[u] = nxtx[u];
        }
        gemv_fma<R>(cur, curx, acc0, acc1);
    }
    if (wave == 0) {
        for (int c = nfull * SC + lane; c < pairs; c += kWave) {
            double2 xr = xv[c];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                double2 a = VEC ? reinterpret_cast<const double2*>(arow[r])[c]
                                : make_double2(arow[r][2 * c], arow[r][2 * c + 1]);
                acc0[r] = fma(a.x, xr.x, acc0[r]);
                acc1[r] = fma(a.y, xr.y, acc1[r]);
            }
        }
        if ((cols & 1) && lane == 0) {
            const double xl = x[cols - 1];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                long rr = row0 + r < rows ? row0 + r : rows - 1;
                acc0[r] = fma(A[rr * lda + cols - 1], xl, acc0[r]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const double s = wave_sum(acc0[r] + acc1[r]);
        if (lane == 0) part[wave][r] = s;
    }
    __syncthreads();
    if (threadIdx.x < R && row0 + threadIdx.x < rows) {
        const int r = threadIdx.x;
        y[row0 + r] = -((part[0][r] + part[1][r]) + (part[2][r] + part[3][r]));
    }
}

template <int R, bool NT>
__global__ __launch_bounds__(256) void k_gemv_neg_wg(const double* __restrict__ A, long lda, int rows, int cols,
                                                     const double* __restrict__ x, double* __restrict__ y) {
    gemv_neg_wg_body<R, NT>(A, lda, rows, cols, x, y);
}

// -J^T F per m-slice (LevMarq / LevMarqMPI, syrk.hip): blockIdx.y = slice s0 + y of J^T (at
// A + s * sstride, row stride lda) against F[s mS, (s + 1) mS) -> y[blockIdx.y * rows + j].
template <int R, bool VEC>
__global__ __launch_bounds__(256) void k_gemv_neg_slices(const double* __restrict__ A, long lda, long sstride, int rows,
                                                         int m, int mS, int s0, const double* __restrict__ x,
                                                         double* __restrict__ y) {
    const int s = s0 + blockIdx.y;
    const int cols = max(0, min(mS, m - s * mS));
    gemv_neg_wg_body<R, true, VEC>(A + (long)s * sstride, lda, rows, cols, x + (long)s * mS,
                                   y + (long)blockIdx.y * rows);
}

// any lda / alignment: one wave per row, 8-byte loads, 4 in flight per lane
__global__ __launch_bounds__(256) void k_gemv_neg_scalar(const double* __restrict__ A, long lda, int rows, int cols,
                                                         const double* __restrict__ x, double* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const double* a = A + row * lda;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    int c = lane;
    for (; c + 3 * kWave < cols; c += 4 * kWave)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = fma(a[c + u * kWave], x[c + u * kWave], acc[u]);
    for (; c < cols; c += kWave) acc[0] = fma(a[c], x[c], acc[0]);
    const double s = wave_sum((acc[0] + acc[1]) + (acc[2] + acc[3]));
    if (lane == 0) y[row] = -s;
}

// reference order: s = 0; s = s + A_ij x_j, j ascending; y = -s  (matrixVectorMultiply + negate)
__global__ void k_gemv_neg_seq(const double* __restrict__ A, long lda, int rows, int cols,
                               const double* __restrict__ x, double* __restrict__ y) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows) return;
    const double* a = A + (long)i * lda;
    double s = 0.0;
    for (int j = 0; j < cols; ++j) s = s + a[j] * x[j];
    y[i] = -s;
}

// ------------------------------------------------------------------------------------
// updateHessianInv in the reference's order (M1 D, then (M1 D) M2 + M3)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ double seq_dot(const double* a, const double* b, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s = s + a[i] * b[i];
    return s;
}

// T = M1 D with M1_il = [i==l] - rho s_i y_l
__global__ void k_bfgs_exact_1(const double* __restrict__ D, long ldd, const double* __restrict__ y,
                               const double* __restrict__ s, int n, double* __restrict__ T) {
    __shared__ double rho_sh;
    if (threadIdx.x == 0 && threadIdx.y == 0) rho_sh = 1 / seq_dot(y, s, n);
    __syncthreads();
    const double rho = rho_sh;
    int i = blockIdx.y * blockDim.y + threadIdx.y;
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || j >= n) return;
    double acc = 0.0;
    for (int l = 0; l < n; ++l) {
        double m1 = (i == l ? 1.0 : 0.0) - rho * s[i] * y[l];
        acc = acc + m1 * D[(long)l * ldd + j];
    }
    T[(long)i * n + j] = acc;
}

// D = T M2 + M3 with M2_lj = [l==j] - rho y_l s_j, M3_ij = rho s_i s_j
__global__ void k_bfgs_exact_2(const double* __restrict__ T, double* __restrict__ D, long ldd,
                               const double* __restrict__ y, const double* __restrict__ s, int n) {
    __shared__ double rho_sh;
    if (threadIdx.x == 0 && threadIdx.y == 0) rho_sh = 1 / seq_dot(y, s, n);
    __syncthreads();
    const double rho = rho_sh;
    int i = blockIdx.y * blockDim.y + threadIdx.y;
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || j >= n) return;
    double acc = 0.0;
    for (int l = 0; l < n; ++l) {
        double m2 = (l == j ? 1.0 : 0.0) - rho * y[l] * s[j];
        acc = acc + T[(long)i * n + l] * m2;
    }
    D[(long)i * ldd + j] = acc + rho * s[i] * s[j];
}

// ------------------------------------------------------------------------------------
// fused BFGS pass
// Tile: 256 rows x 512 columns per 256-thread workgroup; wave w owns 128 columns (2 per
// lane) and walks the 256 rows in groups of 8.  Row partial sums (u = Dc y, v = Dc g) are
// reduced across the wave with a 16-value butterfly (reduce-scatter) and written per
// 128-column strip; column partials (w = Dc^T y) stay in registers and are written per
// 256-row tile.  k_bfgs_pass_finish sums the partials in a fixed order: deterministic.
// ------------------------------------------------------------------------------------
constexpr int kPassCols = 512;
constexpr int kGroup = 8;

// reduce-scatter 16 values across the wave; the lanes with (lane & 3) == 0 end up with the
// full 64-lane sum of value index ((lane>>5)&1)*8 + ((lane>>4)&1)*4 + ((lane>>3)&1)*2 + ((lane>>2)&1)
__device__ __forceinline__ double butterfly16(double (&v)[16], int lane) {
    {
        const bool hi = (lane >> 5) & 1;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            double send = hi ? v[k] : v[k + 8];
            double keep = hi ? v[k + 8] : v[k];
            v[k] = keep + __shfl_xor(send, 32, kWave);
        }
    }
    {
        const bool hi = (lane >> 4) & 1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double send = hi ? v[k] : v[k + 4];
            double keep = hi ? v[k + 4] : v[k];
            v[k] = keep + __shfl_xor(send, 16, kWave);
        }
    }
    {
        const bool hi = (lane >> 3) & 1;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            double send = hi ? v[k] : v[k + 2];
            double keep = hi ? v[k + 2] : v[k];
            v[k] = keep + __shfl_xor(send, 8, kWave);
        }
    }
    {
        const bool hi = (lane >> 2) & 1;
        double send = hi ? v[0] : v[1];
        double keep = hi ? v[1] : v[0];
        v[0] = keep + __shfl_xor(send, 4, kWave);
    }
    double r = v[0];
    r += __shfl_xor(r, 2, kWave);
    r += __shfl_xor(r, 1, kWave);
    return r;
}

template <bool VEC>
__device__ __forceinline__ void pass_load(double2 (&d)[kGroup], const double* __restrict__ D, long ldd, int n, int r0,
                                          int colc, int rlast) {
#pragma unroll
    for (int q = 0; q < kGroup; ++q) {
        const long row = min(r0 + q, rlast);
        if (VEC) {
            // non-temporal: D is streamed once per pass (MI355X: ~1.6x the HBM rate of
            // cached loads for this access pattern, tools/sweep_hg.py)
            const double* p = D + row * ldd + colc;
            d[q].x = __builtin_nontemporal_load(p);
            d[q].y = __builtin_nontemporal_load(p + 1);
        } else {
            d[q].x = colc < n ? D[row * ldd + colc] : 0.0;
            d[q].y = colc + 1 < n ? D[row * ldd + colc + 1] : 0.0;
        }
    }
}

// IDS: the stored D is diag(scale) (I when scale is null) and is synthesised, not read (the
// first fold of a pending correction after a reset writes D without reading it: 8 n^2 bytes)
__device__ __forceinline__ void pass_ident(double2 (&d)[kGroup], const double* __restrict__ scale, int r0, int colc,
                                           int rlast) {
#pragma unroll
    for (int q = 0; q < kGroup; ++q) {
        const int row = min(r0 + q, rlast);
        const double dv = scale ? scale[row] : 1.0;
        d[q].x = row == colc ? dv : 0.0;
        d[q].y = row == colc + 1 ? dv : 0.0;
    }
}

// Rows of a 256-row tile are visited in groups of 8 starting at a tile-dependent group
// (rotation: concurrently running tiles read different HBM channels); the next group's
// 16-byte loads are issued before the current group is reduced (register double buffer).
// Row shard form (BFGS D row-sharded over the ranks): D holds rows [rb, re) of the n x n
// matrix (rb a multiple of the row-tile height); row tiles, partial indices and outputs use global rows,
// so every partial is the one the whole-matrix pass (rb = 0, re = n) would produce.
template <bool PEND, bool WB, bool VEC, bool IDS = false>
__global__ __launch_bounds__(256) void k_bfgs_pass(double* __restrict__ Dsh, long ldd, int n, int rb, int re, int prows,
                                                   const double* __restrict__ sp, const double* __restrict__ ap,
                                                   const double* __restrict__ bp, const double* __restrict__ y,
                                                   const double* __restrict__ g, double* __restrict__ part_u,
                                                   double* __restrict__ part_v, double* __restrict__ part_w,
                                                   const double* __restrict__ id_scale = nullptr) {
    double* __restrict__ D = Dsh - (long)rb * ldd;   // global-row view (only rows [rb, re) touched)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int ncolt = (n + kPassCols - 1) / kPassCols;
    const int rt = rb / prows + blockIdx.x / ncolt;   // global row tile (prows = bfgs_pass_rows(n))
    const int ct = blockIdx.x % ncolt;            // column tile
    const int strip = ct * 4 + wave;              // 128-column strip index
    const int col = strip * 128 + 2 * lane;       // this lane's first column
    const bool c0ok = col < n, c1ok = col + 1 < n;
    // load column: lanes past the last column read column 0 (VEC: the pair (col, col+1) is
    // inside the row because an even ld >= n+1 when n is odd; scalar loads are guarded)
    const int colc = c0ok ? col : 0;

    double yc0 = c0ok ? y[col] : 0.0, yc1 = c1ok ? y[col + 1] : 0.0;
    double gc0 = c0ok ? g[col] : 0.0, gc1 = c1ok ? g[col + 1] : 0.0;
    double ac0 = 0, ac1 = 0, sc0 = 0, sc1 = 0;
    if (PEND) {
        ac0 = c0ok ? ap[col] : 0.0; ac1 = c1ok ? ap[col + 1] : 0.0;
        sc0 = c0ok ? sp[col] : 0.0; sc1 = c1ok ? sp[col + 1] : 0.0;
    }
    double w0 = 0.0, w1 = 0.0;

    const int r_begin = rt * prows;
    const int r_end = min(re, r_begin + prows);
    const int ngroups = (r_end - r_begin + kGroup - 1) / kGroup;
    int grp = rt % ngroups;
    double2 cur[kGroup];
    if (IDS) pass_ident(cur, id_scale, r_begin + grp * kGroup, col, r_end - 1);
    else pass_load<VEC>(cur, D, ldd, n, r_begin + grp * kGroup, colc, r_end - 1);
    for (int t = 0; t < ngroups; ++t) {
        const int r0 = r_begin + grp * kGroup;
        const int gnext = (grp + 1 == ngroups) ? 0 : grp + 1;
        double2 nxt[kGroup];
        if (t + 1 < ngroups) {
            if (IDS) pass_ident(nxt, id_scale, r_begin + gnext * kGroup, col, r_end - 1);
            else pass_load<VEC>(nxt, D, ldd, n, r_begin + gnext * kGroup, colc, r_end - 1);
        }
        double yr[kGroup], sr[kGroup], br[kGroup];
#pragma unroll
        for (int q = 0; q < kGroup; ++q) {
            const int row = min(r0 + q, r_end - 1);
            yr[q] = (r0 + q < r_end) ? y[row] : 0.0;
            if (PEND) { sr[q] = sp[row]; br[q] = bp[row]; }
        }
        double vals[16];
#pragma unroll
        for (int q = 0; q < kGroup; ++q) {
            double e0 = cur[q].x, e1 = cur[q].y;
            const double o0 = e0, o1 = e1;
            if (PEND) {
                e0 = fma(br[q], sc0, fma(sr[q], ac0, e0));
                e1 = fma(br[q], sc1, fma(sr[q], ac1, e1));
            }
            if (!c0ok) { e0 = o0; }
            if (!c1ok) { e1 = o1; }
            if (WB && r0 + q < r_end && c0ok) {
                double* dst = D + (long)(r0 + q) * ldd + col;
                if (VEC) {
                    __builtin_nontemporal_store(e0, dst);
                    __builtin_nontemporal_store(c1ok ? e1 : cur[q].y, dst + 1);
                } else {
                    dst[0] = e0;
                    if (c1ok) dst[1] = e1;
                }
            }
            const double m0 = c0ok ? e0 : 0.0, m1 = c1ok ? e1 : 0.0;
            vals[q] = fma(m1, yc1, m0 * yc0);
            vals[8 + q] = fma(m1, gc1, m0 * gc0);
            w0 = fma(m0, yr[q], w0);
            w1 = fma(m1, yr[q], w1);
        }
        const double red = butterfly16(vals, lane);
        if ((lane & 3) == 0) {
            const int idx = ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
            const int row = r0 + (idx & 7);
            if (row < r_end) {
                if (idx < 8) part_u[(long)strip * n + row] = red;
                else part_v[(long)strip * n + row] = red;
            }
        }
#pragma unroll
        for (int q = 0; q < kGroup; ++q) cur[q] = nxt[q];
        grp = gnext;
    }
    if (c0ok) part_w[(long)rt * n + col] = w0;
    if (c1ok) part_w[(long)rt * n + col + 1] = w1;
}

// Sum the pass partials in a fixed order.  Workgroup = 64 outputs x 4 quarters: quarter q sums
// strips s == q (mod 4) (and row tiles t == q (mod 4)) ascending, then the four quarter sums
// are added (0+1)+(2+3) -- 4x the loads in flight of a thread per output.
__global__ __launch_bounds__(256) void k_bfgs_pass_finish(int n, int nstrips, int nrowt, const double* __restrict__ part_u,
                                                          const double* __restrict__ part_v,
                                                          const double* __restrict__ part_w, double* __restrict__ u,
                                                          double* __restrict__ v, double* __restrict__ w, int ub,
                                                          int ue) {
    __shared__ double red[3][4][64];
    const int il = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + il;
    const int ic = min(i, n - 1);
    double su = 0.0, sv = 0.0, sw = 0.0;
#pragma unroll 4
    for (int s = q; s < nstrips; s += 4) {
        su += part_u[(long)s * n + ic];
        sv += part_v[(long)s * n + ic];
    }
#pragma unroll 4
    for (int t = q; t < nrowt; t += 4) sw += part_w[(long)t * n + ic];
    red[0][q][il] = su;
    red[1][q][il] = sv;
    red[2][q][il] = sw;
    __syncthreads();
    if (q == 0 && i < n) {
        const bool mine = i >= ub && i < ue;   // u, v: this shard's rows only
        if (u && mine) u[i] = (red[0][0][il] + red[0][1][il]) + (red[0][2][il] + red[0][3][il]);
        if (v && mine) v[i] = (red[1][0][il] + red[1][1][il]) + (red[1][2][il] + red[1][3][il]);
        if (w) w[i] = (red[2][0][il] + red[2][1][il]) + (red[2][2][il] + red[2][3][il]);
    }
}

// rows [rb, rb + nrows) of the identity (or diag(scale)), stored from D
__global__ void k_set_identity(double* __restrict__ D, long ldd, int nrows, int rb, const double* __restrict__ scale) {
    long total = (long)nrows * ldd;
    for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += (long)gridDim.x * blockDim.x) {
        long i = rb + k / ldd, j = k % ldd;
        double v = 0.0;
        if (i == j) v = scale ? scale[i] : 1.0;
        D[k] = v;
    }
}

// Dsub[a][b] = D[idx[a]][idx[b]]: one workgroup per destination row (idx ascending, so the
// source reads of a row stay within one row of D and mostly coalesce)
// Dsub[a][b] = D[ridx[a] - rbase][cidx[b]], a < nrows, b < ncols
__global__ void k_gather_sub(const double* __restrict__ D, long ldd, const int* __restrict__ ridx, int nrows,
                             int rbase, const int* __restrict__ cidx, int ncols, double* __restrict__ Dsub, long lds) {
    for (int a = blockIdx.x; a < nrows; a += gridDim.x) {
        const double* row = D + (long)(ridx[a] - rbase) * ldd;
        for (int b = threadIdx.x; b < ncols; b += blockDim.x) Dsub[(long)a * lds + b] = row[cidx[b]];
    }
}

// z = x + y (the LM trial point X + sigma, the same IEEE add as the host's)
__global__ void k_add(const double* __restrict__ x, const double* __restrict__ y, double* __restrict__ z, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) z[i] = x[i] + y[i];
}

__global__ void k_fill(double* __restrict__ p, size_t count, double value) {
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += (size_t)gridDim.x * blockDim.x)
        p[k] = value;
}

}  // namespace

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int launch_gemv_neg(pnol_ctx* ctx, const double* A, int lda, int rows, int cols, const double* x, double* y) {
    if (!A || !x || !y || rows <= 0 || cols <= 0 || lda < cols) return PNOL_ERR_ARG;
    if ((lda & 1) || !aligned16(A) || !aligned16(x)) {
        hipLaunchKernelGGL(k_gemv_neg_scalar, dim3((rows + 3) / 4), dim3(256), 0, ctx->stream, A, (long)lda, rows, cols,
                           x, y);
        return launch_check();
    }
    // rows per wave: enough waves to cover the chip (>= ~2 per SIMD) with long streams each;
    // more rows per wave amortise the x reads (every wave streams all of x from L2).
    // PNOL_GEMV_ROWS=1|2|4 overrides the choice (tuning sweeps, tools/sweep_hg.py).
    static const int forced = [] {
        const char* e = std::getenv("PNOL_GEMV_ROWS");
        return e ? std::atoi(e) : 0;
    }();
    // PNOL_GEMV_MODE (tuning): 0 wave per R rows, 1 workgroup-cooperative rows, 2 (default)
    // = 1 with non-temporal loads: 6.66 TB/s at n = 8192 vs 4.0 for the best cached variant
    // (profiles/r01_sweep_hg.log)
    static const int mode = [] {
        const char* e = std::getenv("PNOL_GEMV_MODE");
        return e ? std::atoi(e) : 2;
    }();
    if (mode == 1 || mode == 2) {
        const int Rw = forced == 1 || forced == 2 || forced == 4 ? forced : 2;
        const int blocks = (rows + Rw - 1) / Rw;
#define PNOL_GEMV_WG(RR, NTT) \
    hipLaunchKernelGGL((k_gemv_neg_wg<RR, NTT>), dim3(blocks), dim3(256), 0, ctx->stream, A, (long)lda, rows, cols, x, y)
        if (mode == 1) {
            if (Rw == 4) PNOL_GEMV_WG(4, false); else if (Rw == 2) PNOL_GEMV_WG(2, false); else PNOL_GEMV_WG(1, false);
        } else {
            if (Rw == 4) PNOL_GEMV_WG(4, true); else if (Rw == 2) PNOL_GEMV_WG(2, true); else PNOL_GEMV_WG(1, true);
        }
#undef PNOL_GEMV_WG
        return launch_check();
    }
    int R = forced == 1 || forced == 2 || forced == 4 ? forced : (rows >= 8192 ? 2 : 1);
    const int blocks = (rows + 4 * R - 1) / (4 * R);
    if (R == 4)
        hipLaunchKernelGGL((k_gemv_neg<4>), dim3(blocks), dim3(256), 0, ctx->stream, A, (long)lda, rows, cols, x, y);
    else if (R == 2)
        hipLaunchKernelGGL((k_gemv_neg<2>), dim3(blocks), dim3(256), 0, ctx->stream, A, (long)lda, rows, cols, x, y);
    else
        hipLaunchKernelGGL((k_gemv_neg<1>), dim3(blocks), dim3(256), 0, ctx->stream, A, (long)lda, rows, cols, x, y);
    return launch_check();
}

int launch_gemv_neg_slices(pnol_ctx* ctx, const double* A, int lda, long sstride, int rows, int m, int mS, int s0,
                           int nsl, const double* x, double* y, hipStream_t stream) {
    if (!stream) stream = ctx->stream;
    if (!A || !x || !y || rows <= 0 || nsl <= 0 || (mS & 1) || !aligned16(x)) return PNOL_ERR_ARG;
    // rows per workgroup (PNOL_JTR_ROWS = 1, 2 or 4; tuning -- each row's sum is the same for all)
    static const int R = [] {
        const char* e = std::getenv("PNOL_JTR_ROWS");
        const int v = e ? std::atoi(e) : 2;
        return (v == 1 || v == 4) ? v : 2;
    }();
    // 16-byte row loads when every row start is 16-byte aligned; the same sums otherwise
    const bool vec = !((lda & 1) || (sstride & 1) || !aligned16(A));
    const dim3 grid((rows + R - 1) / R, nsl);
#define PNOL_SLICES(RR, V) \
    hipLaunchKernelGGL((k_gemv_neg_slices<RR, V>), grid, dim3(256), 0, stream, A, (long)lda, sstride, rows, m, mS, s0, x, y)
    if (vec) {
        if (R == 1) PNOL_SLICES(1, true); else if (R == 4) PNOL_SLICES(4, true); else PNOL_SLICES(2, true);
    } else {
        if (R == 1) PNOL_SLICES(1, false); else if (R == 4) PNOL_SLICES(4, false); else PNOL_SLICES(2, false);
    }
#undef PNOL_SLICES
    return launch_check();
}

int launch_gemv_neg_seq(pnol_ctx* ctx, const double* A, int lda, int rows, int cols, const double* x, double* y) {
    if (!A || !x || !y || rows <= 0 || cols <= 0 || lda < cols) return PNOL_ERR_ARG;
    int blocks = (rows + 63) / 64;
    hipLaunchKernelGGL(k_gemv_neg_seq, dim3(blocks), dim3(64), 0, ctx->stream, A, (long)lda, rows, cols, x, y);
    return launch_check();
}

int launch_bfgs_update_exact(pnol_ctx* ctx, double* D, int ldd, const double* y, const double* s, int n) {
    if (!D || !y || !s || n <= 0 || ldd < n) return PNOL_ERR_ARG;
    void* T = nullptr;
    PNOL_CHECK(ws_get(ctx, "bfgs_exact_T", sizeof(double) * (size_t)n * n, &T));
    dim3 blk(16, 16), grd((n + 15) / 16, (n + 15) / 16);
    hipLaunchKernelGGL(k_bfgs_exact_1, grd, blk, 0, ctx->stream, D, (long)ldd, y, s, n, (double*)T);
    PNOL_CHECK(launch_check());
    hipLaunchKernelGGL(k_bfgs_exact_2, grd, blk, 0, ctx->stream, (const double*)T, D, (long)ldd, y, s, n);
    return launch_check();
}

// Whole matrix (rb = 0, re = n) or the row shard [rb, re) (rb a multiple of bfgs_pass_rows(n)).  With a
// shard, pw_gather (non-null) runs between the pass and the finish: it must fill part_w with
// every rank's row tiles (the LevMarq/BFGS communicator's allgather), and u / v come out for
// rows [rb, re) only.
int bfgs_pass_rows(int n) {
    static const int forced = [] {
        const char* e = std::getenv("PNOL_PASS_ROWS");
        const int v = e ? std::atoi(e) : 0;
        return (v == 32 || v == 64 || v == 128 || v == 256) ? v : 0;
    }();
    if (forced) return forced;
    // measured (tools/pass_sweep.py, cold Infinity Cache, two rounds; profiles/r05_pass_rows_sweep.txt):
    // n = 4096: 128 rows 0.605 of HBM (256: 0.43, 32: 0.55); 8192: 256 rows 0.67 (32: 0.66, 64:
    // 0.61); 16384: 32 rows 0.655 (64: 0.63, 256: 0.59) -- the short tiles of the largest D
    // stream at a better rate despite 8x the w = D^T y partials
    return n >= 12288 ? 32 : (n >= 8192 ? 256 : 128);
}

int launch_bfgs_pass(pnol_ctx* ctx, double* D, int ldd, int n, const double* s_p, const double* a_p,
                     const double* b_p, int write_back, const double* y, const double* g, double* u, double* w,
                     double* v, int rb, int re, int (*pw_gather)(pnol_ctx*, double*, int, int), int ident_src,
                     const double* id_scale) {
    if (re < 0) re = n;
    const int prows = bfgs_pass_rows(n);
    if (!D || n <= 0 || ldd < n || rb < 0 || re > n || rb > re || (rb < re && rb % prows)) return PNOL_ERR_ARG;
    const bool pend = s_p != nullptr;
    if (pend && (!a_p || !b_p)) return PNOL_ERR_ARG;
    // the identity source is only meaningful for a fold with write-back (the only caller)
    if (ident_src && (!pend || !write_back)) return PNOL_ERR_ARG;
    const int ncolt = (n + kPassCols - 1) / kPassCols;
    const int nrowt = (n + prows - 1) / prows;
    const int nstrips = ncolt * 4;
    const int myrowt = (re - rb + prows - 1) / prows;
    void *pu = nullptr, *pv = nullptr, *pw = nullptr, *zeros = nullptr;
    PNOL_CHECK(ws_get(ctx, "pass_part_u", sizeof(double) * (size_t)nstrips * n, &pu));
    PNOL_CHECK(ws_get(ctx, "pass_part_v", sizeof(double) * (size_t)nstrips * n, &pv));
    // room for the allgather's padded layout (rank r's tiles at r * tiles per shard): up to
    // nranks * tiles per shard, which exceeds nrowt for short row tiles and many ranks
    const int wtiles = pw_gather ? pnol_bfgs_pass_part_tiles(n, comm_size()) : nrowt;
    if (wtiles < nrowt) return PNOL_ERR_ARG;
    PNOL_CHECK(ws_get(ctx, "pass_part_w", sizeof(double) * (size_t)wtiles * n, &pw));
    if (!y || !g) {
        PNOL_CHECK(ws_get(ctx, "pass_zeros", sizeof(double) * (size_t)n, &zeros));
        PNOL_CHECK(launch_fill(ctx, (double*)zeros, (size_t)n, 0.0));
        if (!y) y = (const double*)zeros;
        if (!g) g = (const double*)zeros;
    }
    auto* P0 = (double*)pu; auto* P1 = (double*)pv; auto* P2 = (double*)pw;
    if (myrowt > 0) {
        dim3 grd(myrowt * ncolt), blk(256);
        const bool vec = (ldd % 2 == 0) && aligned16(D);
#define PNOL_PASS(PE, W, V)                                                                                        \
    hipLaunchKernelGGL((k_bfgs_pass<PE, W, V>), grd, blk, 0, ctx->stream, D, (long)ldd, n, rb, re, prows, s_p, a_p, b_p, y, \
                       g, P0, P1, P2)
        if (ident_src) {
            if (vec)
                hipLaunchKernelGGL((k_bfgs_pass<true, true, true, true>), grd, blk, 0, ctx->stream, D, (long)ldd, n, rb,
                                   re, prows, s_p, a_p, b_p, y, g, P0, P1, P2, id_scale);
            else
                hipLaunchKernelGGL((k_bfgs_pass<true, true, false, true>), grd, blk, 0, ctx->stream, D, (long)ldd, n, rb,
                                   re, prows, s_p, a_p, b_p, y, g, P0, P1, P2, id_scale);
        } else if (vec) {
            if (pend && write_back) PNOL_PASS(true, true, true);
            else if (pend) PNOL_PASS(true, false, true);
            else if (write_back) PNOL_PASS(false, true, true);
            else PNOL_PASS(false, false, true);
        } else {
            if (pend && write_back) PNOL_PASS(true, true, false);
            else if (pend) PNOL_PASS(true, false, false);
            else if (write_back) PNOL_PASS(false, true, false);
            else PNOL_PASS(false, false, false);
        }
#undef PNOL_PASS
        PNOL_CHECK(launch_check());
    }
    if (pw_gather) PNOL_CHECK(pw_gather(ctx, P2, n, nrowt));
    hipLaunchKernelGGL(k_bfgs_pass_finish, dim3((n + 63) / 64), dim3(256), 0, ctx->stream, n, nstrips, nrowt,
                       (const double*)P0, (const double*)P1, (const double*)P2, u, v, w, rb, re);
    return launch_check();
}

int launch_set_identity(pnol_ctx* ctx, double* D, int ldd, int n, const double* scale, int rb, int re) {
    if (re < 0) re = n;
    if (!D || n <= 0 || ldd < n || rb < 0 || re > n || rb > re) return PNOL_ERR_ARG;
    if (re == rb) return PNOL_OK;
    long total = (long)(re - rb) * ldd;
    int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_set_identity, dim3(blocks), dim3(256), 0, ctx->stream, D, (long)ldd, re - rb, rb, scale);
    return launch_check();
}

int launch_gather_sub(pnol_ctx* ctx, const double* D, int ldd, int n, const int* idx, int nsub, double* Dsub,
                      int lds) {
    if (!D || !idx || !Dsub || nsub < 0 || nsub > n || ldd < n || lds < nsub) return PNOL_ERR_ARG;
    if (nsub == 0) return PNOL_OK;
    hipLaunchKernelGGL(k_gather_sub, dim3(std::min(nsub, 8192)), dim3(256), 0, ctx->stream, D, (long)ldd, idx, nsub, 0,
                       idx, nsub, Dsub, (long)lds);
    return launch_check();
}

int launch_gather_rows(pnol_ctx* ctx, const double* D, int ldd, const int* ridx, int nrows, int rbase, const int* cidx,
                       int ncols, double* Dsub, int lds) {
    if (nrows <= 0 || ncols <= 0) return PNOL_OK;
    if (!D || !ridx || !cidx || !Dsub || lds < ncols) return PNOL_ERR_ARG;
    hipLaunchKernelGGL(k_gather_sub, dim3(std::min(nrows, 8192)), dim3(256), 0, ctx->stream, D, (long)ldd, ridx, nrows,
                       rbase, cidx, ncols, Dsub, (long)lds);
    return launch_check();
}

int launch_add(pnol_ctx* ctx, const double* x, const double* y, double* z, int n) {
    if (!x || !y || !z || n < 0) return PNOL_ERR_ARG;
    if (n == 0) return PNOL_OK;
    hipLaunchKernelGGL(k_add, dim3(std::min((n + 255) / 256, 1024)), dim3(256), 0, ctx->stream, x, y, z, n);
    return launch_check();
}

int launch_fill(pnol_ctx* ctx, double* p, size_t count, double value) {
    if (!p) return PNOL_ERR_ARG;
    if (count == 0) return PNOL_OK;
    int blocks = (int)std::min<size_t>((count + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, ctx->stream, p, count, value);
    return launch_check();
}

}  // namespace pnol
