// syrk.hip -- J^T J on fp64 MFMA (v_mfma_f64_16x16x4_f64), gfx950.
//
// Replaces matrixTranspose(J, JT) + matrixMultiply(JT, J, JTJ) + the Marquardt diagonal
// loop, LevenbergMarquardt.cpp:59-73.  J lives on the device as JT (n x m row-major: one
// finite-difference column per row), so J^T J = JT JT^T is a SYRK whose two operands are
// both read along contiguous rows of JT.
//
//   k_syrk_tile     one 128 x 128 (or 64 x 64) lower-triangle output tile (ti >= tj) per
//                   256-thread workgroup, K split over `split_k` workgroups.  4 waves as 2 x 2, each
//                   64 x 64 = 4 x 4 MFMA tiles (16 fp64 accumulator quads = 128 VGPRs).
//                   K staged 16 columns at a time through double-buffered LDS (rows padded
//                   to 18 doubles: 16-B aligned rows, conflict-free fragment reads).
//   k_syrk_reduce   sums the split-K partial tiles in a fixed order (deterministic), applies
//                   A_ii = (1 + lambda) * JTJ_ii, writes the lower triangle and its mirror.
//   k_jtj_seq       n <= PNOL_SEQ_MAX: the reference's summation order, bitwise.
// The same tile kernel in "direct" mode (C = beta C + alpha X X^T on the lower tiles) is the
// trailing update of the blocked Cholesky in solve.hip.
#include "../pnol_internal.hpp"
#include "../pnol_comm.hpp"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace pnol {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 128;
constexpr int kTK = 16;
constexpr int kPad = 18;   // LDS row stride in doubles

__device__ __forceinline__ void tile_of(int t, int& ti, int& tj) {
    int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    ti = r;
    tj = t - r * (r + 1) / 2;
}

// Stage loader: TILE rows x 16 doubles of X starting at (row0, k0) into registers.
// 256 threads: TPR = 256 / TILE threads per row, each owning 16 / TPR consecutive columns.
// Rows >= nr and columns >= kend read as 0.
template <int TILE, int NT = 256>
struct StageRegs { double2 v[TILE * 8 / NT]; };

template <int TILE, int NT = 256>
__device__ __forceinline__ void load_stage(StageRegs<TILE, NT>& s, const double* __restrict__ X, long ldx, int nr,
                                           int row0, int k0, int kend, bool full) {
    constexpr int TPR = NT / TILE, CPT = 16 / TPR, NV = CPT / 2;
    const int t = threadIdx.x;
    const int row = row0 + t / TPR;
    const int kc = k0 + (t % TPR) * CPT;
    if (row < nr && full) {
        const double2* p = reinterpret_cast<const double2*>(X + (long)row * ldx + kc);
#pragma unroll
        for (int q = 0; q < NV; ++q) s.v[q] = p[q];
    } else {
        const double* p = X + (long)min(row, nr - 1) * ldx;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            int c0 = kc + 2 * q;
            double a = (row < nr && c0 < kend) ? p[c0] : 0.0;
            double b = (row < nr && c0 + 1 < kend) ? p[c0 + 1] : 0.0;
            s.v[q] = make_double2(a, b);
        }
    }
}

template <int TILE, int NT = 256>
__device__ __forceinline__ void store_stage(const StageRegs<TILE, NT>& s, double* __restrict__ lds) {
    constexpr int TPR = NT / TILE, CPT = 16 / TPR, NV = CPT / 2;
    const int t = threadIdx.x;
    double* dst = lds + (t / TPR) * kPad + (t % TPR) * CPT;
#pragma unroll
    for (int q = 0; q < NV; ++q) *reinterpret_cast<double2*>(dst + 2 * q) = s.v[q];
}

// MODE 0: write split-K partial tile to part; MODE 1: C = beta*C + alpha*acc (lower tiles);
// MODE 2: as MODE 0, instantiated separately for the chunked launches of launch_fd_jtj (so a
// kernel trace tells the whole-matrix launches and the pipelined row chunks apart).
// TILE 128: waves 2 x 2 of 64 x 64 (4 x 4 MFMA blocks each); TILE 64: 2 x 2 of 32 x 32.
// NW = 4: waves 2 x 2, each (TILE/2)^2; NW = 8: waves 2 x 4, each TILE/2 x TILE/4 (half the
// accumulators per wave, so twice the waves per SIMD hide the stage boundaries).
// MODE 3: as MODE 0, then the last of a tile's split_k workgroups to finish (counter cnt[t],
// agent-scope release/acquire) sums the tile's partials in slice order -- the same fixed
// order as k_syrk_reduce, so bitwise the same A -- and writes A = the tile with the
// Marquardt diagonal (alpha = lambda) and its mirror; cnt[t] is reset for the next launch.
template <int MODE, int TILE, bool XMAP = false, int NW = 4>
__global__ __launch_bounds__(64 * NW, 2) void k_syrk_tile(const double* __restrict__ X, long ldx, int nr, int K,
                                                      int split_k, int kchunk, double* __restrict__ part,
                                                      double* __restrict__ C, long ldc, double alpha,
                                                      double beta, int tile0, int* __restrict__ cnt = nullptr,
                                                      double* __restrict__ diag_out = nullptr) {
    constexpr int NT = 64 * NW, WC = NW / 2;
    constexpr int WTM = TILE / 2, WTN = TILE / WC, NBM = WTM / 16, NBN = WTN / 16;
    __shared__ __attribute__((aligned(16))) double lds[2][2][TILE * kPad];   // [buf][P/Q]

    // XMAP (split_k a multiple of 8): the K slices s = xcd, xcd + 8, ... go to the XCD that
    // dispatch slot blockIdx % 8 lands on, all tiles of one slice before the next, so the
    // workgroups resident on an XCD stream the same JT columns and share them in its L2.
    // Otherwise consecutive workgroups are the slices of one tile.
    int blk, t, sidx;
    if (XMAP) {
        const int xcd = blockIdx.x % kNumXcd, local = blockIdx.x / kNumXcd;
        const int ntl = gridDim.x / split_k;
        sidx = xcd + kNumXcd * (local / ntl);
        const int tl = local % ntl;
        blk = tl * split_k + sidx;           // partial slot: the same layout as below
        t = tile0 + tl;
    } else {
        blk = blockIdx.x;                    // partial slot (local to this launch)
        t = tile0 + blk / split_k;           // lower-triangle tile index
        sidx = blk % split_k;
    }
    int ti, tj;
    tile_of(t, ti, tj);
    const bool diag = ti == tj;
    const int prow0 = ti * TILE, qrow0 = tj * TILE;
    const int kbeg = sidx * kchunk;
    const int kend = min(K, kbeg + kchunk);
    const int nstages = kend > kbeg ? (kend - kbeg + kTK - 1) / kTK : 0;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wr = wave / WC, wc = wave % WC;
    const bool ldx_even = (ldx & 1) == 0;

    d4 acc[NBM][NBN];
#pragma unroll
    for (int i = 0; i < NBM; ++i)
#pragma unroll
        for (int j = 0; j < NBN; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};

    StageRegs<TILE, NT> ps, qs;
    if (nstages > 0) {
        bool full = ldx_even && (kbeg + kTK <= kend);
        load_stage<TILE, NT>(ps, X, ldx, nr, prow0, kbeg, kend, full);
        if (!diag) load_stage<TILE, NT>(qs, X, ldx, nr, qrow0, kbeg, kend, full);
    }
    const int frow = lane & 15;
    const int fk = lane >> 4;
    for (int st = 0; st < nstages; ++st) {
        const int buf = st & 1;
        double* P = lds[buf][0];
        double* Q = diag ? lds[buf][0] : lds[buf][1];
        store_stage<TILE, NT>(ps, P);
        if (!diag) store_stage<TILE, NT>(qs, Q);
        __syncthreads();
        if (st + 1 < nstages) {
            const int k0 = kbeg + (st + 1) * kTK;
            bool full = ldx_even && (k0 + kTK <= kend);
            load_stage<TILE, NT>(ps, X, ldx, nr, prow0, k0, kend, full);
            if (!diag) load_stage<TILE, NT>(qs, X, ldx, nr, qrow0, k0, kend, full);
        }
#pragma unroll
        for (int kk = 0; kk < kTK / 4; ++kk) {
            double a[NBM], b[NBN];
#pragma unroll
            for (int mi = 0; mi < NBM; ++mi) a[mi] = P[(wr * WTM + mi * 16 + frow) * kPad + kk * 4 + fk];
#pragma unroll
            for (int ni = 0; ni < NBN; ++ni) b[ni] = Q[(wc * WTN + ni * 16 + frow) * kPad + kk * 4 + fk];
#pragma unroll
            for (int mi = 0; mi < NBM; ++mi)
#pragma unroll
                for (int ni = 0; ni < NBN; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
    }

    // f64 MFMA C/D layout: lane l, register r -> row (l >> 4) + 4 r, column l & 15
    const int ocol = lane & 15;
    const int orow = lane >> 4;
    if (MODE == 0 || MODE == 2 || MODE == 3) {
        double* out = part + (long)blk * TILE * TILE;
#pragma unroll
        for (int mi = 0; mi < NBM; ++mi)
#pragma unroll
            for (int ni = 0; ni < NBN; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    int row = wr * WTM + mi * 16 + orow + 4 * r;
                    int col = wc * WTN + ni * 16 + ocol;
                    out[row * TILE + col] = acc[mi][ni][r];
                }
        if (MODE == 3) {
            __shared__ int s_last;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                const int old = __hip_atomic_fetch_add(cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_last = old == split_k - 1;
                if (s_last) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                }
            }
            __syncthreads();
            if (s_last) {
                const double scale = 1 + alpha;
                const double* p0 = part + ((long)(t - tile0) * split_k) * TILE * TILE;
                for (int e = threadIdx.x; e < TILE * TILE; e += NT) {
                    const int r = e / TILE, c = e % TILE;
                    const int i = prow0 + r, j = qrow0 + c;
                    if (i >= nr || j >= nr || j > i) continue;
                    double v = 0.0;
                    for (int s2 = 0; s2 < split_k; ++s2) v += p0[(long)s2 * TILE * TILE + e];
                    if (i == j) {
                        if (diag_out) diag_out[i] = v;
                        C[(long)i * ldc + i] = scale * v;
                    } else {
                        C[(long)i * ldc + j] = v;
                        C[(long)j * ldc + i] = v;
                    }
                }
                if (threadIdx.x == 0) cnt[t] = 0;
            }
        }
    } else {
#pragma unroll
        for (int mi = 0; mi < NBM; ++mi)
#pragma unroll
            for (int ni = 0; ni < NBN; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    int i = prow0 + wr * WTM + mi * 16 + orow + 4 * r;
                    int j = qrow0 + wc * WTN + ni * 16 + ocol;
                    if (i < nr && j < nr && j <= i) {
                        double* c = C + (long)i * ldc + j;
                        *c = beta * (*c) + alpha * acc[mi][ni][r];
                    }
                }
    }
}

// Tile-sharded J^T J (LevMarqMPI): sum one launch's partials per tile in the same fixed
// order, packed[tl * 128^2 + e] = raw (J^T J) tile values (no Marquardt scaling).
__global__ void k_syrk_reduce_packed(const double* __restrict__ part, int split_k, double* __restrict__ packed) {
    const int tl = blockIdx.y;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < kTile * kTile; e += gridDim.x * blockDim.x) {
        const double* p = part + ((long)tl * split_k) * kTile * kTile + e;
        double v = 0.0;
        for (int s = 0; s < split_k; ++s) v += p[(long)s * kTile * kTile];
        packed[(long)tl * kTile * kTile + e] = v;
    }
}

// Unpack the allgathered tile payloads (rank r's slot q holds tile r * tpr + q) into A:
// lower triangle + mirror, A_ii = (1 + lambda) (J^T J)_ii -- the same writes as k_syrk_reduce.
__global__ void k_syrk_unpack(const double* __restrict__ packed, int ntiles, int n, double lambda,
                              double* __restrict__ A, long lda, double* __restrict__ diag_out) {
    const int t = blockIdx.y;
    if (t >= ntiles) return;
    int ti, tj;
    tile_of(t, ti, tj);
    const double scale = 1 + lambda;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < kTile * kTile; e += gridDim.x * blockDim.x) {
        const int r = e / kTile, c = e % kTile;
        const int i = ti * kTile + r, j = tj * kTile + c;
        if (i >= n || j >= n || j > i) continue;
        const double v = packed[(long)t * kTile * kTile + e];
        if (i == j) {
            if (diag_out) diag_out[i] = v;
            A[(long)i * lda + i] = scale * v;
        } else {
            A[(long)i * lda + j] = v;
            A[(long)j * lda + i] = v;
        }
    }
}

// One 32 x 128 strip of a tile per workgroup (blockIdx.x = strip 0..3, blockIdx.y = tile):
// sums the split-K partials in slice order (coalesced 16-byte reads), writes the lower part
// row-wise, and writes the mirror from an LDS transpose so those stores are row-wise too.
__global__ __launch_bounds__(256) void k_syrk_reduce(const double* __restrict__ part, int ntiles, int split_k, int n,
                                                     double lambda, double* __restrict__ A, long lda,
                                                     double* __restrict__ diag_out, int tile0) {
    constexpr int SR = 32;                                 // strip rows
    __shared__ double st[SR][kTile + 1];
    const int t = tile0 + blockIdx.y;                      // part holds this launch's tiles from tile0 on
    int ti, tj;
    tile_of(t, ti, tj);
    const double scale = 1 + lambda;
    const int r0 = blockIdx.x * SR;
    const double* p = part + ((long)(t - tile0) * split_k) * kTile * kTile + (long)r0 * kTile;
    // 32 x 128 doubles = 2048 double2; 256 threads x 8
    for (int q = threadIdx.x; q < SR * kTile / 2; q += 256) {
        const int r = (2 * q) / kTile, c = (2 * q) % kTile;
        double2 v = make_double2(0.0, 0.0);
        for (int s2 = 0; s2 < split_k; ++s2) {
            const double2 w = reinterpret_cast<const double2*>(p + (long)s2 * kTile * kTile)[q];
            v.x += w.x;
            v.y += w.y;
        }
        st[r][c] = v.x;
        st[r][c + 1] = v.y;
        const int i = ti * kTile + r0 + r;
        for (int h = 0; h < 2; ++h) {
            const int j = tj * kTile + c + h;
            const double val = h ? v.y : v.x;
            if (i >= n || j >= n || j > i) continue;
            if (i == j) {
                if (diag_out) diag_out[i] = val;
                A[(long)i * lda + i] = scale * val;
            } else {
                A[(long)i * lda + j] = val;
            }
        }
    }
    __syncthreads();
    // mirror: A[j][i] = tile[i][j] for j > i; row j of A gets 32 consecutive columns i
    for (int q = threadIdx.x; q < SR * kTile; q += 256) {
        const int c = q / SR, r = q % SR;                  // consecutive threads: consecutive i
        const int i = ti * kTile + r0 + r, j = tj * kTile + c;
        if (i < n && j < n && j < i) A[(long)j * lda + i] = st[r][c];
    }
}

// reference order: JTJ_ij = sum_k JT_ik * JT_jk (k ascending, from 0.0); A_ii = (1+lambda) JTJ_ii
__global__ void k_jtj_seq(const double* __restrict__ JT, long ldjt, int m, int n, double lambda,
                          double* __restrict__ A, long lda, double* __restrict__ diag_out) {
    int i = blockIdx.y * blockDim.y + threadIdx.y;
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || j >= n) return;
    const double* a = JT + (long)i * ldjt;
    const double* b = JT + (long)j * ldjt;
    double s = 0.0;
    for (int k = 0; k < m; ++k) s = s + a[k] * b[k];
    if (i == j) {
        if (diag_out) diag_out[i] = s;
        A[(long)i * lda + j] = (1 + lambda) * s;
    } else {
        A[(long)i * lda + j] = s;
    }
}

}  // namespace

// Split-K factor: the workgroups are dispatched in rounds of one per CU, so the kernel takes
// ceil(nwg / ncu) rounds of (K / split) work.  Pick the split whose last round is fullest
// (nwg / (ncu * rounds) closest to 1), with K slices of >= 256 columns and at most 160 MB
// of partial tiles; ties go to the smaller split (less reduce traffic).  At n = 2048
// (136 tiles) on 256 CUs this is 7 (952 WGs, 93% of 4 rounds) instead of 4 (544, 71%).
static int choose_split_k(int ntiles, int K, int ncu) {
    static const int forced = [] {
        const char* e = std::getenv("PNOL_SYRK_SPLIT");
        return e ? std::atoi(e) : 0;
    }();
    if (forced > 0) return std::min(forced, std::max(1, (K + kTK - 1) / kTK));
    if (ncu <= 0) ncu = 256;
    const int kmax = (K + 255) / 256;
    int best = 1;
    double best_time = 1e30;
    for (int s = 1; s <= 64 && s <= kmax; ++s) {
        const double part_mb = (double)ntiles * s * kTile * kTile * 8.0 / 1e6;
        if (s > 1 && part_mb > 160.0) break;
        const long rounds = ((long)ntiles * s + ncu - 1) / ncu;
        const double time = (double)rounds / s;   // in units of one whole-K tile
        if (time < best_time * 0.995) {
            best = s;
            best_time = time;
        }
    }
    return best;
}

// J^T J variant (tuning; every variant sums each element in the same order):
// PNOL_SYRK_NW = 8 (default) or 4 waves per 128 x 128 tile; PNOL_SYRK_FUSED = 1 reduces the
// split-K partials inside the tile kernel (MODE 3), 0 (default) runs k_syrk_reduce after it.
// Measured at m = 16384, n = 2048: 8 waves 1.35 ms vs 4 waves 1.40 ms; the fused reduce 1.51 ms
// vs 1.35 + 0.06 ms -- every tile's last slice finishes in the final round, so the in-kernel
// reduces all land in the tail instead of overlapping the MFMA work.
static int syrk_nw() {
    static const int nw = [] {
        const char* e = std::getenv("PNOL_SYRK_NW");
        return (e && std::atoi(e) == 4) ? 4 : 8;
    }();
    return nw;
}

static bool syrk_fused() {
    static const bool on = [] {
        const char* e = std::getenv("PNOL_SYRK_FUSED");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

static bool syrk_xmap() {
    static const bool on = [] {
        const char* e = std::getenv("PNOL_SYRK_XMAP");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

int launch_jtj(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda, double* A, int lda,
               double* jtj_diag) {
    if (!JT || !A || m <= 0 || n <= 0 || ldjt < m || lda < n) return PNOL_ERR_ARG;
    if (n <= PNOL_SEQ_MAX && m <= 4096) {
        dim3 blk(16, 16), grd((n + 15) / 16, (n + 15) / 16);
        hipLaunchKernelGGL(k_jtj_seq, grd, blk, 0, ctx->stream, JT, (long)ldjt, m, n, lambda, A, (long)lda, jtj_diag);
        return launch_check();
    }
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    const int split_k = choose_split_k(ntiles, m, ctx->num_cu);
    int kchunk = (m + split_k - 1) / split_k;
    kchunk = (kchunk + kTK - 1) / kTK * kTK;
    void* part = nullptr;
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)ntiles * split_k * kTile * kTile, &part));
    if (syrk_fused()) {
        // partial tiles + the last-arriving workgroup's fixed-order reduce in one launch
        void* cnt = nullptr;
        PNOL_CHECK(ws_get_zeroed(ctx, "syrk_cnt", sizeof(int) * (size_t)ntiles, &cnt));
        ScopedTimer tm(ctx, "syrk");
        if (syrk_nw() == 4)
            hipLaunchKernelGGL((k_syrk_tile<3, kTile, false, 4>), dim3(ntiles * split_k), dim3(256), 0, ctx->stream,
                               JT, (long)ldjt, n, m, split_k, kchunk, (double*)part, A, (long)lda, lambda, 0.0, 0,
                               (int*)cnt, jtj_diag);
        else
            hipLaunchKernelGGL((k_syrk_tile<3, kTile, false, 8>), dim3(ntiles * split_k), dim3(512), 0, ctx->stream,
                               JT, (long)ldjt, n, m, split_k, kchunk, (double*)part, A, (long)lda, lambda, 0.0, 0,
                               (int*)cnt, jtj_diag);
        return launch_check();
    }
    {
        ScopedTimer tm(ctx, "syrk");
        if (syrk_nw() == 8)
            hipLaunchKernelGGL((k_syrk_tile<0, kTile, false, 8>), dim3(ntiles * split_k), dim3(512), 0, ctx->stream,
                               JT, (long)ldjt, n, m, split_k, kchunk, (double*)part, (double*)nullptr, 0L, 1.0, 0.0,
                               0);
        else if (syrk_xmap() && split_k % kNumXcd == 0)
            hipLaunchKernelGGL((k_syrk_tile<0, kTile, true>), dim3(ntiles * split_k), dim3(256), 0, ctx->stream, JT,
                               (long)ldjt, n, m, split_k, kchunk, (double*)part, (double*)nullptr, 0L, 1.0, 0.0, 0);
        else
            hipLaunchKernelGGL((k_syrk_tile<0, kTile>), dim3(ntiles * split_k), dim3(256), 0, ctx->stream, JT,
                               (long)ldjt, n, m, split_k, kchunk, (double*)part, (double*)nullptr, 0L, 1.0, 0.0, 0);
    }
    PNOL_CHECK(launch_check());
    ScopedTimer tm(ctx, "syrk_reduce");
    hipLaunchKernelGGL(k_syrk_reduce, dim3(kTile / 32, ntiles), dim3(256), 0, ctx->stream, (const double*)part, ntiles,
                       split_k, n, lambda, A, (long)lda, jtj_diag, 0);
    return launch_check();
}

int launch_jtj_rows(pnol_ctx* ctx, hipStream_t stream, const double* JT, int ldjt, int m, int n, double lambda,
                    double* A, int lda, double* jtj_diag, int row_begin, int row_end) {
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    if (row_begin < 0 || row_end > nt || row_begin >= row_end) return PNOL_ERR_ARG;
    const int split_k = choose_split_k(ntiles, m, ctx->num_cu);
    int kchunk = (m + split_k - 1) / split_k;
    kchunk = (kchunk + kTK - 1) / kTK * kTK;
    const int t0 = row_begin * (row_begin + 1) / 2, t1 = row_end * (row_end + 1) / 2;
    void* part = nullptr;
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)ntiles * split_k * kTile * kTile, &part));
    double* mypart = (double*)part + (size_t)t0 * split_k * kTile * kTile;   // disjoint per row range
    {
        ScopedTimer tm(ctx, "syrk_rows", stream);
        hipLaunchKernelGGL((k_syrk_tile<2, kTile, false, 8>), dim3((t1 - t0) * split_k), dim3(512), 0, stream, JT, (long)ldjt, n,
                           m, split_k, kchunk, mypart, (double*)nullptr, 0L, 1.0, 0.0, t0);
    }
    PNOL_CHECK(launch_check());
    hipLaunchKernelGGL(k_syrk_reduce, dim3(kTile / 32, t1 - t0), dim3(256), 0, stream, (const double*)mypart, t1 - t0, split_k,
                       n, lambda, A, (long)lda, jtj_diag, t0);
    return launch_check();
}

// FD Jacobian + J^T J, pipelined over column chunks.  The FD point tiles are the 128-column
// blocks b = 0 .. nt-1, the same as the J^T J tile rows, so once FD blocks [0, b1) are done the
// tile rows [.., b1) are computable.  Chunk c: FD blocks [b_c, b_{c+1}) on the context stream,
// an event, then on the aux stream the J^T J rows [b_c, b_{c+1}).  The FD GEMM is VALU-bound
// and the J^T J MFMA-bound, so the two overlap on the CUs.  FD costs fall with the column
// index (prefix sharing) while J^T J rows grow, so chunk boundaries are placed at equal FD cost.
// JT and A are bitwise those of launch_fd_jacobian + launch_jtj.
int launch_fd_jtj(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, double* F0, int compute_f0,
                  double* JT, int ldjt, double lambda, double* A, int lda, double* jtj_diag, int nchunks) {
    if (!o || !JT || !A) return PNOL_ERR_ARG;
    const int n = o->n, m = o->m;
    const int nt = (n + kTile - 1) / kTile;
    if (o->kind != PNOL_OBJ_LINRES || nchunks <= 1 || nt < 2 || (n <= PNOL_SEQ_MAX && m <= 4096)) {
        PNOL_CHECK(launch_fd_jacobian(ctx, o, x, h, 0, n, F0, compute_f0, JT, ldjt));
        ScopedTimer tm(ctx, "syrk");
        return launch_jtj(ctx, JT, ldjt, m, n, lambda, A, lda, jtj_diag);
    }
    nchunks = std::min(nchunks, nt);
    if (!ctx->aux_stream) PNOL_HIP(hipStreamCreateWithFlags(&ctx->aux_stream, hipStreamNonBlocking));
    while ((int)ctx->aux_events.size() < nchunks + 1) {
        hipEvent_t e;
        PNOL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->aux_events.push_back(e);
    }
    // chunk boundaries at equal FD cost: block b costs ~ (n - 128 b) chain steps
    std::vector<int> bnd(1, 0);
    {
        double total = 0;
        for (int b = 0; b < nt; ++b) total += n - (double)b * kTile;
        double acc = 0;
        for (int b = 0; b < nt && (int)bnd.size() < nchunks; ++b) {
            acc += n - (double)b * kTile;
            if (acc >= total * bnd.size() / nchunks && b + 1 < nt) bnd.push_back(b + 1);
        }
        bnd.push_back(nt);
    }
    // the aux stream starts after everything already queued on the context stream
    ScopedTimer tm(ctx, "fd_jtj");
    PNOL_HIP(hipEventRecord(ctx->aux_events[nchunks], ctx->stream));
    PNOL_HIP(hipStreamWaitEvent(ctx->aux_stream, ctx->aux_events[nchunks], 0));
    std::vector<int> st, ct;
    for (size_t c = 0; c + 1 < bnd.size(); ++c) {
        st.clear();
        ct.clear();
        for (int b = bnd[c]; b < bnd[c + 1]; ++b) {
            st.push_back(b * kTile);
            ct.push_back(std::min(kTile, n - b * kTile));
        }
        PNOL_CHECK(launch_fd_jacobian_tiles(ctx, o, x, h, st.data(), ct.data(), (int)st.size(), F0, compute_f0, JT, 0,
                                            ldjt, c == 0 ? 1 : 0));
        PNOL_HIP(hipEventRecord(ctx->aux_events[c], ctx->stream));
        PNOL_HIP(hipStreamWaitEvent(ctx->aux_stream, ctx->aux_events[c], 0));
        PNOL_CHECK(launch_jtj_rows(ctx, ctx->aux_stream, JT, ldjt, m, n, lambda, A, lda, jtj_diag, bnd[c], bnd[c + 1]));
    }
    PNOL_HIP(hipEventRecord(ctx->aux_events[nchunks], ctx->aux_stream));
    PNOL_HIP(hipStreamWaitEvent(ctx->stream, ctx->aux_events[nchunks], 0));
    return PNOL_OK;
}

int launch_syrk_lower(pnol_ctx* ctx, const double* X, int ldx, int nr, int K, double alpha, double* C, int ldc,
                      int split_k) {
    (void)split_k;
    if (!X || !C || nr <= 0 || K <= 0) return PNOL_ERR_ARG;
    // 64 x 64 tiles: the Cholesky trailing update has K = 64, so per-workgroup work is small
    // and the launch is latency-bound; 4x more workgroups than 128 x 128 tiles fill the chip.
    constexpr int kT = 64;
    const int nt = (nr + kT - 1) / kT;
    const int ntiles = nt * (nt + 1) / 2;
    hipLaunchKernelGGL((k_syrk_tile<1, kT>), dim3(ntiles), dim3(256), 0, ctx->stream, X, (long)ldx, nr, K, 1, K,
                       (double*)nullptr, C, (long)ldc, alpha, 1.0, 0);
    return launch_check();
}

// J^T J with the 128 x 128 tiles split over the communicator's ranks (contiguous ranges of
// tpr = ceil(ntiles / P) tiles), then one allgather of the packed tiles (P * tpr * 128 KB).
// The split-K factor comes from the global tile count, so every tile is summed exactly as on
// one GPU: A is bitwise independent of P.  n <= PNOL_SEQ_MAX keeps the replicated
// reference-order kernel.
int launch_jtj_sharded(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda, double* A, int lda,
                       double* jtj_diag) {
    const int P = comm_size(), rank = comm_rank();
    if (P <= 1 || (n <= PNOL_SEQ_MAX && m <= 4096)) return launch_jtj(ctx, JT, ldjt, m, n, lambda, A, lda, jtj_diag);
    if (!JT || !A || m <= 0 || n <= 0 || ldjt < m || lda < n) return PNOL_ERR_ARG;
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    const int split_k = choose_split_k(ntiles, m, ctx->num_cu);
    int kchunk = (m + split_k - 1) / split_k;
    kchunk = (kchunk + kTK - 1) / kTK * kTK;
    const int tpr = (ntiles + P - 1) / P;
    const int t0 = std::min(ntiles, rank * tpr), cnt = std::min(ntiles, t0 + tpr) - t0;
    const size_t tile_elems = (size_t)kTile * kTile;
    void *part = nullptr, *packed = nullptr;
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)std::max(cnt, 1) * split_k * tile_elems, &part));
    PNOL_CHECK(ws_get(ctx, "syrk_packed", sizeof(double) * (size_t)P * tpr * tile_elems, &packed));
    double* mine = (double*)packed + (size_t)rank * tpr * tile_elems;
    if (cnt > 0) {
        {
            ScopedTimer tm(ctx, "syrk");
            hipLaunchKernelGGL((k_syrk_tile<0, kTile, false, 8>), dim3(cnt * split_k), dim3(512), 0, ctx->stream, JT, (long)ldjt,
                               n, m, split_k, kchunk, (double*)part, (double*)nullptr, 0L, 1.0, 0.0, t0);
        }
        PNOL_CHECK(launch_check());
        hipLaunchKernelGGL(k_syrk_reduce_packed, dim3(8, cnt), dim3(256), 0, ctx->stream, (const double*)part, split_k,
                           mine);
        PNOL_CHECK(launch_check());
    }
    PNOL_CHECK(comm_allgather_device(ctx, mine, (double*)packed, (size_t)tpr * tile_elems));
    ScopedTimer tm(ctx, "syrk_reduce");
    hipLaunchKernelGGL(k_syrk_unpack, dim3(8, ntiles), dim3(256), 0, ctx->stream, (const double*)packed, ntiles, n,
                       lambda, A, (long)lda, jtj_diag);
    return launch_check();
}

int launch_jtr(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, const double* F, double* rhs) {
    if (n <= PNOL_SEQ_MAX && m <= 4096) return launch_gemv_neg_seq(ctx, JT, ldjt, n, m, F, rhs);
    return launch_gemv_neg(ctx, JT, ldjt, n, m, F, rhs);
}

}  // namespace pnol
