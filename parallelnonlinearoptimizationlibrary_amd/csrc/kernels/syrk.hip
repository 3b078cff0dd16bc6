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
#include "../pnol_internal.hpp"
#include "../pnol_comm.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

namespace pnol {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 128;
constexpr int kTK = 16;
constexpr int kPad = 18;   // LDS row stride in doubles

// Diagonal tiles (ti == tj) of the 8-wave 128-row kernel compute only their 36 lower 16 x 16
// blocks (bi >= bj) of the 64, 5 or 4 per wave so that the two waves of each SIMD (waves w and
// w + 4) hold 9 together -- the busiest SIMD issues 36 MFMAs per stage instead of 64 -- and
// zero the 28 upper blocks (no reader uses them; the partials stay fully defined).  Each block
// runs the same MFMA chain as in the 2 x 4 wave layout, so the partials are bitwise the same.
// wave w's blocks as bi * 8 + bj, 6 bits each (blocks of one block row together: they share
// the A fragment); bits 30..31: 4 or 5 blocks.  Words, not bytes: a scalar load.
__device__ __forceinline__ unsigned diag_blocks(int w) {
    constexpr unsigned T[8] = {
        56u | 57u << 6 | 58u << 12 | 59u << 18 | 60u << 24 | 1u << 30,
        48u | 49u << 6 | 50u << 12 | 51u << 18 | 52u << 24 | 1u << 30,
        40u | 41u << 6 | 42u << 12 | 43u << 18 | 44u << 24 | 1u << 30,
        32u | 33u << 6 | 34u << 12 | 35u << 18 | 36u << 24 | 1u << 30,
        61u | 62u << 6 | 63u << 12 | 0u << 18,
        53u | 54u << 6 | 8u << 12 | 9u << 18,
        45u | 16u << 6 | 17u << 12 | 18u << 18,
        24u | 25u << 6 | 26u << 12 | 27u << 18};
    unsigned v = T[0];
#pragma unroll
    for (int q = 1; q < 8; ++q) v = w == q ? T[q] : v;   // w is wave-uniform: scalar selects
    return v;
}
// the first kDiagSplit[w] blocks share one block row, the rest another (two A fragments)
__device__ __forceinline__ int diag_split(int w) {
    constexpr int S[8] = {5, 5, 5, 5, 3, 2, 1, 4};
    int v = S[0];
#pragma unroll
    for (int q = 1; q < 8; ++q) v = w == q ? S[q] : v;
    return v;
}

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

#ifdef PNOL_SYRK_TIMELINE
// tools/microbench/syrk_timeline.hip only: per workgroup start / end (100 MHz realtime) and
// the hardware ids of the CU it ran on
__device__ unsigned long long g_syrk_tl[3 * 65536];
#endif

// MODE 0: write split-K partial tile to part; MODE 4: 64 x 64 tiles into the 128 x 128 partial
// layout of MODE 0 (see the store below); MODE 2: as MODE 0, instantiated separately for the
// chunked launches of launch_fd_jtj (so a kernel trace tells the whole-matrix launches and the
// pipelined row chunks apart).
// TILE 128: waves 2 x 2 of 64 x 64 (4 x 4 MFMA blocks each); TILE 64: 2 x 2 of 32 x 32.
// NW = 4: waves 2 x 2, each (TILE/2)^2; NW = 8: waves 2 x 4, each TILE/2 x TILE/4 (half the
// accumulators per wave, so twice the waves per SIMD hide the stage boundaries).
// a partial store: non-temporal, or (NTS false) a plain store that may stay in the caches for the
// reduce that reads it next
template <bool NTS, bool SC1 = false>
__device__ __forceinline__ void part_store(double v, double* p) {
    if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // write-through
    else if constexpr (NTS) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// The tile body (k_syrk_tile, and k_syrk_red's SYRK workgroups): workgroup bid of nblk, its
// LDS (lds[buf][P/Q]) passed in; returns the lower-triangle tile index it formed a partial of.
// SC1: the partial stores write through (k_syrk_red's reduce workgroups read them in-launch).
template <int MODE, int TILE, int NW = 4, bool NTS = true, bool SC1 = false, bool DLAST = false>
__device__ __forceinline__ int syrk_tile_body(const double* __restrict__ X, long ldx, int nr, int K, int split_k,
                                              int kfirst, int kchunk, int sub, int slice0, int mS, long sstride,
                                              double* __restrict__ part, int tile0, int bid, int nblk,
                                              double (&lds)[2][2][TILE * kPad]) {
    constexpr int NT = 64 * NW, WC = NW / 2;
    constexpr int WTM = TILE / 2, WTN = TILE / WC, NBM = WTM / 16, NBN = WTN / 16;
#ifdef PNOL_SYRK_TIMELINE
    const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime();
#endif
    // every (tile, slice)'s chunk 0 first, then chunk 1, ...: with a long chunk 0 the short
    // chunks fill the last dispatch round instead of leaving it part-empty
    int blk, t, sidx;
    {
        const int ntl = nblk / split_k, nsl = split_k / sub;
        const int u0 = bid / (ntl * nsl), rest = bid % (ntl * nsl);
        int tl = rest / nsl;
        // DLAST (the whole lower triangle of 128-row tiles): the off-diagonal tiles first, in
        // row order, then the diagonal ones -- the co-resident workgroups of an XCD then do equal
        // work on neighbouring panels in step (the diagonal tiles, 36 of 64 blocks, used to run
        // ahead of the tiles sharing their panels), and the cheap diagonal tiles fill the tail
        if (DLAST) {
            const int nt = (int)((sqrt(8.0 * ntl + 1.0) - 1.0) * 0.5 + 0.5);
            const int noff = ntl - nt;
            if (tl < noff) {
                int r = (int)((sqrt(8.0 * tl + 1.0) + 1.0) * 0.5);   // row r >= 1: r (r - 1) / 2 <= tl
                while (r * (r - 1) / 2 > tl) --r;
                while ((r + 1) * r / 2 <= tl) ++r;
                tl = r * (r + 1) / 2 + (tl - r * (r - 1) / 2);
            } else {
                const int d = tl - noff;
                tl = d * (d + 1) / 2 + d;
            }
        }
        sidx = (rest % nsl) * sub + u0;
        blk = tl * split_k + sidx;           // partial slot (local to this launch)
        t = tile0 + tl;                      // lower-triangle tile index
    }
    int ti, tj;
    tile_of(t, ti, tj);
    const bool diag = ti == tj;
    const int prow0 = ti * TILE, qrow0 = tj * TILE;
    // K slice sidx = sub-chunk u of m-slice `slice` (columns [slice * mS, (slice + 1) * mS) of
    // the operand, stored at X + slice * sstride with row stride ldx; sstride == mS is the
    // plain row-major layout)
    const int slice = slice0 + sidx / sub, u = sidx % sub;
    X += (long)slice * (sstride - mS);
    // sub-chunk 0 is [0, kfirst) of the slice, chunk u >= 1 [kfirst + (u-1) kchunk, + kchunk)
    const int kbeg = slice * mS + (u == 0 ? 0 : kfirst + (u - 1) * kchunk);
    const int kend = min(K, min((slice + 1) * mS, u == 0 ? slice * mS + kfirst : kbeg + kchunk));
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

    constexpr bool kBal = NW == 8 && TILE == 128;
    const bool bal = kBal && diag;
    int dbi[5], dbj[5], dcnt = 0, dsplit = 0;
    {
        const int wv = __builtin_amdgcn_readfirstlane(wave);
        const unsigned code = bal ? diag_blocks(wv) : 0u;
        dcnt = 4 + (int)(code >> 30);
        dsplit = diag_split(wv);
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            dbi[q] = (code >> (6 * q + 3)) & 7;
            dbj[q] = (code >> (6 * q)) & 7;
        }
    }
    const int drow0 = dbi[0], drow1 = dsplit >= 4 ? dbi[4] : dsplit == 3 ? dbi[3] : dsplit == 2 ? dbi[2] : dbi[1];

    // the stage loop, instantiated once per path (diagonal-balanced or 2 x 4 waves) so each copy
    // holds only its own fragments live
    auto stage_loop = [&](auto BAL) {
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
            // one 16-byte fragment read per operand block covers two MFMA K-groups: lane l holds
            // k = 8 kk + 2 (l >> 4) + {0, 1}; the first MFMA takes the even k of the 8-block, the
            // second the odd ones (half the ds_read instructions; the 144-byte row stride keeps the
            // 16 rows of a 16-lane group on distinct bank quads).  Every element's MFMA chain is
            // the same in every mode and tile size, so all paths still sum it identically.
            if constexpr (decltype(BAL)::value) {
#pragma unroll
                for (int kk = 0; kk < kTK / 8; ++kk) {
                    const double2 a0 = *reinterpret_cast<const double2*>(P + (drow0 * 16 + frow) * kPad + kk * 8 + 2 * fk);
                    const double2 a1 = *reinterpret_cast<const double2*>(P + (drow1 * 16 + frow) * kPad + kk * 8 + 2 * fk);
                    double2 b[5];
#pragma unroll
                    for (int q = 0; q < 5; ++q)
                        if (q < 4 || dcnt == 5)
                            b[q] = *reinterpret_cast<const double2*>(P + (dbj[q] * 16 + frow) * kPad + kk * 8 + 2 * fk);
#pragma unroll
                    for (int q = 0; q < 5; ++q)
                        if (q < 4 || dcnt == 5)
                            acc[q >> 1][q & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(q < dsplit ? a0.x : a1.x, b[q].x,
                                                                                      acc[q >> 1][q & 1], 0, 0, 0);
#pragma unroll
                    for (int q = 0; q < 5; ++q)
                        if (q < 4 || dcnt == 5)
                            acc[q >> 1][q & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(q < dsplit ? a0.y : a1.y, b[q].y,
                                                                                      acc[q >> 1][q & 1], 0, 0, 0);
                }
            } else {
#pragma unroll
            for (int kk = 0; kk < kTK / 8; ++kk) {
                double2 a[NBM], b[NBN];
#pragma unroll
                for (int mi = 0; mi < NBM; ++mi)
                    a[mi] = *reinterpret_cast<const double2*>(P + (wr * WTM + mi * 16 + frow) * kPad + kk * 8 + 2 * fk);
#pragma unroll
                for (int ni = 0; ni < NBN; ++ni)
                    b[ni] = *reinterpret_cast<const double2*>(Q + (wc * WTN + ni * 16 + frow) * kPad + kk * 8 + 2 * fk);
#pragma unroll
                for (int mi = 0; mi < NBM; ++mi)
#pragma unroll
                    for (int ni = 0; ni < NBN; ++ni)
                        acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi].x, b[ni].x, acc[mi][ni], 0, 0, 0);
#pragma unroll
                for (int mi = 0; mi < NBM; ++mi)
#pragma unroll
                    for (int ni = 0; ni < NBN; ++ni)
                        acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi].y, b[ni].y, acc[mi][ni], 0, 0, 0);
            }
            }
        }
    };
    if (kBal && bal) stage_loop(std::true_type{});
    else stage_loop(std::false_type{});

    // f64 MFMA C/D layout: lane l, register r -> row (l >> 4) + 4 r, column l & 15
    const int ocol = lane & 15;
    const int orow = lane >> 4;
    {
        // MODE 4 (TILE 64, tile0 = 0): the quadrant (ti & 1, tj & 1) of the 128 x 128 partial
        // tile (ti / 2, tj / 2) -- the same partial layout, and every element summed in the same
        // order as by the 128-row kernel (one MFMA accumulator chain over the same K range)
        double* out;
        int ld;
        if (MODE == 4) {
            const int t128 = (ti >> 1) * ((ti >> 1) + 1) / 2 + (tj >> 1);
            out = part + ((long)t128 * split_k + sidx) * (4 * TILE * TILE) + (long)(ti & 1) * TILE * (2 * TILE) +
                  (tj & 1) * TILE;
            ld = 2 * TILE;
        } else {
            out = part + (long)blk * TILE * TILE;
            ld = TILE;
        }
        if (kBal && bal) {
#pragma unroll
            for (int q = 0; q < 5; ++q)
                if (q < 4 || dcnt == 5)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        part_store<NTS, SC1>(acc[q >> 1][q & 1][r], out + (dbi[q] * 16 + orow + 4 * r) * ld + dbj[q] * 16 + ocol);
            // upper block u = bj (bj - 1) / 2 + bi (bi < bj): blocks wave, wave + 8, ... of the 28
            for (int u = __builtin_amdgcn_readfirstlane(wave); u < 28; u += NW) {
                int bj = 1;
                while ((bj + 1) * bj / 2 <= u) ++bj;
                const int bi = u - bj * (bj - 1) / 2;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    part_store<NTS, SC1>(0.0, out + (bi * 16 + orow + 4 * r) * ld + bj * 16 + ocol);
            }
        } else {
#pragma unroll
            for (int mi = 0; mi < NBM; ++mi)
#pragma unroll
                for (int ni = 0; ni < NBN; ++ni)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        int row = wr * WTM + mi * 16 + orow + 4 * r;
                        int col = wc * WTN + ni * 16 + ocol;
                        part_store<NTS, SC1>(acc[mi][ni][r], out + row * ld + col);
                    }
        }
    }
#ifdef PNOL_SYRK_TIMELINE
    if (threadIdx.x == 0) {
        const unsigned long long tl1 = __builtin_amdgcn_s_memrealtime();
        const unsigned hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));     // HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));    // XCC_ID
        g_syrk_tl[3 * bid] = tl0;
        g_syrk_tl[3 * bid + 1] = tl1;
        g_syrk_tl[3 * bid + 2] = ((unsigned long long)xcc << 32) | hw;
    }
#endif
    return t;
}

template <int MODE, int TILE, int NW = 4, bool NTS = true>
__global__ __launch_bounds__(64 * NW, 2) void k_syrk_tile(const double* __restrict__ X, long ldx, int nr, int K,
                                                      int split_k, int kfirst, int kchunk, int sub, int slice0,
                                                      int mS, long sstride, double* __restrict__ part, int tile0) {
    __shared__ __attribute__((aligned(16))) double lds[2][2][TILE * kPad];   // [buf][P/Q]
    (void)syrk_tile_body<MODE, TILE, NW, NTS>(X, ldx, nr, K, split_k, kfirst, kchunk, sub, slice0, mS, sstride, part,
                                              tile0, blockIdx.x, gridDim.x, lds);
}

// ---- the m-slice summation tree ------------------------------------------------------------
// J^T J and J^T F are summed over the residual rows in kLmSlices m-slices (slice s: rows
// [s mS, (s + 1) mS)).  A slice's value ("leaf") is the sequential sum from 0.0 of its
// sub-chunk partials; the leaves are combined by the fixed pairwise tree
// ((l0 + l1) + (l2 + l3)) + ((l4 + l5) + (l6 + l7)).  A LevMarqMPI rank holding slices [a, b)
// reduces its leaves to the maximal dyadic nodes of that tree inside [a, b) (tree_merge on the
// leaves it has); the owner of an output merges the nodes of all ranks the same way.  Every
// node is the same IEEE sum wherever it is formed, so A and J^T F do not depend on P.
constexpr int kS = kLmSlices;
static_assert(kS == 8, "tree8 spells out the 8-leaf tree");

// v[i]: the node starting at slice i, sz[i] its width (0: none); siblings of equal width merge
// bottom up.  With all kS leaves present this is tree8.
__device__ __forceinline__ void tree_merge(double (&v)[kS], int (&sz)[kS]) {
#pragma unroll
    for (int w = 1; w < kS; w *= 2)
#pragma unroll
        for (int i = 0; i < kS; i += 2 * w)
            if (sz[i] == w && sz[i + w] == w) {
                v[i] = v[i] + v[i + w];
                sz[i] = 2 * w;
                sz[i + w] = 0;
            }
}

__device__ __forceinline__ double tree8(const double (&l)[kS]) {
    return ((l[0] + l[1]) + (l[2] + l[3])) + ((l[4] + l[5]) + (l[6] + l[7]));
}

// Leaves of slices [s0, s1) -- leaf s = sum over u < sub of
// part[unit * ustride + ((s - s0) * sub + u) * sstride + e] -- merged into this range's dyadic
// nodes, written in slice order to out[c * ocstride + unit * oustride + e].  blockIdx.y = unit.
__global__ __launch_bounds__(256) void k_tree_nodes(const double* __restrict__ part, long ustride, long sstride,
                                                    int sub, int s0, int s1, int elems, double* __restrict__ out,
                                                    long ocstride, long oustride) {
    const long unit = blockIdx.y;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < elems; e += gridDim.x * blockDim.x) {
        double v[kS];
        int sz[kS];
#pragma unroll
        for (int i = 0; i < kS; ++i) {
            v[i] = 0.0;
            sz[i] = 0;
            if (i >= s0 && i < s1) {
                const double* p = part + unit * ustride + (long)(i - s0) * sub * sstride + e;
                double a = 0.0;
                for (int u = 0; u < sub; ++u) a += p[(long)u * sstride];
                v[i] = a;
                sz[i] = 1;
            }
        }
        tree_merge(v, sz);
        int c = 0;
#pragma unroll
        for (int i = 0; i < kS; ++i)
            if (sz[i]) out[(long)(c++) * ocstride + unit * oustride + e] = v[i];
    }
}

// The nodes of all ranks (node at slice i: p[i], width w[i]; w[i] = 0 where no node starts)
// merged to the root: out[e].
struct TreeNodes {
    const double* p[kS];
    int w[kS];
};

__global__ __launch_bounds__(256) void k_tree_combine(const TreeNodes tn, long elems, double* __restrict__ out) {
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < elems; e += (long)gridDim.x * blockDim.x) {
        double v[kS];
        int sz[kS];
#pragma unroll
        for (int i = 0; i < kS; ++i) {
            sz[i] = tn.w[i];
            v[i] = sz[i] ? tn.p[i][e] : 0.0;
        }
        tree_merge(v, sz);
        out[e] = v[0];
    }
}

// Tile-sharded J^T J (pnol_jtj_mpi_d): one launch's partials per tile summed by the slice tree,
// packed[tl * 128^2 + e] = raw (J^T J) tile values (no Marquardt scaling).
__global__ void k_syrk_reduce_packed(const double* __restrict__ part, int sub, double* __restrict__ packed) {
    const int tl = blockIdx.y;
    const long E = kTile * kTile;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < kTile * kTile; e += gridDim.x * blockDim.x) {
        const double* p = part + (long)tl * kS * sub * E + e;
        double l[kS];
#pragma unroll
        for (int s = 0; s < kS; ++s) {
            double a = 0.0;
            for (int u = 0; u < sub; ++u) a += p[(long)(s * sub + u) * E];
            l[s] = a;
        }
        packed[(long)tl * E + e] = tree8(l);
    }
}

// Unpack allgathered tile payloads (tile t in rank t / tpr's slot of `slot` doubles, at
// (t % tpr) * 128^2) into A: lower triangle + mirror, A_ii = (1 + lambda) (J^T J)_ii -- the
// same writes as k_syrk_reduce.
__global__ void k_syrk_unpack(const double* __restrict__ packed, int ntiles, int n, double lambda, long slot, int tpr,
                              double* __restrict__ A, long lda, double* __restrict__ diag_out) {
    const int t = blockIdx.y;
    if (t >= ntiles) return;
    int ti, tj;
    tile_of(t, ti, tj);
    const double scale = 1 + lambda;
    const double* src = packed + (long)(t / tpr) * slot + (long)(t % tpr) * kTile * kTile;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < kTile * kTile; e += gridDim.x * blockDim.x) {
        const int r = e / kTile, c = e % kTile;
        const int i = ti * kTile + r, j = tj * kTile + c;
        if (i >= n || j >= n || j > i) continue;
        const double v = src[e];
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
// sums the partials by the slice tree (coalesced 16-byte reads), writes the lower part
// row-wise, and writes the mirror from an LDS transpose so those stores are row-wise too.
// SUB > 0: the sub-chunk count at compile time (all kS * SUB loads of an element in flight at
// once); SUB = 0: runtime `sub`.
// jp / rhs (nullable): one more row of blocks (blockIdx.y == ntiles) forms rhs = the slice
// tree of the 8 -J^T F slice partials jp[s * n + e], exactly as k_tree_nodes over all slices does
// (leaf = 0.0 + partial, then tree8): the tree rides in this launch instead of its own.
// (the body: workgroup (bx, by) of nbx x .., NT threads, the strip staging st[SR][kTile + 1]
// passed in -- k_syrk_reduce, and k_syrk_red's reduce workgroups)
template <int SUB, int SR, int NT>
__device__ __forceinline__ void syrk_reduce_body(const double* __restrict__ part, int ntiles, int sub_rt, int n,
                                                 double lambda, double* __restrict__ A, long lda,
                                                 double* __restrict__ diag_out, int tile0, const double* __restrict__ jp,
                                                 double* __restrict__ rhs, double* __restrict__ rhs2, int bx, int by,
                                                 int nbx, double (*st)[kTile + 1]) {
    if (jp && by == ntiles) {
        for (int e = bx * NT + (int)threadIdx.x; e < n; e += nbx * NT) {
            double l[kS];
#pragma unroll
            for (int s = 0; s < kS; ++s) l[s] = 0.0 + jp[(long)s * n + e];
            const double v = tree8(l);
            rhs[e] = v;
            if (rhs2) rhs2[e] = v;   // (the Cholesky's b when the reduce writes its matrix)
        }
        return;
    }
    const int sub = SUB > 0 ? SUB : sub_rt;                // SR: strip rows
    const int t = tile0 + by;                              // part holds this launch's tiles from tile0 on
    int ti, tj;
    tile_of(t, ti, tj);
    const double scale = 1 + lambda;
    const int r0 = bx * SR;
    const long E = kTile * kTile;
    const double* p = part + ((long)(t - tile0) * kS * sub) * E + (long)r0 * kTile;
    // 32 x 128 doubles = 2048 double2; 256 threads x 8
#pragma unroll 2
    for (int q = threadIdx.x; q < SR * kTile / 2; q += NT) {
        const int r = (2 * q) / kTile, c = (2 * q) % kTile;
        double lx[kS], ly[kS];
#pragma unroll
        for (int s = 0; s < kS; ++s) {
            double ax = 0.0, ay = 0.0;
#pragma unroll
            for (int u = 0; u < (SUB > 0 ? SUB : sub); ++u) {
                const double2 w = reinterpret_cast<const double2*>(p + (long)(s * sub + u) * E)[q];
                ax += w.x;
                ay += w.y;
            }
            lx[s] = ax;
            ly[s] = ay;
        }
        const double vx = tree8(lx), vy = tree8(ly);
        st[r][c] = vx;
        st[r][c + 1] = vy;
        const int i = ti * kTile + r0 + r;
        for (int h = 0; h < 2; ++h) {
            const int j = tj * kTile + c + h;
            const double val = h ? vy : vx;
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
    for (int q = threadIdx.x; q < SR * kTile; q += NT) {
        const int c = q / SR, r = q % SR;                  // consecutive threads: consecutive i
        const int i = ti * kTile + r0 + r, j = tj * kTile + c;
        if (i < n && j < n && j < i) A[(long)j * lda + i] = st[r][c];
    }
}

template <int SUB, int SR = 32>
__global__ __launch_bounds__(256) void k_syrk_reduce(const double* __restrict__ part, int ntiles, int sub_rt, int n,
                                                     double lambda, double* __restrict__ A, long lda,
                                                     double* __restrict__ diag_out, int tile0,
                                                     const double* __restrict__ jp = nullptr,
                                                     double* __restrict__ rhs = nullptr,
                                                     double* __restrict__ rhs2 = nullptr) {
    __shared__ double st[SR][kTile + 1];
    syrk_reduce_body<SUB, SR, 256>(part, ntiles, sub_rt, n, lambda, A, lda, diag_out, tile0, jp, rhs, rhs2, blockIdx.x,
                                   blockIdx.y, gridDim.x, st);
}

// The one-GPU LM trip's J^T J split-K partials AND their reduce in one launch (k_syrk_red):
// workgroups [0, nsyrk) are k_syrk_tile<0, 128, 8>'s; each, after its partial, publishes it by
// the in-launch split-K hand-off (MI355X guide, cdna_hip_programming.md "In-launch split-K
// reduction": plain stores, every wave's vmcnt(0), the barrier, lane 0's agent release and
// vmcnt(0), then a relaxed agent add to its tile's counter -- or, SC1, write-through partial
// stores and no release).  Workgroups [nsyrk, ..) are k_syrk_reduce's (32-row strips, the extra
// row of blocks forming -J^T F): lane 0 polls its tile's counter (relaxed) until all split_k
// partials are in, then one agent acquire, vmcnt(0) and the barrier, then plain loads.  The
// reduce workgroups come after every SYRK workgroup in the grid, so they take the slots of the
// SYRK's last dispatch round as it drains (nothing a SYRK workgroup does waits on them); a poll
// past its cap sets info = kCholTimeout and gives up (the trip then redoes the solve from A formed
// from the partials).  Every value is the sum k_syrk_reduce forms: bitwise the two launches.
constexpr int kRedSR = 32, kRedSpin = 1 << 22;
template <int SUB, bool SC1, bool DLAST = false>
__global__ __launch_bounds__(512, 2) void k_syrk_red(const double* __restrict__ X, long ldx, int nr, int K,
                                                     int split_k, int kfirst, int kchunk, int sub, int mS, long sstride,
                                                     double* __restrict__ part, int nsyrk, int* __restrict__ tcnt,
                                                     int ntiles, int n, double lambda, double* __restrict__ A, long lda,
                                                     const double* __restrict__ jp, double* __restrict__ rhs,
                                                     double* __restrict__ rhs2, int* __restrict__ info) {
    __shared__ __attribute__((aligned(16))) double lds[2][2][kTile * kPad];
    __shared__ int ok_sh;
    const int b = blockIdx.x;
    if (b < nsyrk) {
        const int t = syrk_tile_body<0, kTile, 8, false, SC1, DLAST>(X, ldx, nr, K, split_k, kfirst, kchunk, sub, 0, mS,
                                                                    sstride, part, 0, b, nsyrk, lds);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if constexpr (!SC1) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_fetch_add(tcnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    constexpr int NBX = kTile / kRedSR;
    const int r = b - nsyrk, bx = r % NBX, by = r / NBX;
    if (by < ntiles) {
        if (threadIdx.x == 0) {
            int it = 0, ok = 1;
            while (__hip_atomic_load(tcnt + by, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < split_k) {
                __builtin_amdgcn_s_sleep(2);
                if (++it > kRedSpin) {
                    ok = 0;
                    atomicCAS(info, 0, kCholTimeout);
                    break;
                }
            }
            if (ok) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            ok_sh = ok;
        }
        __syncthreads();
        if (!ok_sh) return;
    }
#ifdef PNOL_SYRK_TIMELINE
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    double(*st)[kTile + 1] = reinterpret_cast<double(*)[kTile + 1]>(&lds[0][0][0]);
    syrk_reduce_body<SUB, kRedSR, 512>(part, ntiles, sub, n, lambda, A, lda, nullptr, 0, jp, rhs, rhs2, bx, by, NBX, st);
#ifdef PNOL_SYRK_TIMELINE
    if (threadIdx.x == 0) {   // the reduce workgroups' entries follow the SYRK ones (start = poll done)
        g_syrk_tl[3 * b] = rt0;
        g_syrk_tl[3 * b + 1] = __builtin_amdgcn_s_memrealtime();
        g_syrk_tl[3 * b + 2] = (unsigned long long)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) << 32;
    }
#endif
}
static_assert(kRedSR * (kTile + 1) <= 2 * 2 * kTile * kPad, "the reduce strip fits the SYRK's LDS");

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

// K split: kLmSlices m-slices of mS rows (a multiple of 64, so an FD row panel never straddles
// two), each cut into `sub` chunks.  sub depends on (m, n) only -- never on the number of
// ranks -- so every A element is summed the same way on any P.  Default: enough workgroups to
// fill the chip (>= 2048 = 256 CUs x 2 resident x 4 rounds), chunks >= 256 columns.  At
// m = 16384, n = 2048 (136 tiles) sub = 2: 2176 workgroups of K = 1024 (measured: SYRK 1.33 ms
// + reduce 0.09 ms, vs 1.42 + 0.05 ms at sub = 1).  PNOL_SYRK_SUB overrides.
struct SliceCfg {
    int mS, sub, kfirst, kchunk;
};

// k_syrk_reduce with the sub-chunk count as a template constant where it is 1, 2 or 4
// (grid.x = 128 / 32 strips per tile at SR = 32; SR = 16 launches twice the workgroups)
template <int SR, typename... Args>
static void launch_reduce_sr(dim3 grid, dim3 block, size_t shm, hipStream_t st, const double* part, int ntiles,
                             int sub, Args... args) {
    grid.x = grid.x * 32 / SR;
    if (sub == 1)
        hipLaunchKernelGGL((k_syrk_reduce<1, SR>), grid, block, shm, st, part, ntiles, sub, args...);
    else if (sub == 2)
        hipLaunchKernelGGL((k_syrk_reduce<2, SR>), grid, block, shm, st, part, ntiles, sub, args...);
    else if (sub == 4)
        hipLaunchKernelGGL((k_syrk_reduce<4, SR>), grid, block, shm, st, part, ntiles, sub, args...);
    else
        hipLaunchKernelGGL((k_syrk_reduce<0, SR>), grid, block, shm, st, part, ntiles, sub, args...);
}

// 16-row strips: 70 us vs 77 us for 32-row strips at n = 2048, sub = 2
template <typename... Args>
static void launch_reduce(dim3 grid, dim3 block, size_t shm, hipStream_t st, const double* part, int ntiles, int sub,
                          Args... args) {
    launch_reduce_sr<16>(grid, block, shm, st, part, ntiles, sub, args...);
}

static SliceCfg slice_cfg(int m, int ntiles) {
    static const int forced = [] {
        const char* e = std::getenv("PNOL_SYRK_SUB");
        return e ? std::atoi(e) : 0;
    }();
    SliceCfg c;
    c.mS = lm_slice_rows(m);
    const int cap = std::max(1, c.mS / 256);
    if (forced > 0) {
        c.sub = std::min(forced, std::max(1, c.mS / kTK));
    } else {
        const int want = (2048 + ntiles * kS - 1) / (ntiles * kS);
        c.sub = std::max(1, std::min(want, cap));
    }
    c.kchunk = ((c.mS + c.sub - 1) / c.sub + kTK - 1) / kTK * kTK;
    c.kfirst = c.kchunk;
    // Chunk 0 takes 75% of the slice (PNOL_SYRK_FIRST = percent; the rest split evenly over
    // chunks 1..sub-1) and is dispatched first (k_syrk_tile's order): 1088 long workgroups, then
    // 1088 short ones that fill the tail of the last dispatch round.  Measured at m = 16384,
    // n = 2048: 1.265 ms vs 1.326 ms for two equal chunks (tools/syrk_sweep.py).
    static const int first_pct = [] {
        const char* e = std::getenv("PNOL_SYRK_FIRST");
        return e ? std::atoi(e) : 75;
    }();
    if (c.sub >= 2 && first_pct > 0 && first_pct < 100) {
        c.kfirst = std::max(kTK, (int)((long)c.mS * first_pct / 100) / kTK * kTK);
        c.kchunk = ((c.mS - c.kfirst + c.sub - 2) / (c.sub - 1) + kTK - 1) / kTK * kTK;
    }
    return c;
}

// 8 waves per 128 x 128 tile (1.35 ms vs 1.40 ms with 4 at m = 16384, n = 2048).  (A split-K
// reduce fused into the tile kernel by the last arriving workgroup measured 1.51 ms vs 1.35 +
// 0.06: every tile's last slice finishes in the final round, so the reduces all land in the
// tail; an XCD-sliced dispatch and 8-byte fragment reads were no faster either; removed.)

// 64 x 64 output tiles (MODE 4) instead of 128 x 128 for the whole-matrix launches: 4x the
// workgroups (4 per CU), the same per-element sums.  Measured at m = 16384, n = 2048 on the
// sliced J^T (16 KB row stride): 1.23 ms vs 1.29 ms, and a rank of an 8-GPU LevMarqMPI (one
// m-slice) gets 1056 workgroups instead of 272; on the row-major J^T (128 KB row stride) the
// 64-row tiles are slower (1.35 vs 1.28 ms), so that layout keeps 128.  PNOL_SYRK_T64 = 0 / 1
// forces either (read per call: tests switch it).
static bool syrk_t64(bool sliced) {
    const char* e = std::getenv("PNOL_SYRK_T64");
    return e ? std::atoi(e) != 0 : sliced;
}

// Partial tiles [tile0, tile0 + ntl) x slices [slice0, slice0 + nsl) x sub-chunks of
// X (nr rows, K columns; slice s at X + s * sstride, row stride ldx) into
// part[((t - tile0) * nsl * sub + (s - slice0) * sub + u) * 128^2].
static void syrk_partials(pnol_ctx* ctx, hipStream_t stream, bool rows_variant, const double* X, long ldx,
                          long sstride, int nr, int K, const SliceCfg& sc, int slice0, int nsl, int tile0, int ntl,
                          double* part, bool t64 = false) {
    const int split = nsl * sc.sub;
    const dim3 grid(ntl * split);
    LaunchTimer tm(ctx, rows_variant ? "syrk_rows" : "syrk");
    if (t64) {   // all tiles (tile0 = 0): ntl counts the 64 x 64 lower tiles
        const int nt64 = (nr + 63) / 64;
        hipExtLaunchKernelGGL((k_syrk_tile<4, 64>), dim3(nt64 * (nt64 + 1) / 2 * split), dim3(256), 0, stream,
                              tm.start(), tm.stop(), 0, X, ldx, nr, K, split, sc.kfirst, sc.kchunk, sc.sub, slice0,
                              sc.mS, sstride, part, 0);
    } else if (rows_variant) {
        hipExtLaunchKernelGGL((k_syrk_tile<2, kTile, 8>), grid, dim3(512), 0, stream, tm.start(), tm.stop(), 0, X, ldx,
                              nr, K, split, sc.kfirst, sc.kchunk, sc.sub, slice0, sc.mS, sstride, part, tile0);
    } else {
        // plain partial stores: the reduce (or the reducing Cholesky) that reads them next finds
        // part of them in the caches -- solve 0.71 vs 0.73 ms, SYRK unchanged, in alternating
        // same-box runs (non-temporal stores for J itself in the FD kernel measured slower; so did
        // non-temporal partials again in round 5: SYRK +10-30 us)
        hipExtLaunchKernelGGL((k_syrk_tile<0, kTile, 8, false>), grid, dim3(512), 0, stream, tm.start(), tm.stop(), 0,
                              X, ldx, nr, K, split, sc.kfirst, sc.kchunk, sc.sub, slice0, sc.mS, sstride, part, tile0);
    }
}

static int jtr_gemv(pnol_ctx* ctx, const double* JT, int ldjt, long sstride, int m, int n, int mS, int s0, int nsl,
                    const double* F, hipStream_t stream = nullptr);
static int jtr_tree(pnol_ctx* ctx, int n, int s0, int nsl, double* out);

int launch_jtj(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda, double* A, int lda,
               double* jtj_diag, const double* F, double* rhs) {
    if (!JT || !A || m <= 0 || n <= 0 || ldjt < m || lda < n) return PNOL_ERR_ARG;
    if (n <= PNOL_SEQ_MAX && m <= 4096) {
        dim3 blk(16, 16), grd((n + 15) / 16, (n + 15) / 16);
        hipLaunchKernelGGL(k_jtj_seq, grd, blk, 0, ctx->stream, JT, (long)ldjt, m, n, lambda, A, (long)lda, jtj_diag);
        PNOL_CHECK(launch_check());
        return rhs ? launch_jtr(ctx, JT, ldjt, m, n, F, rhs) : PNOL_OK;
    }
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    const SliceCfg sc = slice_cfg(m, ntiles);
    void* part = nullptr;
    ctx->lm_trip_tiles.kind = 0;   // the trip's tiles are overwritten below
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)ntiles * kS * sc.sub * kTile * kTile, &part));
    syrk_partials(ctx, ctx->stream, false, JT, ldjt, sc.mS, n, m, sc, 0, kS, 0, ntiles, (double*)part,
                  syrk_t64(false));
    PNOL_CHECK(launch_check());
    if (rhs) PNOL_CHECK(jtr_gemv(ctx, JT, ldjt, sc.mS, m, n, sc.mS, 0, kS, F));
    // -J^T F's slice tree rides in the reduce launch (an extra row of blocks).  (The GEMV on a
    // second stream released by the SYRK's last-dispatched workgroup -- hipStreamWaitValue32 on a
    // tail word -- measured slower, 305-311 vs 314-317 LM iters/s: its HBM stream slowed the
    // SYRK's last workgroups more than it hid; removed.)
    const bool fold = rhs != nullptr;
    void* jp = nullptr;
    if (fold) PNOL_CHECK(ws_get(ctx, "jtr_part", sizeof(double) * (size_t)kS * n, &jp));
    {
        ScopedTimer tm(ctx, "syrk_reduce");
        launch_reduce(dim3(kTile / 32, ntiles + (fold ? 1 : 0)), dim3(256), 0, ctx->stream, (const double*)part,
                      ntiles, sc.sub, n, lambda, A, (long)lda, jtj_diag, 0, (const double*)jp,
                      fold ? rhs : (double*)nullptr);
        PNOL_CHECK(launch_check());
    }
    return PNOL_OK;
}

int launch_jtj_rows(pnol_ctx* ctx, hipStream_t stream, const double* JT, int ldjt, int m, int n, double lambda,
                    double* A, int lda, double* jtj_diag, int row_begin, int row_end) {
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    if (row_begin < 0 || row_end > nt || row_begin >= row_end) return PNOL_ERR_ARG;
    const SliceCfg sc = slice_cfg(m, ntiles);
    const int t0 = row_begin * (row_begin + 1) / 2, t1 = row_end * (row_end + 1) / 2;
    const size_t per_tile = (size_t)kS * sc.sub * kTile * kTile;
    void* part = nullptr;
    ctx->lm_trip_tiles.kind = 0;   // the trip's tiles are overwritten below
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)ntiles * per_tile, &part));
    double* mypart = (double*)part + (size_t)t0 * per_tile;   // disjoint per row range
    syrk_partials(ctx, stream, true, JT, ldjt, sc.mS, n, m, sc, 0, kS, t0, t1 - t0, mypart);
    PNOL_CHECK(launch_check());
    launch_reduce(dim3(kTile / 32, t1 - t0), dim3(256), 0, stream, (const double*)mypart, t1 - t0,
                       sc.sub, n, lambda, A, (long)lda, jtj_diag, t0);
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
                  double* JT, int ldjt, double lambda, double* A, int lda, double* jtj_diag, int nchunks,
                  double* rhs) {
    if (!o || !JT || !A) return PNOL_ERR_ARG;
    const int n = o->n, m = o->m;
    const int nt = (n + kTile - 1) / kTile;
    if (o->kind != PNOL_OBJ_LINRES || nchunks <= 1 || nt < 2 || (n <= PNOL_SEQ_MAX && m <= 4096)) {
        PNOL_CHECK(launch_fd_jacobian(ctx, o, x, h, 0, n, F0, compute_f0, JT, ldjt));
        return launch_jtj(ctx, JT, ldjt, m, n, lambda, A, lda, jtj_diag, F0, rhs);   // times "syrk" itself
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
    return rhs ? launch_jtr(ctx, JT, ldjt, m, n, F0, rhs) : PNOL_OK;
}

// One LM trip's linear algebra with A never formed (single process, n > PNOL_SEQ_MAX,
// LevenbergMarquardt.cpp:55-90): the FD Jacobian, the -J^T F slice partials, the Cholesky's
// prep launch (its words and paddings), the J^T J split-K partials (k_syrk_tile), the reduce
// launch writing A (the Marquardt diagonal) straight into the Cholesky's padded matrix and
// -J^T F into rhs and b, then the persistent tile Cholesky (its chain factors tile 0 itself), the
// backward solve and xnext = x + sigma: no A, no copy of A into the workspace.
// (PNOL_LM_REDUCE=tasks: the persistent launch's first tasks do the reduce themselves, beside the
// chain's first steps -- measured slower, 5/5 same-box trip A/Bs, its 285 MB partial stream in
// front of the chain.)  JT, rhs, sigma, xnext and the solve status are bitwise those of
// launch_fd_jtj (+ rhs) and launch_chol_solve; for the LU fallback launch_jtj_from_partials forms
// A from the trip's partials.
int launch_fd_normal_solve(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, double* F0, int compute_f0,
                           double* JT, int ldjt, double lambda, double* rhs, double* sigma, int* dinfo, double* xnext,
                           bool fd_queued) {
    if (!o || !x || !h || !F0 || !JT || !rhs || !sigma || !dinfo || !xnext || ldjt < o->m) return PNOL_ERR_ARG;
    const int n = o->n, m = o->m;
    if (n <= PNOL_SEQ_MAX) return PNOL_ERR_ARG;
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    const SliceCfg sc = slice_cfg(m, ntiles);
    const int split = kS * sc.sub;
    // the reduce (PNOL_LM_REDUCE, read per call): "tail" (default) its workgroups in the SYRK's
    // own launch (k_syrk_red), taking the slots of the SYRK's last dispatch round -- 3 of 3
    // same-box bench pairs faster than "launch", a reduce launch of its own writing the
    // Cholesky's padded matrix and b (1.18-1.20 ms for both against 1.14-1.16 + 0.07); "tasks":
    // the persistent launch's first tasks (round 4).  PNOL_SYRK_RED_SC1=1: write-through partials
    // and no release fence in the tail form (the same speed).
    const char* er = std::getenv("PNOL_LM_REDUCE");
    const bool tasks = er && std::strcmp(er, "tasks") == 0;
    const bool tail = (!er || std::strcmp(er, "tail") == 0) && !syrk_t64(false);
    // every workspace first: a (re)allocation frees, and a free waits for the device
    void *part = nullptr, *jp = nullptr;
    ctx->lm_trip_tiles.kind = 0;   // the trip's tiles are overwritten below
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)ntiles * split * kTile * kTile, &part));
    PNOL_CHECK(ws_get(ctx, "jtr_part", sizeof(double) * (size_t)kS * n, &jp));
    void* tcnt = nullptr;
    if (tail) PNOL_CHECK(ws_get(ctx, "syrk_tcnt", sizeof(int) * (size_t)ntiles, &tcnt));
    CholRed cr;
    PNOL_CHECK(launch_chol_reducing_prep(ctx, n, dinfo, cr));
    if (fd_queued) PNOL_CHECK(lm_fd_commit(ctx, o, x));   // the Jacobian at x is queued already
    else PNOL_CHECK(launch_fd_jacobian(ctx, o, x, h, 0, n, F0, compute_f0, JT, ldjt));
    PNOL_CHECK(jtr_gemv(ctx, JT, ldjt, sc.mS, m, n, sc.mS, 0, kS, F0));
    // the prep launch (words, paddings, info; the tile counters)
    PNOL_CHECK(launch_chol_reducing_start(ctx, cr, !tasks, (int*)tcnt, ntiles));
    if (tail) {
        const int nsyrk = ntiles * split, nred = (kTile / kRedSR) * (ntiles + 1);
        const char* es = std::getenv("PNOL_SYRK_RED_SC1");
        const bool sc1 = es && std::atoi(es) != 0;
        // the diagonal tiles last (default; PNOL_SYRK_DLAST=0 keeps the row order, read per call):
        // FETCH 1.75 -> 1.39 GB per launch at the same speed (3 same-box pairs, PMC passes of both)
        const char* ed = std::getenv("PNOL_SYRK_DLAST");
        const bool dlast = !ed || std::atoi(ed) != 0;
        {
            LaunchTimer tm(ctx, "syrk");
#define PNOL_RED(SB, SC, DL)                                                                                          \
    hipExtLaunchKernelGGL((k_syrk_red<SB, SC, DL>), dim3(nsyrk + nred), dim3(512), 0, ctx->stream, tm.start(), tm.stop(), 0, \
                          JT, (long)ldjt, n, m, split, sc.kfirst, sc.kchunk, sc.sub, sc.mS, (long)sc.mS, (double*)part,   \
                          nsyrk, (int*)tcnt, ntiles, n, lambda, cr.w.P, cr.w.ldp, (const double*)jp, rhs, cr.w.bv,       \
                          cr.dinfo)
            if (sc.sub == 2) {
                if (dlast) {
                    if (sc1) PNOL_RED(2, true, true); else PNOL_RED(2, false, true);
                } else {
                    if (sc1) PNOL_RED(2, true, false); else PNOL_RED(2, false, false);
                }
            } else {
                if (sc1) PNOL_RED(0, true, false); else PNOL_RED(0, false, false);
            }
#undef PNOL_RED
        }
        PNOL_CHECK(launch_check());
        ScopedTimer tm(ctx, "solve");
        PNOL_CHECK(launch_chol_preloaded_run(ctx, ctx->stream, cr, sigma, x, xnext));
        ctx->lm_trip_tiles = {1, m, n, 1};
        return PNOL_OK;
    }
    syrk_partials(ctx, ctx->stream, false, JT, ldjt, sc.mS, n, m, sc, 0, kS, 0, ntiles, (double*)part,
                  syrk_t64(false));
    PNOL_CHECK(launch_check());
    if (!tasks) {
        {   // A (Marquardt diagonal, mirror) straight into the padded matrix, rhs into rhs and b
            ScopedTimer tm(ctx, "syrk_reduce");
            launch_reduce(dim3(kTile / 32, ntiles + 1), dim3(256), 0, ctx->stream, (const double*)part, ntiles, sc.sub,
                          n, lambda, cr.w.P, cr.w.ldp, (double*)nullptr, 0, (const double*)jp, rhs, cr.w.bv);
            PNOL_CHECK(launch_check());
        }
        ScopedTimer tm(ctx, "solve");
        PNOL_CHECK(launch_chol_preloaded_run(ctx, ctx->stream, cr, sigma, x, xnext));
    } else {
        ScopedTimer tm(ctx, "solve");
        PNOL_CHECK(launch_chol_reducing_run(ctx, ctx->stream, cr, (const double*)part, sc.sub, (const double*)jp,
                                            lambda, rhs, sigma, x, xnext));
    }
    ctx->lm_trip_tiles = {1, m, n, 1};   // pnol_lm_trip_normal_d may form A from these partials
    return PNOL_OK;
}

// A (lower triangle + mirror, the Marquardt diagonal) from the split-K partials of the last
// launch_fd_normal_solve (the same reduce as launch_jtj, so the same A)
int launch_jtj_from_partials(pnol_ctx* ctx, int m, int n, double lambda, double* A, int lda) {
    if (!A || m <= 0 || n <= PNOL_SEQ_MAX || lda < n) return PNOL_ERR_ARG;
    // the partials must still be the last trip's, of this shape (any other J^T J call since
    // overwrote them)
    const auto& tt = ctx->lm_trip_tiles;
    if (tt.kind != 1 || tt.m != m || tt.n != n || tt.nranks != 1) return PNOL_ERR_ARG;
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    const SliceCfg sc = slice_cfg(m, ntiles);
    void* part = nullptr;
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)ntiles * kS * sc.sub * kTile * kTile, &part));
    launch_reduce(dim3(kTile / 32, ntiles), dim3(256), 0, ctx->stream, (const double*)part, ntiles, sc.sub, n, lambda,
                  A, (long)lda, (double*)nullptr, 0);
    return launch_check();
}

// J^T J with the 128 x 128 tiles split over the communicator's ranks (contiguous ranges of
// tpr = ceil(ntiles / P) tiles), then one allgather of the packed tiles (P * tpr * 128 KB).
// Each tile is summed exactly as on one GPU (same K split, same slice tree): A is bitwise
// independent of P.  n <= PNOL_SEQ_MAX keeps the replicated reference-order kernel.
int launch_jtj_sharded(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda, double* A, int lda,
                       double* jtj_diag) {
    const int P = comm_size(), rank = comm_rank();
    if (P <= 1 || (n <= PNOL_SEQ_MAX && m <= 4096)) return launch_jtj(ctx, JT, ldjt, m, n, lambda, A, lda, jtj_diag);
    if (!JT || !A || m <= 0 || n <= 0 || ldjt < m || lda < n) return PNOL_ERR_ARG;
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    const SliceCfg sc = slice_cfg(m, ntiles);
    const int tpr = (ntiles + P - 1) / P;
    const int t0 = std::min(ntiles, rank * tpr), cnt = std::min(ntiles, t0 + tpr) - t0;
    const size_t E = (size_t)kTile * kTile;
    void *part = nullptr, *packed = nullptr;
    ctx->lm_trip_tiles.kind = 0;   // the trip's tiles are overwritten below
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)std::max(cnt, 1) * kS * sc.sub * E, &part));
    PNOL_CHECK(ws_get(ctx, "syrk_packed", sizeof(double) * (size_t)P * tpr * E, &packed));
    double* mine = (double*)packed + (size_t)rank * tpr * E;
    if (cnt > 0) {
        syrk_partials(ctx, ctx->stream, false, JT, ldjt, sc.mS, n, m, sc, 0, kS, t0, cnt, (double*)part);
        PNOL_CHECK(launch_check());
        hipLaunchKernelGGL(k_syrk_reduce_packed, dim3(8, cnt), dim3(256), 0, ctx->stream, (const double*)part, sc.sub,
                           mine);
        PNOL_CHECK(launch_check());
    }
    PNOL_CHECK(comm_allgather_device(ctx, mine, (double*)packed, (size_t)tpr * E));
    ScopedTimer tm(ctx, "syrk_reduce");
    hipLaunchKernelGGL(k_syrk_unpack, dim3(8, ntiles), dim3(256), 0, ctx->stream, (const double*)packed, ntiles, n,
                       lambda, (long)tpr * E, tpr, A, (long)lda, jtj_diag);
    return launch_check();
}

// The dyadic nodes of the slice tree inside [a, b), in slice order: (first slice, width).
static void dyadic_nodes(int a, int b, std::vector<std::pair<int, int>>& out) {
    out.clear();
    int i = a;
    while (i < b) {
        int w = 1;
        while (i % (2 * w) == 0 && i + 2 * w <= b && 2 * w <= kS) w *= 2;
        out.push_back({i, w});
        i += w;
    }
}

// -J^T F on the m-slices [s0, s0 + nsl): jp[(s - s0) * n + j] = -sum_{k in slice s} JT_jk F_k
// (JT slice s at JT + s * sstride, row stride ldjt), then the slice nodes of that range into
// out[c * n + j] (one node = -J^T F itself when the range is all kLmSlices slices).
static int jtr_gemv(pnol_ctx* ctx, const double* JT, int ldjt, long sstride, int m, int n, int mS, int s0, int nsl,
                    const double* F, hipStream_t stream) {
    if (!F) return PNOL_ERR_ARG;
    void* jp = nullptr;
    PNOL_CHECK(ws_get(ctx, "jtr_part", sizeof(double) * (size_t)kS * n, &jp));
    return launch_gemv_neg_slices(ctx, JT, ldjt, sstride, n, m, mS, s0, nsl, F, (double*)jp, stream);
}

static int jtr_tree(pnol_ctx* ctx, int n, int s0, int nsl, double* out) {
    void* jp = nullptr;
    PNOL_CHECK(ws_get(ctx, "jtr_part", sizeof(double) * (size_t)kS * n, &jp));
    hipLaunchKernelGGL(k_tree_nodes, dim3((n + 255) / 256, 1), dim3(256), 0, ctx->stream, (const double*)jp, 0L,
                       (long)n, 1, s0, s0 + nsl, n, out, (long)n, 0L);
    return launch_check();
}

static int jtr_slices(pnol_ctx* ctx, const double* JT, int ldjt, long sstride, int m, int n, int mS, int s0, int nsl,
                      const double* F, double* out) {
    PNOL_CHECK(jtr_gemv(ctx, JT, ldjt, sstride, m, n, mS, s0, nsl, F));
    return jtr_tree(ctx, n, s0, nsl, out);
}

int launch_jtr(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, const double* F, double* rhs) {
    if (n <= PNOL_SEQ_MAX && m <= 4096) return launch_gemv_neg_seq(ctx, JT, ldjt, n, m, F, rhs);
    if (!JT || !F || !rhs || m <= 0 || n <= 0 || ldjt < m) return PNOL_ERR_ARG;
    const int mS = lm_slice_rows(m);
    return jtr_slices(ctx, JT, ldjt, mS, m, n, mS, 0, kS, F, rhs);
}

// LevMarqMPI normal equations on the m-sliced Jacobian (layout of pnol_lm_sliced_layout):
// rank r holds every FD column of its m-slices [s0, s1) (lm_rank_slices).
//   1. partial tiles of J^T J over its slices (all tiles), -J^T F over its slices;
//   2. its slice-tree nodes of every tile; each tile's nodes go to the tile's owner (contiguous
//      tile ranges of tpr tiles) -- one group of point-to-point sends (a reduce-scatter in the
//      tree's order);
//   3. the owner merges the nodes of its tiles; one allgather of (owned tiles + this rank's
//      -J^T F nodes); every rank unpacks A and merges -J^T F.
// Bitwise equal to launch_jtj + launch_jtr on the row-major J^T for every P <= kLmSlices.
// where launch_lm_normal left the summed tiles when asked not to unpack them (A == nullptr)
struct LmTiles {
    bool partials = false;   // one rank: the split-K partials ("syrk_part") and -J^T F partials ("jtr_part")
    const double* part = nullptr;
    const double* jp = nullptr;
    int sub = 0, split = 0;
    const double* packed = nullptr;   // several ranks: the allgathered tiles
    long slot = 0;
    int tpr = 1;
};

static int lm_normal_core(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F, double* A,
                          int lda, double* rhs, double* jtj_diag, LmTiles* out) {
    if (!JTs || !F || !rhs || m <= 0 || n <= 0 || (A && lda < n) || (!A && !out)) return PNOL_ERR_ARG;
    if (n <= PNOL_SEQ_MAX && m <= 4096) return PNOL_ERR_UNSUPPORTED;   // reference-order kernels: row-major J^T
    const int P = comm_size(), me = comm_rank();
    if (P > kS) return PNOL_ERR_UNSUPPORTED;
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    const SliceCfg sc = slice_cfg(m, ntiles);
    const long sstr = (long)n * sc.mS;
    const long E = (long)kTile * kTile;
    int s0, s1;
    lm_rank_slices(P, me, &s0, &s1);
    const int nsl = s1 - s0;
    void* part = nullptr;
    ctx->lm_trip_tiles.kind = 0;   // the trip's tiles are overwritten below
    PNOL_CHECK(ws_get(ctx, "syrk_part", sizeof(double) * (size_t)ntiles * std::max(nsl, 1) * sc.sub * E, &part));
    const bool t64 = syrk_t64(true);
    if (nsl > 0) {
        syrk_partials(ctx, ctx->stream, false, JTs, sc.mS, sstr, n, m, sc, s0, nsl, 0, ntiles, (double*)part, t64);
        PNOL_CHECK(launch_check());
        PNOL_CHECK(jtr_gemv(ctx, JTs, sc.mS, sstr, m, n, sc.mS, s0, nsl, F));
    }
    if (P == 1) {
        // the -J^T F tree rides in the reduce launch
        void* jp = nullptr;
        PNOL_CHECK(ws_get(ctx, "jtr_part", sizeof(double) * (size_t)kS * n, &jp));
        if (!A) {   // the reducing Cholesky sums the partials itself
            out->partials = true;
            out->part = (const double*)part;
            out->jp = (const double*)jp;
            out->sub = sc.sub;
            out->split = kS * sc.sub;
            return PNOL_OK;
        }
        {
            ScopedTimer tm(ctx, "syrk_reduce");
            launch_reduce(dim3(kTile / 32, ntiles + 1), dim3(256), 0, ctx->stream, (const double*)part, ntiles,
                          sc.sub, n, lambda, A, (long)lda, jtj_diag, 0, (const double*)jp, rhs);
        }
        return launch_check();
    }
    // the global node list: rank q's nodes in slice order, ranks in order
    std::vector<std::pair<int, int>> nodes;
    std::vector<int> owner, first(P + 1, 0);
    for (int q = 0; q < P; ++q) {
        int a, b;
        lm_rank_slices(P, q, &a, &b);
        std::vector<std::pair<int, int>> nq;
        dyadic_nodes(a, b, nq);
        first[q] = (int)nodes.size();
        for (auto& nd : nq) {
            nodes.push_back(nd);
            owner.push_back(q);
        }
    }
    first[P] = (int)nodes.size();
    const int NC = (int)nodes.size(), nn = first[me + 1] - first[me];
    constexpr int kMaxNodes = 4;   // dyadic nodes of a slice range of an 8-leaf tree
    const int tpr = (ntiles + P - 1) / P;
    auto t0_of = [&](int d) { return std::min(ntiles, d * tpr); };
    auto cnt_of = [&](int d) { return std::min(ntiles, t0_of(d) + tpr) - t0_of(d); };
    const long slot = (long)tpr * E + (long)kMaxNodes * n;
    void *nodebuf = nullptr, *recv = nullptr, *packed = nullptr;
    PNOL_CHECK(ws_get(ctx, "lm_nodes", sizeof(double) * (size_t)std::max(nn, 1) * ntiles * E, &nodebuf));
    PNOL_CHECK(ws_get(ctx, "lm_nodes_recv", sizeof(double) * (size_t)NC * tpr * E, &recv));
    PNOL_CHECK(ws_get(ctx, "lm_packed", sizeof(double) * (size_t)P * slot, &packed));
    double* mine = (double*)packed + (size_t)me * slot;
    if (nsl > 0) {
        ScopedTimer tm(ctx, "syrk_reduce");
        hipLaunchKernelGGL(k_tree_nodes, dim3(kTile * kTile / 256 / 4, ntiles), dim3(256), 0, ctx->stream,
                           (const double*)part, (long)nsl * sc.sub * E, E, sc.sub, s0, s1, (int)E,
                           (double*)nodebuf, (long)ntiles * E, E);
    }
    PNOL_CHECK(launch_check());
    // -J^T F nodes of my slices into the tail of my allgather slot
    if (nsl > 0) PNOL_CHECK(jtr_tree(ctx, n, s0, nsl, mine + (long)tpr * E));
    // reduce-scatter in tree order: rank q's nodes of owner d's tiles -> d
    {
        ScopedTimer tm(ctx, "exchange_A");
        PNOL_CHECK(comm_exchange(ctx, (const double*)nodebuf, (double*)recv, [&](int q, int d, std::vector<XBlock>& bl) {
            bl.clear();
            if (cnt_of(d) == 0) return;
            for (int c = first[q]; c < first[q + 1]; ++c)
                bl.push_back({(size_t)((c - first[q]) * (long)ntiles + t0_of(d)) * E, (size_t)c * tpr * E,
                              (size_t)cnt_of(d) * E});
        }));
    }
    if (cnt_of(me) > 0) {
        TreeNodes tn{};
        for (int c = 0; c < NC; ++c) {
            const int lo = nodes[c].first;
            tn.w[lo] = nodes[c].second;
            tn.p[lo] = owner[c] == me ? (const double*)nodebuf + ((long)(c - first[me]) * ntiles + t0_of(me)) * E
                                      : (const double*)recv + (long)c * tpr * E;
        }
        ScopedTimer tm(ctx, "syrk_reduce");
        const long el = (long)cnt_of(me) * E;
        hipLaunchKernelGGL(k_tree_combine, dim3((unsigned)std::min<long>((el + 255) / 256, 4096)), dim3(256), 0,
                           ctx->stream, tn, el, mine);
        PNOL_CHECK(launch_check());
    }
    PNOL_CHECK(comm_allgather_device(ctx, mine, (double*)packed, (size_t)slot));
    {
        ScopedTimer tm(ctx, "syrk_reduce");
        if (A) {
            hipLaunchKernelGGL(k_syrk_unpack, dim3(8, ntiles), dim3(256), 0, ctx->stream, (const double*)packed, ntiles,
                               n, lambda, slot, tpr, A, (long)lda, jtj_diag);
            PNOL_CHECK(launch_check());
        } else {   // the reducing Cholesky reads the tiles itself
            out->packed = (const double*)packed;
            out->slot = slot;
            out->tpr = tpr;
        }
        TreeNodes tr{};
        for (int c = 0; c < NC; ++c) {
            const int lo = nodes[c].first;
            tr.w[lo] = nodes[c].second;
            tr.p[lo] = (const double*)packed + (long)owner[c] * slot + (long)tpr * E + (long)(c - first[owner[c]]) * n;
        }
        hipLaunchKernelGGL(k_tree_combine, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, tr, (long)n, rhs);
    }
    return launch_check();
}

int launch_lm_normal(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F, double* A,
                     int lda, double* rhs, double* jtj_diag) {
    if (!A) return PNOL_ERR_ARG;
    return lm_normal_core(ctx, JTs, m, n, lambda, F, A, lda, rhs, jtj_diag, nullptr);
}

// LevMarqMPI's normal equations and damped solve without forming A: the tiles of
// launch_lm_normal (summed by the slice tree over the ranks and allgathered; one rank: its
// partials) go straight into the persistent Cholesky's matrix by its first tasks -- no unpack
// into A, no copy of A -- then the factorisation, the backward solve and xnext = xbase + sigma.
// rhs = -J^T F as launch_lm_normal's.  Bitwise launch_lm_normal + launch_chol_solve.
int launch_lm_normal_solve(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F, double* rhs,
                           double* sigma, int* dinfo, const double* xbase, double* xnext) {
    if (!sigma || !dinfo || !xnext || n <= PNOL_SEQ_MAX) return PNOL_ERR_ARG;
    CholRed cr;
    PNOL_CHECK(launch_chol_reducing_prep(ctx, n, dinfo, cr));
    LmTiles tl;
    PNOL_CHECK(lm_normal_core(ctx, JTs, m, n, lambda, F, nullptr, 0, rhs, nullptr, &tl));
    PNOL_CHECK(launch_chol_reducing_start(ctx, cr));
    ScopedTimer tm(ctx, "solve");
    if (tl.partials)
        PNOL_CHECK(launch_chol_reducing_run(ctx, ctx->stream, cr, tl.part, tl.sub, tl.jp, lambda, rhs, sigma, xbase,
                                            xnext));
    else
        PNOL_CHECK(launch_chol_reducing_run_packed(ctx, ctx->stream, cr, tl.packed, tl.slot, tl.tpr, rhs, lambda, sigma,
                                                   xbase, xnext));
    // pnol_lm_normal_unpack_mpi_d may form A from these tiles
    ctx->lm_trip_tiles = {tl.partials ? 1 : 2, m, n, comm_size()};
    return PNOL_OK;
}

// A from the tiles the last launch_lm_normal_solve left (the LU fallback; the same A as
// launch_lm_normal's)
int launch_lm_normal_unpack(pnol_ctx* ctx, int m, int n, double lambda, double* A, int lda) {
    if (!A || m <= 0 || n <= PNOL_SEQ_MAX || lda < n) return PNOL_ERR_ARG;
    const int P = comm_size();
    if (P == 1) return launch_jtj_from_partials(ctx, m, n, lambda, A, lda);
    const auto& tt = ctx->lm_trip_tiles;   // the last trip's allgathered tiles, of this shape
    if (tt.kind != 2 || tt.m != m || tt.n != n || tt.nranks != P) return PNOL_ERR_ARG;
    const int nt = (n + kTile - 1) / kTile;
    const int ntiles = nt * (nt + 1) / 2;
    const long E = (long)kTile * kTile;
    const int tpr = (ntiles + P - 1) / P;
    constexpr int kMaxNodes = 4;
    const long slot = (long)tpr * E + (long)kMaxNodes * n;
    void* packed = nullptr;
    PNOL_CHECK(ws_get(ctx, "lm_packed", sizeof(double) * (size_t)P * slot, &packed));
    hipLaunchKernelGGL(k_syrk_unpack, dim3(8, ntiles), dim3(256), 0, ctx->stream, (const double*)packed, ntiles, n,
                       lambda, slot, tpr, A, (long)lda, (double*)nullptr);
    return launch_check();
}

}  // namespace pnol
