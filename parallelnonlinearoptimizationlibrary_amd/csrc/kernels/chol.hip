// chol.hip -- the damped LM solve as a lookahead tile Cholesky with explicit diagonal-tile
// inverses (pnol_solve_d method 4, the default for n > PNOL_SEQ_MAX).  Replaces
// luSolve(A, rhs, sigma), LevenbergMarquardt.cpp:83 / LevenbergMarquardtMPI.cpp:88.
//
// A (n x n, SPD) is copied into a zero-padded T*64 x T*64 workspace P (identity on the padded
// diagonal) and factored by 64 x 64 tiles, one launch per panel step k = -1 .. T-2:
//   diag WG      tile (k+1,k+1): L = A_{k+1,k} W_k^T and A_{k+1,k+1} -= L L^T on fp64 MFMA,
//                then the 64-step Cholesky of the tile (wave 0, rows in registers) with its
//                inverse W_{k+1} = L_{k+1,k+1}^{-1} formed one column step behind (wave 1)
//   panel WGs    L_ik = A_ik W_k^T (TRSM as an MFMA product) into a separate factor matrix Lm
//                (the diagonal WG of the same launch still reads A_{k+1,k} from P), published
//                by a per-row flag;
//                they also carry the forward substitution: z_k = W_k b_k, b_i -= L_ik z_k
//   update WGs   A_ij -= L_ik L_jk^T (fp64 MFMA) once rows i and j of the panel are flagged
// The diagonal workgroup recomputes its own L_{k+1,k} instead of waiting for it, so the critical
// path of a step is one workgroup's MFMA + factor + inverse; the trailing update runs beside it.
// A final launch solves L^T x = z by block rows from the bottom up, chained by ready flags, each
// diagonal block applied as the product W_w^T v.
// A non-positive (or NaN) pivot sets *info; the host then solves with Gaussian elimination on
// the untouched A (solve.hip).  Every wait is spin-capped: a wait past the cap sets *info to
// kCholTimeout and the host relaunches the same factorisation (bitwise the same result), never
// the LU -- a timeout is a scheduling event, not a property of A.
#include "../pnol_internal.hpp"
#include "../pnol_comm.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace pnol {
namespace {

constexpr int NB = 64;
constexpr int kPad = 18;             // LDS row stride of a 64 x 16 K-substage (doubles)
constexpr int kSub = NB * kPad;      // doubles per substage
constexpr int kStage = 4 * kSub;     // one 64 x 64 tile as four substages
constexpr int kSpin = 1 << 24;       // polls (each >= one s_sleep(1) + one L2 round trip)
// a wait that ran past kSpin: a scheduling event, never a numerical result -- the first failure
// recorded sticks (atomicCAS), and the host relaunches the same factorisation (launch_solve)
constexpr int kInfoTimeout = kCholTimeout;
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// 1/sqrt(x) to full double precision: the hardware estimate (~2^-24 relative,
// tools/microbench/rsq_acc.hip) and one third-order step, r (1 + e/2 + 3 e^2 / 8) with
// e = 1 - x r^2 (error ~e^3 ~ 2^-72): a 5-deep dependent chain instead of 6 for two Newton steps
__device__ __forceinline__ double rsqrt_nr(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    const double e = fma(-x, r * r, 1.0);
    const double p = fma(e, 0.375, 0.5);
    return fma(r * e, p, r);
}

// SC1: the persistent form's hand-offs between workgroups use sc1 (relaxed agent-scope atomic)
// loads and stores for every handed-off byte instead of release / acquire fences
// (MI355X_MICROARCH.md "Valid forms", table row 1: one workgroup per CU, every storing wave's
// vmcnt(0) wait before the workgroup barrier and the one sc1 flag store).
template <bool SC1>
__device__ __forceinline__ double ldg(const double* p) {
    if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool SC1>
__device__ __forceinline__ void stg(double* p, double v) {
    if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
// 16-byte sc1 load at byte offset `off` from a wave-uniform base (buffer_load_dwordx4 ... sc1;
// 0x00020000: the gfx9 raw-buffer descriptor word 3, 32-bit data format)
typedef int v4i_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double2 ld16_sc1(const double* base, unsigned off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    const v4i_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
    return __builtin_bit_cast(double2, v);
}

// 16-byte sc1 store at byte offset `off` from a wave-uniform base (buffer_store_dwordx4 ... sc1)
//
// Atomicity assumption of the backward solve's granules (x, epoch): one lane's dwordx4 store
// and load at a 16-byte-aligned address lie inside one 128-byte L2 line and travel as one
// request, so a reader sees either the old or the new 16 bytes, never a mix.  The AMDGPU memory
// model does not promise this for dwordx4; it is what MI355X_MICROARCH.md's "Valid forms" row 2
// relies on.  Every granule offset is a multiple of 16 bytes from a hipMalloc base (256-byte
// aligned; asserted on the host, launch_chol_bwd), and tests/test_gpu_kernels.py
// (test_cholesky_bwd_granules_equal_flag_form) compares many solves with the flag form
// (PNOL_BWD_GRANULE=0), which stays selectable as the fallback.
static_assert(sizeof(double2) == 16 && alignof(double2) == 16, "granule = one aligned 16-byte access");
__device__ __forceinline__ void st16_sc1(double* base, unsigned off, double2 v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, v), r, off, 0, 16);
}

// Stage the 64 x 64 tile at (r0, c0) of P into four 64 x 16 substages (row stride kPad):
// thread t owns row t >> 2 and the 16 columns of substage t & 3 (eight 16-byte loads; SC1:
// sixteen 8-byte sc1 loads).
template <bool SC1 = false>
__device__ __forceinline__ void stage_tile(double* __restrict__ dst, const double* __restrict__ P, long ldp, int r0,
                                           int c0) {
    const int t = threadIdx.x, row = t >> 2, sub = t & 3;
    double2 v[8];
    if constexpr (SC1) {
        const double* base = P + (long)r0 * ldp + c0;   // wave-uniform
        const unsigned off = (unsigned)((row * ldp + sub * 16) * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = ld16_sc1(base, off + 16 * q);
    } else {
        const double2* src = reinterpret_cast<const double2*>(P + (long)(r0 + row) * ldp + c0 + sub * 16);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = src[q];
    }
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

template <bool SC1 = false>
__device__ __forceinline__ void acc_load(d4 (&acc)[2][2], const double* __restrict__ P, long ldp, int r0, int c0,
                                         int wr, int wc, int lane) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                acc[mi][ni][r] = ldg<SC1>(P + (long)(r0 + acc_row(wr, mi, lane, r)) * ldp + c0 + acc_col(wc, ni, lane));
}

template <bool SC1 = false>
__device__ __forceinline__ void acc_store(const d4 (&acc)[2][2], double* __restrict__ P, long ldp, int r0, int c0,
                                          int wr, int wc, int lane) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                stg<SC1>(P + (long)(r0 + acc_row(wr, mi, lane, r)) * ldp + c0 + acc_col(wc, ni, lane), acc[mi][ni][r]);
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
                atomicCAS(info, 0, kInfoTimeout);
                return false;
            }
        }
    }
    return true;
}

// Every *f[q] >= tg[q]: all N words are loaded in each round (one memory round trip for the set
// instead of one per word when they are already there); the same cap and info checks.
template <int N>
__device__ __forceinline__ bool spin_all(const int* const (&f)[N], const int (&tg)[N], int* info) {
    int it = 0;
    for (;;) {
        int v[N];
#pragma unroll
        for (int q = 0; q < N; ++q) v[q] = __hip_atomic_load(f[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int q = 0; q < N; ++q) ok = ok && v[q] >= tg[q];
        if (ok) return true;
        __builtin_amdgcn_s_sleep(1);
        if ((++it & 63) == 0) {
            if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
            if (it > kSpin) {
                atomicCAS(info, 0, kInfoTimeout);
                return false;
            }
        }
    }
}

// ---- the diagonal tile: LDS words and copies ------------------------------------------------
constexpr int kHalf = 32;
constexpr int kS = kHalf + 1;   // row stride of the LDS copies of the tile halves

// LDS word store / spin-wait as inline asm: opaque to the scheduler, so the unrolled
// register-resident chains around them stay one basic block (a C++ loop or an atomic here
// splits them and the register rows spill).  One wave's LDS operations are processed in order.
__device__ __forceinline__ void lds_signal(int* cnt, int v) {
    __attribute__((address_space(3))) int* p = (__attribute__((address_space(3))) int*)cnt;
    asm volatile("ds_write_b32 %0, %1" ::"v"(p), "v"(v) : "memory");
}
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

// 16 x 16 block of C = sum_k A(i, k) B(j, k) over K (v_mfma_f64_16x16x4_f64), accumulated into acc.
template <int K, class FA, class FB>
__device__ __forceinline__ d4 mfma_blk(d4 acc, FA fa, FB fb, int lane) {
    const int i = lane & 15, kq = lane >> 4;
    double a[K / 4], b[K / 4];   // all fragments requested first: one LDS latency, not K / 4
#pragma unroll
    for (int q = 0; q < K / 4; ++q) {
        a[q] = fa(i, 4 * q + kq);
        b[q] = fb(i, 4 * q + kq);
    }
    // two independent accumulator chains (even / odd K steps) halve the dependent MFMA latency
    d4 acc2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < K / 4; q += 2) {
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[q], acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q + 1], b[q + 1], acc2, 0, 0, 0);
    }
    return acc + acc2;
}

struct DiagLds {
    double* Sl;    // 64 x 32 left half of the tile, stride kS
    double* S22;   // 32 x 32 bottom-right quarter, stride kS
};

__device__ __forceinline__ DiagLds diag_lds(double* smem) {
    DiagLds L;
    L.Sl = smem;
    L.S22 = smem + 64 * kS;
    return L;
}

// the tile entry (row, col) of the lower triangle into the split LDS copy (upper-right dropped)
__device__ __forceinline__ void diag_put(const DiagLds& L, int row, int col, double v) {
    if (col < kHalf) L.Sl[row * kS + col] = v;
    else if (row >= kHalf) L.S22[(row - kHalf) * kS + col - kHalf] = v;
}

struct NoEarly {
    __device__ void operator()(int, int) const {}
};

// ---- the diagonal tile: Cholesky + inverse in 16-wide micro-panels -------------------------
// Factor the tile held in L.Sl / L.S22 and write W_d = L_dd^{-1} (64 x 64 row-major) to Wd.
// (A 32-wide two-panel form, whose chain wave issued every rank-1 update of its panel itself,
// ran ~290 cycles per pivot, 23k cycles per tile; removed in round 4.)  The tile is four 64 x 16
// micro-panels:
//   wave 0      the pivot chain of micro-panel p (rows 16p .. 63, one row per lane, 16 entries in
//               registers): per pivot at most 14 rank-1 fmas, software-pipelined as panel_step;
//               column c and 1 / L_cc go to LDS, every 2 columns a counter in LDS
//   waves 2, 3  the trailing update by micro-panels 0 and 1 as fp64 MFMA: each owns some lower
//               16 x 16 blocks (ib, q), q >= 1, kept in registers, and applies -L_{ib,p} L_{q,p}^T
//               four columns at a time as wave 0 publishes them (one v_mfma_f64_16x16x4_f64 per
//               block and group); the blocks of micro-panel p+1 go to LDS when panel p is
//               complete.  Micro-panel 2's one block update (3,3) is wave 0's, so waves 2 / 3 are
//               free for the chain's look-ahead (EARLY) from the end of micro-panel 1
//   wave 1      V_p = L_pp^{-1} (16 x 16, lane = column) one column pair behind the chain, then
//               the off-diagonal blocks of W = L^{-1} by block rows, W_ij = -V_i X_ij with
//               X_ij = sum_{k=j}^{i-1} L_ik W_kj accumulated as soon as its operands exist, so only
//               W_3j = -V_3 X_3j (three products, waves 0 and 1) follow the last pivot.
// Every accumulator receives its MFMAs in a fixed order, so W is deterministic; methods 4 and 5
// both use this factor.
// LDS (doubles, from L.Sl): the tile (Sl / S22, 3168), the panels' columns (2560), the W blocks
// (10 x 288), a 64-double discard row; the X hand-off blocks reuse Sl rows 0 .. 26, dead once
// micro-panel 1 is in registers.  Words: cnt[0] final columns, cnt[1] W rows 0..31 done,
// cnt[2] / cnt[3] waves 2 / 3 have stored micro-panel cnt's blocks, cnt[4] V_3 and X_3j in LDS.
constexpr int kMW = 16;            // micro-panel width
constexpr int kBP = 18;            // row stride of a 16 x 16 block in LDS (conflict-free fragments)
constexpr int kBlk = 16 * kBP;     // doubles per block
__host__ __device__ constexpr int lblk(int ib, int jb) { return ib * (ib + 1) / 2 + jb; }
__host__ __device__ constexpr int mp_ld(int p) { return NB - kMW * p; }                 // rows of micro-panel p
__host__ __device__ constexpr int mp_base(int p) { return 1024 * p - 128 * p * (p - 1); }   // sum of kMW * mp_ld(q), q < p

struct MpLds {
    double* Sl;     // the tile, as diag_put leaves it
    double* S22;
    double* Lc;     // micro-panel p's columns at mp_base(p), column-major, rows 16p .. 63 (stride mp_ld(p))
    double* Wb;     // the 10 lower blocks of W, block (ib, jb) at lblk(ib, jb) * kBlk, row stride kBP
    double* Xs;     // 3 hand-off blocks (row stride kBP), in Sl rows 0 .. 26
    double* disc;   // one block (kBlk doubles): stores of lanes outside a micro-panel or a block
};
__device__ __forceinline__ MpLds mp_lds(const DiagLds& L) {
    MpLds M;
    M.Sl = L.Sl;
    M.S22 = L.S22;
    M.Lc = L.S22 + kHalf * kS;
    M.Wb = M.Lc + mp_base(4);
    M.disc = M.Wb + 10 * kBlk;
    M.Xs = L.Sl;
    return M;
}
static_assert(64 * kS + kHalf * kS + mp_base(4) + 11 * kBlk <= 2 * kStage, "micro-panel factor fits the staging LDS");
static_assert(3 * kBlk <= kHalf * kS, "X hand-off blocks fit Sl rows 0..31");

// the W_d rows 0..31 operand of EarlyNext: element (r, c), c <= r block-wise
__device__ __forceinline__ double w11_at(const double* W11, int r, int c) {
    return W11[lblk(r >> 4, c >> 4) * kBlk + (r & 15) * kBP + (c & 15)];
}
__device__ __forceinline__ const double* diag_w11(const DiagLds& L) { return mp_lds(L).Wb; }

// tile entry (row, col), lower triangle, in the diag_put layout
__device__ __forceinline__ double* mp_s(const MpLds& M, int row, int col) {
    return col < kHalf ? M.Sl + row * kS + col : M.S22 + (row - kHalf) * kS + (col - kHalf);
}

// Column J's values as wave 0 reads them back for the deferred part of its rank-1 update:
// entries k >= J + 4 (in pairs from the even K0).
template <int J>
struct ColBuf16 {
    static constexpr int K0 = (J + 4) & ~1, NR = K0 < kMW ? (kMW - K0) / 2 : 0;
    double2 v[NR > 0 ? NR : 1];
};

// column c-2's deferred update (entries k >= J + 2), the pairs q with q % 4 == G
template <int J, int G>
__device__ __forceinline__ void mp_def(double (&a)[kMW], double lp2, const ColBuf16<J - 2>& cp2) {
    if constexpr (J >= 2) {
#pragma unroll
        for (int q = G; q < ColBuf16<J - 2>::NR; q += 4) {
            const int k = ColBuf16<J - 2>::K0 + 2 * q;
            if (k >= J + 2) {
                a[k] = fma(-lp2, cp2.v[q].x, a[k]);
                asm volatile("" : "+v"(a[k]));
            }
            if (k + 1 >= J + 2) {
                a[k + 1] = fma(-lp2, cp2.v[q].y, a[k + 1]);
                asm volatile("" : "+v"(a[k + 1]));
            }
        }
    }
}

// a value defined here: volatile asm statements keep their order, so the IR passes cannot sink
// the computation past this point (sched_barrier alone orders only the machine scheduler)
#define PNOL_PIN(x) asm volatile("" : "+v"(x))
#define PNOL_SB __builtin_amdgcn_sched_barrier(0)

// One pivot of micro-panel P (wave 0): column c = 16P + J from its reciprocal square root r.
// The rank-1 update of column c is split: entries J+1 .. J+3 at once, with the column's values
// from their lanes (v_readlane; entry J+1 is the next pivot, formed in its own lane first), and
// entries k >= J+4 two steps later, with the values read back from the column's LDS copy
// (issued here, consumed at step J+2, so the LDS round trip is off the chain).  Entry k still
// receives every column's update before it is used (columns <= k-4 by step k-2); the order of
// the updates on one entry is fixed by the code, so W is deterministic.
// Issue order is pinned by scheduling barriers: each dependent op of the pivot chain (~12
// cycles of latency each, tools/microbench/piv_chain.hip: 124 cycles per pivot for the bare
// chain) is followed by a group of independent updates that fill its latency; left to itself
// the scheduler issues the chain ops back to back (~280 cycles per pivot).
// Lp and sb alias (a panel lane's sb points into Lp, and the read-back of column J follows its
// store), so neither is __restrict__.
template <int J, int P, bool STAMP>
__device__ __forceinline__ void mp_step(double (&a)[kMW], double r, double lp1, const ColBuf16<J - 1>& cp1, double lp2,
                                        const ColBuf16<J - 2>& cp2, double* Lp, double* sb,
                                        int ss, double* __restrict__ rinv, int* cnt, int lane, bool& bad, long long* st) {
    constexpr int c = kMW * P + J, LD = mp_ld(P);
    if constexpr (STAMP && (J & 7) == 0) st[2 * P + (J >> 3)] = __builtin_amdgcn_s_memtime();
    const double l = a[J] * r;
    a[J] = l;
    double rn = 0.0;
    if constexpr (J + 1 < kMW) {
        const double piv = readlane_d(fma(-l, l, a[J + 1]), c + 1);   // lane c+1's own update
        double r0 = __builtin_amdgcn_rsq(piv);
        PNOL_PIN(r0);
        PNOL_SB;
        a[J + 1] = fma(-l, readlane_d(l, c + 1), a[J + 1]);
        PNOL_PIN(a[J + 1]);
        mp_def<J, 0>(a, lp2, cp2);
        PNOL_SB;
        double r2 = r0 * r0;
        PNOL_PIN(r2);
        PNOL_SB;
        if constexpr (J + 2 < kMW) {
            a[J + 2] = fma(-l, readlane_d(l, c + 2), a[J + 2]);
            PNOL_PIN(a[J + 2]);
        }
        mp_def<J, 1>(a, lp2, cp2);
        PNOL_SB;
        double e = fma(-piv, r2, 1.0);
        PNOL_PIN(e);
        PNOL_SB;
        if constexpr (J + 3 < kMW) {
            a[J + 3] = fma(-l, readlane_d(l, c + 3), a[J + 3]);
            PNOL_PIN(a[J + 3]);
        }
        mp_def<J, 2>(a, lp2, cp2);
        PNOL_SB;
        double pp = fma(e, 0.375, 0.5), re = r0 * e;
        PNOL_PIN(pp);
        PNOL_PIN(re);
        PNOL_SB;
        mp_def<J, 3>(a, lp2, cp2);
        bad |= !(piv > 0.0);
        PNOL_SB;
        rn = fma(re, pp, r0);   // = rsqrt_nr(piv), the same operations
        PNOL_SB;
    }
    // this lane's value of column c: the panel's rows to the column copy, the V_P lanes to row J of
    // W block (P, P), the rest to the discard block (per-lane base and stride: no select here)
    sb[J * ss] = l;
    rinv[c] = r;   // every lane stores the same value: no divergent branch in the chain
    if constexpr ((J & 1) == 1) lds_signal(cnt, c + 1);
    ColBuf16<J> cv;
    if constexpr (ColBuf16<J>::NR > 0) {
#pragma unroll
        for (int q = 0; q < ColBuf16<J>::NR; ++q)
            cv.v[q] = *reinterpret_cast<const double2*>(Lp + J * LD + ColBuf16<J>::K0 + 2 * q);
    }
    asm volatile("" ::: "memory");   // keep the next steps' LDS reads from being hoisted here
    PNOL_SB;
    if constexpr (J + 1 < kMW)
        mp_step<J + 1, P, STAMP>(a, rn, l, cv, lp1, cp1, Lp, sb, ss, rinv, cnt, lane, bad, st);
}

template <int P, bool STAMP>
__device__ __forceinline__ void mp_panel(const MpLds& M, double* __restrict__ rinv, int* cnt, int lane, int d,
                                         int* info, long long* st) {
    if constexpr (P == 1 || P == 2) {   // the owners' blocks of this micro-panel are in LDS
        wait_lds_ge(cnt + 2, P);
        wait_lds_ge(cnt + 3, P);
    } else if constexpr (P == 3) {
        // block (3,3) as wave 2 left it (micro-panels 0, 1 applied); micro-panel 2's update here,
        // from the columns this wave has just written: waves 2 and 3 are free after micro-panel 1
        // for the chain's look-ahead
        wait_lds_ge(cnt + 2, 2);
        d4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = *mp_s(M, 48 + (lane >> 4) + 4 * r, 48 + (lane & 15));
        const double* Lp = M.Lc + mp_base(2);
        acc = mfma_blk<16>(acc, [&](int i, int k) { return -Lp[k * mp_ld(2) + 16 + i]; },
                           [&](int j, int k) { return Lp[k * mp_ld(2) + 16 + j]; }, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r) *mp_s(M, 48 + (lane >> 4) + 4 * r, 48 + (lane & 15)) = acc[r];
    }
    // Lanes 0..15 of micro-panels 1..3 (rows already factored) compute V_P = L_PP^{-1} in the same
    // instruction stream: lane j starts from the unit column e_j, and each pivot's l = a[J] r and
    // rank-1 update a[k] -= l L_kJ are then exactly the forward substitution L_PP y = e_j
    // (y_J = b_J r_J, b_k -= L_kJ y_J), with the column values L_kJ the panel's lanes use, so
    // row J of V_P is these lanes' l of step J.  (Wave 1 forms V_0; it used to form every V_p one
    // column pair behind the chain, which left V_3 ~1.9k cycles after the last pivot.)
    double a[kMW];
    const int row = max(lane, kMW * P);
    const bool vlane = P > 0 && lane < kMW;
#pragma unroll
    for (int k = 0; k < kMW; ++k)
        a[k] = lane >= kMW * P ? *mp_s(M, row, kMW * P + k) : (vlane && k == lane ? 1.0 : 0.0);
    const double piv = readlane_d(a[0], kMW * P);
    bool bad = !(piv > 0.0);
    const ColBuf16<-1> n1{};
    const ColBuf16<-2> n2{};
    double* const Lp = M.Lc + mp_base(P);
    double* const sb = (P == 0 || lane >= kMW * P) ? Lp + (lane - kMW * P)
                                                   : (vlane ? M.Wb + lblk(P, P) * kBlk + lane : M.disc + lane);
    const int ss = (P == 0 || lane >= kMW * P) ? mp_ld(P) : (vlane ? kBP : 0);
    mp_step<0, P, STAMP>(a, rsqrt_nr(piv), 0.0, n1, 0.0, n2, Lp, sb, ss, rinv, cnt, lane, bad, st);
    if (bad && lane == 0) atomicCAS(info, 0, d * NB + kMW * P + 1);
}

// 16 x 16 block (row stride kBP) <-> MFMA accumulator layout
__device__ __forceinline__ void blk_put(double* __restrict__ B, const d4& acc, int lane) {
#pragma unroll
    for (int r = 0; r < 4; ++r) B[((lane >> 4) + 4 * r) * kBP + (lane & 15)] = acc[r];
}

// The trailing update by micro-panels 0 and 1, owned by wave OW (2 or 3), in two phases:
//   A  the block column 1 -- wave 2: (1,1) (3,1); wave 3: (2,1) -- micro-panel 0 applied four
//      columns at a time as wave 0 publishes them, then stored to LDS (cnt[OW] = 1: micro-panel
//      1 may start);
//   B  (3,3) (wave 2), (3,2) (2,2) (wave 3): micro-panel 0 (final by then), then micro-panel 1
//      as it is published, stored (cnt[OW] = 2); block (3,3)'s micro-panel 2 update is wave 0's
//      (mp_panel<3>).
// Lsrc / kb0 (the persistent chain, Lsrc non-null): the prepare left these blocks without their
// K blocks kb0 .. 3 of -L L^T (deferred, so the chain's first micro-panel starts after only the
// block column 0 products); each block takes them first, from L in the substage layout at Lsrc
// -- the same MFMAs in the same order as diag_prepare / late_prepare, so the blocks and W are
// bitwise unchanged.  kb0 = 4: nothing deferred.
template <int OW>
__device__ __forceinline__ void mp_owner(const MpLds& M, int* cnt, int lane, const double* __restrict__ Lsrc, int kb0) {
    const int frow = lane & 15, fk = lane >> 4;
    // block (ib, q): its LDS value, then the deferred K blocks of -L L^T
    auto lld = [&](d4& acc, int ib, int q) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = *mp_s(M, 16 * ib + (lane >> 4) + 4 * r, 16 * q + (lane & 15));
        if (Lsrc && kb0 < 4) {
            double fa[4][4], fb[4][4];
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
                if (kb >= kb0)
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) {
                        fa[kb][kk] = -Lsrc[kb * kSub + (ib * 16 + frow) * kPad + kk * 4 + fk];
                        fb[kb][kk] = Lsrc[kb * kSub + (q * 16 + frow) * kPad + kk * 4 + fk];
                    }
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
                if (kb >= kb0)
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
                        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[kb][kk], fb[kb][kk], acc, 0, 0, 0);
        }
    };
    // group g (columns 4g .. 4g+3) of micro-panel P applied to block (ib, q)
    auto upd = [&](d4& acc, int ib, int q, auto pc, int g) {
        constexpr int P = decltype(pc)::value, LD = mp_ld(P);
        const double* Lp = M.Lc + mp_base(P);
        const double x = -Lp[(4 * g + fk) * LD + 16 * ib - kMW * P + frow];
        const double y = Lp[(4 * g + fk) * LD + 16 * q - kMW * P + frow];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
    };
    auto put = [&](const d4& acc, int ib, int q) {
#pragma unroll
        for (int r = 0; r < 4; ++r) *mp_s(M, 16 * ib + (lane >> 4) + 4 * r, 16 * q + (lane & 15)) = acc[r];
    };
    constexpr int NA = OW == 2 ? 2 : 1;
    const int ia[2] = {OW == 2 ? 1 : 2, 3};
    d4 a[NA];
#pragma unroll
    for (int b = 0; b < NA; ++b) lld(a[b], ia[b], 1);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        wait_lds_ge(cnt, 4 * g + 4);
#pragma unroll
        for (int b = 0; b < NA; ++b) upd(a[b], ia[b], 1, std::integral_constant<int, 0>(), g);
    }
#pragma unroll
    for (int b = 0; b < NA; ++b) put(a[b], ia[b], 1);
    lds_signal(cnt + OW, 1);   // in order after the block stores (one wave's LDS ops are ordered)
    constexpr int NB2 = OW == 2 ? 1 : 2;
    const int ibb[2] = {3, OW == 2 ? 3 : 2}, qb[2] = {OW == 2 ? 3 : 2, 2};
    d4 c[NB2];
#pragma unroll
    for (int b = 0; b < NB2; ++b) lld(c[b], ibb[b], qb[b]);
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int b = 0; b < NB2; ++b) upd(c[b], ibb[b], qb[b], std::integral_constant<int, 0>(), g);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        wait_lds_ge(cnt, kMW + 4 * g + 4);
#pragma unroll
        for (int b = 0; b < NB2; ++b) upd(c[b], ibb[b], qb[b], std::integral_constant<int, 1>(), g);
    }
#pragma unroll
    for (int b = 0; b < NB2; ++b) put(c[b], ibb[b], qb[b]);
    lds_signal(cnt + OW, 2);
}

// V_P = L_PP^{-1} (wave 1, lane j = column j; lanes >= 16 compute zeros) into W block (P, P)
template <int P>
__device__ __forceinline__ void mp_inverse(const MpLds& M, const double* __restrict__ rinv, const int* cnt, int lane) {
    constexpr int LD = mp_ld(P);
    const double* Lp = M.Lc + mp_base(P);   // row 16P + k of column 16P + J at Lp[J * LD + k]
    double y[kMW];
#pragma unroll
    for (int k = 0; k < kMW; ++k) y[k] = (k == lane) ? 1.0 : 0.0;
    auto step = [&](auto jc) {
        constexpr int J = decltype(jc)::value, K0 = J, NR = (kMW - K0) / 2;
        wait_lds_ge(cnt, kMW * P + J + 2);
        double2 c0[NR], c1[NR];
#pragma unroll
        for (int q = 0; q < NR; ++q) {
            c0[q] = *reinterpret_cast<const double2*>(Lp + J * LD + K0 + 2 * q);
            c1[q] = *reinterpret_cast<const double2*>(Lp + (J + 1) * LD + K0 + 2 * q);
        }
        const double r0 = rinv[kMW * P + J], r1 = rinv[kMW * P + J + 1];
        __builtin_amdgcn_sched_barrier(0);
        const double w0 = y[J] * r0;
        y[J] = w0;
        y[J + 1] = fma(-c0[0].y, w0, y[J + 1]);
        const double w1 = y[J + 1] * r1;
        y[J + 1] = w1;
#pragma unroll
        for (int q = 1; q < NR; ++q) {
            const int k = K0 + 2 * q;
            y[k] = fma(-c0[q].x, w0, y[k]);
            y[k + 1] = fma(-c0[q].y, w0, y[k + 1]);
            y[k] = fma(-c1[q].x, w1, y[k]);
            y[k + 1] = fma(-c1[q].y, w1, y[k + 1]);
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    step(std::integral_constant<int, 0>());
    step(std::integral_constant<int, 2>());
    step(std::integral_constant<int, 4>());
    step(std::integral_constant<int, 6>());
    step(std::integral_constant<int, 8>());
    step(std::integral_constant<int, 10>());
    step(std::integral_constant<int, 12>());
    step(std::integral_constant<int, 14>());
    // lanes >= 16 (zero columns) store into the discard block: one base, immediate offsets
    double* dst = (lane < kMW ? M.Wb + lblk(P, P) * kBlk : M.disc) + (lane & 15);
#pragma unroll
    for (int k = 0; k < kMW; ++k) dst[k * kBP] = y[k];
}

// acc += L_{I,K} W_{K,J} (K = 16): L from micro-panel K's columns, W from its block
template <int I, int K, int J>
__device__ __forceinline__ d4 mp_lw(d4 acc, const MpLds& M, int lane) {
    const double* Lp = M.Lc + mp_base(K);
    const double* Wk = M.Wb + lblk(K, J) * kBlk;
    return mfma_blk<16>(acc, [&](int i, int k) { return Lp[k * mp_ld(K) + 16 * (I - K) + i]; },
                        [&](int j, int k) { return Wk[k * kBP + j]; }, lane);
}
// W_{I,J} = -V_I X (X a block in LDS) into W block (I, J)
template <int I, int J>
__device__ __forceinline__ void mp_vx(const MpLds& M, const double* __restrict__ X, int lane) {
    const double* Vi = M.Wb + lblk(I, I) * kBlk;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = mfma_blk<16>(acc, [&](int i, int k) { return -Vi[i * kBP + k]; }, [&](int j, int k) { return X[k * kBP + j]; },
                       lane);
    blk_put(M.Wb + lblk(I, J) * kBlk, acc, lane);
}

// W_d's block row IB (rows 16 IB .. 16 IB + 15, final) to Wd: lane = column, zeros right of the
// diagonal block; one coalesced 512-byte row per store
template <bool SC1, int IB>
__device__ __forceinline__ void mp_w_rows(const MpLds& M, double* __restrict__ Wd, int lane) {
    const int jb = lane >> 4, c = lane & 15;
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = jb <= IB ? M.Wb[lblk(IB, jb <= IB ? jb : 0) * kBlk + q * kBP + c] : 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) stg<SC1>(Wd + (16 * IB + q) * NB + lane, v[q]);
}

template <bool STAMP = false, bool SC1 = false, class EARLY = NoEarly>
__device__ __forceinline__ void factor_diag16(const DiagLds& L, double* __restrict__ rinv, int* cnt,
                                              double* __restrict__ Wd, int d, int* info, long long* st = nullptr,
                                              const EARLY& early = EARLY(), double* __restrict__ Wst = nullptr,
                                              const double* __restrict__ Lsrc = nullptr, int kb0 = 4) {
    const int t = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const MpLds M = mp_lds(L);
    if (wave == 0) {
        mp_panel<0, STAMP>(M, rinv, cnt, lane, d, info, st);
        mp_panel<1, STAMP>(M, rinv, cnt, lane, d, info, st);
        mp_panel<2, STAMP>(M, rinv, cnt, lane, d, info, st);
        mp_panel<3, STAMP>(M, rinv, cnt, lane, d, info, st);
        if constexpr (STAMP) st[8] = __builtin_amdgcn_s_memtime();
        wait_lds_ge(cnt + 4, 1);
        mp_vx<3, 0>(M, M.Xs, lane);
        mp_vx<3, 1>(M, M.Xs + kBlk, lane);
        if constexpr (STAMP) st[9] = __builtin_amdgcn_s_memtime();
    } else if (wave == 1) {
        // V_0 here; V_1 .. V_3 come from the chain wave's idle lanes (mp_panel), final once the
        // column counter passes their micro-panel.  W's block rows 0..2 go to Wd as soon as they
        // are final (rows 48..63 follow the barrier), so the publish after the last pivot drains
        // a quarter of W's stores.
        const d4 z = {0.0, 0.0, 0.0, 0.0};
        mp_inverse<0>(M, rinv, cnt, lane);
        d4 x10 = mp_lw<1, 0, 0>(z, M, lane), x20 = mp_lw<2, 0, 0>(z, M, lane), x30 = mp_lw<3, 0, 0>(z, M, lane);
        wait_lds_ge(cnt, 2 * kMW);   // V_1
        if constexpr (STAMP) st[10] = __builtin_amdgcn_s_memtime();
        blk_put(M.Xs, x10, lane);
        mp_vx<1, 0>(M, M.Xs, lane);
        lds_signal(cnt + 1, 1);   // W rows 0 .. 31 (blocks (0,0), (1,0), (1,1)) are final
        mp_w_rows<SC1, 0>(M, Wd, lane);
        mp_w_rows<SC1, 1>(M, Wd, lane);
        d4 x21 = mp_lw<2, 1, 1>(z, M, lane), x31 = mp_lw<3, 1, 1>(z, M, lane);
        x20 = mp_lw<2, 1, 0>(x20, M, lane);
        x30 = mp_lw<3, 1, 0>(x30, M, lane);
        wait_lds_ge(cnt, 3 * kMW);   // V_2
        if constexpr (STAMP) st[11] = __builtin_amdgcn_s_memtime();
        blk_put(M.Xs, x20, lane);
        blk_put(M.Xs + kBlk, x21, lane);
        mp_vx<2, 0>(M, M.Xs, lane);
        mp_vx<2, 1>(M, M.Xs + kBlk, lane);
        d4 x32 = mp_lw<3, 2, 2>(z, M, lane);
        x30 = mp_lw<3, 2, 0>(x30, M, lane);
        x31 = mp_lw<3, 2, 1>(x31, M, lane);
        blk_put(M.Xs, x30, lane);   // after mp_vx<2, *>'s reads of Xs (one wave's LDS ops are ordered)
        blk_put(M.Xs + kBlk, x31, lane);
        blk_put(M.Xs + 2 * kBlk, x32, lane);
        lds_signal(cnt + 4, 1);
        mp_w_rows<SC1, 2>(M, Wd, lane);
        wait_lds_ge(cnt, 4 * kMW);   // V_3
        if constexpr (STAMP) st[12] = __builtin_amdgcn_s_memtime();
        mp_vx<3, 2>(M, M.Xs + 2 * kBlk, lane);
    } else {
        if (wave == 2) mp_owner<2>(M, cnt, lane, Lsrc, kb0);
        else mp_owner<3>(M, cnt, lane, Lsrc, kb0);
        wait_lds_ge(cnt + 1, 1);   // EarlyNext reads W rows 0..31
        early(wave, lane);
    }
    __syncthreads();
    if constexpr (STAMP) if (wave == 0) st[13] = __builtin_amdgcn_s_memtime();
    // W_d to HBM: rows 48..63 (wave 3; wave 1 stored rows 0..47 as they became final), lane =
    // column (each store one coalesced 512-byte row; zeros above the diagonal blocks); with Wst,
    // every wave's 16 rows also go to LDS in the substage layout (the next tile's L = A W^T
    // operand: late_prepare reads rows 32..63, diag_prepare all of it).  Wst overlaps the column
    // and W areas: every value is read before the barrier.
    {
        const int jb = lane >> 4, c = lane & 15;
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int ib = wave;
            v[q] = jb <= ib ? M.Wb[lblk(ib, jb <= ib ? jb : 0) * kBlk + q * kBP + c] : 0.0;
        }
        if (wave == 3)
#pragma unroll
            for (int q = 0; q < 16; ++q) stg<SC1>(Wd + (16 * wave + q) * NB + lane, v[q]);
        if (Wst) {
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 16; ++q) Wst[jb * kSub + (16 * wave + q) * kPad + c] = v[q];
        }
    }
}

template <bool STAMP = false, bool SC1 = false, class EARLY = NoEarly>
__device__ __forceinline__ void factor_diag(const DiagLds& L, double* __restrict__ rinv, int* cnt,
                                            double* __restrict__ Wd, int d, int* info, long long* st = nullptr,
                                            const EARLY& early = EARLY(), double* __restrict__ Wst = nullptr,
                                            const double* __restrict__ Lsrc = nullptr, int kb0 = 4) {
    factor_diag16<STAMP, SC1, EARLY>(L, rinv, cnt, Wd, d, info, st, early, Wst, Lsrc, kb0);
}

// ---- the diagonal workgroup's two products, balanced over its 4 waves --------------------
// L = A_{d,k} W_k^T with W_k lower triangular: wave w forms the 16-row strip w of L; output
// block column jb needs only K blocks kb <= jb, so every wave issues 4 (1 + 2 + 3 + 4) = 40
// MFMAs instead of the 64 of a 32 x 32 quadrant over the full K.  Each element's K steps run in
// ascending order in one accumulator.
__device__ __forceinline__ void diag_l_strip(d4 (&acc)[4], const double* __restrict__ X, const double* __restrict__ Y,
                                             int w, int lane) {
    const int frow = lane & 15, fk = lane >> 4;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) acc[jb] = d4{0.0, 0.0, 0.0, 0.0};
    // every operand read from LDS before the first MFMA: one wait instead of one LDS round trip
    // per K step (the MFMAs and their order are unchanged)
    double a[4][4], b[10][4];   // b: the pairs (kb, jb <= kb .. 3) in order
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            a[kb][kk] = X[kb * kSub + (w * 16 + frow) * kPad + kk * 4 + fk];
#pragma unroll
            for (int jb = kb; jb < 4; ++jb)
                b[kb * 4 - kb * (kb - 1) / 2 + jb - kb][kk] = Y[kb * kSub + (jb * 16 + frow) * kPad + kk * 4 + fk];
        }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int jb = kb; jb < 4; ++jb)
                acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kb][kk], b[kb * 4 - kb * (kb - 1) / 2 + jb - kb][kk], acc[jb],
                                                               0, 0, 0);
}

// the strip into LDS in the substage layout (L as the operand of the second product)
__device__ __forceinline__ void diag_strip_to_stage(const d4 (&acc)[4], double* __restrict__ X, int w, int lane) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) X[jb * kSub + (w * 16 + (lane >> 4) + 4 * r) * kPad + (lane & 15)] = acc[jb][r];
}

// Two blocks (strip s, column blocks j0 and j1) of diag_l_strip's product -- each block's MFMA
// chain exactly as diag_l_strip forms it (K blocks kb <= jb ascending, kk ascending), so the
// same bits; a half critical update task forms its half of L_ik this way, two blocks per wave.
__device__ __forceinline__ void diag_l_blocks(d4 (&acc)[2], const double* __restrict__ X, const double* __restrict__ Y,
                                              int s, int j0, int j1, int lane) {
    const int frow = lane & 15, fk = lane >> 4;
    acc[0] = acc[1] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const double a = X[kb * kSub + (s * 16 + frow) * kPad + kk * 4 + fk];
            if (kb <= j0)
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Y[kb * kSub + (j0 * 16 + frow) * kPad + kk * 4 + fk],
                                                              acc[0], 0, 0, 0);
            if (kb <= j1)
                acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Y[kb * kSub + (j1 * 16 + frow) * kPad + kk * 4 + fk],
                                                              acc[1], 0, 0, 0);
        }
}

// acc[mi] (output block row 2 h + mi, column block w) -= X Y^T over the 64-wide K: the per-block
// MFMA chain of mfma_xyt<true> (the same operands in the same order), for a half tile
__device__ __forceinline__ void mfma_xyt_half(d4 (&acc)[2], const double* __restrict__ X, const double* __restrict__ Y,
                                              int h, int w, int lane) {
    const int frow = lane & 15, fk = lane >> 4;
#pragma unroll
    for (int sub = 0; sub < 4; ++sub)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const double b = Y[sub * kSub + (w * 16 + frow) * kPad + kk * 4 + fk];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                const double a = -X[sub * kSub + ((2 * h + mi) * 16 + frow) * kPad + kk * 4 + fk];
                acc[mi] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[mi], 0, 0, 0);
            }
        }
}

// a panel's L strip (this wave's 16 rows of L_ik, from diag_l_strip) to the factor matrix, and
// into LDS row-major 64 x 65 (the forward substitution's copy)
template <bool SC1 = false>
__device__ __forceinline__ void strip_store(const d4 (&acc)[4], double* __restrict__ Lm, long ldp, int r0, int c0, int w,
                                            int lane) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            stg<SC1>(Lm + (long)(r0 + w * 16 + (lane >> 4) + 4 * r) * ldp + c0 + jb * 16 + (lane & 15), acc[jb][r]);
}
__device__ __forceinline__ void strip_to_rows(const d4 (&acc)[4], double* __restrict__ S, int w, int lane) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) S[(w * 16 + (lane >> 4) + 4 * r) * (NB + 1) + jb * 16 + (lane & 15)] = acc[jb][r];
}

// A_dd - L L^T on the 10 lower 16 x 16 blocks (ib >= jb) only -- the factor never reads the
// upper ones -- 3 / 3 / 2 / 2 blocks per wave (48 MFMAs on the busiest wave instead of 64)
__device__ __forceinline__ int diag_blk(int w, int s) {   // (ib << 2) | jb, or -1
    constexpr int tab[4][3] = {{(3 << 2) | 0, (3 << 2) | 1, 0}, {(3 << 2) | 2, (3 << 2) | 3, (1 << 2) | 0},
                               {(2 << 2) | 0, (2 << 2) | 1, -1}, {(2 << 2) | 2, (1 << 2) | 1, -1}};
    return tab[w][s];
}
// the deferred form (the persistent chain): only the block column jb = 0 gets -L L^T here, one
// block per wave (listed first); the other blocks are stored as they are and their owners in
// factor_diag16 (mp_owner) apply the products during the first micro-panel
__device__ __forceinline__ int diag_blk_def(int w, int s) {
    constexpr int tab[4][3] = {{0, (3 << 2) | 1, (1 << 2) | 1}, {(1 << 2) | 0, (3 << 2) | 2, (3 << 2) | 3},
                               {(2 << 2) | 0, (2 << 2) | 1, -1}, {(3 << 2) | 0, (2 << 2) | 2, -1}};
    return tab[w][s];
}

#ifdef PNOL_CHOL_TIMELINE
// tools/microbench/chol_timeline.hip only: per launch k + 1 and workgroup class (0 diagonal,
// 1 panel, 2 update): first start, last end (100 MHz realtime)
__device__ unsigned long long g_chol_tl[64 * 3 * 2];
__device__ unsigned long long g_chol_clk[64 * 8];   // the diagonal workgroup's shader-clock stamps
// persistent form, per step k (100 MHz realtime): [0] W_k published, panel (k+2, k) [1] claimed
// [2] flags ok [3] stored; update (k+2, k+1, k) [4] claimed [5] flags ok [6] stored; [7] panel
// (k+1, k) stored
__device__ unsigned long long g_chol_crit[64 * 8];
// the chain's look-ahead inside step d's factor (wave 2, shader clock): [0] polling starts,
// [1] tiles ready, [2] staged in LDS, [3] its MFMAs done
__device__ unsigned long long g_chol_la[64 * 4];
#define PNOL_LA_STAMP(d, i) \
    if (threadIdx.x == 128 && (d) < 64) g_chol_la[4 * (d) + (i)] = __builtin_amdgcn_s_memtime();
#define PNOL_CRIT(k, i) \
    if (threadIdx.x == 0 && (k) >= 0 && (k) < 64) g_chol_crit[8 * (k) + (i)] = __builtin_amdgcn_s_memrealtime();
#define PNOL_CHOL_STAMP(k, i) \
    if (threadIdx.x == 0 && (k) + 1 < 64) g_chol_clk[8 * ((k) + 1) + (i)] = __builtin_amdgcn_s_memtime();
__device__ __forceinline__ void chol_tl_mark(int k, int cls, unsigned long long t0) {
    if (threadIdx.x == 0 && k + 1 < 64) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        atomicMin(&g_chol_tl[((k + 1) * 3 + cls) * 2], t0);
        atomicMax(&g_chol_tl[((k + 1) * 3 + cls) * 2 + 1], t1);
    }
}
#else
#define PNOL_CHOL_STAMP(k, i)
#define PNOL_CRIT(k, i)
#define PNOL_LA_STAMP(d, i)
#endif
#ifdef PNOL_CHOL_TASKTRACE
// tools/microbench/chol_tasktrace.hip: per worker task (claim index g) the claim, the end of its
// dependency waits and its publish (100 MHz realtime), its step and kind
__device__ unsigned long long g_chol_tasks[16384 * 4];
#define PNOL_TASK_T0(g) const unsigned long long tt0_ = __builtin_amdgcn_s_memrealtime(); const int tg_ = (g);
#define PNOL_TASK_READY() const unsigned long long tt1_ = __builtin_amdgcn_s_memrealtime();
#define PNOL_TASK_END(k, kind)                                                                         \
    if (threadIdx.x == 0 && tg_ < 16384) {                                                              \
        g_chol_tasks[4 * tg_] = tt0_;                                                                  \
        g_chol_tasks[4 * tg_ + 1] = tt1_;                                                              \
        g_chol_tasks[4 * tg_ + 2] = __builtin_amdgcn_s_memrealtime();                                  \
        g_chol_tasks[4 * tg_ + 3] = ((unsigned long long)(k) << 8) | (unsigned long long)(kind);       \
    }
#else
#define PNOL_TASK_T0(g)
#define PNOL_TASK_READY()
#define PNOL_TASK_END(k, kind)
#endif

// The diagonal tile d = k + 1 (k >= 0) ready for factor_diag: L = A_{d,k} W_k^T (recomputed
// here rather than waited for), A_dd - L L^T on its 10 lower 16 x 16 blocks, into the split LDS
// copy L.  X / Y: the two staging areas (smem, smem + kStage).
// w_in_lds: Y already holds W_k in the substage layout (the previous factor_diag16 of the chain
// left it there), so only A_{d,k} is staged.
// Ldef (the persistent chain): L goes to Ldef (substage layout) and only block column 0 gets
// -L L^T here (diag_blk_def); factor_diag16's owners apply the rest (mp_owner, kb0 = 0).
// Astg / Cstg (the persistent chain after a staged-only look-ahead): A_{d,k} already in Astg
// (the substage layout) and A_dd's lower blocks in Cstg (16 x 16 row-major each, lower-block
// order) -- nothing is loaded from memory but W_k when it is not in LDS.
template <bool SC1 = false>
__device__ __forceinline__ void diag_prepare(const double* __restrict__ P, long ldp, const double* __restrict__ W,
                                             int k, double* __restrict__ X, double* __restrict__ Y, const DiagLds& L,
                                             int wave, int lane, bool w_in_lds = false, double* __restrict__ Ldef = nullptr,
                                             const double* __restrict__ Astg = nullptr,
                                             const double* __restrict__ Cstg = nullptr) {
    const int d0 = (k + 1) * NB;
    const int k0 = k * NB;
    const bool def = Ldef != nullptr;
    if (!Astg) stage_tile<SC1>(X, P, ldp, d0, k0);
    if (!w_in_lds) stage_tile<SC1>(Y, W + (long)k * NB * NB, NB, 0, 0);
    d4 cdd[3];   // this wave's lower blocks of A_dd, in flight during the first product
#pragma unroll
    for (int sb = 0; sb < 3; ++sb) {
        const int bl = def ? diag_blk_def(wave, sb) : diag_blk(wave, sb), ib = bl >> 2, jb = bl & 3;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            cdd[sb][r] = bl < 0  ? 0.0
                         : Cstg ? Cstg[(ib * (ib + 1) / 2 + jb) * 256 + ((lane >> 4) + 4 * r) * 16 + (lane & 15)]
                                : ldg<SC1>(P + (long)(d0 + ib * 16 + (lane >> 4) + 4 * r) * ldp + d0 + jb * 16 + (lane & 15));
    }
    __syncthreads();
    PNOL_CHOL_STAMP(k, 1)
    d4 lst[4];
    diag_l_strip(lst, Astg ? Astg : X, Y, wave, lane);   // L_{d,k} = A_{d,k} W_k^T, strip `wave`
    __syncthreads();
    PNOL_CHOL_STAMP(k, 2)
    double* const Ls = def ? Ldef : X;
    diag_strip_to_stage(lst, Ls, wave, lane);
    __syncthreads();
    const int frow = lane & 15, fk = lane >> 4;
#pragma unroll
    for (int sb = 0; sb < 3; ++sb) {           // A_dd - L L^T, lower blocks
        const int bl = def ? diag_blk_def(wave, sb) : diag_blk(wave, sb), ib = bl >> 2, jb = bl & 3;
        if (bl < 0 || (def && jb != 0)) continue;   // wave-uniform
        double fa[4][4], fb[4][4];              // the block's operands, read before its MFMAs
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                fa[kb][kk] = -Ls[kb * kSub + (ib * 16 + frow) * kPad + kk * 4 + fk];
                fb[kb][kk] = Ls[kb * kSub + (jb * 16 + frow) * kPad + kk * 4 + fk];
            }
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) cdd[sb] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[kb][kk], fb[kb][kk], cdd[sb], 0, 0, 0);
    }
    __syncthreads();                            // X / Y are rewritten below
#pragma unroll
    for (int sb = 0; sb < 3; ++sb) {
        const int bl = def ? diag_blk_def(wave, sb) : diag_blk(wave, sb), ib = bl >> 2, jb = bl & 3;
        if (bl < 0) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            diag_put(L, ib * 16 + (lane >> 4) + 4 * r, jb * 16 + (lane & 15), cdd[sb][r]);
    }
}

// ---- the persistent chain's look-ahead --------------------------------------------------------
// While tile d is factored, waves 2 and 3 (idle once T is formed) start the next tile's products:
// once tiles (d+1, d) and (d+1, d+1) carry the updates of columns < d (their version words), they
// stage A_{d+1,d} and the lower 16 x 16 blocks of A_{d+1,d+1}, form the left half of
// L = A_{d+1,d} W_d^T (block columns 0, 1 need only W11, which wave 1 has finished) and apply
// its part of A_dd - L L^T (K blocks 0, 1).  After the factor, late_prepare forms the right half
// of L (K blocks up to 3, W_d's rows 32..63 from the LDS copy Wst) and the rest of L L^T.  Every
// accumulator receives the same MFMAs in the same order as diag_prepare's, so the factor is
// bitwise method 4's.  Waves 2 / 3 wait for the tiles inside the factor (their dependencies are
// tasks of step d-1, which never wait on W_d); with a finite cutoff (PNOL_CHOL_LOOKAHEAD = c)
// they give up once wave 0 has c columns of the tile final, and the next step stages as before.
constexpr int kLowerBlks = 10;   // lower 16 x 16 blocks of a 64 x 64 tile, index ib (ib + 1) / 2 + jb

__device__ __forceinline__ void blk_ij(int b, int& ib, int& jb) {
    ib = b >= 6 ? 3 : (b >= 3 ? 2 : (b >= 1 ? 1 : 0));
    jb = b - ib * (ib + 1) / 2;
}

__device__ __forceinline__ int lds_peek(const int* w) {
    const __attribute__((address_space(3))) int* p = (const __attribute__((address_space(3))) int*)w;
    int v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

struct EarlyLds {
    double* pfx;   // A_{d+1,d} in the substage layout (then L's right half, substages 2, 3)
    double* pll;   // L's left half, substages 0, 1
    double* pfc;   // the lower blocks of A_{d+1,d+1} (16 x 16 row-major each), then minus L_left L_left^T
    int* w;        // [0] decision (1 go, 2 skip), [1] / [2] wave 2 / 3's L_left stored
};

struct EarlyNext {
    const double* P;
    long ldp;
    int T, d;
    const int* ver;
    const double* W11;   // W_d rows 0..31 of the tile being factored (diag_w11, read by w11_at)
    const int* cnt;      // factor_diag's column counter (wave 0's progress)
    int cutoff;          // give up once cnt reaches this (> 64: wait for the tiles)
    EarlyLds E;
    __device__ void operator()(int wave, int lane) const {
        const int dn = d + 1;
        if (dn >= T) return;
        if (wave == 2) {
            PNOL_LA_STAMP(d, 0)
            // 1: the tiles came before `cutoff` columns of this factor were final -- stage them and
            // start their products; 3: they came later, before the factor's last column -- stage
            // them only (the next step's diag_prepare takes them from LDS instead of memory);
            // 2: not in time
            int ready = 0, late = 0;
            for (int it = 0;; ++it) {
                ready = __hip_atomic_load(ver + dn * T + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= d &&
                        __hip_atomic_load(ver + dn * T + dn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= d;
                ready = __builtin_amdgcn_readfirstlane(ready);
                const int c = __builtin_amdgcn_readfirstlane(lds_peek(cnt));
                if (ready) {
                    late = c >= cutoff;
                    break;
                }
                if (it > 4096 || (cutoff <= NB && c >= NB)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            PNOL_LA_STAMP(d, 1)
            lds_signal(E.w, ready ? (late ? 3 : 1) : 2);
        } else {
            wait_lds_ge(E.w, 1);
        }
        const int mode = __builtin_amdgcn_readfirstlane(lds_peek(E.w));
        if (mode != 1 && mode != 3) return;
        const int h = wave - 2;   // wave 2: rows 0..31 and blocks 0..4; wave 3: rows 32..63, blocks 5..9
        {
            // an opaque copy of the lane id: keeps the (loop-invariant) load offsets from being
            // hoisted out of the chain loop and held in registers across the factor
            int ln = lane;
            asm volatile("" : "+v"(ln));
            // the 26 16-byte sc1 loads per lane in one round
            const double* base = P + (long)(dn * NB + 32 * h) * ldp + d * NB;   // wave-uniform
            const double* cb = P + (long)(dn * NB) * ldp + dn * NB;
            double2 v[16], u[10];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int id = q * 64 + ln, row = id >> 5, col = (id & 31) * 2;
                v[q] = ld16_sc1(base, (unsigned)((row * ldp + col) * 8));
            }
#pragma unroll
            for (int q = 0; q < 10; ++q) {
                int ib, jb;
                blk_ij(5 * h + (q >> 1), ib, jb);
                const int id = (q & 1) * 64 + ln, row = id >> 3, col = (id & 7) * 2;
                u[q] = ld16_sc1(cb, (unsigned)(((ib * 16 + row) * ldp + jb * 16 + col) * 8));
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int id = q * 64 + ln, row = 32 * h + (id >> 5), col = (id & 31) * 2;
                *reinterpret_cast<double2*>(E.pfx + (col >> 4) * kSub + row * kPad + (col & 15)) = v[q];
            }
#pragma unroll
            for (int q = 0; q < 10; ++q) {
                const int id = (q & 1) * 64 + ln, row = id >> 3, col = (id & 7) * 2;
                *reinterpret_cast<double2*>(E.pfc + (5 * h + (q >> 1)) * 256 + row * 16 + col) = u[q];
            }
        }
        PNOL_LA_STAMP(d, 2)
        if (mode == 3) return;   // staged only
        const int frow = lane & 15, fk = lane >> 4;
        // Every MFMA operand of a phase is read from LDS before its first MFMA (one wait, not one
        // LDS round trip per K step); each accumulator takes the same MFMAs in the same order.
        // L's left half for this wave's strips (block columns jb = 0, 1: K blocks kb <= jb)
        {
            double av[2][2][4], bw[3][4];   // av[s][kb][kk]; bw: (kb, jb) = (0, 0), (0, 1), (1, 1)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                bw[0][kk] = w11_at(W11, frow, kk * 4 + fk);
                bw[1][kk] = w11_at(W11, 16 + frow, kk * 4 + fk);
                bw[2][kk] = w11_at(W11, 16 + frow, 16 + kk * 4 + fk);
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb)
                        av[s][kb][kk] = E.pfx[kb * kSub + ((2 * h + s) * 16 + frow) * kPad + kk * 4 + fk];
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int strip = 2 * h + s;
                d4 acc[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                        for (int jb = kb; jb < 2; ++jb)
                            acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s][kb][kk], bw[kb + jb][kk], acc[jb], 0, 0, 0);
#pragma unroll
                for (int jb = 0; jb < 2; ++jb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        E.pll[jb * kSub + (strip * 16 + (lane >> 4) + 4 * r) * kPad + (lane & 15)] = acc[jb][r];
            }
        }
        lds_signal(E.w + 1 + h, 1);
        wait_lds_ge(E.w + 2 - h, 1);
        // this wave's five blocks of A_dd - L_left L_left^T (K blocks 0, 1): the fragments of the
        // row blocks they touch, then the blocks
        auto llt = [&](auto hc) {
            constexpr int H = decltype(hc)::value, RB = H == 0 ? 3 : 4;
            double fr[RB][2][4];
            d4 c[5];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) fr[rb][kb][kk] = E.pll[kb * kSub + (rb * 16 + frow) * kPad + kk * 4 + fk];
#pragma unroll
            for (int q = 0; q < 5; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) c[q][r] = E.pfc[(5 * H + q) * 256 + ((lane >> 4) + 4 * r) * 16 + (lane & 15)];
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                constexpr int b0 = 5 * H;
                const int b = b0 + q;
                const int ib = b >= 6 ? 3 : (b >= 3 ? 2 : (b >= 1 ? 1 : 0)), jb = b - ib * (ib + 1) / 2;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
                        c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(-fr[ib][kb][kk], fr[jb][kb][kk], c[q], 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 5; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) E.pfc[(5 * H + q) * 256 + ((lane >> 4) + 4 * r) * 16 + (lane & 15)] = c[q][r];
        };
        if (h == 0) llt(std::integral_constant<int, 0>());
        else llt(std::integral_constant<int, 1>());
        PNOL_LA_STAMP(d, 3)
    }
};

// The rest of diag_prepare after a look-ahead: L's right half (block columns 2, 3) from the staged
// A_{d,k} (E.pfx) and W_k's rows 32..63 (Wst), then K blocks 2, 3 of A_dd - L L^T on the partial
// blocks in E.pfc, into the split LDS copy L.
// def: only block column 0 gets K blocks 2, 3 here (diag_blk_def); factor_diag16's owners apply
// the rest from E.pfx (mp_owner, kb0 = 2)
__device__ __forceinline__ void late_prepare(const EarlyLds& E, const double* __restrict__ Wst, const DiagLds& L,
                                             int wave, int lane, bool def = false) {
    const int frow = lane & 15, fk = lane >> 4;
    // each phase's MFMA operands are read from LDS before its first MFMA (as in EarlyNext)
    {
        double a[4][4], b[7][4];   // b: (kb, jb) = (0,2) (0,3) (1,2) (1,3) (2,2) (2,3) (3,3)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                a[kb][kk] = E.pfx[kb * kSub + (wave * 16 + frow) * kPad + kk * 4 + fk];
#pragma unroll
                for (int jb = (kb > 2 ? kb : 2); jb < 4; ++jb)
                    b[kb < 3 ? 2 * kb + jb - 2 : 6][kk] = Wst[kb * kSub + (jb * 16 + frow) * kPad + kk * 4 + fk];
            }
        d4 lr[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int jb = (kb > 2 ? kb : 2); jb < 4; ++jb)
                    lr[jb - 2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kb][kk], b[kb < 3 ? 2 * kb + jb - 2 : 6][kk], lr[jb - 2], 0, 0, 0);
        // this wave's own rows of substages 2, 3 (only it reads them above)
#pragma unroll
        for (int jb = 2; jb < 4; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                E.pfx[jb * kSub + (wave * 16 + (lane >> 4) + 4 * r) * kPad + (lane & 15)] = lr[jb - 2][r];
    }
    __syncthreads();
    double fa[3][2][4], fb[3][2][4];
    d4 c[3];
#pragma unroll
    for (int sb = 0; sb < 3; ++sb) {
        const int b0 = def ? diag_blk_def(wave, sb) : diag_blk(wave, sb);
        const int bl = b0, ib = bl < 0 ? 0 : bl >> 2, jb = bl < 0 ? 0 : bl & 3;
        const int b = ib * (ib + 1) / 2 + jb;
#pragma unroll
        for (int r = 0; r < 4; ++r) c[sb][r] = E.pfc[b * 256 + ((lane >> 4) + 4 * r) * 16 + (lane & 15)];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                fa[sb][kb][kk] = -E.pfx[(kb + 2) * kSub + (ib * 16 + frow) * kPad + kk * 4 + fk];
                fb[sb][kb][kk] = E.pfx[(kb + 2) * kSub + (jb * 16 + frow) * kPad + kk * 4 + fk];
            }
    }
#pragma unroll
    for (int sb = 0; sb < 3; ++sb) {
        const int bl = def ? diag_blk_def(wave, sb) : diag_blk(wave, sb), ib = bl >> 2, jb = bl & 3;
        if (bl < 0) continue;   // wave-uniform
        if (!def || jb == 0)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    c[sb] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[sb][kb][kk], fb[sb][kb][kk], c[sb], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) diag_put(L, ib * 16 + (lane >> 4) + 4 * r, jb * 16 + (lane & 15), c[sb][r]);
    }
}

// ---- one panel step ---------------------------------------------------------------------
// Launch k (-1 <= k <= T-2), R = T-1-k.  blockIdx 0: the diagonal tile k+1; 1..R: panel rows
// i = k+1 .. T-1; then the update tiles (i, j), k+1 <= j <= i, (i, j) != (k+1, k+1), by columns.
// Waits only ever target lower blockIdx (the panel workgroups), and every wait is capped.
// Launch -1 is also the prep: block 0 resets info and factors tile 0 straight from A while
// blocks 1.. copy A into the padded P (identity on the padded diagonal) and rhs into bv.
__global__ __launch_bounds__(256, 2) void k_chol_step(double* __restrict__ P, double* __restrict__ Lm, long ldp,
                                                   int T, int k, double* __restrict__ W, double* __restrict__ bv,
                                                   double* __restrict__ zv, int* __restrict__ rowflag, int epoch,
                                                   int* __restrict__ info, const double* __restrict__ A, long lda,
                                                   int n, const double* __restrict__ rhs, int* __restrict__ pflags,
                                                   int npflags) {
    __shared__ __attribute__((aligned(16))) double smem[2 * kStage];   // 73.7 KB
    __shared__ double rinv[NB];
    __shared__ double zsh[NB];
    __shared__ int cnt[6];   // diagonal-tile phase words (factor_diag)
    __shared__ int ok_sh;
    const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), wr = wave >> 1, wc = wave & 1;
#ifdef PNOL_CHOL_TIMELINE
    const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime(), ck0 = __builtin_amdgcn_s_memtime();
#endif
    if (k < 0 && blockIdx.x > 0) {   // prep: rows b-1, b-1+G, ... of P
        const int N = T * NB, G = gridDim.x - 1;
        // 16-byte loads and stores, all of a row's loads issued before its stores (N is a multiple
        // of 64; the pairs past n -- the padding -- are formed per element)
        const bool vec = ((lda & 1) == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
        for (int r = blockIdx.x - 1; r < N; r += G) {
            double* pr = P + (long)r * ldp;
            const double* ar = A + (long)r * lda;
            if (vec && r < n) {
                double2 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int c = 2 * (t + 256 * u);
                    v[u] = c + 1 < n ? *reinterpret_cast<const double2*>(ar + c)
                                     : make_double2(c < n ? ar[c] : (r == c ? 1.0 : 0.0), r == c + 1 ? 1.0 : 0.0);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int c = 2 * (t + 256 * u);
                    if (c < N) *reinterpret_cast<double2*>(pr + c) = v[u];
                }
                for (int c = 2 * (t + 1024); c < N; c += 512) {   // rows past 2048 columns
                    const double2 w = c + 1 < n ? *reinterpret_cast<const double2*>(ar + c)
                                                : make_double2(c < n ? ar[c] : (r == c ? 1.0 : 0.0), r == c + 1 ? 1.0 : 0.0);
                    *reinterpret_cast<double2*>(pr + c) = w;
                }
            } else {
                for (int c = t; c < N; c += 256) pr[c] = (r < n && c < n) ? ar[c] : (r == c ? 1.0 : 0.0);
            }
        }
        if (blockIdx.x == 1)
            for (int r = t; r < N; r += 256) bv[r] = r < n ? rhs[r] : 0.0;
        if (blockIdx.x == gridDim.x - 1)   // the persistent form's progress words (k_chol_persist)
            for (int q = t; q < npflags; q += 256) pflags[q] = 0;
        return;
    }
    if (k < 0) {
        if (t == 0) __hip_atomic_store(info, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        return;
    }
    double* X = smem;
    double* Y = smem + kStage;
    const int R = T - 1 - k;
    const int b = blockIdx.x;

    if (b == 0) {   // ---------------- diagonal tile d = k + 1
        const int d = k + 1;
        const DiagLds L = diag_lds(smem);
        if (t < 6) cnt[t] = 0;
        if (k >= 0) {
            diag_prepare(P, ldp, W, k, X, Y, L, wave, lane);
        } else {
            const int row = t >> 2, c0 = (t & 3) * 16;
            double v[16];   // all 16 loads in flight before the first LDS store (clamped addresses)
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = A[(long)min(row, n - 1) * lda + min(c0 + q, n - 1)];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int c = c0 + q;
                diag_put(L, row, c, (row < n && c < n) ? v[q] : (row == c ? 1.0 : 0.0));
            }
        }
        __syncthreads();
        PNOL_CHOL_STAMP(k, 3)
        factor_diag(L, rinv, cnt, W + (long)d * NB * NB, d, info);
        PNOL_CHOL_STAMP(k, 4)
#ifdef PNOL_CHOL_TIMELINE
        __syncthreads();
        chol_tl_mark(k, 0, tl0);
        if (threadIdx.x == 0 && k + 1 < 64) g_chol_clk[8 * (k + 1)] = ck0;
        PNOL_CHOL_STAMP(k, 7)
#endif
        return;
    }

    if (b <= R) {   // ---------------- panel row i: L_ik = A_ik W_k^T, forward-solve update
        const int i = k + b, k0 = k * NB, i0 = i * NB;
        stage_tile(X, P, ldp, i0, k0);
        stage_tile(Y, W + (long)k * NB * NB, NB, 0, 0);
        __syncthreads();
        // W_k is lower triangular: each wave forms a 16-row strip of L_ik over the nonzero K
        // blocks only (40 MFMAs instead of 64; the diagonal workgroup's own L uses the same
        // products, so both copies of L_{k+1,k} carry the same bits)
        d4 acc[4];
        diag_l_strip(acc, X, Y, wave, lane);
        strip_store(acc, Lm, ldp, i0, k0, wave, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                                 // every wave's stores have drained
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(rowflag + i, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // forward substitution carried by the panel: z_k = W_k b_k, b_i -= L_ik z_k
        strip_to_rows(acc, X, wave, lane);   // X is free (the MFMA finished before the barrier)
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
#ifdef PNOL_CHOL_TIMELINE
        chol_tl_mark(k, 1, tl0);
#endif
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
    stage_tile(X, Lm, ldp, i * NB, k0);
    if (i != j) stage_tile(Y, Lm, ldp, j * NB, k0);
    d4 acc[2][2];
    acc_load(acc, P, ldp, i * NB, j * NB, wr, wc, lane);
    __syncthreads();
    mfma_xyt<true>(acc, X, i != j ? Y : X, wr, wc, lane);
    acc_store(acc, P, ldp, i * NB, j * NB, wr, wc, lane);
#ifdef PNOL_CHOL_TIMELINE
    chol_tl_mark(k, 2, tl0);
#endif
}

// ---- the persistent form (method 5) --------------------------------------------------------
// The steps k = 0 .. T-2 of k_chol_step as ONE launch after the prep launch (k = -1, which also
// factors tile 0 and zeroes the progress words):
//   blockIdx 0     the diagonal chain: for d = 1 .. T-1, once tiles (d, d-1) and (d, d) hold
//                  the updates of columns < d-1, diag_prepare + factor_diag -> W_d, published;
//                  no launch boundary and no wait for the rest of step d-1's work;
//   blockIdx >= 1  workers taking tasks from an atomic counter (task_of's order) -- step k's
//                  panel rows i = k+1 .. T-1 and its update tiles by columns (the same task set as
//                  the blocks of launch k), each step's four critical tasks handed out one step
//                  early -- each waiting on the diagonal chain (which itself waits only on tasks of
//                  steps <= d-2) or on tasks handed out before it, except that the <= 4 early
//                  tasks may wait on their predecessor step's later tasks: the queue drains once
//                  5 workers are resident (order 0, PNOL_CHOL_ORDER=0: with any number).
// Progress words (int, zeroed by the prep): wdone[d] (W_d published), lcnt[i] (panels of row i
// stored in Lm), bcnt[i] (forward-substitution updates applied to b_i), ver[i * T + j] (update
// steps applied to tile (i, j)); plus the task counter.  Hand-offs without fences: every byte
// another workgroup reads (P, Lm, W, b) is stored and loaded sc1, every storing wave waits
// vmcnt(0) before the workgroup barrier behind which one lane stores the word (sc1), and the
// consumer's lane 0 polls it with sc1 loads before a barrier (MI355X_MICROARCH.md "Valid forms",
// row 1; one workgroup per CU: __launch_bounds__(256, 1) and the register count).  Every tile, panel and b update is the same arithmetic in the same order as in
// the per-step launches, so the result is bitwise method 4's.
struct PersistWords {
    int *wdone, *lcnt, *bcnt, *ver, *counter, *half;
};
// half: per tile, the halves of a split critical update stored (0, 1, 2)
__device__ __forceinline__ PersistWords persist_words(int* f, int T) {
    return {f, f + T, f + 2 * T, f + 3 * T, f + 3 * T + T * T, f + 3 * T + T * T + 1};
}

// publish `v` into *w after every wave's (sc1) stores of this workgroup have completed
__device__ __forceinline__ void publish(int* w, int v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a worker task's last publish: lane 0 also claims the worker's next task, so the claim's
// round trip overlaps the store drain the publish waits for anyway (the claim order is unchanged)
__device__ __forceinline__ void publish_claim(int* w, int v, int* counter, int& pre) {
    if (threadIdx.x == 0) pre = atomicAdd(counter, 1);
    publish(w, v);
}
// a half critical update's publish: the second half to finish publishes the tile's version (each
// half's sc1 stores have completed before its arrival count, so both halves are in L2 by then)
__device__ __forceinline__ void publish_half_claim(int* hc, int* w, int v, int* counter, int& pre) {
    if (threadIdx.x == 0) pre = atomicAdd(counter, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && __hip_atomic_fetch_add(hc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1)
        __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every *f[q] >= tg[q] in one round of loads (no waiting)
template <int N>
__device__ __forceinline__ bool ready_all(const int* const (&f)[N], const int (&tg)[N]) {
    int v[N];
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = __hip_atomic_load(f[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool ok = true;
#pragma unroll
    for (int q = 0; q < N; ++q) ok = ok && v[q] >= tg[q];
    return ok;
}

// The reducing form (launch_chol_reducing, the LM trip): A is not formed -- the persistent
// launch's first tasks sum the J^T J split-K partials of k_syrk_tile into the padded matrix P
// themselves, one 64 x 64 tile each in column order (its version word leaves -1 when it is
// stored: every step task's wait ver >= k also waits for it), after one task forming
// b = -J^T F from the slice partials (b's block-row words leave -1).  The chain factors tile 0
// itself.  Every value is the sum of k_syrk_reduce and k_tree_nodes (leaf = the sub-chunks from
// 0.0 in order, then tree8; the Marquardt diagonal), and P's upper half inside the diagonal
// tiles is the mirror, as the copy of A in the prep launch gives -- so the factorisation is
// bitwise the one of A.
struct RedArgs {
    const double* part = nullptr;   // nullptr: not the reducing form
    int sub = 0, n = 0;
    double lambda = 0.0;
    const double* jp = nullptr;     // the 8 -J^T F slice partials (jp[s n + e])
    double* rhs = nullptr;          // rhs = -J^T F, for the LU fallback
    // LevMarqMPI: the J^T J tiles already summed (the allgathered packed tiles: tile t at
    // packed + (t / tpr) slot + (t % tpr) 128^2) and rhs already formed (rhs_in)
    const double* packed = nullptr;
    long slot = 0;
    int tpr = 1;
    const double* rhs_in = nullptr;
    // the matrix and b already in P / bv (a reduce launch wrote them; every version and b word
    // starts at 0): no reduce tasks, the chain factors tile 0 itself
    bool preloaded = false;
    // the worker claim order (task_of): 1 (default) each step's critical tasks one step early,
    // 0 by step (PNOL_CHOL_ORDER=0)
    int order = 1;
    // the two critical update tasks of each step form their L panels themselves
    // (PNOL_CHOL_SELFL=0: they wait for the panel tasks' stored L)
    bool selfl = true;
    // ... and run as two tasks each, one per 32-row half of the tile (selfl only; PNOL_CHOL_SPLIT)
    bool split = true;
    // each step's other updates claimed by tile row (task_local; PNOL_CHOL_ROWMAJOR)
    bool rowmajor = true;
};

template <int SUB>
__device__ __forceinline__ void red_pair(const double* __restrict__ p, long off, int sub, double& vx, double& vy) {
    constexpr long E = 128L * 128L;
    double lx[8], ly[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        double ax = 0.0, ay = 0.0;
#pragma unroll
        for (int u = 0; u < (SUB > 0 ? SUB : sub); ++u) {
            const double2 w = *reinterpret_cast<const double2*>(p + (long)(s * sub + u) * E + off);
            ax += w.x;
            ay += w.y;
        }
        lx[s] = ax;
        ly[s] = ay;
    }
    vx = ((lx[0] + lx[1]) + (lx[2] + lx[3])) + ((lx[4] + lx[5]) + (lx[6] + lx[7]));
    vy = ((ly[0] + ly[1]) + (ly[2] + ly[3])) + ((ly[4] + ly[5]) + (ly[6] + ly[7]));
}

// reduce task u of the reducing form: u = 0 b, u >= 1 the (u-1)-th lower 64 x 64 tile in column order
__device__ void red_task(int u, const RedArgs& red, double* __restrict__ P, long ldp, int T, double* __restrict__ bv,
                         const PersistWords& pw, int* __restrict__ info) {
    const int t = threadIdx.x;
    if (u == 0 && red.rhs_in) {   // b = the rhs the caller formed
        for (int e = t; e < red.n; e += 256) stg<true>(bv + e, red.rhs_in[e]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int i = t; i < T; i += 256) __hip_atomic_store(pw.bcnt + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (u == 0) {
        for (int e = t; e < red.n; e += 256) {
            double l[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) l[s] = 0.0 + red.jp[(long)s * red.n + e];
            const double v = ((l[0] + l[1]) + (l[2] + l[3])) + ((l[4] + l[5]) + (l[6] + l[7]));
            red.rhs[e] = v;
            stg<true>(bv + e, v);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int i = t; i < T; i += 256) __hip_atomic_store(pw.bcnt + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    int r = u - 1, J = 0;
    while (r >= T - J) {
        r -= T - J;
        ++J;
    }
    const int I = J + r, ti = I >> 1, tj = J >> 1;
    const long tt = (long)ti * (ti + 1) / 2 + tj;
    const double* p = red.part ? red.part + tt * 8 * red.sub * (128L * 128L) : nullptr;
    const double* pk = red.packed ? red.packed + (tt / red.tpr) * red.slot + (tt % red.tpr) * (128L * 128L) : nullptr;
    const double scale = 1 + red.lambda;
    // two element pairs per step (the loads of both in flight; 2 x 8 x sub 16-byte loads)
    auto pairs = [&](auto SUBC) {
        constexpr int S = decltype(SUBC)::value;
        for (int q0 = t; q0 < NB * NB / 2; q0 += 512) {   // element pairs (r, c), (r, c + 1)
            double v[2][2];
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                const int q = q0 + 256 * w, rr = q >> 5, c = 2 * (q & 31);
                const long off = (long)(64 * (I & 1) + rr) * 128 + 64 * (J & 1) + c;
                if (pk) {   // the summed tile (k_syrk_unpack's values)
                    const double2 pv = *reinterpret_cast<const double2*>(pk + off);
                    v[w][0] = pv.x;
                    v[w][1] = pv.y;
                } else {
                    red_pair<S>(p, off, red.sub, v[w][0], v[w][1]);
                }
            }
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                const int q = q0 + 256 * w, rr = q >> 5, c = 2 * (q & 31);
                const int i = I * NB + rr;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int j = J * NB + c + h;
                    if (i >= red.n || j >= red.n || j > i) continue;
                    stg<true>(P + (long)i * ldp + j, i == j ? scale * v[w][h] : v[w][h]);
                    if (j < i && I == J) stg<true>(P + (long)j * ldp + i, v[w][h]);   // the mirror inside the diagonal tile
                }
            }
        }
    };
    if (red.sub == 2) pairs(std::integral_constant<int, 2>{});
    else pairs(std::integral_constant<int, 0>{});
    publish(pw.ver + I * T + J, 0);
}


// The workers' claim order: claim index g -> step k and task -- a panel row i (L_ik, b_i), or
// an update tile (i, j) -= L_ik L_jk^T.  Step k (R = T-1-k panel rows) holds
// S_k = R + R (R + 1) / 2 - 1 tasks, local index l: panels l < R, then the update tiles in
// column order with the two the chain needs next first (l = R: (k+2, k+1), l = R+1: (k+2, k+2)).
//   order 0: step by step (every task waits only on tasks claimed before it).
//   order 1: each step's critical set C_k (l in {0, 1, R, R+1}; {0} for R = 1) one step early:
//            C_0, C_1, rest_0, C_2, rest_1, ..., C_{T-2}, rest_{T-3}, rest_{T-2}.  A task of C_{k+1}
//            may wait on a task of rest_k claimed after it: up to 4 workers can wait on unclaimed
//            tasks, so this order needs more than 4 workers.
// (By tile column -- all of a column's updates before the next column's panels, every
// dependency claimed first -- measured 1.23 ms per solve against 0.60: the workers pile up on
// far-column tasks waiting for the chain while runnable updates stay unclaimed.)
// Order 1 against order 0: 6 of 6 same-box bench pairs faster, +0.5-1% LM iters/s.
struct Task {
    int k, i, j;   // j < 0: panel row i of step k
    int h;         // >= 0: the 32-row half h of a split critical update
};
// split: the two critical updates (l = R, R + 1) are four half tasks (l = R .. R + 3), the other
// updates one index later by two.  rowmajor: the updates after the critical two by tile row
// (rows k+3, k+4, ..., each from column k+1 to the diagonal) instead of by tile column: the chain
// needs row d's tiles at step d - 1, so the rows near the diagonal come first.
__device__ __forceinline__ Task task_local(int k, int l, int T, bool split, bool rowmajor = false) {
    const int R = T - 1 - k;
    if (l < R) return {k, k + 1 + l, -1, -1};
    int q = l - R;
    if (split && R >= 2) {
        if (q < 4) return {k, k + 2, q < 2 ? k + 1 : k + 2, q & 1};
        q -= 2;
    }
    if (rowmajor && q >= 2) {
        int r = q - 2, i = k + 3;   // row i holds the tiles (i, k+1) .. (i, i): i - k of them
        while (r >= i - k) {
            r -= i - k;
            ++i;
        }
        return {k, i, k + 1 + r, -1};
    }
    // full column order f: column k+1 holds f = 0 .. R-1 (f = 0 is the chain's), column k+2
    // starts at f = R, ...
    int u = q == 0 ? 1 : (q == 1 ? R : (q < R ? q : q + 1));
    int j = k + 1;
    while (u >= T - j) {
        u -= T - j;
        ++j;
    }
    return {k, j + u, j, -1};
}
// tasks of step k (R = T - 1 - k panel rows), with the split critical updates
__host__ __device__ __forceinline__ int step_tasks(int R, bool split) {
    return R + R * (R + 1) / 2 - 1 + (split && R >= 2 ? 2 : 0);
}
__device__ __forceinline__ Task task_of(int g, int T, int order, bool split, bool rowmajor = false) {
    if (order == 1) {
        const int nc = split ? 6 : 4;   // the critical set: panels k+1, k+2 and the updates (halves)
        auto csz = [&](int kk) { return T - 1 - kk >= 2 ? nc : 1; };
        auto cmap = [&](int x, int RR) { return x < 2 ? x : RR + x - 2; };
        if (g < csz(0)) return task_local(0, cmap(g, T - 1), T, split, rowmajor);
        g -= csz(0);
        for (int kk = 0;; ++kk) {
            if (kk + 1 <= T - 2) {
                const int c1 = csz(kk + 1);
                if (g < c1) return task_local(kk + 1, cmap(g, T - 2 - kk), T, split, rowmajor);
                g -= c1;
            }
            const int RR = T - 1 - kk, S = step_tasks(RR, split), rest = S - csz(kk);
            if (g < rest || kk >= T - 2)
                return task_local(kk, g < RR - 2 ? g + 2 : g + (split && RR >= 2 ? 6 : 4), T, split, rowmajor);
            g -= rest;
        }
    }
    int k = 0, R = T - 1;
    for (;;) {
        const int S = step_tasks(R, split);
        if (g < S || R <= 1) break;
        g -= S;
        ++k;
        --R;
    }
    return task_local(k, g, T, split, rowmajor);
}

__global__ __launch_bounds__(256, 1) void k_chol_persist(double* __restrict__ P, double* __restrict__ Lm, long ldp,
                                                      int T, double* __restrict__ W, double* __restrict__ bv,
                                                      double* __restrict__ zv, int* __restrict__ flags, int ntasks,
                                                      int* __restrict__ info, int lookahead,
                                                      const RedArgs red) {
    __shared__ __attribute__((aligned(16))) double smem[2 * kStage];   // 73.7 KB
    // the chain's look-ahead areas (EarlyNext / late_prepare): 75.8 KB
    __shared__ __attribute__((aligned(16))) double pfx[kStage];
    __shared__ __attribute__((aligned(16))) double pll[2 * kSub];
    __shared__ __attribute__((aligned(16))) double pfc[kLowerBlks * 256];
    __shared__ double rinv[NB];
    __shared__ double zsh[NB];
    __shared__ int cnt[6];
    __shared__ int ew[4];
    __shared__ int task_sh, ok_sh;
    const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), wr = wave >> 1, wc = wave & 1;
    const PersistWords pw = persist_words(flags, T);
    double* X = smem;
    double* Y = smem + kStage;

    if (blockIdx.x == 0) {   // ---------------- the diagonal chain
        const EarlyLds E{pfx, pll, pfc, ew};
        if (t < 4) ew[t] = 0;
        const bool smode = red.part || red.packed || red.preloaded;   // the chain also factors tile 0
        for (int d = smode ? 0 : 1; d < T; ++d) {
            const int k = d - 1;
#ifdef PNOL_CHOL_TIMELINE
            const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime(), ck0 = __builtin_amdgcn_s_memtime();
#endif
            if (t == 0) {
                const bool ok = __hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
                                (d == 0 ? spin_ge(pw.ver, 0, info)
                                        : spin_all<2>({pw.ver + d * T + k, pw.ver + d * T + d}, {k, k}, info));
                ok_sh = ok;
            }
            __syncthreads();
            if (!ok_sh) return;
            PNOL_CHOL_STAMP(k, 5)
            const DiagLds L = diag_lds(smem);
            // the previous factor's waves 2 / 3 staged this tile and did half of its products
            const bool pre = lookahead && ew[0] == 1;
            const bool staged = lookahead && ew[0] == 3;   // the tiles only, in pfx / pfc
#ifdef PNOL_CHOL_TIMELINE
            if (t == 0 && k + 1 < 64) g_chol_clk[8 * (k + 1) + 6] = pre ? 1 : (staged ? 2 : 0);
#endif
            if (d == 0) {   // tile 0 as the reduce tasks stored it (sc1 loads)
                const int row = t >> 2, c0 = (t & 3) * 16;
                double v[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) v[q] = ldg<true>(P + (long)row * ldp + c0 + q);
#pragma unroll
                for (int q = 0; q < 16; ++q) diag_put(L, row, c0 + q, v[q]);
            } else if (pre) {
                late_prepare(E, Y, L, wave, lane, true);
            } else {   // W_{d-1} stays in Y after the chain's own factor
                diag_prepare<true>(P, ldp, W, k, X, Y, L, wave, lane, d > 1 || smode, pfx, staged ? pfx : nullptr,
                                   staged ? pfc : nullptr);
            }
            if (t < 6) cnt[t] = 0;   // every read of cnt / ew above is behind a barrier inside
            if (t < 4) ew[t] = 0;    // either prepare
            __syncthreads();
            PNOL_CHOL_STAMP(k, 3)
            // the owners' deferred -L L^T: K blocks 0..3 after diag_prepare, 2..3 after late_prepare,
            // none for tile 0 (stored whole)
            const int kb0 = d == 0 ? 4 : (pre ? 2 : 0);
            if (lookahead)
                factor_diag<false, true, EarlyNext>(L, rinv, cnt, W + (long)d * NB * NB, d, info, nullptr,
                                                    EarlyNext{P, ldp, T, d, pw.ver, diag_w11(L), cnt, lookahead, E}, Y,
                                                    pfx, kb0);
            else   // micro-panel factor: W_d also stays in Y for the next diag_prepare
                factor_diag<false, true>(L, rinv, cnt, W + (long)d * NB * NB, d, info, nullptr, NoEarly(), Y, pfx, kb0);
            PNOL_CHOL_STAMP(k, 4)
            publish(pw.wdone + d, 1);   // its barrier also ends every read of this step's LDS
            PNOL_CRIT(d, 0)
#ifdef PNOL_CHOL_TIMELINE
            chol_tl_mark(k, 0, tl0);
            if (threadIdx.x == 0 && k + 1 < 64) g_chol_clk[8 * (k + 1)] = ck0;
            PNOL_CHOL_STAMP(k, 7)
#endif
        }
        return;
    }

    const int nred = (red.part || red.packed) ? 1 + T * (T + 1) / 2 : 0;   // the reducing form's first tasks
    int pre = -1;   // lane 0: the next task, claimed during the last one's publish (publish_claim)
    for (;;) {   // ---------------- workers
        if (t == 0) {
            task_sh = pre >= 0 ? pre : atomicAdd(pw.counter, 1);
            pre = -1;
        }
        __syncthreads();
        int g = task_sh;
        __syncthreads();   // task_sh is rewritten by the next claim
        if (g >= nred + ntasks) return;
        if (g < nred) {
            red_task(g, red, P, ldp, T, bv, pw, info);
            continue;
        }
        g -= nred;
        PNOL_TASK_T0(g)
        const bool split = red.selfl && red.split;
        // order 1 lets each critical set's tasks (4, or 6 split) wait on unclaimed ones: more
        // workers than that, or step order
        const Task tk = task_of(g, T, red.order == 1 && gridDim.x <= (split ? 7 : 5) ? 0 : red.order, split, red.rowmajor);
        const int k = tk.k;
        const int k0 = k * NB;
        if (tk.j < 0) {   // ---- panel row i: L_ik = A_ik W_k^T, then b_i -= L_ik (W_k b_k)
            const int i = tk.i, i0 = i * NB;
#ifdef PNOL_CHOL_TIMELINE
            const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime();
            if (i == k + 2) PNOL_CRIT(k, 1)
#endif
            // A_ik through column k-1, b_k complete and b_i's earlier updates: usually long
            // before W_k, so A_ik is staged while the workgroup waits for the diagonal chain
            if (t == 0) ok_sh = spin_all<3>({pw.ver + i * T + k, pw.bcnt + k, pw.bcnt + i}, {k, k, k}, info);
            __syncthreads();
            if (!ok_sh) return;
            stage_tile<true>(X, P, ldp, i0, k0);
            if (t == 0) {   // W_k (tile 0 comes from the prep launch)
                ok_sh = (k == 0 && !red.part && !red.packed && !red.preloaded) || spin_ge(pw.wdone + k, 1, info);
#ifdef PNOL_CHOL_TIMELINE
                if (i == k + 2) PNOL_CRIT(k, 2)
#endif
            }
            __syncthreads();
            if (!ok_sh) return;
            stage_tile<true>(Y, W + (long)k * NB * NB, NB, 0, 0);
            __syncthreads();
            PNOL_TASK_READY()
            d4 acc[4];   // this wave's 16-row strip of L_ik (nonzero K blocks of W_k^T only)
            diag_l_strip(acc, X, Y, wave, lane);
            strip_store<true>(acc, Lm, ldp, i0, k0, wave, lane);
            publish(pw.lcnt + i, k + 1);
#ifdef PNOL_CHOL_TIMELINE
            if (i == k + 2) PNOL_CRIT(k, 3)
            if (i == k + 1) PNOL_CRIT(k, 7)
#endif
            strip_to_rows(acc, X, wave, lane);   // X is free (the products finished before the barrier)
            if (t < NB) {
                double s = 0.0;
#pragma unroll 16
                for (int j = 0; j < NB; ++j) s = fma(Y[(j >> 4) * kSub + t * kPad + (j & 15)], ldg<true>(bv + k0 + j), s);
                zsh[t] = s;
            }
            __syncthreads();
            if (t < NB) {
                double s = 0.0;
#pragma unroll 16
                for (int j = 0; j < NB; ++j) s = fma(X[t * (NB + 1) + j], zsh[j], s);
                stg<true>(bv + i0 + t, ldg<true>(bv + i0 + t) - s);
                if (i == k + 1) stg<true>(zv + k0 + t, zsh[t]);
            }
            publish_claim(pw.bcnt + i, k + 1, pw.counter, pre);
            PNOL_TASK_END(k, 0)
#ifdef PNOL_CHOL_TIMELINE
            chol_tl_mark(k, 1, tl0);
#endif
            continue;
        }
        // ---- update tile (i, j) -= L_ik L_jk^T (task_of's order)
        const int i = tk.i, j = tk.j;
#ifdef PNOL_CHOL_TIMELINE
        const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime();
        const bool crit = i == k + 2 && j == k + 1;
        if (crit) PNOL_CRIT(k, 4)
#endif
        if (tk.h >= 0) {
            // Half h (rows 32 h .. 32 h + 31) of a critical update tile (k+2, k+1) or (k+2, k+2):
            // as the whole-tile task below (L_ik and L_jk formed here from A and W_k), on half the
            // output rows -- L_ik's half only (two blocks per wave, diag_l_blocks) for (k+2, k+1),
            // L_jk whole (the output's columns); the diagonal tile needs L_ik whole on both sides.
            // Every output block's MFMA chain is the whole-tile task's (mfma_xyt_half), so the tile
            // is bitwise the same; the second half to finish publishes its version.
            const int h = tk.h, w = wave;
            double* Z = pfx;
            if (t == 0)
                ok_sh = spin_all<3>({pw.ver + i * T + j, pw.ver + i * T + k, pw.ver + j * T + k}, {k, k, k}, info);
            __syncthreads();
            if (!ok_sh) return;
            d4 acc[2];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    acc[mi][r] = ldg<true>(P + (long)(i * NB + (2 * h + mi) * 16 + (lane >> 4) + 4 * r) * ldp + j * NB +
                                           w * 16 + (lane & 15));
            stage_tile<true>(X, P, ldp, i * NB, k0);
            if (i != j) stage_tile<true>(Z, P, ldp, j * NB, k0);
            if (t == 0) ok_sh = (k == 0 && !red.part && !red.packed && !red.preloaded) || spin_ge(pw.wdone + k, 1, info);
            __syncthreads();
            if (!ok_sh) return;
#ifdef PNOL_CHOL_TIMELINE
            if (crit && h == 0) PNOL_CRIT(k, 5)
#endif
            stage_tile<true>(Y, W + (long)k * NB * NB, NB, 0, 0);
            __syncthreads();
            PNOL_TASK_READY()
            if (i != j) {
                const int s = 2 * h + (w >> 1), j0 = (w & 1) ? 1 : 0, j1 = (w & 1) ? 2 : 3;
                d4 lh[2], lj[4];
                diag_l_blocks(lh, X, Y, s, j0, j1, lane);
                diag_l_strip(lj, Z, Y, w, lane);
                __syncthreads();   // every read of the A staging areas is done
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    X[j0 * kSub + (s * 16 + (lane >> 4) + 4 * r) * kPad + (lane & 15)] = lh[0][r];
                    X[j1 * kSub + (s * 16 + (lane >> 4) + 4 * r) * kPad + (lane & 15)] = lh[1][r];
                }
                diag_strip_to_stage(lj, Z, w, lane);
            } else {
                d4 li[4];
                diag_l_strip(li, X, Y, w, lane);
                __syncthreads();
                diag_strip_to_stage(li, X, w, lane);
            }
            __syncthreads();
            mfma_xyt_half(acc, X, i != j ? Z : X, h, w, lane);
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    stg<true>(P + (long)(i * NB + (2 * h + mi) * 16 + (lane >> 4) + 4 * r) * ldp + j * NB + w * 16 +
                                  (lane & 15),
                              acc[mi][r]);
            publish_half_claim(pw.half + i * T + j, pw.ver + i * T + j, k + 1, pw.counter, pre);
            PNOL_TASK_END(k, 2)
#ifdef PNOL_CHOL_TIMELINE
            if (crit) PNOL_CRIT(k, 6)
            chol_tl_mark(k, 2, tl0);
#endif
            continue;
        }
        if (red.selfl && i == k + 2 && j >= k + 1) {
            // The two tiles the chain needs next, (k+2, k+1) and (k+2, k+2): this task forms the L
            // panels it needs itself -- L_ik = A_ik W_k^T (and L_jk), diag_l_strip exactly as the
            // panel tasks form them, so the same bits -- instead of waiting for the panel tasks to
            // store them: the tiles are ready one store / flag / poll / staging round trip earlier
            // (the panel tasks still store L for every other update and run the forward
            // substitution).  A_ik, A_jk and the tile are final through column k - 1 long before
            // W_k, so they are staged while the workgroup waits for the chain.
            double* Z = pfx;   // the chain's look-ahead area (unused by workers) holds A_jk / L_jk
            if (t == 0)
                ok_sh = spin_all<3>({pw.ver + i * T + j, pw.ver + i * T + k, pw.ver + j * T + k}, {k, k, k}, info);
            __syncthreads();
            if (!ok_sh) return;
            d4 acc[2][2];
            acc_load<true>(acc, P, ldp, i * NB, j * NB, wr, wc, lane);
            stage_tile<true>(X, P, ldp, i * NB, k0);
            if (i != j) stage_tile<true>(Z, P, ldp, j * NB, k0);
            if (t == 0) ok_sh = (k == 0 && !red.part && !red.packed && !red.preloaded) || spin_ge(pw.wdone + k, 1, info);
            __syncthreads();
            if (!ok_sh) return;
#ifdef PNOL_CHOL_TIMELINE
            if (crit) PNOL_CRIT(k, 5)
#endif
            stage_tile<true>(Y, W + (long)k * NB * NB, NB, 0, 0);
            __syncthreads();
            PNOL_TASK_READY()
            d4 li[4], lj[4];
            diag_l_strip(li, X, Y, wave, lane);
            if (i != j) diag_l_strip(lj, Z, Y, wave, lane);
            __syncthreads();   // every read of the A staging areas is done
            diag_strip_to_stage(li, X, wave, lane);
            if (i != j) diag_strip_to_stage(lj, Z, wave, lane);
            __syncthreads();
            mfma_xyt<true>(acc, X, i != j ? Z : X, wr, wc, lane);
            acc_store<true>(acc, P, ldp, i * NB, j * NB, wr, wc, lane);
            publish_claim(pw.ver + i * T + j, k + 1, pw.counter, pre);
            PNOL_TASK_END(k, 3)
#ifdef PNOL_CHOL_TIMELINE
            if (crit) PNOL_CRIT(k, 6)
            chol_tl_mark(k, 2, tl0);
#endif
            continue;
        }
        // the tile's earlier updates first: its loads stay in flight while the workgroup waits
        // for the two panels; when all three words are already there (one round of loads), the
        // tile and both panels are loaded together
        if (t == 0) {
            ok_sh = ready_all<3>({pw.ver + i * T + j, pw.lcnt + i, pw.lcnt + j}, {k, k + 1, k + 1})
                        ? 2
                        : spin_ge(pw.ver + i * T + j, k, info);
        }
        __syncthreads();
        const int st0 = ok_sh;
        if (!st0) return;
        d4 acc[2][2];
        acc_load<true>(acc, P, ldp, i * NB, j * NB, wr, wc, lane);
        if (st0 != 2) {
            __syncthreads();   // every read of ok_sh above is done
            if (t == 0) {
                ok_sh = spin_all<2>({pw.lcnt + i, pw.lcnt + j}, {k + 1, k + 1}, info);
#ifdef PNOL_CHOL_TIMELINE
                if (crit) PNOL_CRIT(k, 5)
#endif
            }
            __syncthreads();
            if (!ok_sh) return;
        }
#ifdef PNOL_CHOL_TIMELINE
        else if (crit) PNOL_CRIT(k, 5)
#endif
        stage_tile<true>(X, Lm, ldp, i * NB, k0);
        if (i != j) stage_tile<true>(Y, Lm, ldp, j * NB, k0);
        __syncthreads();
        PNOL_TASK_READY()
        mfma_xyt<true>(acc, X, i != j ? Y : X, wr, wc, lane);
        acc_store<true>(acc, P, ldp, i * NB, j * NB, wr, wc, lane);
        publish_claim(pw.ver + i * T + j, k + 1, pw.counter, pre);
        PNOL_TASK_END(k, 1)
#ifdef PNOL_CHOL_TIMELINE
        if (crit) PNOL_CRIT(k, 6)
        chol_tl_mark(k, 2, tl0);
#endif
    }
}

// ---- backward substitution L^T x = z ------------------------------------------------------
// Workgroup b owns block w = T-1-b.  For c = T-1 .. w+1 it waits for x_c (flag), accumulating
// s_w += L_cw^T x_c with the next L_cw tile prefetched; then x_w = W_w^T (z_w - s_w).
// z_{T-1} = W_{T-1} b_{T-1} is formed here (the factor launches form z_0 .. z_{T-2}).
// The x_c hand-off is the fence-free form of MI355X_MICROARCH.md "Valid forms", table row 1:
// x_w stored with sc1 (relaxed agent atomic) stores by the one storing wave, its vmcnt(0)
// wait, then lane 0's sc1 flag store; the consumer's lane 0 polls with sc1 loads, the block
// barrier follows, and every load of x_c is an sc1 load.  No release / acquire fence (each
// costs ~1.7 us) sits on the 32-step chain.
// GRAN (the default): x_w goes out as 16-byte granules (x_w[t], epoch) -- one sc1 store per
// lane, no vmcnt wait, no flag -- and each consumer wave polls the 16 granules it needs itself
// (MI355X_MICROARCH.md "Valid forms": R2's granule needs no ordering), so a hop costs one
// memory round trip instead of store-drain + flag + poll + load.  xg holds 2 T*64 doubles,
// zeroed whenever the epoch restarts.  The arithmetic is the same either way.
template <bool GRAN>
__global__ __launch_bounds__(256) void k_chol_bwd(const double* __restrict__ Lm, long ldp, int T, int n,
                                                  const double* __restrict__ W, const double* __restrict__ bv,
                                                  const double* __restrict__ zv, double* xw, double* __restrict__ x,
                                                  int* flags, int epoch, int* info,
                                                  const double* __restrict__ xbase = nullptr,
                                                  double* __restrict__ xnext = nullptr,
                                                  double* __restrict__ x_host = nullptr) {
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
        for (int r = 0; r < 16; ++r) dst[r] = Lm[(long)(c * NB + q * 16 + r) * ldp + w0 + j];
    };
    if (w + 1 < T) load_blk(Lv, T - 1);
    double wr[16];   // W_w's column j, rows q*16 .. +16: requested before the chain, not after it
#pragma unroll
    for (int r = 0; r < 16; ++r) wr[r] = Ww[(q * 16 + r) * NB + j];
    const double ep = (double)epoch;
    for (int c = T - 1; c > w; --c) {
        if (c - 1 > w) load_blk(Ln, c - 1);
        double xr[16];
        if constexpr (GRAN) {
            // lanes 0..15 of wave q poll the granules of x_c[q*16 .. q*16+15]
            double* g = xw + 2 * ((long)c * NB + q * 16);   // wave-uniform
            double v = 0.0;
            int it = 0;
            for (;;) {
                const double2 gv = j < 16 ? ld16_sc1(g, (unsigned)(j * 16)) : make_double2(0.0, ep);
                if (__all(gv.y == ep)) {
                    v = gv.x;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                if ((++it & 63) == 0) {
                    if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
                    if (it > kSpin) {
                        atomicCAS(info, 0, kInfoTimeout);
                        return;   // every wave leaves (waves that ended no longer hold the barrier)
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) xr[r] = readlane_d(v, r);
        } else {
            if (t == 0) ok_sh = spin_ge(flags + c, epoch, info);
            __syncthreads();
            if (!ok_sh) return;
            const double* xc = xw + c * NB + q * 16;
#pragma unroll
            for (int r = 0; r < 16; ++r) xr[r] = __hip_atomic_load(xc + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) s = fma(Lv[r], xr[r], s);
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
    for (int r = 0; r < 16; ++r) s = fma(wr[r], vsh[q * 16 + r], s);
    part[q][j] = s;
    __syncthreads();
    if (t < NB) {   // wave 0 alone stores x_w
        const double xv = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
        if constexpr (GRAN) {
            st16_sc1(xw + 2 * (long)w0, (unsigned)(t * 16), make_double2(xv, ep));
        } else {
            __hip_atomic_store(xw + w0 + t, xv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (w0 + t < n) {
            x[w0 + t] = xv;
            if (x_host) x_host[w0 + t] = xv;   // the LM trip's pinned result block (TripMirror)
            // the LM trial point X + sigma (LevenbergMarquardt.cpp:87-90), the add of pnol_add_d
            if (xnext) xnext[w0 + t] = xbase[w0 + t] + xv;
        }
        if constexpr (!GRAN) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (t == 0) __hip_atomic_store(flags + w, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void k_flag_info(int* info, int v) { *info = v; }

}  // namespace

// Solve A sigma = rhs (A SPD, untouched) by the lookahead tile Cholesky; *dinfo (device) != 0
// afterwards when a pivot failed or a chain timed out.
// PNOL_CHOL_PERSIST = 0 / 1 (read per call: the tests switch it) selects the per-step launches
// (method 4) or the persistent form; `variant` 4 / 5 forces one.
static bool chol_persistent(int variant) {
    if (variant == 4) return false;
    if (variant == 5) return true;
    const char* e = std::getenv("PNOL_CHOL_PERSIST");
    return e ? std::atoi(e) != 0 : true;
}

// PNOL_BWD_GRANULE = 0: the backward solve's flag hand-off instead of granules (read per call)
static bool bwd_granules() {
    const char* e = std::getenv("PNOL_BWD_GRANULE");
    return !e || std::atoi(e) != 0;
}

int launch_chol_solve(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo,
                      const double* xbase, double* xnext) {
    return launch_chol_solve_v(ctx, A, lda, rhs, sigma, n, dinfo, 0, xbase, xnext);
}

// The tile Cholesky's workspace (CholWs, pnol_internal.hpp): the per-step / persistent forms and
// the reducing form

static int chol_ws(pnol_ctx* ctx, int n, bool persist, CholWs& w) {
    w.T = (n + NB - 1) / NB;
    w.N = w.T * NB;
    w.ldp = w.N;
    const int T = w.T, N = w.N;
    void *P = nullptr, *Lm = nullptr, *W = nullptr, *bv = nullptr, *zv = nullptr, *xw = nullptr, *pf = nullptr;
    PNOL_CHECK(ws_get(ctx, "chol4_P", sizeof(double) * (size_t)N * w.ldp, &P));
    PNOL_CHECK(ws_get(ctx, "chol4_L", sizeof(double) * (size_t)N * w.ldp, &Lm));
    PNOL_CHECK(ws_get(ctx, "chol4_W", sizeof(double) * (size_t)T * NB * NB, &W));
    PNOL_CHECK(ws_get(ctx, "chol4_b", sizeof(double) * (size_t)N, &bv));
    PNOL_CHECK(ws_get(ctx, "chol4_z", sizeof(double) * (size_t)N, &zv));
    // the backward solve's hand-off words: x granules (x, epoch) -- 2 N doubles, zeroed when
    // allocated and whenever the epoch restarts (a stale granule must never match)
    // (the flag form keeps its own buffer, so the two layouts never share memory)
    w.gran = bwd_granules();
    if (w.gran) {
        auto it = ctx->ws.bufs.find("chol4_xg");
        const void* before = it == ctx->ws.bufs.end() ? nullptr : it->second.first;
        PNOL_CHECK(ws_get(ctx, "chol4_xg", sizeof(double) * 2 * (size_t)N, &xw));
        if (xw != before) PNOL_HIP(hipMemsetAsync(xw, 0, sizeof(double) * 2 * (size_t)N, ctx->stream));
    } else {
        PNOL_CHECK(ws_get(ctx, "chol4_x", sizeof(double) * (size_t)N, &xw));
    }
    if (T > ctx->chol4_cap || ctx->chol4_epoch > (1 << 29)) {
        void* f = nullptr;
        const int cap = std::max(T, ctx->chol4_cap);
        PNOL_CHECK(ws_get(ctx, "chol4_flags", sizeof(int) * (size_t)2 * cap, &f));
        PNOL_HIP(hipMemsetAsync(f, 0, sizeof(int) * (size_t)2 * cap, ctx->stream));
        if (w.gran) PNOL_HIP(hipMemsetAsync(xw, 0, sizeof(double) * 2 * (size_t)N, ctx->stream));   // epoch restarts
        ctx->chol4_flags = (int*)f;
        ctx->chol4_cap = cap;
        ctx->chol4_epoch = 0;
    }
    w.rowflag = ctx->chol4_flags;
    w.bwdflag = ctx->chol4_flags + ctx->chol4_cap;
    w.npf = 3 * T + 2 * T * T + 1;   // [wdone | lcnt | bcnt | ver | claim counter | half counts]
    if (persist) PNOL_CHECK(ws_get(ctx, "chol5_words", sizeof(int) * (size_t)w.npf, &pf));
    w.P = (double*)P; w.Lm = (double*)Lm; w.W = (double*)W; w.bv = (double*)bv; w.zv = (double*)zv;
    w.xw = (double*)xw; w.pf = (int*)pf;
    return PNOL_OK;
}

// k_chol_persist: steps 0 .. T-2 (the reducing form: the reduce tasks first, and tile 0 too)
static int chol_persist_launch(pnol_ctx* ctx, hipStream_t st, const CholWs& w, int* dinfo, const RedArgs& red) {
    const int T = w.T;
    RedArgs rp = red;
    {
        const char* es = std::getenv("PNOL_CHOL_SELFL");   // read per call (A/B, tests)
        rp.selfl = !es || std::atoi(es) != 0;
        const char* eh = std::getenv("PNOL_CHOL_SPLIT");
        rp.split = !eh || std::atoi(eh) != 0;
        const char* er = std::getenv("PNOL_CHOL_ROWMAJOR");
        rp.rowmajor = !er || std::atoi(er) != 0;
    }
    int ntasks = 0;
    for (int R = T - 1; R >= 1; --R) ntasks += step_tasks(R, rp.selfl && rp.split);
    // tuning knob (read per call): PNOL_CHOL5_WORKERS = worker workgroups; one per CU
    // (the look-ahead areas already hold the static LDS to one workgroup per CU).
    // PNOL_CHOL_LOOKAHEAD = 0 turns the diagonal chain's look-ahead off (read per call).
    const char* ew = std::getenv("PNOL_CHOL5_WORKERS");
    const char* el = std::getenv("PNOL_CHOL_LOOKAHEAD");
    // > 0: the look-ahead gives up once wave 0 has finished that many columns of the tile
    // (0 off; above 64: the factor waits for the next tiles).  The next tiles wait on a panel and
    // an update task (~6 us each after W_{d-1}), so a look-ahead that starts late runs past the
    // factor (its staging and MFMAs take ~9k cycles) and costs more than the prepare it saves.
    // Measured at n = 2048 with the micro-panel factor (tools/microbench/chol_timeline.hip, two
    // rounds, profiles/r05_lookahead_sweep.txt): 0: 0.585-0.587 ms, 32: 0.582-0.587, 40: 0.579-
    // 0.585, 48: 0.571-0.578 (default), 56: 0.588-0.597, 64: 0.596-0.601; LM bench 52 vs 64: 3
    // of 3 same-box pairs faster (327-328 vs 324-328 LM iters/s).  (Round 2's factor: 64 best.)
    // Tiles that come after the cutoff but before the factor's last column are still staged
    // (EarlyNext mode 3): their step's prepare skips the loads, ~4.5k of its ~10.5k cycles, and
    // the solve goes 0.559-0.561 -> 0.553-0.556 ms; with it every cutoff from 1 to 48 measures
    // the same (56: 0.562-0.566), profiles/r05_lookahead_sweep.txt.
    const int lookahead = el ? std::max(0, std::atoi(el)) : 48;
    {
        // order 1 (each step's critical tasks a step early) lets up to four workers wait on tasks
        // nobody has claimed yet, so it needs more than four workers resident.  A GPU shared by
        // several processes may hold fewer (a 4-process run at cfg 3 stalled one trip until the
        // spin cap, profiles/r06_chol_contention_4p_cfg3.json): ranks sharing the GPU over the
        // host backend, and a context that has seen a timed-out wait, claim in step order.
        const char* eo = std::getenv("PNOL_CHOL_ORDER");
        rp.order = eo ? (std::atoi(eo) != 0 ? 1 : 0) : ((ctx->chol_order0 || comm_shares_device()) ? 0 : 1);
    }
    const int slots = std::max(ctx->num_cu, 1) - 1;
    const int want = ew ? std::atoi(ew) : slots;
    const int nred = (red.part || red.packed) ? 1 + T * (T + 1) / 2 : 0;
    const int workers = std::max(1, std::min(ntasks + nred, want));
    hipLaunchKernelGGL(k_chol_persist, dim3(1 + workers), dim3(256), 0, st, w.P, w.Lm, w.ldp, T, w.W, w.bv, w.zv, w.pf,
                       ntasks, dinfo, lookahead, rp);
    return launch_check();
}

// the backward solve (+ the trial point)
static int chol_bwd_launch(pnol_ctx* ctx, hipStream_t st, const CholWs& w, int n, double* sigma, int* dinfo,
                           const double* xbase, double* xnext, bool trip = false) {
    const int epoch = ++ctx->chol4_epoch;
    if (w.gran && ((uintptr_t)w.xw & 15) != 0) return PNOL_ERR_ARG;   // granules need 16-byte alignment
    if (w.gran)
        hipLaunchKernelGGL(k_chol_bwd<true>, dim3(w.T), dim3(256), 0, st, (const double*)w.Lm, w.ldp, w.T, n,
                           (const double*)w.W, (const double*)w.bv, (const double*)w.zv, w.xw, sigma, w.bwdflag, epoch,
                           dinfo, xbase, xnext, ctx->trip_mirror.sigma);
    else
        hipLaunchKernelGGL(k_chol_bwd<false>, dim3(w.T), dim3(256), 0, st, (const double*)w.Lm, w.ldp, w.T, n,
                           (const double*)w.W, (const double*)w.bv, (const double*)w.zv, w.xw, sigma, w.bwdflag, epoch,
                           dinfo, xbase, xnext, ctx->trip_mirror.sigma);
    PNOL_CHECK(launch_check());
    // test hook (tests/test_gpu_solvers.py, tests/test_gpu_mpi.py; read per call: the tests flip
    // it, per rank too): a value > 0 reports a non-positive pivot on every Cholesky solve, so the
    // callers' LU paths run on an SPD system; kCholTimeout (-7) reports a timed-out wait on the LM
    // trip's solves only (`trip`: the reducing form, pnol_solve_step_d), so the caller's relaunch
    // -- pnol_solve_d, which is not forced -- runs
    if (const char* e = std::getenv("PNOL_CHOL_FORCE_FALLBACK")) {
        const int v = std::atoi(e);
        if (v > 0 || (v == kCholTimeout && trip)) {
            hipLaunchKernelGGL(k_flag_info, dim3(1), dim3(1), 0, st, dinfo, v);
            return launch_check();
        }
    }
    return PNOL_OK;
}

int launch_chol_solve_v(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo,
                        int variant, const double* xbase, double* xnext) {
    CholWs w;
    const bool persist = chol_persistent(variant) && (n + NB - 1) / NB >= 2;
    PNOL_CHECK(chol_ws(ctx, n, persist, w));
    const int T = w.T, N = w.N;
    for (int k = -1; k <= (persist ? -1 : T - 2); ++k) {
        const int R = T - 1 - k;
        const int grid = k < 0 ? 2 + std::min(N, 1024) : R + R * (R + 1) / 2;
        const int epoch = ++ctx->chol4_epoch;
        hipLaunchKernelGGL(k_chol_step, dim3(grid), dim3(256), 0, ctx->stream, w.P, w.Lm, w.ldp, T, k, w.W, w.bv, w.zv,
                           w.rowflag, epoch, dinfo, A, (long)lda, n, rhs, w.pf, persist ? w.npf : 0);
    }
    if (persist) PNOL_CHECK(chol_persist_launch(ctx, ctx->stream, w, dinfo, RedArgs{}));
    // (xnext: the LM loop's trip solve -- pnol_solve_step_d -- which the timeout test hook may force)
    return chol_bwd_launch(ctx, ctx->stream, w, n, sigma, dinfo, xbase, xnext, xnext != nullptr);
}

// The reducing form's prep: the persistent form's progress words -- the tile versions and b's
// block-row words at -1 (not yet stored by the reduce tasks), the rest 0 --, b's padding past n,
// P's padding (identity on the diagonal past n, as the copy of A gives), info = 0.
__global__ __launch_bounds__(256) void k_chol_reducing_prep(double* __restrict__ P, long ldp, int T, int n,
                                                            double* __restrict__ bv, int* __restrict__ pflags,
                                                            int npflags, int* __restrict__ info, int vinit,
                                                            int* __restrict__ zc, int nz) {
    const int N = T * NB, tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    const int b0 = 2 * T, v1 = 3 * T + T * T;   // [bcnt | ver]
    for (int q = tid; q < npflags; q += nth) pflags[q] = (q >= b0 && q < v1) ? vinit : 0;
    for (int q = tid; q < nz; q += nth) zc[q] = 0;   // the caller's counters (k_syrk_red's tile counts)
    for (int r = n + tid; r < N; r += nth) bv[r] = 0.0;
    if (n < N) {
        const long pad = (long)(N - n) * N + (long)n * (N - n);   // rows >= n, then columns >= n of rows < n
        for (long e = tid; e < pad; e += nth) {
            int r, c;
            if (e < (long)(N - n) * N) {
                r = n + (int)(e / N);
                c = (int)(e % N);
            } else {
                const long f = e - (long)(N - n) * N;
                r = (int)(f / (N - n));
                c = n + (int)(f % (N - n));
            }
            P[(long)r * ldp + c] = r == c ? 1.0 : 0.0;
        }
    }
    if (tid == 0) *info = 0;
}

int launch_chol_reducing_prep(pnol_ctx* ctx, int n, int* dinfo, CholRed& cr) {
    if (!dinfo || n <= NB) return PNOL_ERR_ARG;
    cr.n = n;
    cr.dinfo = dinfo;
    return chol_ws(ctx, n, true, cr.w);
}

int launch_chol_reducing_start(pnol_ctx* ctx, const CholRed& cr, bool preloaded, int* zc, int nz) {
    const CholWs& w = cr.w;
    const int n = cr.n;
    const long pad = (long)(w.N - n) * w.N + (long)n * (w.N - n), work = std::max<long>(pad, w.npf);
    hipLaunchKernelGGL(k_chol_reducing_prep, dim3((unsigned)std::max<long>(1, std::min<long>(1024, (work + 255) / 256))),
                       dim3(256), 0, ctx->stream, w.P, w.ldp, w.T, n, w.bv, w.pf, w.npf, cr.dinfo, preloaded ? 0 : -1,
                       zc, zc ? nz : 0);
    return launch_check();
}

// the persistent factorisation of the matrix a reduce launch left in P (and b in bv), then the
// backward solve and xnext = xbase + sigma (launch_chol_reducing_start(preloaded) first)
int launch_chol_preloaded_run(pnol_ctx* ctx, hipStream_t st, const CholRed& cr, double* sigma, const double* xbase,
                              double* xnext) {
    if (!sigma) return PNOL_ERR_ARG;
    RedArgs red;
    red.n = cr.n;
    red.preloaded = true;
    PNOL_CHECK(chol_persist_launch(ctx, st, cr.w, cr.dinfo, red));
    return chol_bwd_launch(ctx, st, cr.w, cr.n, sigma, cr.dinfo, xbase, xnext, true);
}

int launch_chol_reducing_run(pnol_ctx* ctx, hipStream_t st, const CholRed& cr, const double* part, int sub,
                             const double* jp, double lambda, double* rhs, double* sigma, const double* xbase,
                             double* xnext) {
    if (!part || !jp || !rhs || !sigma || sub < 1) return PNOL_ERR_ARG;
    RedArgs red;
    red.part = part;
    red.sub = sub;
    red.n = cr.n;
    red.lambda = lambda;
    red.jp = jp;
    red.rhs = rhs;
    PNOL_CHECK(chol_persist_launch(ctx, st, cr.w, cr.dinfo, red));
    return chol_bwd_launch(ctx, st, cr.w, cr.n, sigma, cr.dinfo, xbase, xnext, true);
}

// LevMarqMPI: the same from the allgathered, summed tiles (packed) and the formed rhs
int launch_chol_reducing_run_packed(pnol_ctx* ctx, hipStream_t st, const CholRed& cr, const double* packed, long slot,
                                    int tpr, const double* rhs, double lambda, double* sigma, const double* xbase,
                                    double* xnext) {
    if (!packed || !rhs || !sigma || tpr < 1) return PNOL_ERR_ARG;
    RedArgs red;
    red.packed = packed;
    red.slot = slot;
    red.tpr = tpr;
    red.rhs_in = rhs;
    red.n = cr.n;
    red.lambda = lambda;
    PNOL_CHECK(chol_persist_launch(ctx, st, cr.w, cr.dinfo, red));
    return chol_bwd_launch(ctx, st, cr.w, cr.n, sigma, cr.dinfo, xbase, xnext, true);
}

}  // namespace pnol
