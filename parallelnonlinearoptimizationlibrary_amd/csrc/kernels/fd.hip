// fd.hip -- device objectives and the batched forward-difference engine (gfx950).
//
// Replaces the N+1 sequential objEval calls of Objective::gradientApproximation
// (PNOL_Objective.cpp:12-34) and MultiObjective::gradientApproximation (:165-197), and their
// round-robin MPI forms (:88-159, :202-299): every perturbed point x + h_j e_j of a column
// block [j0, j0+cnt) is evaluated in one launch.  Each point's objective value is computed
// in the objective's own sequential operation order (one thread or one register tile per
// point), so the device FD values equal the host objEval's bit for bit wherever the
// objective uses no transcendental (Rosenbrock, quadratic, cubic with pow(x,3) tabulated on
// the host, the fma-chain linear residual).  The perturbed coordinate is formed exactly as
// the reference forms XdX[j] = X[j] + dX[j].
//
//   k_scalar_fd_values   scalar objectives: one thread per point, x staged through LDS
//   k_multi_fd           ExpCurve / Cubic (tiny n): one thread per (point, residual)
//   k_linres_eval        r = A x - y: one thread per residual row, A tiles staged in LDS
//   k_linres_fdP         all points of a tile list at once on the row-panel copy of A: one
//                        residual row per lane, each point's fma chain in a register
//                        (R = A [x + h_j e_j]_j, epilogue J = ((R - y) - F0) / h; no MFMA:
//                        this is the objective, evaluated like user code would be); waves
//                        resume from base-chain checkpoints and broadcast x outside the
//                        perturbation window
#include "../pnol_internal.hpp"
#include "../pnol_comm.hpp"

#include <algorithm>
#include <cstring>
#include <functional>
#include <memory>
#include <cstdlib>
#include <vector>

namespace pnol {
namespace {

__device__ __forceinline__ double u01(unsigned long long seed, unsigned long long idx) {
    unsigned long long z = seed + (idx + 1ULL) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    return (double)(z >> 11) * 0x1.0p-53;
}

// ---- scalar objectives ------------------------------------------------------------------
constexpr int kChunk = 1024;

// Point p in [0, cnt] (p == cnt: the base point); vals[p] = f(x_p).
template <int KIND>
__global__ __launch_bounds__(256) void k_scalar_fd_values(const double* __restrict__ x, const double* __restrict__ h,
                                                          int n, int i0, int cnt, const double* __restrict__ p0,
                                                          const double* __restrict__ p1, double power,
                                                          double* __restrict__ vals) {
    __shared__ double xs[kChunk + 1];
    __shared__ double ds[KIND == PNOL_OBJ_QUADRATIC ? kChunk : 1];
    __shared__ double bs[KIND == PNOL_OBJ_QUADRATIC ? kChunk : 1];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = p <= cnt;
    const int j = (active && p < cnt) ? i0 + p : -1;          // perturbed coordinate, -1 = base
    const double xj = (j >= 0) ? x[j] + h[j] : 0.0;            // XdX[j] = X[j] + dX[j]
    double f = 0.0;
    for (int c0 = 0; c0 < n; c0 += kChunk) {
        const int len = min(kChunk, n - c0);
        __syncthreads();
        for (int e = threadIdx.x; e <= len && c0 + e < n; e += blockDim.x) xs[e] = x[c0 + e];
        if (KIND == PNOL_OBJ_QUADRATIC)
            for (int e = threadIdx.x; e < len; e += blockDim.x) { ds[e] = p0[c0 + e]; bs[e] = p1[c0 + e]; }
        __syncthreads();
        if (!active) continue;
        if (KIND == PNOL_OBJ_ROSENBROCK) {
            // value += 100 (x_{k+1} - x_k^2)^2 + (1 - x_k)^2, k < n-1  (ExampleObjectives.hpp:93-96)
            const int kmax = min(len, n - 1 - c0);
            for (int e = 0; e < kmax; ++e) {
                const int k = c0 + e;
                double xk = (k == j) ? xj : xs[e];
                double xk1 = (k + 1 == j) ? xj : xs[e + 1];
                double t = xk1 - xk * xk;
                double u = 1.0 - xk;
                f = f + (100.0 * (t * t) + u * u);
            }
        } else if (KIND == PNOL_OBJ_QUADRATIC) {
            for (int e = 0; e < len; ++e) {
                const int k = c0 + e;
                double xk = (k == j) ? xj : xs[e];
                double t = (0.5 * ds[e] * xk) * xk - bs[e] * xk;
                if (k + 1 < n) {
                    double xk1 = (k + 1 == j) ? xj : xs[e + 1];
                    t = t + (0.25 * xk) * xk1;
                }
                f = f + t;
            }
        } else {  // PNOL_OBJ_POWER (ExampleObjectives.hpp:219-222)
            for (int e = 0; e < len; ++e) {
                const int k = c0 + e;
                double xk = (k == j) ? xj : xs[e];
                f = f + (power == 2.0 ? xk * xk : pow(xk, power));
            }
        }
    }
    if (active) vals[p] = f;
}

// vals[k] = f(X_k) for the row-major points Xs (npts x n): a batch of single evaluations
// (line-search trial points, pool entries).  One workgroup per point: the terms of a 2048-
// coordinate chunk are formed in parallel into LDS, then one lane adds them in index order --
// the objective's own sequential sum, so the host objEval's bits.
constexpr int kEvChunk = 2048;
template <int KIND>
__global__ __launch_bounds__(256) void k_eval_batch(const double* __restrict__ Xs, int n,
                                                    const double* __restrict__ p0, const double* __restrict__ p1,
                                                    double power, double* __restrict__ vals) {
    __shared__ double terms[kEvChunk];
    const double* __restrict__ X = Xs + (long)blockIdx.x * n;
    const int nt = KIND == PNOL_OBJ_ROSENBROCK ? n - 1 : n;   // Rosenbrock: k < n - 1
    double f = 0.0;
    for (int c0 = 0; c0 < nt; c0 += kEvChunk) {
        const int len = min(kEvChunk, nt - c0);
        for (int e = threadIdx.x; e < len; e += blockDim.x) {
            const int i = c0 + e;
            const double xi = X[i];
            double t;
            if (KIND == PNOL_OBJ_ROSENBROCK) {
                const double a = X[i + 1] - xi * xi, u = 1.0 - xi;
                t = 100.0 * (a * a) + u * u;
            } else if (KIND == PNOL_OBJ_QUADRATIC) {
                t = (0.5 * p0[i] * xi) * xi - p1[i] * xi;
                if (i + 1 < n) t = t + (0.25 * xi) * X[i + 1];
            } else {
                t = power == 2.0 ? xi * xi : pow(xi, power);
            }
            terms[e] = t;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int e = 0;
            for (; e + 8 <= len; e += 8) {
                double t8[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) t8[q] = terms[e + q];
#pragma unroll
                for (int q = 0; q < 8; ++q) f = f + t8[q];
            }
            for (; e < len; ++e) f = f + terms[e];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) vals[blockIdx.x] = f;
}

// ---- FD gradient of the scalar objectives, term form ------------------------------------
// f = sum_k t_k is accumulated in k order; perturbing coordinate j changes at most the terms
// touching x_j (Rosenbrock / quadratic: t_{j-1} and t_j; power: t_j).  So every point's sum is
// the sequence of the base terms T_k = t_k(x) with those two replaced, and T is formed once
// (k_scalar_terms).  A wave owns 64 consecutive points: outside the window of terms any of its
// lanes perturbs, the addend T_k is the same for all lanes -- one scalar load feeding one
// v_add_f64 per term; inside the window each lane forms its own perturbed terms exactly as the
// objective does.  Same additions in the same order as evaluating each point from scratch
// (bitwise), one dependent add per term on the critical path instead of the whole term.
template <int KIND>
__device__ __forceinline__ int scalar_nterms(int n) { return KIND == PNOL_OBJ_ROSENBROCK ? max(n - 1, 0) : n; }

// term k at the point whose coordinates k, k + 1 are xk, xk1 (the objective's own expression)
template <int KIND>
__device__ __forceinline__ double scalar_term(int k, int n, double xk, double xk1, const double* __restrict__ p0,
                                              const double* __restrict__ p1, double power) {
    if (KIND == PNOL_OBJ_ROSENBROCK) {
        const double t = xk1 - xk * xk, u = 1.0 - xk;   // ExampleObjectives.hpp:93-96
        return 100.0 * (t * t) + u * u;
    } else if (KIND == PNOL_OBJ_QUADRATIC) {
        double t = (0.5 * p0[k] * xk) * xk - p1[k] * xk;
        if (k + 1 < n) t = t + (0.25 * xk) * xk1;
        return t;
    } else {
        return power == 2.0 ? xk * xk : pow(xk, power);
    }
}

// xcopy (the host-pointer gradient): x is the caller's pinned host block, read once here over
// PCIe and copied to device memory for the chain kernel -- no separate host-to-device copy;
// likewise hsrc -> hdst, the step vector when it changed since the last call
template <int KIND>
__global__ __launch_bounds__(256) void k_scalar_terms(const double* __restrict__ x, int n, const double* __restrict__ p0,
                                                      const double* __restrict__ p1, double power,
                                                      double* __restrict__ T, double* __restrict__ xcopy = nullptr,
                                                      const double* __restrict__ hsrc = nullptr,
                                                      double* __restrict__ hdst = nullptr) {
    const int nt = scalar_nterms<KIND>(n);
    const int lane = threadIdx.x & 63;
    const int stride = gridDim.x * blockDim.x;
    for (int k0 = blockIdx.x * blockDim.x; k0 < n; k0 += stride) {   // whole waves (uniform trip count)
        const int k = k0 + threadIdx.x;
        const double xk = k < n ? x[k] : 0.0;
        // x[k + 1] from the next lane (one read of host memory per element); lane 63 reads its own
        double xk1 = __shfl_down(xk, 1, 64);
        if (lane == 63) xk1 = k + 1 < n ? x[k + 1] : 0.0;
        if (k + 1 >= n) xk1 = 0.0;
        if (xcopy && k < n) xcopy[k] = xk;
        if (hsrc && k < n) hdst[k] = hsrc[k];
        if (k < nt) T[k] = scalar_term<KIND>(k, n, xk, xk1, p0, p1, power);
    }
}

// Points q in [0, cnt] (q == cnt: the base point): vals[q] = f(x + h_j e_j), j = i0 + q.
// T streams through LDS in double-buffered chunks (cooperative coalesced loads of chunk c + 1
// in flight while chunk c is summed); the uniform addends are LDS broadcast reads, which --
// unlike scalar loads, whose completion order is not fixed -- stay in flight sixteen at a time
// ahead of the dependent add chain.  Each lane forms its two perturbed terms (t_{j-1}, t_j at
// x + h_j e_j) before the chain, so inside the window the substitution is two selects.
// Measured chain step (tools/microbench/add_chain.hip, one wave): 5.3 cycles with the addends in
// VGPRs (the dependent v_add_f64 latency), 9.7 from LDS 16 ahead, 12.7 from LDS 8 ahead, ~21
// from scalar loads.
constexpr int kTermChunk = 2048;   // 16 KB of terms per LDS stage (two stages)
constexpr int kChainAhead = 16;

// f + Tc[k0] + Tc[k0 + 1] + ... + Tc[k1 - 1], left to right.  Three register blocks of
// kChainAhead addends rotate (no copies): the LDS reads of block b + 2 are issued before the adds
// of block b, so two blocks of reads are in flight across each block of the dependent chain.
// The sched_barriers keep the compiler from sinking the reads behind the adds (which left one
// block's latency exposed per iteration).
__device__ __forceinline__ void chain_ld(double (&v)[kChainAhead], const double* __restrict__ Tc, int k) {
#pragma unroll
    for (int q = 0; q < kChainAhead; q += 2) {
        const double2 w = *reinterpret_cast<const double2*>(Tc + k + q);
        v[q] = w.x;
        v[q + 1] = w.y;
    }
}
__device__ __forceinline__ double chain_add(double f, const double (&v)[kChainAhead]) {
#pragma unroll
    for (int q = 0; q < kChainAhead; ++q) f = f + v[q];
    return f;
}
__device__ __forceinline__ double chain_sum(double f, const double* __restrict__ Tc, int k0, int k1) {
    constexpr int D = kChainAhead;
    int k = k0;
    // scalar head up to a 16-byte boundary of the LDS chunk (Tc + k even)
    if ((k & 1) && k < k1) f = f + Tc[k++];
    if (k1 - k >= 3 * D) {
        double A[D], B[D], C[D];
        chain_ld(A, Tc, k);
        chain_ld(B, Tc, k + D);
        for (; k + 6 * D <= k1; k += 3 * D) {
            __builtin_amdgcn_sched_barrier(0);
            chain_ld(C, Tc, k + 2 * D);
            __builtin_amdgcn_sched_barrier(0);
            f = chain_add(f, A);
            __builtin_amdgcn_sched_barrier(0);
            chain_ld(A, Tc, k + 3 * D);
            __builtin_amdgcn_sched_barrier(0);
            f = chain_add(f, B);
            __builtin_amdgcn_sched_barrier(0);
            chain_ld(B, Tc, k + 4 * D);
            __builtin_amdgcn_sched_barrier(0);
            f = chain_add(f, C);
        }
        // A, B hold [k, k + 2D); k + 3D <= k1 < k + 6D
        __builtin_amdgcn_sched_barrier(0);
        chain_ld(C, Tc, k + 2 * D);
        f = chain_add(f, A);
        f = chain_add(f, B);
        f = chain_add(f, C);
        k += 3 * D;
    }
    for (; k < k1; ++k) f = f + Tc[k];
    return f;
}

template <int KIND>
__global__ __launch_bounds__(256) void k_scalar_fd_chain(const double* __restrict__ x, const double* __restrict__ h,
                                                         int n, int i0, int cnt, const double* __restrict__ p0,
                                                         const double* __restrict__ p1, double power,
                                                         const double* __restrict__ T, double* __restrict__ vals) {
    __shared__ __attribute__((aligned(16))) double Ts[2][kTermChunk];
    constexpr int kPer = kTermChunk / 2 / 256;   // double2 loads per thread per chunk
    const int lane = threadIdx.x & 63;
    const int q0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)) * 64);
    const int q = q0 + lane;
    const bool active = q <= cnt;
    const int j = (active && q < cnt) ? i0 + q : -1;            // perturbed coordinate, -1: base
    const int nt = scalar_nterms<KIND>(n);
    // this lane's perturbed terms at XdX[j] = X[j] + dX[j]: t_j and (not for power) t_{j-1}
    double tj = 0.0, tjm1 = 0.0;
    if (j >= 0) {
        const double xj = x[j] + h[j];
        if (j < nt) tj = scalar_term<KIND>(j, n, xj, j + 1 < n ? x[j + 1] : 0.0, p0, p1, power);
        if (KIND != PNOL_OBJ_POWER && j >= 1 && j - 1 < nt) tjm1 = scalar_term<KIND>(j - 1, n, x[j - 1], xj, p0, p1, power);
    }
    // terms some lane of the wave perturbs: [w0, w1) (empty for a wave of base / idle lanes)
    const int jlo = i0 + q0, jhi = i0 + min(q0 + 63, cnt - 1);
    int w0 = nt, w1 = nt;
    if (q0 < cnt) {
        w0 = max(0, min(KIND == PNOL_OBJ_POWER ? jlo : jlo - 1, nt));
        w1 = max(w0, min(jhi + 1, nt));
    }
    // chunk c of T into registers (zero past nt; only [c0, c1) is ever read)
    double2 pre[kPer];
    auto fetch = [&](int c0) {
#pragma unroll
        for (int r = 0; r < kPer; ++r) {
            const int e = c0 + 2 * (threadIdx.x + 256 * r);
            pre[r] = make_double2(e < nt ? T[e] : 0.0, e + 1 < nt ? T[e + 1] : 0.0);
        }
    };
    auto stash = [&](double* dst) {
#pragma unroll
        for (int r = 0; r < kPer; ++r) reinterpret_cast<double2*>(dst)[threadIdx.x + 256 * r] = pre[r];
    };
    double f = 0.0;
    fetch(0);
    stash(Ts[0]);
    __syncthreads();
    for (int c0 = 0, cb = 0; c0 < nt; c0 += kTermChunk, cb ^= 1) {
        const int c1 = min(c0 + kTermChunk, nt);
        const bool more = c1 < nt;
        if (more) fetch(c1);                       // in flight during this chunk's chain
        const double* __restrict__ Tc = Ts[cb] - c0;   // Tc[k] = T[k] for k in [c0, c1)
        const int e0 = min(max(w0, c0), c1);
        f = chain_sum(f, Tc, c0, e0);
        const int e1 = min(max(w1, c0), c1);
        for (int k = e0; k < e1; ++k) {
            double t = Tc[k];
            t = k == j ? tj : t;
            if (KIND != PNOL_OBJ_POWER) t = k + 1 == j ? tjm1 : t;
            f = f + t;
        }
        f = chain_sum(f, Tc, e1, c1);
        if (more) stash(Ts[cb ^ 1]);
        __syncthreads();
    }
    if (active) vals[q] = f;
}

__global__ void k_scalar_fd_finish(const double* __restrict__ vals, const double* __restrict__ h, int i0, int cnt,
                                   double* __restrict__ f0, double* __restrict__ g) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const double F = vals[cnt];
    if (p == 0 && f0) *f0 = F;
    if (p < cnt) g[p] = (vals[p] - F) / h[i0 + p];
}

// ---- small residual objectives (ExpCurve, Cubic) ---------------------------------------
template <int KIND>
__device__ __forceinline__ double multi_residual(const double* X, int k, const double* xd, const double* yd,
                                                 const double* p3) {
    if (KIND == PNOL_OBJ_EXPCURVE) {
        double func = X[0] * exp(X[1] * xd[k]) + X[2];        // ExampleObjectives.hpp:128
        return yd[k] - func;
    } else {
        double xv = xd[k];                                      // :175, pow(x,3) tabulated
        double func = X[0] * p3[k] + X[1] * (xv * xv) + X[2] * xv + X[3];
        return yd[k] - func;
    }
}

template <int KIND>
__global__ void k_multi_eval(const double* __restrict__ x, int n, int m, const double* __restrict__ xd,
                             const double* __restrict__ yd, const double* __restrict__ p3, double* __restrict__ F) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    double X[4] = {0, 0, 0, 0};
    for (int q = 0; q < n && q < 4; ++q) X[q] = x[q];
    F[k] = multi_residual<KIND>(X, k, xd, yd, p3);
}

template <int KIND>
__global__ void k_multi_fd(const double* __restrict__ x, const double* __restrict__ h, int n, int m, int j0, int cnt,
                           const double* __restrict__ xd, const double* __restrict__ yd, const double* __restrict__ p3,
                           const double* __restrict__ F0, double* __restrict__ JT, long ldjt) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int p = blockIdx.y;
    if (k >= m || p >= cnt) return;
    const int j = j0 + p;
    double X[4] = {0, 0, 0, 0};
    for (int q = 0; q < n && q < 4; ++q) X[q] = x[q];
    X[j] = x[j] + h[j];
    const double Fj = multi_residual<KIND>(X, k, xd, yd, p3);
    JT[(long)p * ldjt + k] = (Fj - F0[k]) / h[j];
}

// ---- linear residual r = A x - y --------------------------------------------------------
// One residual per lane of wave 0, an fma chain over k ascending (the objective's definition).
// 64 rows per 256-thread workgroup: all four waves stream the next 64 x 128 tile of A into
// registers (coalesced 1 KiB row segments, 16-byte loads) while wave 0 runs the chains of
// the current tile out of LDS -- the chain is sequential, the bytes are not.
constexpr int kEvRows = 64, kEvK = 128, kEvPad = kEvK + 1;
constexpr int kCkpt = 16;   // checkpoint stride of the base chain (== the FD kernel's K stage)

// CKPT: also store the chain value before every 16th column, C[(k / 16) * m + row] for
// k = 16, 32, ... (the prefix every FD point with a perturbed column >= k shares).
template <bool VEC, bool CKPT>
__global__ __launch_bounds__(256) void k_linres_eval(const double* __restrict__ A, const double* __restrict__ x,
                                                     const double* __restrict__ y, int m, int n,
                                                     double* __restrict__ F, double* __restrict__ C) {
    __shared__ double As[kEvRows * kEvPad];
    __shared__ double xs[kEvK];
    const int t = threadIdx.x;
    const int r0 = blockIdx.x * kEvRows;
    // thread t stages rows (t >> 6) + 4q, columns 2*(t & 63) .. +1  (q = 0..15)
    const int lr = t >> 6, lc = 2 * (t & 63);
    double2 reg[16];
    auto load = [&](int k0) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = min(r0 + lr + 4 * q, m - 1);
            const int c = k0 + lc;
            const double* p = A + (long)row * n + c;
            if (VEC && c + 1 < n) {
                // A is streamed once per evaluation: non-temporal 16-byte loads
                reg[q].x = __builtin_nontemporal_load(p);
                reg[q].y = __builtin_nontemporal_load(p + 1);
            } else {
                reg[q].x = c < n ? p[0] : 0.0;
                reg[q].y = c + 1 < n ? p[1] : 0.0;
            }
        }
    };
    double acc = 0.0;
    const int nk = (n + kEvK - 1) / kEvK;
    load(0);
    for (int kc = 0; kc < nk; ++kc) {
        const int k0 = kc * kEvK;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            As[(lr + 4 * q) * kEvPad + lc] = reg[q].x;
            As[(lr + 4 * q) * kEvPad + lc + 1] = reg[q].y;
        }
        if (t < kEvK) xs[t] = k0 + t < n ? x[k0 + t] : 0.0;
        __syncthreads();
        if (kc + 1 < nk) load(k0 + kEvK);
        if (t < 64) {
            const int len = min(kEvK, n - k0);
            const double* a = As + t * kEvPad;
            if (CKPT) {
                const int row = r0 + t;
                for (int e0 = 0; e0 < len; e0 += kCkpt) {
                    if (k0 + e0 > 0 && row < m) C[(long)((k0 + e0) / kCkpt) * m + row] = acc;
                    const int e1 = min(e0 + kCkpt, len);
                    for (int e = e0; e < e1; ++e) acc = fma(a[e], xs[e], acc);
                }
            } else {
                for (int e = 0; e < len; ++e) acc = fma(a[e], xs[e], acc);
            }
        }
    }
    const int row = r0 + t;
    if (t < 64 && row < m && F) F[row] = y ? acc - y[row] : acc;
}

// Batched FD GEMM.  Prefix sharing: the chain of point j equals the base chain for every k < j
// (x is only perturbed at k = j), so a tile whose first point is column jmin starts at
// ks = 16 * floor(jmin / 16) from the base chain's checkpoint C[ks / 16] and runs k = ks..n-1.
// Same fma sequence per point, hence bit-identical output; about half the flops of the
// full-length chains.
constexpr int kBK = 16;
constexpr int kFdTile = PNOL_FD_TILE;   // columns per point tile (BN of every launched variant)

// Point tiles of one FD GEMM launch (kernel argument): columns [start[t], start[t] + count[t]).
constexpr int kFdMaxTiles = 64;
struct FdTiles {
    int ntiles;
    int jbase;   // JT row of column c is c - jbase
    int start[kFdMaxTiles];
    int count[kFdMaxTiles];
};

// ---- row-panel k-major forms: one residual row per lane, no LDS --------------------------
// AP holds A in 64-row panels, k-major inside a panel: AP[(rb * n + k) * 64 + r] = A[64 rb + r][k]
// (rows past m are zero).  A wave owning a panel streams it front to back -- 512 contiguous
// bytes per k -- and the x_k operand is wave-uniform (scalar loads, the SGPR operand of
// v_fmac_f64), so the FD GEMM's broadcast stages are pure VALU: 32 fmas per 8-byte load.
constexpr int kPanel = 64;

__device__ __forceinline__ const double* panel_col(const double* AP, int n, int rb, int k) {
    return AP + ((long)rb * n + k) * kPanel;
}

// A (m x n row-major) -> AP, through 64 x 64 LDS tiles (padded against bank conflicts)
__global__ __launch_bounds__(256) void k_to_panels(const double* __restrict__ A, int m, int n, double* __restrict__ AP) {
    __shared__ double tile[64][65];
    const int rb = blockIdx.y, r0 = rb * 64, c0 = blockIdx.x * 64;
    const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6;
    for (int r = tr; r < 64; r += 4) tile[r][tc] = (r0 + r < m && c0 + tc < n) ? A[(long)(r0 + r) * n + c0 + tc] : 0.0;
    __syncthreads();
    for (int c = tr; c < 64; c += 4)
        if (c0 + c < n) AP[((long)rb * n + c0 + c) * kPanel + tc] = tile[tc][c];
}

// r = A x - y from AP: lane = row, the objective's fma chain over k ascending; CKPT also
// stores the chain value before every kCkpt-th column (C[(k / kCkpt) * m + row], k > 0).
// One wave per panel (m / 64 waves, about one per CU): the chain is sequential, so the panel
// stream is kept deep -- a ring of kRing 16-column blocks (kRing * 8 KB per wave) in flight
// while one is consumed.
constexpr int kRing = 6;

// xsave (nullable): block 0 records x there -- the content the checkpoints belong to.
// xcheck (nullable): the reuse check of a compute_f0 = 2 call -- every block first compares x
// with the recorded copy bit for bit and stops when they agree (the checkpoints and F in place
// are x's); otherwise it recomputes F and its checkpoints (the record is left as it was).
template <bool CKPT>
__global__ __launch_bounds__(64) void k_linres_evalP(const double* __restrict__ AP, const double* __restrict__ x,
                                                     const double* __restrict__ y, int m, int n,
                                                     double* __restrict__ F, double* __restrict__ C,
                                                     double* __restrict__ xsave = nullptr,
                                                     const double* __restrict__ xcheck = nullptr, int rb0 = 0,
                                                     double* __restrict__ Fh = nullptr,
                                                     const int* __restrict__ info_d = nullptr,
                                                     int* __restrict__ info_h = nullptr) {
    // rb0: the first row panel of this launch (a row-sharded LevMarqMPI rank evaluates its
    // m-slices only; the grid covers its panels)
    const int rb = rb0 + blockIdx.x, row = rb * kPanel + threadIdx.x;
    if (xcheck) {
        bool diff = false;
        const unsigned long long* xa = reinterpret_cast<const unsigned long long*>(x);
        const unsigned long long* xb = reinterpret_cast<const unsigned long long*>(xcheck);
        for (int k = threadIdx.x; k < n; k += 64) diff |= xa[k] != xb[k];
        if (!__any(diff)) return;   // one wave per block: uniform
    }
    if (xsave && blockIdx.x == 0)
        for (int k = threadIdx.x; k < n; k += 64) xsave[k] = x[k];
    // the LM trip's pinned result block (TripMirror): the solve status word, final by now (every
    // kernel that writes it ran before this one)
    if (info_h && blockIdx.x == 0 && threadIdx.x == 0) info_h[0] = info_d[0];
    const double* a = panel_col(AP, n, rb, 0) + threadIdx.x;
    constexpr int U = kCkpt;
    double acc = 0.0;
    const int nb = n / U;   // full blocks
    double ring[kRing][U];
    auto load = [&](int r, int blk) {
        const double* ak = a + (size_t)blk * U * kPanel;
#pragma unroll
        for (int q = 0; q < U; ++q) ring[r][q] = __builtin_nontemporal_load(ak + q * kPanel);
    };
    auto step = [&](int r, int blk) {
        const int k = blk * U;
        if (CKPT && k > 0 && row < m) C[(long)(k / kCkpt) * m + row] = acc;
#pragma unroll
        for (int q = 0; q < U; ++q) acc = fma(ring[r][q], x[k + q], acc);
    };
#pragma unroll
    for (int r = 0; r < kRing; ++r)
        if (r < nb) load(r, r);
    int blk = 0;
    for (; blk + kRing <= nb; blk += kRing) {
#pragma unroll
        for (int r = 0; r < kRing; ++r) {
            step(r, blk + r);
            if (blk + r + kRing < nb) load(r, blk + r + kRing);
        }
    }
#pragma unroll
    for (int r = 0; r < kRing; ++r)
        if (blk + r < nb) step(r, blk + r);
    int k = nb * U;
    if (CKPT && k > 0 && k < n && row < m) C[(long)(k / kCkpt) * m + row] = acc;
    for (; k < n; ++k) acc = fma(a[(size_t)k * kPanel], x[k], acc);
    if (row < m && F) {
        const double v = y ? acc - y[row] : acc;
        F[row] = v;
        if (Fh) Fh[row] = v;
    }
}

// FD GEMM from AP.  Workgroup = 4 waves on the same 64-row panel (one row per lane), wave w
// owning points [32w, 32w + 32) of the tile and starting from the base-chain checkpoint at
// its own first column.  Per k a lane does 32 fmas:
// x_k for every point except the one whose column is k, which gets x_k + h_k
// (XdX[j] = X[j] + dX[j]).  The next 8 k of the panel are in flight while the current 8 are
// consumed.  Bit-identical to the host evaluation.
// PW points per wave: 32 (the tile's 128 columns over 4 waves), or 16 (8 waves) for launches
// too small to fill the chip -- a LevMarqMPI rank's share at P >= 8, or one tile of the phased
// columns-mode launch: there the makespan is the longest chain's single-wave latency (a wave
// starting at column 0 runs ~n k-steps of PW fmas each), and 16 points per wave halve it while
// the chip still holds >= 2 waves per SIMD.  Every point's chain is the same either way.
constexpr int kPW = 32;

template <int PW = kPW>
__global__ __launch_bounds__(64 * (PNOL_FD_TILE / PW)) void k_linres_fdP(
    const double* __restrict__ AP, const double* __restrict__ y, const double* __restrict__ x,
    const double* __restrict__ h, int m, int n, const FdTiles tl, const double* __restrict__ F0,
    const double* __restrict__ C, double* __restrict__ JT, long ldjt, int mS, long sstride, int mt0, int nmt,
    const int* __restrict__ sel, const double* __restrict__ x1, const double* __restrict__ F01,
    const double* __restrict__ C1) {
    // sel (the LM loop's pre-queued Jacobian, pnol_ctx::FdGate): the point k_trip_gate passed on
    if (sel) {
        const int v = __builtin_amdgcn_readfirstlane(*sel);
        if (v < 0) return;
        if (v == 1) {
            x = x1;
            F0 = F01;
            C = C1;
        }
    }
    // Longest work first: the host sorts the tiles by first column (the chains of tile t run
    // k = ks_t .. n-1), and blockIdx walks all panels of tile 0, then of tile 1, ..., so the
    // short tiles fill the tail.  Panel mt lands on XCD mt % 8 for every tile (L2 reuse).
    // Panels [mt0, mt0 + nmt): the launch's rows (all of them, or a row-sharded rank's slices).
    const int nt = blockIdx.x / nmt, mt = mt0 + blockIdx.x % nmt;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int j0 = tl.start[nt], cnt = tl.count[nt];
    const int pw0 = w * PW;
    if (pw0 >= cnt) return;                 // wave-uniform; the kernel has no barriers
    const int np = min(PW, cnt - pw0);
    const int c0 = j0 + pw0;                // first column of this wave
    const int ks = (c0 / kBK) * kBK;
    const int row = mt * kPanel + lane, rowc = min(row, m - 1);
    const double* a = panel_col(AP, n, mt, 0) + lane;

    double acc[PW];
    {
        const double c = ks > 0 ? C[(long)(ks / kCkpt) * m + rowc] : 0.0;
#pragma unroll
        for (int j = 0; j < PW; ++j) acc[j] = c;
    }
    // k in [kb, ke): every point multiplies by x_k; blocks of 8, ping-pong prefetch of the
    // next block (no register copies)
    auto step8 = [&](const double (&av)[8], int k) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const double xk = x[k + q];
#pragma unroll
            for (int j = 0; j < PW; ++j) acc[j] = fma(av[q], xk, acc[j]);
        }
    };
    auto load8 = [&](double (&av)[8], int k) {
        const double* ak = a + (size_t)k * kPanel;   // one address, immediate offsets q * 512 B
#pragma unroll
        for (int q = 0; q < 8; ++q) av[q] = ak[q * kPanel];
    };
    auto bcast = [&](int kb, int ke) {
        int k = kb;
        const int nblk = (ke - k) / 8;   // whole blocks of 8
        if (nblk > 0) {
            // pairs of blocks with one loop exit: the accumulators keep their registers across
            // the back edge (a loop with an exit after each block made the compiler copy all 32
            // of them once per pair).  The load of the block after the pair is clamped to the
            // last block, so it is always in bounds and unused when past the end.
            const int klast = kb + (nblk - 1) * 8;
            double p0[8], p1[8];
            load8(p0, k);
            for (int b = 0; b + 2 <= nblk; b += 2) {
                load8(p1, k + 8);
                step8(p0, k);
                load8(p0, min(k + 16, klast));
                step8(p1, k + 8);
                k += 16;
            }
            if (nblk & 1) {
                step8(p0, k);
                k += 8;
            }
        }
        for (; k < ke; ++k) {
            const double av = a[(long)k * kPanel], xk = x[k];
#pragma unroll
            for (int j = 0; j < PW; ++j) acc[j] = fma(av, xk, acc[j]);
        }
    };
    bcast(ks, c0);
    // the window: point kk is perturbed at k = c0 + kk
    const int klen = min(PW, n - c0);
    if (klen == PW) {
#pragma unroll
        for (int q0 = 0; q0 < PW; q0 += 8) {
            double av[8];
            load8(av, c0 + q0);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int kk = q0 + q;
                const double xk = x[c0 + kk], xp = xk + h[c0 + kk];
#pragma unroll
                for (int j = 0; j < PW; ++j) acc[j] = fma(av[q], j == kk ? xp : xk, acc[j]);
            }
        }
    } else {
        for (int kk = 0; kk < klen; ++kk) {
            const double av = a[(long)(c0 + kk) * kPanel];
            const double xk = x[c0 + kk], xp = xk + h[c0 + kk];
#pragma unroll
            for (int j = 0; j < PW; ++j) acc[j] = fma(av, j == kk ? xp : xk, acc[j]);
        }
    }
    bcast(c0 + klen, n);
    // epilogue: F = acc - y; J = (F - F0) / h
    if (row < m) {
        const double yr = y[row], f0 = F0[row];
        // row r of J: slice r / mS of the sliced layout (mS >= m: plain row-major J^T)
        const int sl = (mt * kPanel) / mS;
        double* out = JT + (long)sl * sstride + (row - sl * mS);
#pragma unroll
        for (int j = 0; j < PW; ++j)
            if (j < np) {
                const int col = c0 + j;
                __builtin_nontemporal_store(((acc[j] - yr) - f0) / h[col], out + (long)(col - tl.jbase) * ldjt);
            }
    }
}

// The LM loop's pre-queued Jacobian (pnol_ctx::FdGate): one lane polls the host's word
// {seq, choice} (system-scope loads of pinned memory) until it carries this gate's seq, then
// hands the choice to the FD launch queued behind it (sel) and reports it to the host (res).  A
// host that never answers is given up on after cap ticks of the 100 MHz clock (choice -2: the FD
// launch returns, and the host's check of res sees it).  (The same poll inside the FD launch --
// workgroup 0 polling the host, the others a device word -- measured slower: the FD launch 20-40
// us longer with its resident workgroups spinning, profiles/r06_lm_gate_ab.txt.)
__global__ void k_trip_gate(const int* hw, int seq, int* sel, int* res, unsigned long long cap) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int v = -2;
    for (;;) {
        if (__hip_atomic_load(hw, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == seq) {
            v = __hip_atomic_load(hw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > cap) break;
        __builtin_amdgcn_s_sleep(4);
    }
    sel[0] = v;
    res[0] = v;
    res[1] = seq;
}

// ---- synthetic data, splitmix64 counter stream ---------------------------
__global__ void k_synth_quadratic(unsigned long long seed, int n, double bscale, double* d, double* b) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        d[i] = 1.0 + 3.0 * u01(seed, (unsigned long long)i);
        b[i] = (2.0 * u01(seed, (unsigned long long)(n + i)) - 1.0) * bscale;
    }
}

__global__ void k_synth_linres(unsigned long long seed, int m, int n, double scale, double* A, double* xstar) {
    const long mn = (long)m * n;
    for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; k < mn + n; k += (long)gridDim.x * blockDim.x) {
        if (k < mn) A[k] = (2.0 * u01(seed, (unsigned long long)k) - 1.0) * scale;
        else xstar[k - mn] = 2.0 * u01(seed, (unsigned long long)k) - 1.0;
    }
}

}  // namespace

// ---- launchers ------------------------------------------------------------------------------
static bool is_scalar_kind(int k) { return k == PNOL_OBJ_ROSENBROCK || k == PNOL_OBJ_POWER || k == PNOL_OBJ_QUADRATIC; }

int launch_dobj_eval(pnol_ctx* ctx, pnol_dobj* o, const double* x, double* out) {
    if (!o || !x || !out) return PNOL_ERR_ARG;
    switch (o->kind) {
        case PNOL_OBJ_ROSENBROCK:
        case PNOL_OBJ_POWER:
        case PNOL_OBJ_QUADRATIC:
            return launch_eval_batch(ctx, o, x, 1, out);   // one point: terms in parallel, summed in order
        case PNOL_OBJ_EXPCURVE:
            hipLaunchKernelGGL((k_multi_eval<PNOL_OBJ_EXPCURVE>), dim3((o->m + 255) / 256), dim3(256), 0, ctx->stream, x, o->n,
                               o->m, o->p0, o->p1, o->p2, out);
            return launch_check();
        case PNOL_OBJ_CUBIC:
            hipLaunchKernelGGL((k_multi_eval<PNOL_OBJ_CUBIC>), dim3((o->m + 255) / 256), dim3(256), 0, ctx->stream, x, o->n,
                               o->m, o->p0, o->p1, o->p2, out);
            return launch_check();
        case PNOL_OBJ_LINRES: {
            ScopedTimer tm(ctx, "linres_eval");
            if (o->at)
                hipLaunchKernelGGL((k_linres_evalP<false>), dim3((o->m + kPanel - 1) / kPanel), dim3(64), 0, ctx->stream,
                                   (const double*)o->at, x, o->p1, o->m, o->n, out, (double*)nullptr, (double*)nullptr,
                                   (const double*)nullptr);
            else if (o->n % 2 == 0)
                hipLaunchKernelGGL((k_linres_eval<true, false>), dim3((o->m + kEvRows - 1) / kEvRows), dim3(256), 0, ctx->stream,
                                   o->p0, x, o->p1, o->m, o->n, out, (double*)nullptr);
            else
                hipLaunchKernelGGL((k_linres_eval<false, false>), dim3((o->m + kEvRows - 1) / kEvRows), dim3(256), 0,
                                   ctx->stream, o->p0, x, o->p1, o->m, o->n, out, (double*)nullptr);
            return launch_check();
        }
        default:
            return PNOL_ERR_UNSUPPORTED;
    }
}

int launch_eval_batch(pnol_ctx* ctx, pnol_dobj* o, const double* Xs, int npts, double* out) {
    if (!o || !Xs || !out || npts < 0) return PNOL_ERR_ARG;
    if (npts == 0) return PNOL_OK;
    if (!is_scalar_kind(o->kind)) {   // residual kinds: F of each point, rows of out (npts x m)
        for (int k = 0; k < npts; ++k) PNOL_CHECK(launch_dobj_eval(ctx, o, Xs + (size_t)k * o->n, out + (size_t)k * o->m));
        return PNOL_OK;
    }
    const dim3 grid(npts), blk(256);
    if (o->kind == PNOL_OBJ_ROSENBROCK)
        hipLaunchKernelGGL((k_eval_batch<PNOL_OBJ_ROSENBROCK>), grid, blk, 0, ctx->stream, Xs, o->n, o->p0, o->p1,
                           o->power, out);
    else if (o->kind == PNOL_OBJ_POWER)
        hipLaunchKernelGGL((k_eval_batch<PNOL_OBJ_POWER>), grid, blk, 0, ctx->stream, Xs, o->n, o->p0, o->p1,
                           o->power, out);
    else
        hipLaunchKernelGGL((k_eval_batch<PNOL_OBJ_QUADRATIC>), grid, blk, 0, ctx->stream, Xs, o->n, o->p0, o->p1,
                           o->power, out);
    return launch_check();
}

// The row-panel k-major copy of a linear residual's A (objective data never changes after creation).
static int ensure_panels(pnol_ctx* ctx, pnol_dobj* o) {
    if (o->at) return PNOL_OK;
    const int nrb = (o->m + kPanel - 1) / kPanel;
    PNOL_HIP(hipMalloc(&o->at, sizeof(double) * (size_t)nrb * kPanel * o->n));
    hipLaunchKernelGGL(k_to_panels, dim3((o->n + 63) / 64, nrb), dim3(256), 0, ctx->stream, (const double*)o->p0, o->m,
                       o->n, o->at);
    return launch_check();
}

// The two checkpoint slots.  An LM trip holds the checkpoints of its Jacobian point x_s and
// writes those of the trial point x_t: with two slots a rejected step (x_s stands) finds x_s's
// still in place and skips the base-chain pass.  A slot is tagged with the objective's creation
// id (never reused, unlike its address) and the device x pointer, and keeps a copy of x's
// content (written by the kernel that makes the checkpoints), so a compute_f0 = 2 caller that
// changed x in place gets a recomputation instead of stale checkpoints.
static int ckpt_find(pnol_ctx* ctx, const pnol_dobj* o, const double* x, int r0, int r1) {
    for (int s = 0; s < 2; ++s)
        if (o && ctx->ckpt_oid[s] == o->id && ctx->ckpt_x[s] == x && ctx->ckpt_r0[s] <= r0 && ctx->ckpt_r1[s] >= r1)
            return s;
    return -1;
}
static int ckpt_buf(pnol_ctx* ctx, const pnol_dobj* o, int slot, void** C, void** xcopy) {
    const int ncp = (o->n + kCkpt - 1) / kCkpt;
    ctx->ckpt_use[slot] = ++ctx->ckpt_clock;
    PNOL_CHECK(ws_get(ctx, slot ? "linres_ckx1" : "linres_ckx0", sizeof(double) * (size_t)o->n, xcopy));
    return ws_get(ctx, slot ? "linres_ckpt1" : "linres_ckpt0", sizeof(double) * (size_t)o->m * (ncp > 1 ? ncp : 1), C);
}
// the slot the checkpoints of (o, x) on rows [r0, r1) are written to: its own if tagged, else
// the least recent; tagged (o, x, rows) (reusable false: written but never reused)
static int ckpt_claim(pnol_ctx* ctx, const pnol_dobj* o, const double* x, bool reusable, void** C, void** xcopy,
                      int r0, int r1) {
    int s = ckpt_find(ctx, o, x, r0, r1);
    if (s < 0) s = ctx->ckpt_use[0] <= ctx->ckpt_use[1] ? 0 : 1;
    ctx->ckpt_oid[s] = reusable ? o->id : 0;
    ctx->ckpt_x[s] = x;
    ctx->ckpt_r0[s] = r0;
    ctx->ckpt_r1[s] = r1;
    ctx->ckpt_last = s;
    return ckpt_buf(ctx, o, s, C, xcopy);
}

// F = F(x), and for a linear residual also the prefix checkpoints of x, kept in the context
// for the next FD call on (o, x) with compute_f0 == 2 (the LM trial point becomes the next
// Jacobian point when the step is accepted).
int launch_dobj_eval_ckpt(pnol_ctx* ctx, pnol_dobj* o, const double* x, double* out, int r0, int r1) {
    if (!o || !x || !out) return PNOL_ERR_ARG;
    if (o->kind != PNOL_OBJ_LINRES) return launch_dobj_eval(ctx, o, x, out);
    if (r1 < 0) {
        r0 = 0;
        r1 = o->m;
    }
    if (r0 == r1) r0 = r1 = o->m;   // no rows
    if (r0 < 0 || (r0 % kPanel && r0 != o->m) || r1 > o->m || r0 > r1 || (r1 % kPanel && r1 != o->m))
        return PNOL_ERR_ARG;
    PNOL_CHECK(ensure_panels(ctx, o));
    void *C = nullptr, *xc = nullptr;
    PNOL_CHECK(ckpt_claim(ctx, o, x, true, &C, &xc, r0, r1));
    const int nb = (r1 - r0 + kPanel - 1) / kPanel;
    if (nb > 0) {
        ScopedTimer tm(ctx, "linres_eval");
        const auto& tm_ = ctx->trip_mirror;
        hipLaunchKernelGGL((k_linres_evalP<true>), dim3(nb), dim3(64), 0, ctx->stream, (const double*)o->at, x, o->p1,
                           o->m, o->n, out, (double*)C, (double*)xc, (const double*)nullptr, r0 / kPanel, tm_.F,
                           tm_.info_d, tm_.info_h);
    }
    return launch_check();
}


template <int KIND>
static int launch_fd_chain(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, int i0, int cnt, double* T,
                           double* V, double* xdev, const double* hsrc) {
    const int nt = std::max(o->n, 1);
    hipLaunchKernelGGL((k_scalar_terms<KIND>), dim3(std::min((nt + 255) / 256, 1024)), dim3(256), 0, ctx->stream, x, o->n,
                       o->p0, o->p1, o->power, T, xdev, hsrc, hsrc ? const_cast<double*>(h) : (double*)nullptr);
    PNOL_CHECK(launch_check());
    const int waves = (cnt + 1 + 63) / 64;
    hipLaunchKernelGGL((k_scalar_fd_chain<KIND>), dim3((waves + 3) / 4), dim3(256), 0, ctx->stream,
                       xdev ? (const double*)xdev : x, h, o->n, i0, cnt, o->p0, o->p1, o->power, (const double*)T, V);
    return launch_check();
}

int launch_fd_gradient(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, int i0, int cnt, double* f0,
                       double* g, double* xdev, const double* hsrc) {
    if (!o || !x || !h || !is_scalar_kind(o->kind)) return PNOL_ERR_ARG;
    if (i0 < 0 || cnt < 0 || i0 + cnt > o->n) return PNOL_ERR_ARG;
    void *vals = nullptr, *terms = nullptr;
    PNOL_CHECK(ws_get(ctx, "fd_vals", sizeof(double) * (size_t)(cnt + 1), &vals));
    PNOL_CHECK(ws_get(ctx, "fd_terms", sizeof(double) * (size_t)o->n, &terms));
    double *V = (double*)vals, *T = (double*)terms;
    // PNOL_FD_SCALAR=0: the point-per-thread form (every term recomputed; tuning / cross-check)
    static const bool chain = [] {
        const char* e = std::getenv("PNOL_FD_SCALAR");
        return !e || std::atoi(e) != 0;
    }();
    if (xdev && !chain) {   // the point-per-thread form reads x throughout: bring it to the device
        PNOL_HIP(hipMemcpyAsync(xdev, x, sizeof(double) * (size_t)o->n, hipMemcpyHostToDevice, ctx->stream));
        x = xdev;
    }
    if (hsrc && !chain) {
        PNOL_HIP(hipMemcpyAsync(const_cast<double*>(h), hsrc, sizeof(double) * (size_t)o->n, hipMemcpyHostToDevice,
                                ctx->stream));
        hsrc = nullptr;
    }
    if (chain) {
        if (o->kind == PNOL_OBJ_ROSENBROCK)
            PNOL_CHECK(launch_fd_chain<PNOL_OBJ_ROSENBROCK>(ctx, o, x, h, i0, cnt, T, V, xdev, hsrc));
        else if (o->kind == PNOL_OBJ_POWER)
            PNOL_CHECK(launch_fd_chain<PNOL_OBJ_POWER>(ctx, o, x, h, i0, cnt, T, V, xdev, hsrc));
        else PNOL_CHECK(launch_fd_chain<PNOL_OBJ_QUADRATIC>(ctx, o, x, h, i0, cnt, T, V, xdev, hsrc));
    } else {
        const int blocks = (cnt + 1 + 255) / 256;
        if (o->kind == PNOL_OBJ_ROSENBROCK)
            hipLaunchKernelGGL((k_scalar_fd_values<PNOL_OBJ_ROSENBROCK>), dim3(blocks), dim3(256), 0, ctx->stream, x, h,
                               o->n, i0, cnt, o->p0, o->p1, o->power, V);
        else if (o->kind == PNOL_OBJ_POWER)
            hipLaunchKernelGGL((k_scalar_fd_values<PNOL_OBJ_POWER>), dim3(blocks), dim3(256), 0, ctx->stream, x, h, o->n,
                               i0, cnt, o->p0, o->p1, o->power, V);
        else
            hipLaunchKernelGGL((k_scalar_fd_values<PNOL_OBJ_QUADRATIC>), dim3(blocks), dim3(256), 0, ctx->stream, x, h,
                               o->n, i0, cnt, o->p0, o->p1, o->power, V);
        PNOL_CHECK(launch_check());
    }
    hipLaunchKernelGGL(k_scalar_fd_finish, dim3((cnt + 255) / 256 + 1), dim3(256), 0, ctx->stream, (const double*)V, h, i0,
                       cnt, f0, g);
    return launch_check();
}

// FD Jacobian rows for the point tiles [start[t], start[t] + count[t]) (count <= kFdTile),
// column c written to JT row c - jbase.  Linear residual: one base-chain pass (F0 and the
// prefix checkpoints), then the FD GEMM over all tiles in launches of <= kFdMaxTiles tiles.
int launch_fd_jacobian_tiles(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, const int* start,
                             const int* count, int ntiles, double* F0, int compute_f0, double* JT, int jbase,
                             int ldjt, int ckpt, int mS, long sstride, int r0, int r1,
                             const std::function<int(int)>* after_tile) {
    const bool sliced = mS > 0;
    const bool rows_all = r1 < 0;
    if (!o) return PNOL_ERR_ARG;
    if (rows_all) {
        r0 = 0;
        r1 = o->m;
    }
    if (!rows_all && r0 == r1) r0 = r1 = o->m;   // no rows (a rank past the last residual)
    if (!rows_all && (!sliced || r0 < 0 || (r0 % kPanel && r0 != o->m) || r1 > o->m || r0 > r1 ||
                      (r1 % kPanel && r1 != o->m)))
        return PNOL_ERR_ARG;
    if (!o || !x || !h || !F0 || is_scalar_kind(o->kind) || ntiles < 0 || ldjt < (sliced ? mS : o->m))
        return PNOL_ERR_ARG;
    if (sliced && (o->kind != PNOL_OBJ_LINRES || mS % kPanel != 0 || sstride < (long)o->n * ldjt))
        return PNOL_ERR_UNSUPPORTED;
    if (!sliced) {
        mS = o->m;   // one slice: plain row-major J^T
        sstride = 0;
    }
    for (int t = 0; t < ntiles; ++t)
        if (start[t] < 0 || count[t] < 0 || count[t] > kFdTile || start[t] + count[t] > o->n || start[t] < jbase)
            return PNOL_ERR_ARG;
    int total = 0;
    for (int t = 0; t < ntiles; ++t) total += count[t];
    if (total > 0 && !JT) return PNOL_ERR_ARG;
    if (o->kind != PNOL_OBJ_LINRES || total == 0) {
        if (compute_f0 == 1) PNOL_CHECK(launch_dobj_eval(ctx, o, x, F0));
        for (int t = 0; t < ntiles; ++t)
            if (count[t] > 0)
                PNOL_CHECK(launch_fd_jacobian(ctx, o, x, h, start[t], count[t], F0, 0,
                                              JT + (size_t)(start[t] - jbase) * ldjt, ldjt));
        return PNOL_OK;
    }
    PNOL_CHECK(ensure_panels(ctx, o));
    // one pass of the base chain: F0 (when asked) and the prefix checkpoints.  compute_f0 == 3
    // (the library's own LM loop: x untouched since pnol_dobj_eval_ckpt_d) reuses a tagged
    // slot outright; compute_f0 == 2 (ABI callers) reuses it only if x's content still matches
    // the slot's record (checked on the device, else F0 and the checkpoints are recomputed);
    // untagged, both recompute -- 2 including F0, which then cannot be trusted either.
    void *C = nullptr, *xc = nullptr;
    double* f0_out = (compute_f0 == 1 || compute_f0 == 2) ? F0 : nullptr;
    const double* xcheck = nullptr;
    const int have = compute_f0 >= 2 ? ckpt_find(ctx, o, x, r0, r1) : -1;
    // the pre-queued form (lm_prequeue_fd): both points' checkpoints in place, one batched launch
    const pnol_ctx::FdGate gate = ctx->fd_gate;
    void* C1 = nullptr;
    if (gate.hw) {
        const int have1 = ckpt_find(ctx, o, gate.x1, r0, r1);
        if (have < 0 || have1 < 0 || have1 == have || compute_f0 != 3 || after_tile || sliced || !rows_all ||
            ntiles > kFdMaxTiles)
            return PNOL_ERR_UNSUPPORTED;
        const int ncp = (o->n + kCkpt - 1) / kCkpt;
        PNOL_CHECK(ws_get(ctx, have1 ? "linres_ckpt1" : "linres_ckpt0", sizeof(double) * (size_t)o->m * (ncp > 1 ? ncp : 1),
                          &C1));
    }
    if (have >= 0) {
        ctx->ckpt_last = have;
        PNOL_CHECK(ckpt_buf(ctx, o, have, &C, &xc));
        if (compute_f0 == 3 || !ckpt) ckpt = 0;
        else xcheck = (const double*)xc;   // verify, recompute on a mismatch
    } else if (ckpt) {
        PNOL_CHECK(ckpt_claim(ctx, o, x, true, &C, &xc, r0, r1));
        if (compute_f0 == 3) f0_out = nullptr;
    } else {   // the caller's previous call on (o, x) wrote them (chunked FD: chunks after the first)
        PNOL_CHECK(ckpt_buf(ctx, o, ctx->ckpt_last, &C, &xc));
    }
    const int mt0 = r0 / kPanel, nmt = (r1 - r0 + kPanel - 1) / kPanel;   // this call's row panels
    if (ckpt && nmt > 0) {
        LaunchTimer tm(ctx, "fd_ckpt");
        hipExtLaunchKernelGGL((k_linres_evalP<true>), dim3(nmt), dim3(64), 0, ctx->stream, tm.start(), tm.stop(), 0,
                              (const double*)o->at, x, (const double*)o->p1, o->m, o->n, f0_out, (double*)C,
                              xcheck ? (double*)nullptr : (double*)xc, xcheck, mt0, (double*)nullptr,
                              (const int*)nullptr, (int*)nullptr);
        PNOL_CHECK(launch_check());
    }
    if (nmt == 0) return PNOL_OK;   // a rank without rows
    const double* Cc = (const double*)C;
    // Launch order: batched (after_tile == nullptr) -- the tiles sorted by first column (longest
    // chains first), up to kFdMaxTiles per launch; phased -- one launch per tile in the caller's
    // order, after_tile(t) called behind each (the columns-mode exchange of that tile's rows).
    std::vector<int> ord(ntiles);
    for (int t = 0; t < ntiles; ++t) ord[t] = t;
    if (!after_tile)
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return start[a] < start[b]; });
    const int per_launch = after_tile ? 1 : kFdMaxTiles;
    // 16 points per wave when a launch would hold <= 2 waves per SIMD at 32 (k_linres_fdP);
    // PNOL_FD_PW = 16 / 32 forces either (A/B measurement)
    static const int force_pw = [] {
        const char* e = std::getenv("PNOL_FD_PW");
        return e ? std::atoi(e) : 0;
    }();
    if (gate.hw) {
        hipLaunchKernelGGL(k_trip_gate, dim3(1), dim3(64), 0, ctx->stream, gate.hw, gate.seq, gate.sel, gate.res,
                           gate.cap);
        PNOL_CHECK(launch_check());
    }
    LaunchTimer lt(ctx, "fd_jacobian");
    for (int t0 = 0; t0 < ntiles; t0 += per_launch) {
        FdTiles tl;
        tl.ntiles = std::min(per_launch, ntiles - t0);
        tl.jbase = jbase;
        for (int t = 0; t < tl.ntiles; ++t) {
            tl.start[t] = start[ord[t0 + t]];
            tl.count[t] = count[ord[t0 + t]];
        }
        const dim3 grid(nmt * tl.ntiles);
        const hipEvent_t ea = t0 == 0 ? lt.start() : nullptr;
        const hipEvent_t eb = t0 + per_launch >= ntiles ? lt.stop() : nullptr;
        const long waves32 = (long)nmt * tl.ntiles * (kFdTile / kPW);
        const bool pw16 = force_pw ? force_pw == 16 : waves32 <= 8L * std::max(ctx->num_cu, 1);
        if (pw16)
            hipExtLaunchKernelGGL((k_linres_fdP<16>), grid, dim3(64 * (kFdTile / 16)), 0, ctx->stream, ea, eb, 0,
                                  (const double*)o->at, (const double*)o->p1, x, h, o->m, o->n, tl, (const double*)F0,
                                  Cc, JT, (long)ldjt, mS, sstride, mt0, nmt, (const int*)gate.sel, gate.x1,
                                  gate.F01, (const double*)C1);
        else
            hipExtLaunchKernelGGL((k_linres_fdP<kPW>), grid, dim3(64 * (kFdTile / kPW)), 0, ctx->stream, ea, eb, 0,
                                  (const double*)o->at, (const double*)o->p1, x, h, o->m, o->n, tl, (const double*)F0,
                                  Cc, JT, (long)ldjt, mS, sstride, mt0, nmt, (const int*)gate.sel, gate.x1,
                                  gate.F01, (const double*)C1);
        PNOL_CHECK(launch_check());
        if (after_tile) PNOL_CHECK((*after_tile)(ord[t0]));
    }
    return PNOL_OK;
}

int launch_fd_jacobian(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, int j0, int cnt, double* F0,
                       int compute_f0, double* JT, int ldjt) {
    if (!o || !x || !h || !F0 || is_scalar_kind(o->kind)) return PNOL_ERR_ARG;
    if (j0 < 0 || cnt < 0 || j0 + cnt > o->n || ldjt < o->m) return PNOL_ERR_ARG;
    if (o->kind == PNOL_OBJ_LINRES && cnt > 0) {
        // the contiguous block as consecutive kFdTile-column tiles
        std::vector<int> st, ct;
        for (int c = j0; c < j0 + cnt; c += kFdTile) {
            st.push_back(c);
            ct.push_back(std::min(kFdTile, j0 + cnt - c));
        }
        return launch_fd_jacobian_tiles(ctx, o, x, h, st.data(), ct.data(), (int)st.size(), F0, compute_f0, JT, j0,
                                        ldjt);
    }
    if (compute_f0) PNOL_CHECK(launch_dobj_eval(ctx, o, x, F0));
    if (cnt == 0) return PNOL_OK;
    if (!JT) return PNOL_ERR_ARG;
    switch (o->kind) {
        case PNOL_OBJ_EXPCURVE:
            hipLaunchKernelGGL((k_multi_fd<PNOL_OBJ_EXPCURVE>), dim3((o->m + 255) / 256, cnt), dim3(256), 0, ctx->stream, x, h,
                               o->n, o->m, j0, cnt, o->p0, o->p1, o->p2, (const double*)F0, JT, (long)ldjt);
            return launch_check();
        case PNOL_OBJ_CUBIC:
            hipLaunchKernelGGL((k_multi_fd<PNOL_OBJ_CUBIC>), dim3((o->m + 255) / 256, cnt), dim3(256), 0, ctx->stream, x, h,
                               o->n, o->m, j0, cnt, o->p0, o->p1, o->p2, (const double*)F0, JT, (long)ldjt);
            return launch_check();
        default:
            return PNOL_ERR_UNSUPPORTED;
    }
}

int lm_prequeue_fd(pnol_ctx* ctx, pnol_dobj* o, const double* x0, double* F00, const double* x1, double* F01,
                   const double* h, double* JT, int ldjt, const int* hw, int seq, int* sel, int* res,
                   unsigned long long cap) {
    if (!o || o->kind != PNOL_OBJ_LINRES || !x0 || !F00 || !x1 || !F01 || !hw || !sel || !res) return PNOL_ERR_ARG;
    ctx->fd_gate = {hw, seq, sel, res, x1, F01, cap};
    const int st = launch_fd_jacobian(ctx, o, x0, h, 0, o->n, F00, 3, JT, ldjt);
    ctx->fd_gate = {};
    return st;
}

int lm_fd_commit(pnol_ctx* ctx, pnol_dobj* o, const double* x) {
    const int have = ckpt_find(ctx, o, x, 0, o->m);
    if (have < 0) return PNOL_ERR_ARG;
    ctx->ckpt_last = have;
    void *C = nullptr, *xc = nullptr;
    return ckpt_buf(ctx, o, have, &C, &xc);
}

int launch_synthetic_quadratic(pnol_ctx* ctx, unsigned long long seed, int n, double bscale, double* d, double* b) {
    hipLaunchKernelGGL(k_synth_quadratic, dim3(std::min(1024, (n + 255) / 256)), dim3(256), 0, ctx->stream, seed, n, bscale,
                       d, b);
    return launch_check();
}

int launch_synthetic_linres(pnol_ctx* ctx, unsigned long long seed, int m, int n, double* A, double* xstar, double* y) {
    const double scale = 1.0 / std::sqrt((double)n);
    hipLaunchKernelGGL(k_synth_linres, dim3(4096), dim3(256), 0, ctx->stream, seed, m, n, scale, A, xstar);
    PNOL_CHECK(launch_check());
    // y = A x* with the residual's own fma chain (no y offset)
    if (n % 2 == 0)
        hipLaunchKernelGGL((k_linres_eval<true, false>), dim3((m + kEvRows - 1) / kEvRows), dim3(256), 0, ctx->stream,
                           (const double*)A, (const double*)xstar, (const double*)nullptr, m, n, y, (double*)nullptr);
    else
        hipLaunchKernelGGL((k_linres_eval<false, false>), dim3((m + kEvRows - 1) / kEvRows), dim3(256), 0, ctx->stream,
                           (const double*)A, (const double*)xstar, (const double*)nullptr, m, n, y, (double*)nullptr);
    return launch_check();
}

int lm_phased_env() {
    const char* e = std::getenv("PNOL_LM_PHASED");
    if (e && std::atoi(e) == 0) return 0;
    const char* s = std::getenv("PNOL_LM_SUBPHASES");   // column groups of each rank's last tile
    const int v = s ? std::atoi(s) : kLmSubphases;
    return std::min(8, std::max(1, v));
}

int lm_fd_mode_env() {
    const char* e = std::getenv("PNOL_LM_FD");
    return (e && std::strcmp(e, "rows") == 0) ? 1 : 0;
}

bool lm_rows_mode(pnol_ctx* ctx) {
    if (ctx->lm_fd_mode < 0) ctx->lm_fd_mode = lm_fd_mode_env();
    return ctx->lm_fd_mode == 1;
}

// this rank's residual rows [r0, r1) in rows mode: its m-slices
static void lm_my_rows(int m, int* r0, int* r1) {
    const int P = comm_size(), me = comm_rank(), mS = lm_slice_rows(m);
    int s0 = 0, s1 = 0;
    lm_rank_slices(P, me, &s0, &s1);
    *r0 = std::min(m, s0 * mS);
    *r1 = std::min(m, s1 * mS);
}

// Rank q's FD tiles in phase order: cheapest first (the latest first column: the shortest
// prefix-shared chains), so the exchange of the early tiles runs while the expensive ones compute
// and only the last phase's exchange is left after the FD.  sub >= 2 cuts the last tile into
// `sub` column groups (multiples of 16 columns, the prefix checkpoints' stride), each its own
// launch and exchange phase: only the last group's slices are then exposed, 1/sub of a tile's
// (the same columns, the same bits).
static void lm_phase_tiles(int n, int P, int q, std::vector<int>& st, std::vector<int>& ct, int sub = 1) {
    fd_tiles_of(n, P, q, st, ct);   // ascending first column
    std::reverse(st.begin(), st.end());
    std::reverse(ct.begin(), ct.end());
    if (sub < 2 || st.empty()) return;
    const int s0 = st.back(), c = ct.back();
    const int w = std::max(16, (c / sub + 15) / 16 * 16);
    st.pop_back();
    ct.pop_back();
    for (int a = 0; a < c; a += w) {
        st.push_back(s0 + a);
        ct.push_back(std::min(w, c - a));
    }
}

static int lm_comm_stream(pnol_ctx* ctx, int nphase) {
    if (!ctx->comm_stream) PNOL_HIP(hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking));
    while ((int)ctx->phase_events.size() < nphase) {
        hipEvent_t e;
        PNOL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->phase_events.push_back(e);
    }
    if (!ctx->comm_done) PNOL_HIP(hipEventCreateWithFlags(&ctx->comm_done, hipEventDisableTiming));
    return PNOL_OK;
}

// LevMarqMPI Jacobian on the sliced J^T layout (pnol_lm_sliced_layout), LevenbergMarquardtMPI.cpp:60
// -> PNOL_Objective.cpp:202-299.
// Columns mode (default; the reference's decomposition, its round-robin columns dealt as
// cost-balanced tiles): this rank evaluates its FD tiles for every residual row, one launch per
// tile, cheapest first; behind each launch an event, and on the communication stream, gated by
// it, that tile's m-slices go to the ranks holding them (one group of point-to-point transfers
// per tile: phase k carries every rank's k-th tile).  Each rank ends with every FD column of its
// own slices -- all launch_lm_normal reads -- having moved 1/P of the J^T an allgather would,
// and all but the last tile's transfer overlapped with the FD launches.  Rows mode (linear
// residuals): every FD column on this rank's own m-slices, no Jacobian exchange at all.
int launch_lm_jacobian(pnol_ctx* ctx, pnol_dobj* o, const double* x, const double* h, double* F0, int compute_f0,
                       double* JTs) {
    if (!o || !JTs || o->kind != PNOL_OBJ_LINRES) return PNOL_ERR_UNSUPPORTED;
    const int P = comm_size(), me = comm_rank(), n = o->n;
    if (P > kLmSlices) return PNOL_ERR_UNSUPPORTED;
    const int mS = lm_slice_rows(o->m);
    const long sstr = (long)n * mS;
    std::vector<int> st, ct;
    if (lm_rows_mode(ctx)) {
        // Every residual row of the linear residual is its own fma chain over x, so the FD
        // column j on rows [r0, r1) is exactly the rows [r0, r1) of the whole column: each rank
        // evaluates all n FD columns on its m-slices -- 1/P of the FD work, balanced, and the
        // sliced J^T it needs (launch_lm_normal) is complete with no exchange.
        int r0 = 0, r1 = 0;
        lm_my_rows(o->m, &r0, &r1);
        fd_tiles_of(n, 1, 0, st, ct);
        return launch_fd_jacobian_tiles(ctx, o, x, h, st.data(), ct.data(), (int)st.size(), F0, compute_f0, JTs, 0, mS,
                                        1, mS, sstr, r0, r1);
    }
    if (P == 1) {
        fd_tiles_of(n, 1, 0, st, ct);
        return launch_fd_jacobian_tiles(ctx, o, x, h, st.data(), ct.data(), (int)st.size(), F0, compute_f0, JTs, 0,
                                        mS, 1, mS, sstr);
    }
    // ctx->lm_phased (read once per LevMarqMPI solve and agreed over the ranks): 0 (PNOL_LM_PHASED=0)
    // one tile-list launch, then every tile's slices in one exchange on the context stream after
    // it -- no second stream, no events; S >= 1 one launch and exchange phase per tile, the last
    // tile cut into S column groups (PNOL_LM_SUBPHASES); the same bits either way
    if (ctx->lm_phased < 0) ctx->lm_phased = lm_phased_env();
    std::vector<std::vector<int>> pst(P), pct(P);
    int nphase = 0;
    for (int q = 0; q < P; ++q) {
        lm_phase_tiles(n, P, q, pst[q], pct[q], ctx->lm_phased);
        nphase = std::max(nphase, (int)pst[q].size());
    }
    if (ctx->lm_phased == 0) {
            const int mine = (int)pst[me].size();
            PNOL_CHECK(launch_fd_jacobian_tiles(ctx, o, x, h, pst[me].data(), pct[me].data(), mine, F0, compute_f0,
                                                JTs, 0, mS, 1, mS, sstr));
            ScopedTimer tm(ctx, "exchange_J");
            return comm_exchange(ctx, JTs, JTs, [&](int q, int d, std::vector<XBlock>& bl) {
                bl.clear();
                int s0, s1;
                lm_rank_slices(P, d, &s0, &s1);
                for (size_t k = 0; k < pst[q].size(); ++k) {
                    const size_t c0 = (size_t)pst[q][k], cc = (size_t)pct[q][k];
                    for (int s = s0; s < s1; ++s) {
                        if ((long)s * mS >= o->m) break;
                        const size_t off = (size_t)s * sstr + c0 * mS;
                        bl.push_back({off, off, cc * mS});
                    }
                }
            });
        }
    PNOL_CHECK(lm_comm_stream(ctx, nphase + 1));
    const int mine = (int)pst[me].size();
    // phase k is gated by the event behind this rank's k-th tile; phases past its last tile
    // (and every phase of a rank without tiles) by the event behind its last launch
    int launched = 0;
    const std::function<int(int)> after = [&](int) {
        PNOL_HIP(hipEventRecord(ctx->phase_events[launched++], ctx->stream));
        return PNOL_OK;
    };
    PNOL_CHECK(launch_fd_jacobian_tiles(ctx, o, x, h, pst[me].data(), pct[me].data(), mine, F0, compute_f0, JTs, 0,
                                        mS, 1, mS, sstr, 0, -1, &after));
    if (launched < mine) return PNOL_ERR_UNSUPPORTED;   // (linear residuals launch per tile)
    if (mine == 0) PNOL_HIP(hipEventRecord(ctx->phase_events[0], ctx->stream));
    const hipEvent_t fd_end = timer_event(ctx, "exchange_J", ctx->stream);
    hipEvent_t busy0 = nullptr;
    for (int k = 0; k < nphase; ++k) {
        PNOL_HIP(hipStreamWaitEvent(ctx->comm_stream, ctx->phase_events[std::min(k, std::max(mine - 1, 0))], 0));
        if (k == 0) busy0 = timer_event(ctx, "exchange_J_busy", ctx->comm_stream);
        PNOL_CHECK(comm_exchange(ctx, JTs, JTs, [&](int q, int d, std::vector<XBlock>& bl) {
            bl.clear();
            if (k >= (int)pst[q].size()) return;
            const size_t c0 = (size_t)pst[q][k], cc = (size_t)pct[q][k];
            int s0, s1;
            lm_rank_slices(P, d, &s0, &s1);
            for (int s = s0; s < s1; ++s) {
                if ((long)s * mS >= o->m) break;
                const size_t off = (size_t)s * sstr + c0 * mS;
                bl.push_back({off, off, cc * mS});
            }
        }, ctx->comm_stream));
    }
    timer_pair(ctx, "exchange_J_busy", busy0, timer_event(ctx, "exchange_J_busy", ctx->comm_stream));
    timer_pair(ctx, "exchange_J", fd_end, timer_event(ctx, "exchange_J", ctx->comm_stream));
    PNOL_HIP(hipEventRecord(ctx->comm_done, ctx->comm_stream));
    PNOL_HIP(hipStreamWaitEvent(ctx->stream, ctx->comm_done, 0));
    return PNOL_OK;
}

// The LevMarqMPI trial point: F(x) and its checkpoints on this rank's rows, then each rank's
// rows to every other rank (the host's chi^2 sums all m residuals on every rank).  Columns mode:
// every rank evaluates all rows, as the one-GPU loop does.
int launch_lm_eval(pnol_ctx* ctx, pnol_dobj* o, const double* x, double* F) {
    if (!o || !x || !F) return PNOL_ERR_ARG;
    const int P = comm_size();
    if (P == 1 || !lm_rows_mode(ctx) || o->kind != PNOL_OBJ_LINRES) return launch_dobj_eval_ckpt(ctx, o, x, F);
    int r0 = 0, r1 = 0;
    lm_my_rows(o->m, &r0, &r1);
    PNOL_CHECK(launch_dobj_eval_ckpt(ctx, o, x, F, r0, r1));
    ScopedTimer tm(ctx, "exchange_F");
    return comm_exchange(ctx, F, F, [&](int q, int d, std::vector<XBlock>& bl) {
        (void)d;
        bl.clear();
        const int m = o->m, mS = lm_slice_rows(m);
        int s0 = 0, s1 = 0;
        lm_rank_slices(comm_size(), q, &s0, &s1);
        const int a = std::min(m, s0 * mS), b = std::min(m, s1 * mS);
        if (b > a) bl.push_back({(size_t)a, (size_t)a, (size_t)(b - a)});
    });
}

}  // namespace pnol
