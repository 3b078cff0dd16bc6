// solve.hip -- the damped LM solve, sigma = A^{-1} rhs (replaces luSolve, LevenbergMarquardt.cpp:83).
//
// A = J^T J + lambda diag(J^T J) is symmetric positive definite whenever J has full column
// rank, so the fast path is a blocked right-looking Cholesky (nb = 64):
//   k_potrf_diag   factor the 64 x 64 diagonal block in LDS (one workgroup)
//   k_trsm_panel   L21 = A21 L11^{-T}, one row per thread, row held in registers
//   syrk (MODE 1)  A22 -= L21 L21^T on the lower tiles, fp64 MFMA (syrk.hip)
//   k_chol_solve   forward / backward substitution, one workgroup, 64-row blocks
// A non-positive (or NaN) pivot flips to Gaussian elimination with partial pivoting in the
// reference's operation order (k_lu_*), which is also the method for n <= PNOL_SEQ_MAX so
// the small ExampleObjectives problems are bitwise equal to the CPU path.
#include "../pnol_internal.hpp"

namespace pnol {
namespace {

constexpr int kNB = 64;

// ---- Cholesky ---------------------------------------------------------------------------
// Diagonal block, one wave: lane t owns row t; left-looking (Crout) column steps
//   s_t = a_tj - sum_{k<j} L_tk L_jk ;  L_jj = sqrt(s_j) ;  L_tj = s_t / L_jj  (t > j)
// with row j read as an LDS broadcast.  A single wave needs no workgroup barrier between
// steps, only LDS ordering (s_barrier with one wave is free).
__global__ __launch_bounds__(64) void k_potrf_diag(double* __restrict__ A, long lda, int k0, int nbe,
                                                   int* __restrict__ info) {
    __shared__ double L[kNB][kNB + 1];
    const int t = threadIdx.x;
    for (int r = 0; r < kNB; ++r)
        L[r][t] = (r < nbe && t <= r) ? A[(long)(k0 + r) * lda + k0 + t] : 0.0;
    __syncthreads();
    if (*info != 0) return;   // an earlier block already failed
    bool bad = false;
    for (int j = 0; j < nbe; ++j) {
        double s = (t >= j && t < nbe) ? L[t][j] : 0.0;
        for (int k = 0; k < j; ++k) s = fma(-L[t][k], L[j][k], s);
        const double sjj = __shfl(s, j, 64);
        if (!(sjj > 0.0)) {          // not positive definite (or NaN): uniform exit
            if (t == 0) *info = k0 + j + 1;
            bad = true;
            break;
        }
        const double d = sqrt(sjj);
        if (t == j) L[j][j] = d;
        else if (t > j && t < nbe) L[t][j] = s / d;
        __syncthreads();
    }
    if (bad) return;
    for (int r = 0; r < nbe; ++r)
        if (t <= r) A[(long)(k0 + r) * lda + k0 + t] = L[r][t];
}

// Panel below the diagonal block: x L11^T = a for every row, one thread per row with the
// row in registers (fully unrolled right-looking substitution, L11 read as LDS broadcasts).
// 64 rows per workgroup, loaded and stored through LDS in coalesced 512-byte row segments.
__global__ __launch_bounds__(64) void k_trsm_panel(double* __restrict__ A, long lda, int n, int k0, int nbe,
                                                   const int* __restrict__ info) {
    __shared__ double L[kNB][kNB + 1];
    __shared__ double X[kNB][kNB + 1];
    if (*info != 0) return;
    const int t = threadIdx.x;
    const int rbase = k0 + nbe + blockIdx.x * kNB;
    for (int r = 0; r < kNB; ++r) {
        L[r][t] = (r < nbe && t < nbe) ? A[(long)(k0 + r) * lda + k0 + t] : (r == t ? 1.0 : 0.0);
        const int row = rbase + r;
        X[r][t] = (row < n && t < nbe) ? A[(long)row * lda + k0 + t] : 0.0;
    }
    __syncthreads();
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
    __syncthreads();
    for (int r = 0; r < kNB; ++r) {
        const int row = rbase + r;
        if (row < n && t < nbe) A[(long)row * lda + k0 + t] = X[r][t];
    }
}

// Forward then backward substitution with the lower factor; one 1024-thread workgroup.
// Per 64-row block: the 64 x 64 diagonal block is staged in LDS and solved by wave 0
// (lane i owns row i, pivots broadcast by shuffle); the rest of the right-hand side is then
// updated by all 16 waves with coalesced reads (forward: a wave per row, lanes over the
// block's columns; backward: a thread per remaining entry, lanes over a row of L).
__global__ __launch_bounds__(1024) void k_chol_solve(const double* __restrict__ L, long lda, int n,
                                                     const double* __restrict__ rhs, double* __restrict__ x,
                                                     double* __restrict__ work, const int* __restrict__ info) {
    __shared__ double T[64][65];
    __shared__ double zb[64];
    if (*info != 0) return;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6, nwaves = blockDim.x >> 6;
    double* b = work;   // n doubles
    for (int i = t; i < n; i += blockDim.x) b[i] = rhs[i];
    __syncthreads();
    // forward: L z = b
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int nb = min(64, n - i0);
        for (int e = t; e < 64 * 64; e += blockDim.x) {
            const int r = e >> 6, c = e & 63;
            T[r][c] = (r < nb && c <= r) ? L[(long)(i0 + r) * lda + i0 + c] : 0.0;
        }
        __syncthreads();
        if (wave == 0) {
            double bi = lane < nb ? b[i0 + lane] : 0.0;
            for (int j = 0; j < nb; ++j) {
                const double zj = __shfl(bi, j, 64) / T[j][j];
                if (lane == j) bi = zj;
                else if (lane > j) bi = fma(-T[lane][j], zj, bi);
            }
            if (lane < nb) { b[i0 + lane] = bi; zb[lane] = bi; }
        }
        __syncthreads();
        const double zl = lane < nb ? zb[lane] : 0.0;
        for (int i = i0 + nb + wave; i < n; i += nwaves) {
            double s = lane < nb ? L[(long)i * lda + i0 + lane] * zl : 0.0;
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
            if (lane == 0) b[i] = b[i] - s;
        }
        __syncthreads();
    }
    // backward: L^T x = z
    for (int iend = n; iend > 0; iend -= 64) {
        const int i0 = max(0, iend - 64);
        const int nb = iend - i0;
        for (int e = t; e < 64 * 64; e += blockDim.x) {
            const int r = e >> 6, c = e & 63;
            T[r][c] = (r < nb && c <= r) ? L[(long)(i0 + r) * lda + i0 + c] : 0.0;
        }
        __syncthreads();
        if (wave == 0) {
            double zi = lane < nb ? b[i0 + lane] : 0.0;
            for (int j = nb - 1; j >= 0; --j) {
                const double xj = __shfl(zi, j, 64) / T[j][j];
                if (lane == j) zi = xj;
                else if (lane < j) zi = fma(-T[j][lane], xj, zi);
            }
            if (lane < nb) { b[i0 + lane] = zi; zb[lane] = zi; }
        }
        __syncthreads();
        for (int i = t; i < i0; i += blockDim.x) {
            double s = 0.0;
            for (int j = 0; j < nb; ++j) s = fma(L[(long)(i0 + j) * lda + i], zb[j], s);
            b[i] = b[i] - s;
        }
        __syncthreads();
    }
    for (int i = t; i < n; i += blockDim.x) x[i] = b[i];
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

int launch_solve(pnol_ctx* ctx, double* A, int lda, const double* rhs, double* sigma, int n, int method,
                 int* info) {
    if (!A || !rhs || !sigma || n <= 0 || lda < n) return PNOL_ERR_ARG;
    void* dinfo_v = nullptr;
    PNOL_CHECK(ws_get(ctx, "solve_info", sizeof(int) * 4, &dinfo_v));
    int* dinfo = (int*)dinfo_v;
    int used = 0;
    if (method == 0) method = (n <= PNOL_SEQ_MAX) ? 2 : 1;
    if (method == 1) {
        // keep a copy of A so a failed factorisation can fall back to LU on the original
        void* Acopy = nullptr;
        PNOL_CHECK(ws_get(ctx, "chol_Acopy", sizeof(double) * (size_t)n * n, &Acopy));
        long total = (long)n * n;
        hipLaunchKernelGGL(k_copy_matrix, dim3((int)std::min<long>((total + 255) / 256, 4096)), dim3(256), 0,
                           ctx->stream, (const double*)A, (long)lda, (double*)Acopy, n);
        hipLaunchKernelGGL(k_set_int, dim3(1), dim3(1), 0, ctx->stream, dinfo, 0);
        for (int k0 = 0; k0 < n; k0 += kNB) {
            const int nbe = std::min(kNB, n - k0);
            hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(64), 0, ctx->stream, A, (long)lda, k0, nbe, dinfo);
            const int below = n - k0 - nbe;
            if (below > 0) {
                hipLaunchKernelGGL(k_trsm_panel, dim3((below + kNB - 1) / kNB), dim3(kNB), 0, ctx->stream, A, (long)lda, n,
                                   k0, nbe, (const int*)dinfo);
                PNOL_CHECK(launch_syrk_lower(ctx, A + (long)(k0 + nbe) * lda + k0, lda, below, nbe, -1.0,
                                             A + (long)(k0 + nbe) * lda + k0 + nbe, lda, 1));
            }
        }
        void* work = nullptr;
        PNOL_CHECK(ws_get(ctx, "chol_work", sizeof(double) * (size_t)n, &work));
        hipLaunchKernelGGL(k_chol_solve, dim3(1), dim3(1024), 0, ctx->stream, (const double*)A, (long)lda, n, rhs,
                           sigma, (double*)work, (const int*)dinfo);
        PNOL_CHECK(launch_check());
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
