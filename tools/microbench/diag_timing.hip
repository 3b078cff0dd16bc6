// Times the diagonal-tile factor of the method-4 Cholesky (chol.hip factor_diag) in one
// workgroup with s_memtime stamps; checks W = L^{-1} against the host.  Build:
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I include \
//     -I parallelnonlinearoptimizationlibrary_amd/csrc tools/microbench/diag_timing.hip -o tools/microbench/diag_timing
#include "../../parallelnonlinearoptimizationlibrary_amd/csrc/kernels/chol.hip"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace pnol {
int ws_get(pnol_ctx*, const char*, size_t, void**, bool*) { return PNOL_ERR_ARG; }   // unused here
}

__global__ __launch_bounds__(256, 2) void k_diag_time(const double* A, double* W, int* info, long long* st) {
    using namespace pnol;
    __shared__ __attribute__((aligned(16))) double smem[2 * kStage];
    __shared__ double rinv[NB];
    __shared__ int cnt[6];
    const int t = threadIdx.x;
    const DiagLds L = diag_lds(smem);
    if (t < 6) cnt[t] = 0;
    const int row = t >> 2, c0 = (t & 3) * 16;
    for (int q = 0; q < 16; ++q) diag_put(L, row, c0 + q, A[row * 64 + c0 + q]);
    __syncthreads();
    if (t == 0) st[31] = __builtin_amdgcn_s_memtime();
    factor_diag<true>(L, rinv, cnt, W, 0, info, st);
}

#if PNOL_CHOL_MP
// wave 0's chain alone (waves 1..3 idle, the owners' words preset): the pivot chain's cost
// without the other waves' LDS polling and MFMA traffic beside it
__global__ __launch_bounds__(256, 2) void k_chain_solo(const double* A, int* info, long long* st) {
    using namespace pnol;
    __shared__ __attribute__((aligned(16))) double smem[2 * kStage];
    __shared__ double rinv[NB];
    __shared__ int cnt[6];
    const int t = threadIdx.x;
    const DiagLds L = diag_lds(smem);
    if (t < 6) cnt[t] = t >= 2 ? 99 : 0;
    const int row = t >> 2, c0 = (t & 3) * 16;
    for (int q = 0; q < 16; ++q) diag_put(L, row, c0 + q, A[row * 64 + c0 + q]);
    __syncthreads();
    if (t >= 64) return;
    const MpLds M = mp_lds(L);
    const int lane = t;
    if (t == 0) st[31] = __builtin_amdgcn_s_memtime();
    mp_panel<0, true>(M, rinv, cnt, lane, 0, info, st);
    mp_panel<1, true>(M, rinv, cnt, lane, 0, info, st);
    mp_panel<2, true>(M, rinv, cnt, lane, 0, info, st);
    mp_panel<3, true>(M, rinv, cnt, lane, 0, info, st);
    if (t == 0) st[8] = __builtin_amdgcn_s_memtime();
}
#endif

int main() {
    const int n = 64;
    std::vector<double> M(n * n), A(n * n);
    unsigned long long s = 12345;
    for (auto& v : M) { s = s * 6364136223846793005ULL + 1442695040888963407ULL; v = ((s >> 11) * 0x1.0p-53) - 0.5; }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = (i == j) ? 1.0 : 0.0;
            for (int k = 0; k < n; ++k) acc += M[i * n + k] * M[j * n + k];
            A[i * n + j] = acc;
        }
    double *dA, *dW; int* dinfo; long long* dst;
    hipMalloc(&dA, 8 * n * n); hipMalloc(&dW, 8 * n * n); hipMalloc(&dinfo, 4); hipMalloc(&dst, 8 * 32);
    hipMemcpy(dA, A.data(), 8 * n * n, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        hipMemset(dinfo, 0, 4); hipMemset(dst, 0, 8 * 32);
        hipLaunchKernelGGL(k_diag_time, dim3(1), dim3(256), 0, 0, dA, dW, dinfo, dst);
        hipDeviceSynchronize();
    }
    std::vector<long long> st(32); std::vector<double> W(n * n); int info = 0;
    hipMemcpy(st.data(), dst, 8 * 32, hipMemcpyDeviceToHost);
    hipMemcpy(W.data(), dW, 8 * n * n, hipMemcpyDeviceToHost);
    hipMemcpy(&info, dinfo, 4, hipMemcpyDeviceToHost);
    // check: W A W^T = I  (W = L^{-1}, A = L L^T)
    double err = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = 0;
            for (int k = 0; k < n; ++k) {
                double wa = 0;
                for (int l = 0; l < n; ++l) wa += W[i * n + l] * A[l * n + k];
                acc += wa * W[j * n + k];
            }
            err = std::fmax(err, std::fabs(acc - (i == j)));
        }
    const long long b = st[31];
    unsigned long long h = 1469598103934665603ULL;   // FNV-1a of W's bits (A/B builds must agree)
    for (double v : W) { unsigned long long u; memcpy(&u, &v, 8); h = (h ^ u) * 1099511628211ULL; }
    printf("{\"info\": %d, \"max|W A W^T - I|\": %.3e, \"w_hash\": \"%016llx\", \"cycles\": {", info, err, h);
#if PNOL_CHOL_MP
    const char* names[] = {"p0_j0", "p0_j8", "p1_j0", "p1_j8", "p2_j0", "p2_j8", "p3_j0", "p3_j8", "chain_end",
                           "w30_w31_end", "v1_end", "v2_end", "v3_end", "barrier"};
    const int nn = 14;
#else
    const char* names[] = {"p1_j0", "p1_j8", "p1_j16", "p1_j24", "p1_end", "w11_end", "p2_q00_end", "-", "p3_start",
                           "p3_j0", "p3_j8", "p3_j16", "p3_j24", "p3_end", "w22_end", "b3", "p4_end"};
    const int nn = 17;
#endif
    for (int i = 0; i < nn; ++i)
        if (names[i][0] != '-') printf("%s\"%s\": %lld", i ? ", " : "", names[i], st[i] ? st[i] - b : -1LL);
    printf("}");
#if PNOL_CHOL_MP
    hipMemset(dst, 0, 8 * 32);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_chain_solo, dim3(1), dim3(256), 0, 0, dA, dinfo, dst);
    hipDeviceSynchronize();
    hipMemcpy(st.data(), dst, 8 * 32, hipMemcpyDeviceToHost);
    printf(", \"chain_solo\": {");
    for (int i = 0; i < 9; ++i) printf("%s\"%s\": %lld", i ? ", " : "", names[i], st[i] - st[31]);
    printf("}");
#endif
    printf("}\n");
    return (info == 0 && err < 1e-12) ? 0 : 1;
}
