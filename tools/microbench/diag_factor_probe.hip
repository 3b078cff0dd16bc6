// The diagonal tile's factor alone (factor_diag16, STAMP): shader-clock stamps every 8 pivots of
// each 16-wide micro-panel (wave 0), at the end of micro-panel 3, after V_3 X_3j, and wave 1's
// milestones -- where a chain step's ~28k cycles go.  One 256-thread workgroup, R repetitions
// on an SPD 64 x 64 tile; prints one JSON line of per-stamp cycles from the factor's start.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -I include \
//     -I parallelnonlinearoptimizationlibrary_amd/csrc tools/microbench/diag_factor_probe.hip \
//     -L parallelnonlinearoptimizationlibrary_amd -lpnol_amd \
//     -Wl,-rpath,'$ORIGIN/../../parallelnonlinearoptimizationlibrary_amd' -o tools/microbench/diag_factor_probe
#include "../../parallelnonlinearoptimizationlibrary_amd/csrc/kernels/chol.hip"

#include <cstdio>

namespace pnol {
namespace {
__global__ __launch_bounds__(256, 1) void k_diag_probe(int reps, double* Wd, int* info, long long* out) {
    __shared__ __attribute__((aligned(16))) double smem[2 * kStage];
    __shared__ double rinv[NB];
    __shared__ int cnt[6];
    __shared__ long long st[16];
    const int t = threadIdx.x;
    const DiagLds L = diag_lds(smem);
    for (int r = 0; r < reps; ++r) {
        // SPD: A_ii = 64, A_ij = 1 / (1 + i + j) (lower triangle into the split copy)
        for (int e = t; e < NB * NB; e += 256) {
            const int i = e / NB, j = e % NB;
            if (j <= i) diag_put(L, i, j, i == j ? 64.0 : 1.0 / (1 + i + j));
        }
        if (t < 6) cnt[t] = 0;
        if (t < 16) st[t] = 0;
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        factor_diag<true, false>(L, rinv, cnt, Wd, 0, info, st);
        __syncthreads();
        if (t < 14 && r == reps - 1) out[t] = st[t] ? st[t] - t0 : -1;
        if (t == 0 && r == reps - 1) out[14] = __builtin_amdgcn_s_memtime() - t0;
        __syncthreads();
    }
}
}  // namespace
}  // namespace pnol

int main() {
    using namespace pnol;
    double* Wd;
    int* info;
    long long* out;
    hipMalloc(&Wd, sizeof(double) * NB * NB);
    hipMalloc(&info, sizeof(int));
    hipMalloc(&out, sizeof(long long) * 16);
    hipMemset(info, 0, sizeof(int));
    hipLaunchKernelGGL(k_diag_probe, dim3(1), dim3(256), 0, 0, 20, Wd, info, out);
    long long h[16];
    int hinfo = 0;
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    double w[NB * NB];
    hipMemcpy(w, Wd, sizeof(w), hipMemcpyDeviceToHost);
    unsigned long long fnv = 1469598103934665603ull;   // FNV-1a over W's bytes: bitwise comparisons across builds
    const unsigned char* wb = reinterpret_cast<const unsigned char*>(w);
    for (size_t i = 0; i < sizeof(w); ++i) fnv = (fnv ^ wb[i]) * 1099511628211ull;
    hipMemcpy(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost);
    std::printf("{\"info\": %d, \"w_fnv\": \"%016llx\", \"stamps_cycles\": {", hinfo, fnv);
    const char* names[15] = {"p0_j0", "p0_j8", "p1_j0", "p1_j8", "p2_j0", "p2_j8", "p3_j0", "p3_j8", "w0_panels_done",
                             "w0_vx_done", "w1_inv1", "w1_inv2", "w1_inv3", "after_barrier", "total"};
    for (int i = 0; i < 15; ++i) std::printf("%s\"%s\": %lld", i ? ", " : "", names[i], h[i]);
    std::printf("}}\n");
    return 0;
}
