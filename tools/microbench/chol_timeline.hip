// Per-step timeline of the method-4 tile Cholesky (chol.hip k_chol_step, one launch per panel
// step): for every launch, when its diagonal / panel / update workgroups ran, and the gap from
// one step's diagonal tile to the next -- the split between the factor chain and launch overhead.
// Prints one JSON line.  Build (after the library):
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -I include \
//     -I parallelnonlinearoptimizationlibrary_amd/csrc tools/microbench/chol_timeline.hip \
//     -L parallelnonlinearoptimizationlibrary_amd -lpnol_amd \
//     -Wl,-rpath,'$ORIGIN/../../parallelnonlinearoptimizationlibrary_amd' -o tools/microbench/chol_timeline
#define PNOL_CHOL_TIMELINE 1
#include "../../parallelnonlinearoptimizationlibrary_amd/csrc/kernels/chol.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

// symmetric, diagonally dominant: A_ij = A_ji in [-0.5, 0.5), A_ii = n
__global__ void k_spd(double* A, int n) {
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < (long)n * n; e += (long)gridDim.x * blockDim.x) {
        const long i = e / n, j = e % n, a = i < j ? i : j, b = i < j ? j : i;
        unsigned long long z = (unsigned long long)(a * n + b) * 0x9E3779B97F4A7C15ull + 7;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        A[e] = i == j ? (double)n : (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    }
}

int main(int argc, char** argv) {
    using namespace pnol;
    const int n = argc > 1 ? std::atoi(argv[1]) : 2048;
    pnol_ctx* ctx = nullptr;
    if (pnol_ctx_create(0, &ctx) != PNOL_OK) {
        std::fprintf(stderr, "no device\n");
        return 1;
    }
    double *A, *b, *x;
    int* info;
    hipMalloc(&A, sizeof(double) * (size_t)n * n);
    hipMalloc(&b, sizeof(double) * n);
    hipMalloc(&x, sizeof(double) * n);
    hipMalloc(&info, sizeof(int));
    hipLaunchKernelGGL(k_spd, dim3(2048), dim3(256), 0, ctx->stream, A, n);
    std::vector<double> ones(n, 1.0);
    hipMemcpy(b, ones.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    const int T = (n + NB - 1) / NB;
    std::vector<unsigned long long> init(64 * 3 * 2);
    for (size_t i = 0; i < init.size(); i += 2) {
        init[i] = ~0ull;
        init[i + 1] = 0;
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms[6];
    std::vector<unsigned long long> zero(64 * 8, 0);
    for (int r = 0; r < 6; ++r) {
        hipStreamSynchronize(ctx->stream);
        hipMemcpyToSymbol(HIP_SYMBOL(g_chol_clk), zero.data(), sizeof(unsigned long long) * zero.size());
        hipMemcpyToSymbol(HIP_SYMBOL(g_chol_tl), init.data(), sizeof(unsigned long long) * init.size());
        hipMemcpyToSymbol(HIP_SYMBOL(g_chol_crit), zero.data(), sizeof(unsigned long long) * zero.size());
        hipMemcpyToSymbol(HIP_SYMBOL(g_chol_la), zero.data(), sizeof(unsigned long long) * 64 * 4);
        hipEventRecord(e0, ctx->stream);
        if (launch_chol_solve(ctx, A, n, b, x, n, info) != PNOL_OK) return 1;
        hipEventRecord(e1, ctx->stream);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms[r], e0, e1);
    }
    int hinfo = 0;
    hipMemcpy(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost);
    std::vector<unsigned long long> tl(init.size());
    hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(g_chol_tl), sizeof(unsigned long long) * tl.size());
    std::vector<unsigned long long> ck(64 * 8);
    hipMemcpyFromSymbol(ck.data(), HIP_SYMBOL(g_chol_clk), sizeof(unsigned long long) * ck.size());
    auto at = [&](int s, int c, int e) { return tl[(s * 3 + c) * 2 + e]; };
    const unsigned long long base = at(0, 0, 0);
    std::printf("{\"n\": %d, \"steps\": %d, \"info\": %d, \"ms_events\": [", n, T, hinfo);
    for (int r = 0; r < 6; ++r) std::printf("%s%.4f", r ? ", " : "", ms[r]);
    std::printf("], \"steps_us\": [");
    double sum_diag = 0, sum_gap = 0;
    for (int s = 0; s < T && s < 64; ++s) {
        const double ds = (at(s, 0, 0) - base) * 0.01, de = (at(s, 0, 1) - base) * 0.01;
        const bool hp = at(s, 1, 1) != 0, hu = at(s, 2, 1) != 0;
        const double gap = s + 1 < T ? (at(s + 1, 0, 0) - at(s, 0, 1)) * 0.01 : 0.0;
        sum_diag += de - ds;
        sum_gap += gap;
        std::printf("%s{\"k\": %d, \"diag\": [%.2f, %.2f], \"panel\": [%.2f, %.2f], \"update\": [%.2f, %.2f], "
                    "\"gap_to_next_diag\": %.2f, \"diag_cycles\": %llu, \"diag_clock_ghz\": %.3f, "
                    "\"stamps\": [%lld, %lld, %lld, %lld, %lld, %lld], \"lookahead_used\": %llu}",
                    s ? ", " : "", s - 1, ds, de, hp ? (at(s, 1, 0) - base) * 0.01 : -1.0,
                    hp ? (at(s, 1, 1) - base) * 0.01 : -1.0, hu ? (at(s, 2, 0) - base) * 0.01 : -1.0,
                    hu ? (at(s, 2, 1) - base) * 0.01 : -1.0, gap, ck[8 * s + 7] - ck[8 * s],
                    (double)(ck[8 * s + 7] - ck[8 * s]) / ((at(s, 0, 1) - at(s, 0, 0)) * 10.0),
                    // cycles from the start: staged, L strip, A_dd - L L^T in LDS, factor done, end
                    s ? (long long)(ck[8 * s + 1] - ck[8 * s]) : 0LL, s ? (long long)(ck[8 * s + 2] - ck[8 * s]) : 0LL,
                    (long long)(ck[8 * s + 3] - ck[8 * s]), (long long)(ck[8 * s + 4] - ck[8 * s]),
                    (long long)(ck[8 * s + 7] - ck[8 * s]),
                    // persistent form: the end of the wait for the two tiles (0 in method 4)
                    ck[8 * s + 5] ? (long long)(ck[8 * s + 5] - ck[8 * s]) : 0LL, ck[8 * s + 6]);
    }
    std::vector<unsigned long long> la(64 * 4);
    hipMemcpyFromSymbol(la.data(), HIP_SYMBOL(g_chol_la), sizeof(unsigned long long) * la.size());
    // the look-ahead inside step s's factor, cycles from the factor's start: polling starts,
    // tiles ready, staged, MFMAs done (-1: not run)
    std::printf("], \"lookahead_cycles\": [");
    for (int s = 1; s < T && s < 64; ++s) {
        auto dc = [&](int i) { return la[4 * s + i] ? (long long)la[4 * s + i] - (long long)ck[8 * s + 3] : -1LL; };
        std::printf("%s[%d, %lld, %lld, %lld, %lld]", s > 1 ? ", " : "", s, dc(0), dc(1), dc(2), dc(3));
    }
    std::vector<unsigned long long> cr(64 * 8);
    hipMemcpyFromSymbol(cr.data(), HIP_SYMBOL(g_chol_crit), sizeof(unsigned long long) * cr.size());
    std::printf("], \"critical_us_after_W\": [");
    for (int k = 1; k + 2 < T && k < 64; ++k) {
        auto dt = [&](int i) { return cr[8 * k + i] ? ((long long)cr[8 * k + i] - (long long)cr[8 * k]) * 0.01 : -1.0; };
        std::printf("%s[%d, %.2f, %.2f, %.2f, %.2f, %.2f, %.2f, %.2f]", k > 1 ? ", " : "", k, dt(1), dt(2), dt(3), dt(4),
                    dt(5), dt(6), dt(7));
    }
    std::printf("], \"sum_diag_us\": %.1f, \"sum_gap_us\": %.1f, \"workers\": \"%s\", \"solo\": \"%s\", "
                "\"persist\": \"%s\", \"lookahead\": \"%s\"}\n", sum_diag, sum_gap, std::getenv("PNOL_CHOL5_WORKERS") ? std::getenv("PNOL_CHOL5_WORKERS") : "",
                std::getenv("PNOL_CHOL5_SOLO") ? std::getenv("PNOL_CHOL5_SOLO") : "",
                std::getenv("PNOL_CHOL_PERSIST") ? std::getenv("PNOL_CHOL_PERSIST") : "",
                std::getenv("PNOL_CHOL_LOOKAHEAD") ? std::getenv("PNOL_CHOL_LOOKAHEAD") : "");
    return 0;
}
