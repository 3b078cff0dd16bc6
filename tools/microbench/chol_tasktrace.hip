// Per-task trace of the persistent tile Cholesky's workers (chol.hip k_chol_persist, method 5) at
// n = 2048: for every claimed task its claim time, the end of its dependency waits ("ready") and
// its publish, with the diagonal chain's W_k publish times -- whether the early steps' worker
// tasks are late because they wait (dependencies) or because they work (throughput).  Prints
// one JSON line: per step the task counts and the median wait / work per kind, and when the
// step's last update task publishes relative to W_k.  Build (after the library):
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -I include \
//     -I parallelnonlinearoptimizationlibrary_amd/csrc tools/microbench/chol_tasktrace.hip \
//     -L parallelnonlinearoptimizationlibrary_amd -lpnol_amd \
//     -Wl,-rpath,'$ORIGIN/../../parallelnonlinearoptimizationlibrary_amd' -o tools/microbench/chol_tasktrace
#define PNOL_CHOL_TIMELINE 1
#define PNOL_CHOL_TASKTRACE 1
#include "../../parallelnonlinearoptimizationlibrary_amd/csrc/kernels/chol.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

static double median(std::vector<double> v) {
    if (v.empty()) return -1.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
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
    std::vector<unsigned long long> init(64 * 3 * 2), zt(16384 * 4, 0);
    for (size_t i = 0; i < init.size(); i += 2) {
        init[i] = ~0ull;
        init[i + 1] = 0;
    }
    float ms = 0;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 4; ++r) {   // the last run's trace
        hipStreamSynchronize(ctx->stream);
        hipMemcpyToSymbol(HIP_SYMBOL(g_chol_tl), init.data(), sizeof(unsigned long long) * init.size());
        hipMemcpyToSymbol(HIP_SYMBOL(g_chol_tasks), zt.data(), sizeof(unsigned long long) * zt.size());
        hipEventRecord(e0, ctx->stream);
        if (launch_chol_solve(ctx, A, n, b, x, n, info) != PNOL_OK) return 1;
        hipEventRecord(e1, ctx->stream);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    std::vector<unsigned long long> tl(init.size()), tk(zt.size());
    hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(g_chol_tl), sizeof(unsigned long long) * tl.size());
    hipMemcpyFromSymbol(tk.data(), HIP_SYMBOL(g_chol_tasks), sizeof(unsigned long long) * tk.size());
    // W_k publish = the end of the chain's step d = k (g_chol_tl class 0 of slot d; slot 0 is the
    // first tile's factor, before the persistent launch)
    auto wk = [&](int k) { return tl[(k * 3 + 0) * 2 + 1]; };
    const unsigned long long base = tl[0];
    std::printf("{\"n\": %d, \"steps\": %d, \"ms\": %.4f, \"per_step\": [", n, T, ms);
    bool first = true;
    for (int k = 0; k + 1 < T && k < 63; ++k) {
        std::vector<double> wait[4], work[4];
        int cnt[4] = {0, 0, 0, 0};
        double upd_last = -1e30, claim_first = 1e30;
        for (int g = 0; g < 16384; ++g) {
            const unsigned long long* r = &tk[4 * g];
            if (!r[2]) continue;
            const int kk = (int)(r[3] >> 8), kind = (int)(r[3] & 255);
            if (kk != k || kind > 3) continue;
            cnt[kind]++;
            wait[kind].push_back((r[1] - r[0]) * 0.01);
            work[kind].push_back((r[2] - r[1]) * 0.01);
            claim_first = std::min(claim_first, ((double)r[0] - (double)wk(k)) * 0.01);
            if (kind != 0) upd_last = std::max(upd_last, ((double)r[2] - (double)wk(k)) * 0.01);
        }
        std::printf("%s{\"k\": %d, \"W_us\": %.2f, \"next_W_after_us\": %.2f, \"panels\": %d, \"updates\": %d, "
                    "\"half_updates\": %d, \"first_claim_rel_W\": %.2f, \"last_update_rel_W\": %.2f, "
                    "\"wait_med_us\": [%.2f, %.2f, %.2f], \"work_med_us\": [%.2f, %.2f, %.2f]}",
                    first ? "" : ", ", k, (wk(k) - base) * 0.01,
                    k + 2 < T ? ((double)wk(k + 1) - (double)wk(k)) * 0.01 : -1.0, cnt[0], cnt[1], cnt[2], claim_first,
                    upd_last, median(wait[0]), median(wait[1]), median(wait[2]), median(work[0]), median(work[1]),
                    median(work[2]));
        first = false;
    }
    std::printf("]}\n");
    return 0;
}
