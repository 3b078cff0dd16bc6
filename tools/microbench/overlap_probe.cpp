// Probe: can the damped solve run beside the J^T J SYRK on a disjoint set of CUs?
// Times J^T J (pnol_jtj_d) and the method-4 solve (pnol_solve_async_d) alone on the full chip,
// alone on CU-masked streams, and both at once on complementary masks.  Prints one JSON line.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/microbench/overlap_probe.cpp \
//     -L parallelnonlinearoptimizationlibrary_amd -lpnol_amd \
//     -Wl,-rpath,'$ORIGIN/../../parallelnonlinearoptimizationlibrary_amd' -o tools/microbench/overlap_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include "pnol_amd.h"

static void on_segv(int) {
    void* bt[64];
    const int k = backtrace(bt, 64);
    backtrace_symbols_fd(bt, k, 2);
    _exit(3);
}

static hipStream_t masked(int ncu, int first, int count, int stride) {
    std::vector<uint32_t> m((ncu + 31) / 32, 0u);
    for (int c = 0, k = first; c < count; ++c, k += stride) m[(k % ncu) / 32] |= 1u << ((k % ncu) % 32);
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()) != hipSuccess) return nullptr;
    return s;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// median of reps wall times of f() (launch + device sync)
static double timeit(const std::function<void()>& f, int reps = 7) {
    std::vector<double> t;
    f();
    hipDeviceSynchronize();
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_ms();
        f();
        hipDeviceSynchronize();
        t.push_back(now_ms() - t0);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

__global__ void k_fill(double* x, long count) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < count; i += (long)gridDim.x * blockDim.x) {
        unsigned long long z = (unsigned long long)i * 0x9E3779B97F4A7C15ull + 0x5EED;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    }
}

#define STEP(x) std::fprintf(stderr, "step %s\n", x)
int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    signal(SIGSEGV, on_segv);
    STEP("start");
    const int m = 16384, n = 2048;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    STEP("attr");
    pnol_ctx *ca = nullptr, *cb = nullptr;
    if (pnol_ctx_create(0, &ca) || pnol_ctx_create(0, &cb)) return 1;
    STEP("ctx");
    double *JT, *A, *A2, *rhs, *sig;
    int* dinfo;
    hipMalloc(&JT, sizeof(double) * (size_t)n * m);
    STEP("malloc JT");
    hipMalloc(&A, sizeof(double) * (size_t)n * n);
    hipMalloc(&A2, sizeof(double) * (size_t)n * n);
    hipMalloc(&rhs, sizeof(double) * n);
    hipMalloc(&sig, sizeof(double) * n);
    hipMalloc(&dinfo, sizeof(int));
    STEP("mallocs");
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, JT, (long)n * m);
    STEP("fill");
    hipLaunchKernelGGL(k_fill, dim3(8), dim3(256), 0, 0, rhs, (long)n);
    hipDeviceSynchronize();
    STEP("alloc");
    pnol_jtj_d(ca, JT, m, m, n, 1e-3, A2, n, nullptr);   // an SPD system for the solve
    pnol_ctx_synchronize(ca);
    auto jtj = [&](pnol_ctx* c) { pnol_jtj_d(c, JT, m, m, n, 1e-3, A, n, nullptr); };
    auto solve = [&](pnol_ctx* c) { pnol_solve_async_d(c, A2, n, rhs, sig, n, dinfo); };
    std::printf("{\"cus\": %d", ncu);
    pnol_ctx_set_stream(ca, nullptr);
    pnol_ctx_set_stream(cb, nullptr);
    STEP("spd");
    std::printf(", \"jtj_full_ms\": %.4f", timeit([&] { jtj(ca); }));
    std::printf(", \"solve_full_ms\": %.4f", timeit([&] { solve(cb); }));
    std::printf(", \"serial_full_ms\": %.4f", timeit([&] { jtj(ca); solve(ca); }));
    struct Split { const char* name; int a_first, a_count, a_stride, b_first, b_count, b_stride; };
    // masks: B gets `count` CUs (contiguous low ids, or spread by stride), A the rest
    const Split splits[] = {
        {"b16_low", 16, ncu - 16, 1, 0, 16, 1},
        {"b16_spread", 1, ncu - 16, 1, 0, 16, 16},
        {"b32_low", 32, ncu - 32, 1, 0, 32, 1},
        {"b8_low", 8, ncu - 8, 1, 0, 8, 1},
    };
    for (const Split& s : splits) {
        hipStream_t sa, sb;
        if (s.b_stride == 1) {
            sa = masked(ncu, s.a_first, s.a_count, 1);
            sb = masked(ncu, s.b_first, s.b_count, 1);
        } else {   // B = every stride-th CU from 0, A = the others
            std::vector<uint32_t> ma((ncu + 31) / 32, 0u), mb((ncu + 31) / 32, 0u);
            for (int c = 0; c < ncu; ++c) {
                if (c % s.b_stride == 0 && c / s.b_stride < s.b_count) mb[c / 32] |= 1u << (c % 32);
                else ma[c / 32] |= 1u << (c % 32);
            }
            hipExtStreamCreateWithCUMask(&sa, (uint32_t)ma.size(), ma.data());
            hipExtStreamCreateWithCUMask(&sb, (uint32_t)mb.size(), mb.data());
        }
        if (!sa || !sb) {
            std::printf(", \"%s\": \"mask refused\"", s.name);
            continue;
        }
        STEP(s.name);
        pnol_ctx_set_stream(ca, sa);
        pnol_ctx_set_stream(cb, sb);
        const double ja = timeit([&] { jtj(ca); });
        const double sbm = timeit([&] { solve(cb); });
        const double both = timeit([&] { jtj(ca); solve(cb); });
        std::printf(", \"%s\": {\"jtj_ms\": %.4f, \"solve_ms\": %.4f, \"concurrent_ms\": %.4f}", s.name, ja, sbm, both);
        pnol_ctx_set_stream(ca, nullptr);
        pnol_ctx_set_stream(cb, nullptr);
        hipStreamDestroy(sa);
        hipStreamDestroy(sb);
    }
    int hinfo = 0;
    hipMemcpy(&hinfo, dinfo, sizeof(int), hipMemcpyDeviceToHost);
    std::printf(", \"solve_info\": %d}\n", hinfo);
    return 0;
}
