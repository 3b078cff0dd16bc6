// fp64 peak microbenchmark for gfx950: v_mfma_f64_16x16x4_f64 and VALU v_fma_f64 throughput
// (confirm the 78.6 TF denominator).  Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 fp64_peak.hip -o fp64_peak
//
// The sustained TFLOP/s of a saturating kernel depends on the clock the chip holds under that
// load (DVFS), so every wave also records the shader clock counter (s_memtime) and the constant
// 100 MHz reference (s_memrealtime) around its loop.  That gives the clock actually sustained
// and the issue rate in flops per cycle per CU -- the hardware rate, which times the 2.4 GHz peak
// clock is the spec-sheet peak.  Launch configurations sweep waves per SIMD and independent
// accumulator chains so the rate is the MFMA pipe's, not a latency bound.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

// CH independent accumulators; each chain has its own A / B operand registers (DISTINCT), or
// all chains share one pair
template <int CH, bool DISTINCT = false>
__global__ __launch_bounds__(256) void k_mfma(double* out, long long* clk, int iters, double a0) {
    d4 acc[CH];
    double a[DISTINCT ? CH : 1], b[DISTINCT ? CH : 1];
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = (d4){0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < (DISTINCT ? CH : 1); ++i) {
        a[i] = a0 + threadIdx.x * 1e-9 + i * 1e-12;
        b[i] = 1.0 - threadIdx.x * 1e-9 - i * 1e-12;
    }
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i)   // accumulators pinned in VGPRs (the builtin's form moved
                                       // every accumulator VGPR <-> AGPR each iteration)
            asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0"
                         : "+v"(acc[i])
                         : "v"(a[DISTINCT ? i : 0]), "v"(b[DISTINCT ? i : 0]));
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        clk[2 * w] = t1 - t0;
        clk[2 * w + 1] = r1 - r0;
    }
    if (s == 12345.678) out[0] = s;
}

__global__ __launch_bounds__(256) void k_valu(double* out, long long* clk, int iters, double a0) {
    double acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = i;
    const double a = a0 + threadIdx.x * 1e-12, b = 1.0 - 1e-12;
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = fma(acc[i], b, a);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i];
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        clk[2 * w] = t1 - t0;
        clk[2 * w + 1] = r1 - r0;
    }
    if (s == 12345.678) out[0] = s;
}

struct Run {
    double ms, tflops, clock_ghz, flops_per_cycle_cu;
};

// flop_per_wave: flops one wave executes in the timed launch
template <class Launch>
static Run run(Launch launch, int blocks, double flop_per_wave, int ncu, long long* dclk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch(10);   // warm
    hipEventRecord(e0);
    launch(-1);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const int waves = blocks * 4;
    std::vector<long long> h(2 * (size_t)waves);
    hipMemcpy(h.data(), dclk, sizeof(long long) * h.size(), hipMemcpyDeviceToHost);
    double cyc = 0, real = 0;
    for (int w = 0; w < waves; ++w) {
        cyc += (double)h[2 * w];
        real += (double)h[2 * w + 1];
    }
    cyc /= waves;                   // shader clocks per wave loop
    real /= waves;                  // 100 MHz ticks per wave loop
    Run r;
    r.ms = ms;
    r.tflops = flop_per_wave * waves / (ms * 1e-3) / 1e12;
    r.clock_ghz = cyc / real * 0.1;
    // every wave runs its loop concurrently (all resident): the chip's flops per shader cycle
    r.flops_per_cycle_cu = flop_per_wave * waves / cyc / ncu;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return r;
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    double* out;
    long long* clk;
    hipMalloc(&out, 8);
    hipMalloc(&clk, sizeof(long long) * 2 * ncu * 64);
    std::printf("{\"cus\": %d, \"mfma_f64_16x16x4\": [", ncu);
    bool first = true;
    double best_fpc = 0, best_tf = 0;
    for (int wps : {1, 2, 4}) {            // workgroups of 4 waves per CU = waves per SIMD requested
        for (int var = 0; var < 4; ++var) {   // chains 4 / 8 / 16, 8 with distinct operands
            const int ch = var == 0 ? 4 : (var == 2 ? 16 : 8);
            const bool dist = var == 3;
            const int blocks = ncu * wps;
            const int iters = 4000 * 8 / ch;
            auto launch = [&](int it) {
                const int n = it < 0 ? iters : it;
                if (var == 0) hipLaunchKernelGGL((k_mfma<4>), dim3(blocks), dim3(256), 0, 0, out, clk, n, 1.0);
                else if (var == 1) hipLaunchKernelGGL((k_mfma<8>), dim3(blocks), dim3(256), 0, 0, out, clk, n, 1.0);
                else if (var == 2) hipLaunchKernelGGL((k_mfma<16>), dim3(blocks), dim3(256), 0, 0, out, clk, n, 1.0);
                else hipLaunchKernelGGL((k_mfma<8, true>), dim3(blocks), dim3(256), 0, 0, out, clk, n, 1.0);
            };
            const Run r = run(launch, blocks, (double)iters * ch * 2048.0, ncu, clk);
            // flops per shader cycle per CU from the kernel time and the clock the waves measured
            const double fpc = r.tflops * 1e12 / (r.clock_ghz * 1e9) / ncu;
            if (fpc > best_fpc) best_fpc = fpc;
            if (r.tflops > best_tf) best_tf = r.tflops;
            std::printf("%s{\"waves_per_simd\": %d, \"chains\": %d, \"distinct_operands\": %s, \"ms\": %.3f, "
                        "\"tflops\": %.2f, \"clock_ghz\": %.3f, \"flops_per_cycle_per_cu\": %.1f}",
                        first ? "" : ", ", wps, ch, dist ? "true" : "false", r.ms, r.tflops, r.clock_ghz, fpc);
            first = false;
        }
    }
    auto vlaunch = [&](int it) {
        hipLaunchKernelGGL(k_valu, dim3(ncu * 8), dim3(256), 0, 0, out, clk, it < 0 ? 20000 : it, 1.0);
    };
    const Run v = run(vlaunch, ncu * 8, 20000.0 * 16 * 2 * 64, ncu, clk);
    std::printf("], \"valu_fma_f64\": {\"tflops\": %.2f, \"clock_ghz\": %.3f, \"flops_per_cycle_per_cu\": %.1f}, "
                "\"mfma_best_sustained_tflops\": %.2f, \"mfma_flops_per_cycle_per_cu\": %.1f, "
                "\"mfma_peak_tflops_at_2p4ghz\": %.2f}\n",
                v.tflops, v.clock_ghz, v.tflops * 1e12 / (v.clock_ghz * 1e9) / ncu, best_tf, best_fpc,
                best_fpc * ncu * 2.4e9 / 1e12);
    return 0;
}
