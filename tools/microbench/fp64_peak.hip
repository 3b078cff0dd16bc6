// fp64 peak microbenchmark for gfx950: v_mfma_f64_16x16x4_f64 and VALU v_fma_f64 throughput
// with independent accumulator chains on every SIMD (confirm the 78.6 TF
// denominator).  Prints one JSON line.   hipcc --offload-arch=gfx950 -O3 fp64_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma(double* out, int iters, double a0) {
    d4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (d4){0, 0, 0, 0};
    double a = a0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.678) out[0] = s;
}

__global__ __launch_bounds__(256) void k_valu(double* out, int iters, double a0) {
    double acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = i;
    const double a = a0 + threadIdx.x * 1e-12, b = 1.0 - 1e-12;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = fma(acc[i], b, a);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i];
    if (s == 12345.678) out[0] = s;
}

int main() {
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    double* out;
    hipMalloc(&out, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = ncu * 8;   // 8 WGs x 4 waves per CU = 8 waves per SIMD
    const int it_m = 4000, it_v = 20000;
    float ms = 0;
    // MFMA: per wave per iteration 8 x (16*16*4*2) flop
    hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out, it_m, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double mf = (double)blocks * 4 * it_m * 8 * 2048.0;
    const double tf_mfma = mf / (ms * 1e-3) / 1e12;
    // VALU: per thread per iteration 16 fma = 32 flop
    hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, out, it_v, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms2 = 0;
    hipEventElapsedTime(&ms2, e0, e1);
    const double vf = (double)blocks * 256 * it_v * 32.0;
    const double tf_valu = vf / (ms2 * 1e-3) / 1e12;
    std::printf("{\"cus\": %d, \"mfma_f64_16x16x4_tflops\": %.2f, \"mfma_ms\": %.3f, \"valu_fma_f64_tflops\": %.2f, "
                "\"valu_ms\": %.3f}\n", ncu, tf_mfma, ms, tf_valu, ms2);
    return 0;
}
