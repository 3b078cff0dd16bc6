// Latency of the Cholesky pivot chain's pieces on gfx950 (one wave, shader cycles per step):
// l = a * r; piv = readlane(fma(-l, l, b), 1); r = rsqrt_nr(piv) and variants.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 tools/microbench/piv_chain.hip -o tools/microbench/piv_chain
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rsqrt_nr(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    const double e = fma(-x, r * r, 1.0);
    const double p = fma(e, 0.375, 0.5);
    return fma(r * e, p, r);
}

template <int V>
__global__ void k_chain(const double* in, double* out, long long* cyc) {
    const int lane = threadIdx.x;
    double a = in[lane], b = in[64 + lane], r = 1.0 / sqrt(in[lane]);
    double acc = 0.0;
    double x[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = in[(lane + q) & 127];
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < 256; ++it) {
        const double l = a * r;
        double piv;
        if constexpr (V == 0 || V == 2 || V == 3 || V >= 4) piv = readlane_d(fma(-l, l, b), 1);
        else piv = fma(-l, l, b);
        if constexpr (V == 0 || V == 1 || V >= 4) r = rsqrt_nr(piv);
        else if constexpr (V == 2) r = __builtin_amdgcn_rsq(piv);
        else r = piv * 0.5 + 0.25;   // V 3: no transcendental (readlane + 4 VALU ops)
        if constexpr (V >= 4) {   // independent work beside the chain: NF fmas (+ readlane pairs)
            constexpr int NF = V == 4 ? 8 : 16;
#pragma unroll
            for (int q = 0; q < NF; ++q) {
                double c = V == 6 && q < 6 ? readlane_d(l, q + 2) : x[(q + 3) & 15];
                x[q] = fma(-l, c, x[q]);
            }
        }
        acc += l;
        asm volatile("" : "+v"(r));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double xs = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) xs += x[q];
    out[lane] = acc + r + xs;
    if (lane == 0) cyc[V] = t1 - t0;
}

int main() {
    double h[128];
    for (int i = 0; i < 64; ++i) { h[i] = 1.0 + 0.001 * i; h[64 + i] = 2.0 + 0.001 * i; }
    double *din, *dout; long long* dc;
    hipMalloc(&din, sizeof h); hipMalloc(&dout, 8 * 64); hipMalloc(&dc, 8 * 8);
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, din, dout, dc);
        hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, din, dout, dc);
        hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, din, dout, dc);
        hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, din, dout, dc);
        hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(64), 0, 0, din, dout, dc);
        hipLaunchKernelGGL(k_chain<5>, dim3(1), dim3(64), 0, 0, din, dout, dc);
        hipLaunchKernelGGL(k_chain<6>, dim3(1), dim3(64), 0, 0, din, dout, dc);
        hipDeviceSynchronize();
    }
    long long c[8];
    hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
    printf("{\"cycles_per_step\": {\"readlane+rsqrt_nr\": %.1f, \"rsqrt_nr_only\": %.1f, \"readlane+rsq\": %.1f, "
           "\"readlane+valu\": %.1f, \"chain+8fma\": %.1f, \"chain+16fma\": %.1f, \"chain+16fma_6readlane\": %.1f}}\n",
           c[0] / 256.0, c[1] / 256.0, c[2] / 256.0, c[3] / 256.0, c[4] / 256.0, c[5] / 256.0, c[6] / 256.0);
    return 0;
}
