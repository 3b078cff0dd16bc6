// Dependent fp64 add chains on gfx950: how many shader cycles one sequential f = f + t_k step
// costs (the objective's own summation order -- the FD gradient's and the line-search
// evaluations' critical path), with the addends
//   reg   in VGPRs (the pure v_add_f64 dependent latency),
//   lds8  from LDS, the next 8 in flight while 8 are added (fd.hip chain_sum),
//   lds16 the same with 16 / 32 in flight,
// for C independent chains per lane interleaved (C = 1, 2, 4).  One wave per launch, s_memtime
// around the loop.  Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 add_chain.hip -o add_chain
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kN = 8192;

template <int C>
__global__ void k_reg(double* out, double a0, long long* clk) {
    double t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = a0 * (i + 1) + threadIdx.x * 1e-9;
    double f[C];
#pragma unroll
    for (int c = 0; c < C; ++c) f[c] = c;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < kN; k += 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
#pragma unroll
            for (int c = 0; c < C; ++c) f[c] = f[c] + t[(i + c) & 15];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += f[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) clk[0] = t1 - t0;
}

// addends from LDS (every lane the same address: a broadcast), D in flight
template <int C, int D>
__global__ void k_lds(const double* __restrict__ T, double* out, long long* clk) {
    __shared__ double Ts[kN];
    for (int e = threadIdx.x; e < kN; e += blockDim.x) Ts[e] = T[e];
    __syncthreads();
    double f[C];
#pragma unroll
    for (int c = 0; c < C; ++c) f[c] = c;
    const long long t0 = __builtin_amdgcn_s_memtime();
    double cur[D];
#pragma unroll
    for (int q = 0; q < D; ++q) cur[q] = Ts[q];
    for (int k = 0; k + 2 * D <= kN; k += D) {
        double nxt[D];
#pragma unroll
        for (int q = 0; q < D; ++q) nxt[q] = Ts[k + D + q];
#pragma unroll
        for (int q = 0; q < D; ++q)
#pragma unroll
            for (int c = 0; c < C; ++c) f[c] = f[c] + cur[q];
#pragma unroll
        for (int q = 0; q < D; ++q) cur[q] = nxt[q];
    }
#pragma unroll
    for (int q = 0; q < D; ++q)
#pragma unroll
        for (int c = 0; c < C; ++c) f[c] = f[c] + cur[q];
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += f[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) clk[0] = t1 - t0;
}


// ping-pong register buffers (no cur = nxt copies), D in flight; B128: double2 LDS reads
template <int D, bool B128>
__global__ void k_lds_pp(const double* __restrict__ T, double* out, long long* clk) {
    __shared__ __attribute__((aligned(16))) double Ts[kN];
    for (int e = threadIdx.x; e < kN; e += blockDim.x) Ts[e] = T[e];
    __syncthreads();
    double f = 0.0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    double a[D], b[D];
    auto ld = [&](double (&dst)[D], int k) {
        if (B128) {
#pragma unroll
            for (int q = 0; q < D; q += 2) {
                const double2 v = *reinterpret_cast<const double2*>(Ts + k + q);
                dst[q] = v.x;
                dst[q + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int q = 0; q < D; ++q) dst[q] = Ts[k + q];
        }
    };
    ld(a, 0);
    for (int k = 0; k + 2 * D <= kN; k += 2 * D) {
        ld(b, k + D);
#pragma unroll
        for (int q = 0; q < D; ++q) f = f + a[q];
        if (k + 3 * D <= kN) ld(a, k + 2 * D);
#pragma unroll
        for (int q = 0; q < D; ++q) f = f + b[q];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = f;
    if (threadIdx.x == 0) clk[0] = t1 - t0;
}

// addends by scalar loads straight from global memory (uniform index), D per block
template <int D>
__global__ void k_sld(const double* __restrict__ T, double* out, long long* clk) {
    double f = 0.0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < kN; k += D) {
#pragma unroll
        for (int q = 0; q < D; ++q) f = f + T[k + q];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = f;
    if (threadIdx.x == 0) clk[0] = t1 - t0;
}


// DPP broadcast: each 16-lane row holds 16 terms (lane l: T[k + (l & 15)]); the add takes term q
// with row_newbcast:q -- one v_add_f64 per term, no LDS read on the chain
template <int Q>
__device__ __forceinline__ double add_bcast(double f, double t) {
    double b;
    asm("v_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(b) : "v"(t), "i"(Q));
    f = f + b;
    return f;
}
template <int Q = 0>
__device__ __forceinline__ double add16(double f, double t) {
    f = add_bcast<Q>(f, t);
    if constexpr (Q + 1 < 16) return add16<Q + 1>(f, t);
    else return f;
}
__global__ void k_dpp(const double* __restrict__ T, double* out, long long* clk) {
    __shared__ __attribute__((aligned(16))) double Ts[kN];
    for (int e = threadIdx.x; e < kN; e += blockDim.x) Ts[e] = T[e];
    __syncthreads();
    const int r = threadIdx.x & 15;
    double f = 0.0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    double a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = Ts[16 * q + r];
    for (int k = 0; k + 128 <= kN; k += 128) {
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = Ts[k + 64 + 16 * q + r];
#pragma unroll
        for (int q = 0; q < 4; ++q) f = add16(f, a[q]);
        if (k + 192 <= kN) {
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = Ts[k + 128 + 16 * q + r];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) f = add16(f, b[q]);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = f;
    if (threadIdx.x == 0) clk[0] = t1 - t0;
}


// the shader clock under this load: s_memtime cycles over 100 MHz s_memrealtime ticks around a
// k_lds<1, 16>-style chain, for G workgroups of W waves
__global__ void k_clock(const double* __restrict__ T, double* out, long long* clk) {
    __shared__ double Ts[kN];
    for (int e = threadIdx.x; e < kN; e += blockDim.x) Ts[e] = T[e];
    __syncthreads();
    double f = 0.0;
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int rep = 0; rep < 8; ++rep) {
        double cur[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) cur[q] = Ts[q];
        for (int k = 0; k + 32 <= kN; k += 16) {
            double nxt[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) nxt[q] = Ts[k + 16 + q];
#pragma unroll
            for (int q = 0; q < 16; ++q) f = f + cur[q];
#pragma unroll
            for (int q = 0; q < 16; ++q) cur[q] = nxt[q];
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) f = f + cur[q];
    }
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = f;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

static void clock_probe(const double* T, int G, int W) {
    double* out;
    long long* clk;
    hipMalloc(&out, sizeof(double) * G * W * 64);
    hipMalloc(&clk, 16);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_clock, dim3(G), dim3(64 * W), 0, 0, T, out, clk);
    hipDeviceSynchronize();
    long long c[2];
    hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    std::printf(", \"clock_G%d_W%d\": {\"cycles_per_step\": %.2f, \"MHz\": %.0f}", G, W, (double)c[0] / (8.0 * kN),
                c[1] > 0 ? (double)c[0] / (double)c[1] * 100.0 : 0.0);
    hipFree(out);
    hipFree(clk);
}


// readlane broadcast: lane l holds T[k + l]; term q of the block goes to every lane through two
// v_readlane_b32 (SGPR operand of the add) -- no LDS read on the chain
__device__ __forceinline__ double rl(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
__global__ void k_rl(const double* __restrict__ T, double* out, long long* clk) {
    const int lane = threadIdx.x & 63;
    double f = 0.0;
    double a = T[lane], b;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k + 128 <= kN; k += 128) {
        b = T[k + 64 + lane];
#pragma unroll
        for (int q = 0; q < 64; ++q) f = f + rl(a, q);
        if (k + 192 <= kN) a = T[k + 128 + lane];
#pragma unroll
        for (int q = 0; q < 64; ++q) f = f + rl(b, q);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = f;
    if (threadIdx.x == 0) clk[0] = t1 - t0;
}

template <class K, class... A>
static double run(K kern, int threads, A... a) {
    long long* clk;
    hipMalloc(&clk, 8);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, a..., clk);
    hipDeviceSynchronize();
    long long c = 0;
    hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
    hipFree(clk);
    return (double)c / kN;   // cycles per step of one chain
}

int main() {
    double *T, *out;
    hipMalloc(&T, sizeof(double) * kN);
    hipMalloc(&out, sizeof(double) * 256);
    {
        double h[kN];
        for (int i = 0; i < kN; ++i) h[i] = 1.0 / (i + 3) + (i % 7) * 1e-3;
        hipMemcpy(T, h, sizeof(h), hipMemcpyHostToDevice);
        double ref = 0.0;
        for (int i = 0; i < kN; ++i) ref = ref + h[i];
        long long* c;
        hipMalloc(&c, 8);
        hipLaunchKernelGGL(k_dpp, dim3(1), dim3(64), 0, 0, (const double*)T, out, c);
        double got[64];
        hipMemcpy(got, out, sizeof(got), hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l) bad += got[l] != ref;
        std::fprintf(stderr, "dpp chain vs host sequential sum: %d of 64 lanes differ (ref %.17g got %.17g)\n", bad, ref, got[0]);
        hipFree(c);
    }
    std::printf("{\"cycles_per_step\": {");
    std::printf("\"reg_c1\": %.2f, ", run(k_reg<1>, 64, out, 1e-3));
    std::printf("\"reg_c2\": %.2f, ", run(k_reg<2>, 64, out, 1e-3));
    std::printf("\"reg_c4\": %.2f, ", run(k_reg<4>, 64, out, 1e-3));
    std::printf("\"lds8_c1\": %.2f, ", run(k_lds<1, 8>, 64, (const double*)T, out));
    std::printf("\"lds16_c1\": %.2f, ", run(k_lds<1, 16>, 64, (const double*)T, out));
    std::printf("\"lds32_c1\": %.2f, ", run(k_lds<1, 32>, 64, (const double*)T, out));
    std::printf("\"lds16_c2\": %.2f, ", run(k_lds<2, 16>, 64, (const double*)T, out));
    std::printf("\"lds16_c4\": %.2f, ", run(k_lds<4, 16>, 64, (const double*)T, out));
    std::printf("\"pp8\": %.2f, ", run(k_lds_pp<8, false>, 64, (const double*)T, out));
    std::printf("\"pp16\": %.2f, ", run(k_lds_pp<16, false>, 64, (const double*)T, out));
    std::printf("\"pp16_b128\": %.2f, ", run(k_lds_pp<16, true>, 64, (const double*)T, out));
    std::printf("\"pp32_b128\": %.2f, ", run(k_lds_pp<32, true>, 64, (const double*)T, out));
    std::printf("\"pp16_b128_4waves\": %.2f, ", run(k_lds_pp<16, true>, 256, (const double*)T, out));
    std::printf("\"sld8\": %.2f, ", run(k_sld<8>, 64, (const double*)T, out));
    std::printf("\"sld16\": %.2f, ", run(k_sld<16>, 64, (const double*)T, out));
    std::printf("\"sld32\": %.2f, ", run(k_sld<32>, 64, (const double*)T, out));
    std::printf("\"dpp\": %.2f, ", run(k_dpp, 64, (const double*)T, out));
    std::printf("\"dpp_4waves\": %.2f, ", run(k_dpp, 256, (const double*)T, out));
    std::printf("\"readlane\": %.2f, ", run(k_rl, 64, (const double*)T, out));
    std::printf("\"readlane_4waves\": %.2f", run(k_rl, 256, (const double*)T, out));
    std::printf("}");
    clock_probe(T, 1, 1);
    clock_probe(T, 1, 4);
    clock_probe(T, 65, 4);
    clock_probe(T, 256, 4);
    clock_probe(T, 1024, 4);
    std::printf("}\n");
    return 0;
}
