// Does streaming 256 contiguous 1 MB row panels in lockstep (the k_linres_evalP pattern: wave b
// reads panel b front to back, 512 B per step) lose bandwidth to HBM channel camping, against the
// same bytes block-interleaved (step k of wave b at (k * nw + b) * 512)?  One wave per workgroup,
// 16 independent 8-byte loads in flight per lane per step group, a sum per lane to keep them.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/panel_stride_probe.hip -o tools/microbench/panel_stride_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool INTERLEAVED>
__global__ __launch_bounds__(64) void k_stream(const double* __restrict__ a, int steps, int nw, double* out) {
    const int b = blockIdx.x, lane = threadIdx.x;
    double acc = 0.0;
    for (int k0 = 0; k0 < steps; k0 += 16) {
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const long k = k0 + q;
            const long off = INTERLEAVED ? (k * nw + b) * 64 : ((long)b * steps + k) * 64;
            v[q] = __builtin_nontemporal_load(a + off + lane);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) acc += v[q];
    }
    out[b * 64 + lane] = acc;
}

int main() {
    const int nw = 256, steps = 2048;   // 256 panels x 2048 steps x 512 B = 268 MB (cfg 3's A)
    const size_t n = (size_t)nw * steps * 64;
    double *a, *out;
    hipMalloc(&a, n * sizeof(double));
    hipMalloc(&out, nw * 64 * sizeof(double));
    hipMemset(a, 0, n * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 2; ++mode) {
            float best = 1e9f;
            for (int it = 0; it < 10; ++it) {
                hipEventRecord(e0);
                if (mode) k_stream<true><<<nw, 64>>>(a, steps, nw, out);
                else k_stream<false><<<nw, 64>>>(a, steps, nw, out);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            std::printf("{\"layout\": \"%s\", \"us\": %.1f, \"GBps\": %.0f}\n", mode ? "interleaved" : "contiguous panels",
                        best * 1e3, n * 8.0 / (best * 1e-3) / 1e9);
        }
    hipFree(a);
    hipFree(out);
    return 0;
}
