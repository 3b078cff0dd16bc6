// Per-workgroup timeline of the J^T J split-K SYRK (syrk.hip k_syrk_tile, the bench's
// configuration): where the gap between the MFMA-busy fraction and the kernel time goes --
// per-workgroup duration of the long / short K chunks, concurrency over time, the tail after
// the last dispatch, the balance over the XCDs.  Prints one JSON line.  Build (after the library):
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -I include \
//     -I parallelnonlinearoptimizationlibrary_amd/csrc tools/microbench/syrk_timeline.hip \
//     -L parallelnonlinearoptimizationlibrary_amd -lpnol_amd \
//     -Wl,-rpath,'$ORIGIN/../../parallelnonlinearoptimizationlibrary_amd' -o tools/microbench/syrk_timeline
#define PNOL_SYRK_TIMELINE 1
#include "../../parallelnonlinearoptimizationlibrary_amd/csrc/kernels/syrk.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_fill(double* x, long count) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < count; i += (long)gridDim.x * blockDim.x) {
        unsigned long long z = (unsigned long long)i * 0x9E3779B97F4A7C15ull + 0x5EED;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    }
}

int main(int argc, char** argv) {
    using namespace pnol;
    const int m = argc > 1 ? std::atoi(argv[1]) : 16384, n = argc > 2 ? std::atoi(argv[2]) : 2048;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
    pnol_ctx* ctx = nullptr;
    if (pnol_ctx_create(0, &ctx) != PNOL_OK) {
        std::fprintf(stderr, "no device\n");
        return 1;
    }
    const int nt = (n + kTile - 1) / kTile, ntiles = nt * (nt + 1) / 2;
    const SliceCfg sc = slice_cfg(m, ntiles);
    const int split = kS * sc.sub, grid = ntiles * split;
    if (grid > 65536) {
        std::fprintf(stderr, "grid too large for the timeline buffer\n");
        return 1;
    }
    double *JT, *part;
    hipMalloc(&JT, sizeof(double) * (size_t)n * m);
    hipMalloc(&part, sizeof(double) * (size_t)grid * kTile * kTile);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, ctx->stream, JT, (long)n * m);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ms(reps);
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(e0, ctx->stream);
        syrk_partials(ctx, ctx->stream, false, JT, m, sc.mS, n, m, sc, 0, kS, 0, ntiles, part, false);
        hipEventRecord(e1, ctx->stream);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms[r], e0, e1);
    }
    std::vector<unsigned long long> tl(3 * (size_t)grid);
    hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(g_syrk_tl), sizeof(unsigned long long) * tl.size());
    // the last repetition's timeline (10 ns ticks)
    unsigned long long t0 = ~0ull, t1 = 0, last_start = 0;
    for (int b = 0; b < grid; ++b) {
        t0 = std::min(t0, tl[3 * b]);
        t1 = std::max(t1, tl[3 * b + 1]);
        last_start = std::max(last_start, tl[3 * b]);
    }
    // K chunk of each workgroup (u = 0: the long first chunk) from the dispatch mapping
    const int ntl = grid / split, nsl = split / sc.sub;
    double dur_sum[2] = {0, 0}, dur_max[2] = {0, 0}, dur_min[2] = {1e30, 1e30};
    int cnt[2] = {0, 0};
    std::vector<std::pair<unsigned long long, int>> ev;
    double busy = 0, xbusy[8] = {0};
    int xcnt[8] = {0};
    for (int b = 0; b < grid; ++b) {
        const int u = b / (ntl * nsl);   // k_syrk_tile's dispatch order: every chunk 0 first
        const int c = u == 0 ? 0 : 1;
        const double d = (double)(tl[3 * b + 1] - tl[3 * b]) * 0.01;   // us
        dur_sum[c] += d;
        dur_max[c] = std::max(dur_max[c], d);
        dur_min[c] = std::min(dur_min[c], d);
        cnt[c]++;
        busy += d;
        const int x = (int)(tl[3 * b + 2] >> 32) & 7;
        xbusy[x] += d;
        xcnt[x]++;
        ev.push_back({tl[3 * b], +1});
        ev.push_back({tl[3 * b + 1], -1});
    }
    std::sort(ev.begin(), ev.end());
    int run = 0, peak = 0;
    double area = 0;
    unsigned long long prev = t0, drop = 0;
    for (auto& e : ev) {
        area += (double)run * (e.first - prev);
        prev = e.first;
        run += e.second;
        peak = std::max(peak, run);
    }
    // the tail: from the first moment after the last dispatch that fewer than peak - 8 run
    run = 0;
    for (auto& e : ev) {
        run += e.second;
        if (e.first >= last_start && run < peak - 8 && !drop) drop = e.first;
    }
    const double span = (t1 - t0) * 0.01;
    const double flops = (double)m * n * (n + 1);
    std::printf("{\"m\": %d, \"n\": %d, \"tiles\": %d, \"sub\": %d, \"kfirst\": %d, \"kchunk\": %d, \"workgroups\": %d, "
                "\"ms_events\": [", m, n, ntiles, sc.sub, sc.kfirst, sc.kchunk, grid);
    for (int r = 0; r < reps; ++r) std::printf("%s%.4f", r ? ", " : "", ms[r]);
    std::printf("], \"span_us\": %.1f, \"tflops_span\": %.2f, \"peak_concurrency\": %d, \"mean_concurrency\": %.1f, "
                "\"slot_fill\": %.4f, \"last_dispatch_us\": %.1f, \"tail_us\": %.1f, "
                "\"long_chunk_us\": {\"count\": %d, \"mean\": %.1f, \"min\": %.1f, \"max\": %.1f}, "
                "\"short_chunk_us\": {\"count\": %d, \"mean\": %.1f, \"min\": %.1f, \"max\": %.1f}, \"xcd\": [",
                span, flops / (span * 1e-6) / 1e12, peak, area / (t1 - t0), area / ((double)peak * (t1 - t0)),
                (last_start - t0) * 0.01, drop ? (t1 - drop) * 0.01 : 0.0, cnt[0], cnt[0] ? dur_sum[0] / cnt[0] : 0,
                cnt[0] ? dur_min[0] : 0, dur_max[0], cnt[1], cnt[1] ? dur_sum[1] / cnt[1] : 0, cnt[1] ? dur_min[1] : 0,
                dur_max[1]);
    for (int x = 0; x < 8; ++x) std::printf("%s{\"wgs\": %d, \"busy_us\": %.0f}", x ? ", " : "", xcnt[x], xbusy[x]);
    std::printf("]}\n");
    return 0;
}
