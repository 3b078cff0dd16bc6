// Per-workgroup timeline of the LM trip's k_syrk_red launch (syrk.hip: the split-K SYRK workgroups
// and, after them in the grid, the in-launch reduce workgroups), the bench's configuration
// (sub = 2, diagonal tiles last).  Where the launch's time goes beyond the MFMA work: slot fill
// while the SYRK workgroups run, the per-chunk durations against the MFMA-bound time of the same
// chunk, the reduce tail after the last SYRK workgroup.  Prints one JSON line.  Build (after the
// library):
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -I include \
//     -I parallelnonlinearoptimizationlibrary_amd/csrc tools/microbench/syrk_red_timeline.hip \
//     -L parallelnonlinearoptimizationlibrary_amd -lpnol_amd \
//     -Wl,-rpath,'$ORIGIN/../../parallelnonlinearoptimizationlibrary_amd' -o tools/microbench/syrk_red_timeline
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
    if (sc.sub != 2) {
        std::fprintf(stderr, "this driver launches the sub = 2 instance\n");
        return 1;
    }
    const int noff = nt * (nt - 1) / 2;
    const int split = kS * sc.sub, nsyrk = ntiles * split, nred = (kTile / kRedSR) * (ntiles + 1);
    const int grid = nsyrk + nred;
    if (grid > 65536) {
        std::fprintf(stderr, "grid too large for the timeline buffer\n");
        return 1;
    }
    double *JT, *part, *A, *jp, *rhs, *rhs2;
    int *tcnt, *info;
    hipMalloc(&JT, sizeof(double) * (size_t)n * m);
    hipMalloc(&part, sizeof(double) * (size_t)nsyrk * kTile * kTile);
    hipMalloc(&A, sizeof(double) * (size_t)n * n);
    hipMalloc(&jp, sizeof(double) * (size_t)kS * n);
    hipMalloc(&rhs, sizeof(double) * n);
    hipMalloc(&rhs2, sizeof(double) * n);
    hipMalloc(&tcnt, sizeof(int) * ntiles);
    hipMalloc(&info, sizeof(int));
    hipMemset(jp, 0, sizeof(double) * (size_t)kS * n);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, ctx->stream, JT, (long)n * m);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ms(reps);
    for (int r = 0; r < reps; ++r) {
        hipMemsetAsync(tcnt, 0, sizeof(int) * ntiles, ctx->stream);
        hipMemsetAsync(info, 0, sizeof(int), ctx->stream);
        hipEventRecord(e0, ctx->stream);
        hipLaunchKernelGGL((k_syrk_red<2, false, true>), dim3(grid), dim3(512), 0, ctx->stream, JT, (long)m, n, m, split,
                           sc.kfirst, sc.kchunk, sc.sub, sc.mS, (long)sc.mS, part, nsyrk, tcnt, ntiles, n, 0.01, A,
                           (long)n, (const double*)jp, rhs, rhs2, info);
        hipEventRecord(e1, ctx->stream);
        if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess) {
            std::fprintf(stderr, "launch failed\n");
            return 1;
        }
        hipEventElapsedTime(&ms[r], e0, e1);
    }
    int hinfo = 0;
    hipMemcpy(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost);
    std::vector<unsigned long long> tl(3 * (size_t)grid);
    hipMemcpyFromSymbol(tl.data(), HIP_SYMBOL(g_syrk_tl), sizeof(unsigned long long) * tl.size());
    // the last repetition (10 ns ticks)
    unsigned long long t0 = ~0ull, t1 = 0, syrk_end = 0, last_syrk_start = 0, red_first = ~0ull;
    for (int b = 0; b < grid; ++b) {
        t0 = std::min(t0, tl[3 * b]);
        t1 = std::max(t1, tl[3 * b + 1]);
        if (b < nsyrk) {
            syrk_end = std::max(syrk_end, tl[3 * b + 1]);
            last_syrk_start = std::max(last_syrk_start, tl[3 * b]);
        } else {
            red_first = std::min(red_first, tl[3 * b]);
        }
    }
    // SYRK workgroups by chunk (u = 0 long) and diagonal / off-diagonal tile (the DLAST order:
    // local tile index tl >= noff is a diagonal tile)
    const int nsl = split / sc.sub;
    double dsum[2][2] = {{0, 0}, {0, 0}}, dmax[2][2] = {{0, 0}, {0, 0}};
    int cnt[2][2] = {{0, 0}, {0, 0}};
    std::vector<std::pair<unsigned long long, int>> ev;
    double busy = 0;
    for (int b = 0; b < nsyrk; ++b) {
        const int u = b / (ntiles * nsl), tl_ = (b % (ntiles * nsl)) / nsl;
        const int c = u == 0 ? 0 : 1, dg = tl_ >= noff ? 1 : 0;
        const double d = (double)(tl[3 * b + 1] - tl[3 * b]) * 0.01;
        dsum[c][dg] += d;
        dmax[c][dg] = std::max(dmax[c][dg], d);
        cnt[c][dg]++;
        busy += d;
        ev.push_back({tl[3 * b], +1});
        ev.push_back({tl[3 * b + 1], -1});
    }
    std::sort(ev.begin(), ev.end());
    int run = 0, peak = 0;
    for (auto& e : ev) peak = std::max(peak, run += e.second);
    // slot fill of the SYRK phase: SYRK workgroup-time / (peak x [t0, syrk_end])
    const double syrk_span = (syrk_end - t0) * 0.01, span = (t1 - t0) * 0.01;
    // time from the last SYRK dispatch on which fewer than peak - 8 SYRK workgroups run
    run = 0;
    unsigned long long drop = 0;
    for (auto& e : ev) {
        run += e.second;
        if (e.first >= last_syrk_start && run < peak - 8 && !drop) drop = e.first;
    }
    double rsum = 0, rmax = 0;
    for (int b = nsyrk; b < grid; ++b) {
        const double d = (double)(tl[3 * b + 1] - tl[3 * b]) * 0.01;
        rsum += d;
        rmax = std::max(rmax, d);
    }
    // MFMA-bound time of a chunk with two workgroups per CU sharing the pipes: blocks x K/4 MFMAs
    // of 64 cycles over 4 SIMDs, x2, at 2.4 GHz
    auto ideal_us = [&](int k, bool dg) { return (dg ? 36.0 : 64.0) * (k / 4.0) * 64.0 / 4.0 * 2.0 / 2400.0; };
    const int klong = sc.kfirst, kshort = sc.mS - sc.kfirst;
    const double flops = (double)m * n * (n + 1);
    std::printf("{\"m\": %d, \"n\": %d, \"tiles\": %d, \"kfirst\": %d, \"kshort\": %d, \"syrk_wgs\": %d, \"reduce_wgs\": %d, "
                "\"info\": %d, \"ms_events\": [",
                m, n, ntiles, klong, kshort, nsyrk, nred, hinfo);
    for (int r = 0; r < reps; ++r) std::printf("%s%.4f", r ? ", " : "", ms[r]);
    std::printf("], \"span_us\": %.1f, \"tflops_span\": %.2f, \"syrk_phase_us\": %.1f, \"peak_concurrency\": %d, "
                "\"syrk_slot_fill\": %.4f, \"syrk_tail_us\": %.1f, \"reduce_after_syrk_us\": %.1f, "
                "\"first_reduce_start_us\": %.1f, \"reduce_wg_us\": {\"mean\": %.2f, \"max\": %.2f}, \"chunks\": [",
                span, flops / (span * 1e-6) / 1e12, syrk_span, peak, busy / ((double)peak * syrk_span),
                drop ? (syrk_end - drop) * 0.01 : 0.0, (t1 - syrk_end) * 0.01, (red_first - t0) * 0.01,
                rsum / nred, rmax);
    bool first = true;
    for (int c = 0; c < 2; ++c)
        for (int dg = 0; dg < 2; ++dg) {
            if (!cnt[c][dg]) continue;
            const double mean = dsum[c][dg] / cnt[c][dg], id = ideal_us(c ? kshort : klong, dg);
            std::printf("%s{\"chunk\": \"%s\", \"diag\": %s, \"count\": %d, \"mean_us\": %.1f, \"max_us\": %.1f, "
                        "\"mfma_bound_us_2p4\": %.1f, \"efficiency\": %.3f}",
                        first ? "" : ", ", c ? "short" : "long", dg ? "true" : "false", cnt[c][dg], mean, dmax[c][dg],
                        id, id / mean);
            first = false;
        }
    std::printf("]}\n");
    return 0;
}
