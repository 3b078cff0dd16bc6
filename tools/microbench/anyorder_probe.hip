// Does a kernel launched with hipExtAnyOrderLaunch (no AQL barrier bit) start on the CUs the
// previous kernel of the same stream frees during its last dispatch round, before that kernel
// has finished?  Kernel A: G workgroups, 2 per CU (64 KB LDS each), each busy for D realtime
// ticks (100 MHz) -- several dispatch rounds.  Kernel B: 256 small workgroups that stamp their
// start.  Printed (microseconds, relative to A's first start): A's last workgroup start (its
// last dispatch), A's last end, B's first start -- for B launched plainly and with the flag.
//   hipcc --offload-arch=gfx950 -O3 anyorder_probe.hip -o anyorder_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__global__ __launch_bounds__(256) void k_busy(unsigned long long* st, unsigned long long* en, long ticks,
                                             double* sink) {
    __shared__ double pad[8192];   // 64 KB: two workgroups per CU
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    pad[threadIdx.x] = (double)threadIdx.x;
    __syncthreads();
    double a = pad[(threadIdx.x + 1) & 255];
    // the spin is bounded by the realtime counter alone: every wave leaves after `ticks`
    while ((long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) a = a * 0.999 + 1e-3;
    if (a == 12345.678) sink[0] = a;
    if (threadIdx.x == 0) {
        st[blockIdx.x] = t0;
        en[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    }
}

__global__ __launch_bounds__(256) void k_stamp(unsigned long long* st) {
    if (threadIdx.x == 0) st[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

int main() {
    const int G = 2048, GB = 256;
    const long ticks = 2000;   // 20 us per workgroup: 4 rounds at 2 per CU
    unsigned long long *st, *en, *bst;
    double* sink;
    CK(hipMalloc(&st, G * 8));
    CK(hipMalloc(&en, G * 8));
    CK(hipMalloc(&bst, GB * 8));
    CK(hipMalloc(&sink, 8));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<unsigned long long> hs(G), he(G), hb(GB);
    std::printf("{");
    for (int flag = 0; flag < 2; ++flag) {
        for (int rep = 0; rep < 4; ++rep) {
            hipExtLaunchKernelGGL(k_busy, dim3(G), dim3(256), 0, s, nullptr, nullptr, 0, st, en, ticks, sink);
            hipExtLaunchKernelGGL(k_stamp, dim3(GB), dim3(256), 0, s, nullptr, nullptr, flag ? hipExtAnyOrderLaunch : 0,
                                  bst);
            CK(hipGetLastError());
            CK(hipStreamSynchronize(s));
        }
        CK(hipMemcpy(hs.data(), st, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(he.data(), en, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), bst, GB * 8, hipMemcpyDeviceToHost));
        const unsigned long long a0 = *std::min_element(hs.begin(), hs.end());
        const unsigned long long alast = *std::max_element(hs.begin(), hs.end());
        const unsigned long long aend = *std::max_element(he.begin(), he.end());
        const unsigned long long b0 = *std::min_element(hb.begin(), hb.end());
        std::printf("%s\"%s\": {\"a_last_start_us\": %.2f, \"a_end_us\": %.2f, \"b_first_start_us\": %.2f}",
                    flag ? ", " : "", flag ? "any_order" : "plain", (alast - a0) / 100.0, (aend - a0) / 100.0,
                    ((double)b0 - (double)a0) / 100.0);
    }
    std::printf("}\n");
    return 0;
}
