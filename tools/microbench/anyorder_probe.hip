// Does a kernel launched with hipExtAnyOrderLaunch (no AQL barrier bit) start on the CUs the
// previous kernel of the same stream frees during its last dispatch round, before that kernel
// has finished?  Kernel A: G workgroups, 2 per CU (64 KB LDS each), each busy for D realtime
// ticks (100 MHz) -- several dispatch rounds.  Kernel B: 256 small workgroups that stamp their
// start.  Printed (microseconds, relative to A's first start): A's last workgroup start (its
// last dispatch), A's last end, B's first start -- for B launched plainly and with the flag,
// and for B on a second stream gated by hipStreamWaitValue32 on a word that A's last
// workgroup stores (system scope) when it starts ("wait_value").
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
                                             double* sink, unsigned* flag, unsigned epoch) {
    __shared__ double pad[8192];   // 64 KB: two workgroups per CU
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (flag && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
        __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    unsigned* flag = nullptr;
    // signal memory is one 8-byte word; plain device memory as a fallback
    bool sig = hipExtMallocWithFlags((void**)&flag, 8, hipMallocSignalMemory) == hipSuccess;
    if (!sig) {
        (void)hipGetLastError();
        CK(hipMalloc((void**)&flag, 64));
    }
    CK(hipMemset(flag, 0, 8));
    std::fprintf(stderr, "flag memory: %s\n", sig ? "signal" : "device");
    unsigned epoch = 0;
    std::vector<unsigned long long> hs(G), he(G), hb(GB);
    std::printf("{");
    const char* names[3] = {"plain", "any_order", "wait_value"};
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 4; ++rep) {
            ++epoch;
            hipExtLaunchKernelGGL(k_busy, dim3(G), dim3(256), 0, s, nullptr, nullptr, 0, st, en, ticks, sink,
                                  mode == 2 ? flag : (unsigned*)nullptr, epoch);
            if (mode == 2) {
                CK(hipStreamWaitValue32(s2, flag, epoch, hipStreamWaitValueGte, 0xffffffffu));
                hipLaunchKernelGGL(k_stamp, dim3(GB), dim3(256), 0, s2, bst);
            } else {
                hipExtLaunchKernelGGL(k_stamp, dim3(GB), dim3(256), 0, s, nullptr, nullptr,
                                      mode ? hipExtAnyOrderLaunch : 0, bst);
            }
            CK(hipGetLastError());
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
        }
        CK(hipMemcpy(hs.data(), st, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(he.data(), en, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), bst, GB * 8, hipMemcpyDeviceToHost));
        const unsigned long long a0 = *std::min_element(hs.begin(), hs.end());
        const unsigned long long alast = *std::max_element(hs.begin(), hs.end());
        const unsigned long long aend = *std::max_element(he.begin(), he.end());
        const unsigned long long b0 = *std::min_element(hb.begin(), hb.end());
        std::printf("%s\"%s\": {\"a_last_start_us\": %.2f, \"a_end_us\": %.2f, \"b_first_start_us\": %.2f}",
                    mode ? ", " : "", names[mode], (alast - a0) / 100.0, (aend - a0) / 100.0,
                    ((double)b0 - (double)a0) / 100.0);
    }
    std::printf("}\n");
    return 0;
}
