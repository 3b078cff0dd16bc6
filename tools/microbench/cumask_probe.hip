// Probe: which XCD (XCC_ID) and CU (HW_ID) the workgroups of a CU-masked stream land on, for
// masks of contiguous CU indices and of every 8th index.  Prints one JSON line.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/cumask_probe.hip -o tools/microbench/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <set>
#include <string>
#include <vector>

__global__ void k_where(unsigned* out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));   // XCC_ID
        const unsigned hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));    // HW_ID
        out[2 * blockIdx.x] = xcc & 15;
        out[2 * blockIdx.x + 1] = hw;
    }
    // keep the workgroup resident a little so the dispatcher spreads the grid
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 5000) __builtin_amdgcn_s_sleep(10);
}

static std::string run(int ncu, const std::vector<int>& cus) {
    std::vector<uint32_t> m((ncu + 31) / 32, 0u);
    for (int c : cus) m[c / 32] |= 1u << (c % 32);
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()) != hipSuccess) return "\"refused\"";
    const int grid = 2048;
    unsigned* d = nullptr;
    hipMalloc(&d, sizeof(unsigned) * 2 * grid);
    hipLaunchKernelGGL(k_where, dim3(grid), dim3(64), 0, s, d);
    std::vector<unsigned> h(2 * grid);
    hipMemcpy(h.data(), d, sizeof(unsigned) * 2 * grid, hipMemcpyDeviceToHost);
    std::set<unsigned> cu;
    std::vector<std::set<unsigned>> per(16);
    for (int b = 0; b < grid; ++b) {
        // HW_ID: CU_ID bits 8..11, SH_ID bit 12, SE_ID bits 13..14 (gfx9 layout)
        const unsigned phys = (h[2 * b + 1] >> 8) & 0x7f;
        cu.insert((h[2 * b] << 16) | phys);
        per[h[2 * b] & 15].insert(phys);
    }
    hipFree(d);
    hipStreamDestroy(s);
    std::string r = "{\"distinct_cus\": " + std::to_string(cu.size()) + ", \"per_xcc\": [";
    for (int x = 0; x < 8; ++x) r += (x ? ", " : "") + std::to_string(per[x].size());
    r += "]}";
    return r;
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    std::printf("{\"cus\": %d", ncu);
    struct M { const char* name; std::vector<int> cus; };
    std::vector<M> ms;
    for (int first : {0, 32, 224}) {
        M a{nullptr, {}};
        for (int c = first; c < first + 32; ++c) a.cus.push_back(c);
        ms.push_back(a);
    }
    for (int r : {0, 1, 7}) {
        M a{nullptr, {}};
        for (int c = r; c < ncu; c += 8) a.cus.push_back(c);
        ms.push_back(a);
    }
    {   // all but 0..31
        M a{nullptr, {}};
        for (int c = 32; c < ncu; ++c) a.cus.push_back(c);
        ms.push_back(a);
    }
    {   // all but every 8th
        M a{nullptr, {}};
        for (int c = 0; c < ncu; ++c) if (c % 8) a.cus.push_back(c);
        ms.push_back(a);
    }
    {   // 0..3
        M a{nullptr, {}};
        for (int c = 0; c < 4; ++c) a.cus.push_back(c);
        ms.push_back(a);
    }
    {   // 0, 1, 2, 3 of each 32
        M a{nullptr, {}};
        for (int c = 0; c < ncu; ++c) if (c % 32 < 4) a.cus.push_back(c);
        ms.push_back(a);
    }
    {   // all
        M a{nullptr, {}};
        for (int c = 0; c < ncu; ++c) a.cus.push_back(c);
        ms.push_back(a);
    }
    const char* names[] = {"cu0_31", "cu32_63", "cu224_255", "every8_from0", "every8_from1", "every8_from7",
                           "not0_31", "not_every8", "cu0_3", "cu0_3_of_each32", "all"};
    for (size_t i = 0; i < ms.size(); ++i) std::printf(", \"%s\": %s", names[i], run(ncu, ms[i].cus).c_str());
    std::printf("}\n");
    return 0;
}
