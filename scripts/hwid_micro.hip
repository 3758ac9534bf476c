// Diagnostic micro-benchmark (not product): where do workgroups land?
// Launches G workgroups of 512 threads holding 144 KiB of LDS (one per CU, as
// tsg_jit_kernel), records per workgroup HW_ID (CU/SH/SE) and XCC_ID, and the
// shader-clock start time, then prints the placement of blockIdx 0..G-1.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/hwid_micro.hip -o scripts/hwid_micro.bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <set>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);            \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__global__ __launch_bounds__(512) void where(uint32_t *out, int spin)
{
    extern __shared__ char lds[];
    asm volatile("; %0" ::"v"(lds));
    if (threadIdx.x == 0) {
        uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        uint64_t t = __builtin_amdgcn_s_memrealtime();
        out[blockIdx.x * 4 + 0] = hw;
        out[blockIdx.x * 4 + 1] = xcc;
        out[blockIdx.x * 4 + 2] = (uint32_t)t;
    }
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) {
    }
}

int main()
{
    const int lds = 144 * 1024;
    CHECK(hipFuncSetAttribute((const void *)where, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    for (int G : {256, 1024}) {
        uint32_t *d;
        CHECK(hipMalloc(&d, G * 16));
        hipLaunchKernelGGL(where, dim3(G), dim3(512), lds, 0, d, 2000);  // 2000 ticks of 100 MHz = 20 us
        CHECK(hipDeviceSynchronize());
        std::vector<uint32_t> h(G * 4);
        CHECK(hipMemcpy(h.data(), d, G * 16, hipMemcpyDeviceToHost));
        printf("G=%d\n", G);
        std::map<uint32_t, std::vector<int>> by_loc;
        std::set<uint32_t> cus;
        for (int i = 0; i < G; i++) {
            uint32_t hw = h[i * 4], xcc = h[i * 4 + 1] & 0xf;
            uint32_t cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            uint32_t loc = xcc << 12 | se << 8 | sh << 4 | cu;
            by_loc[loc].push_back(i);
            if (G == 256 || i < 64)
                printf("b%4d xcc %u se %u sh %u cu %2u t %u\n", i, xcc, se, sh, cu, h[i * 4 + 2]);
        }
        printf("distinct locations %zu\n", by_loc.size());
        for (auto &kv : by_loc) {
            printf("loc xcc %u se %u sh %u cu %2u :", kv.first >> 12, (kv.first >> 8) & 15, (kv.first >> 4) & 15,
                   kv.first & 15);
            for (int b : kv.second) printf(" %d", b);
            printf("\n");
        }
        CHECK(hipFree(d));
    }
    return 0;
}
