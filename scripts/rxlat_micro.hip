// Micro-benchmark (diagnostic): issue rate of the rx walk's entry pattern at
// 2 waves per SIMD (512-thread workgroups, 1 per CU).
//   A: s_set_gpr_idx_idx + 2 v_pk_add_f32, one column chain (dependent)
//   B: same, 8 columns rotating (independent chains)
//   C: B without s_set_gpr_idx_idx
//   D: A without s_set_gpr_idx_idx
//   E: B with the index set one entry ahead of a 2-column interleave
// Build: hipcc --offload-arch=gfx950 -O3 scripts/rxlat_micro.hip -o scripts/rxlat_micro.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef float X32 __attribute__((ext_vector_type(32)));

#define ENT(S, A) "s_set_gpr_idx_idx " S "\n v_pk_add_f32 v[" A "], v[" A "], v[32:33]\n"
#define ENT2(S, A, B) "s_set_gpr_idx_idx " S "\n v_pk_add_f32 v[" A "], v[" A "], v[32:33]\n v_pk_add_f32 v[" B "], v[" B "], v[34:35]\n"
#define PL2(A, B) "v_pk_add_f32 v[" A "], v[" A "], v[40:41]\n v_pk_add_f32 v[" B "], v[" B "], v[42:43]\n"
#define A8 ENT2("%[i0]","96:97","98:99") ENT2("%[i1]","96:97","98:99") ENT2("%[i2]","96:97","98:99") ENT2("%[i3]","96:97","98:99") \
           ENT2("%[i0]","96:97","98:99") ENT2("%[i1]","96:97","98:99") ENT2("%[i2]","96:97","98:99") ENT2("%[i3]","96:97","98:99")
#define B8 ENT2("%[i0]","96:97","98:99") ENT2("%[i1]","100:101","102:103") ENT2("%[i2]","104:105","106:107") ENT2("%[i3]","108:109","110:111") \
           ENT2("%[i0]","112:113","114:115") ENT2("%[i1]","116:117","118:119") ENT2("%[i2]","120:121","122:123") ENT2("%[i3]","124:125","126:127")
#define C8 PL2("96:97","98:99") PL2("100:101","102:103") PL2("104:105","106:107") PL2("108:109","110:111") \
           PL2("112:113","114:115") PL2("116:117","118:119") PL2("120:121","122:123") PL2("124:125","126:127")
#define D8 PL2("96:97","98:99") PL2("96:97","98:99") PL2("96:97","98:99") PL2("96:97","98:99") \
           PL2("96:97","98:99") PL2("96:97","98:99") PL2("96:97","98:99") PL2("96:97","98:99")

template <int MODE>
__global__ __launch_bounds__(512, 1) void kern(float *out, int iters, uint32_t p0)
{
    const int lane = threadIdx.x & 63;
    X32 x, acc;
#pragma unroll
    for (int k = 0; k < 32; k++) { x[k] = k * 0.5f + lane; acc[k] = 0.f; }
    uint32_t i0 = p0 & 0xff, i1 = (p0 >> 8) & 0xff, i2 = (p0 >> 16) & 0xff, i3 = p0 >> 24;
    uint32_t n = iters;
#define RUN(BODY) asm volatile("s_set_gpr_idx_on %[i0], gpr_idx(SRC1)\n.Ll%=:\n" BODY BODY \
        "s_sub_u32 %[n], %[n], 1\n s_cmp_lg_u32 %[n], 0\n s_cbranch_scc1 .Ll%=\n s_set_gpr_idx_off\n" \
        : "+{v[32:63]}"(x), "+{v[96:127]}"(acc), [n] "+s"(n) \
        : [i0] "s"(i0), [i1] "s"(i1), [i2] "s"(i2), [i3] "s"(i3) : "scc")
    if (MODE == 0) RUN(A8);
    else if (MODE == 1) RUN(B8);
    else if (MODE == 2) RUN(C8);
    else RUN(D8);
    out[blockIdx.x * 512 + threadIdx.x] = acc[0] + acc[5] + acc[31];
}

template <int MODE>
int run(const char *name, float *dout)
{
    const int blocks = 1024, iters = 20000;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(512), 0, 0, dout, iters, 0x0a060202u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(512), 0, 0, dout, iters, 0x0a060202u);
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double adds = (double)blocks * 8 * iters * 32;  // wave pk_adds
    printf("%s: %.3f ms  %.3f pk_add/clk/CU (2.4 GHz)\n", name, ms, adds / (ms * 1e-3) / 2.4e9 / 256);
    return 0;
}
int main()
{
    float *d; CHECK(hipMalloc(&d, 1024 * 512 * 4));
    if (run<0>("A set_idx, 1 chain  ", d) || run<1>("B set_idx, 8 chains ", d) ||
        run<2>("C plain,   8 chains ", d) || run<3>("D plain,   1 chain  ", d)) return 1;
    return 0;
}
