// Micro-benchmark (diagnostic, not part of the product): X rows held in
// VGPRs and gathered by s_set_gpr_idx relative addressing (SRC1) into
// v_pk_add_f32 chains -- correctness of the indexed packed add on gfx950 and
// its throughput with 16 waves per CU, against plain packed adds.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/gpridx_micro.hip -o scripts/gpridx_micro.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef float X32 __attribute__((ext_vector_type(32)));
typedef float F4 __attribute__((ext_vector_type(4)));

// 8 indexed adds alternating two chains; idx SGPRs i0..i7 (already 2*k)
#define IDX8                                                                   \
    "s_set_gpr_idx_idx %[i0]\n v_pk_add_f32 v[96:97], v[96:97], v[32:33]\n"     \
    "s_set_gpr_idx_idx %[i1]\n v_pk_add_f32 v[98:99], v[98:99], v[32:33]\n"     \
    "s_set_gpr_idx_idx %[i2]\n v_pk_add_f32 v[96:97], v[96:97], v[32:33]\n"     \
    "s_set_gpr_idx_idx %[i3]\n v_pk_add_f32 v[98:99], v[98:99], v[32:33]\n"     \
    "s_set_gpr_idx_idx %[i4]\n v_pk_add_f32 v[96:97], v[96:97], v[32:33]\n"     \
    "s_set_gpr_idx_idx %[i5]\n v_pk_add_f32 v[98:99], v[98:99], v[32:33]\n"     \
    "s_set_gpr_idx_idx %[i6]\n v_pk_add_f32 v[96:97], v[96:97], v[32:33]\n"     \
    "s_set_gpr_idx_idx %[i7]\n v_pk_add_f32 v[98:99], v[98:99], v[32:33]\n"
// same with the index extracted from a packed word each time (s_lshr)
#define IDX8S                                                                  \
    "s_set_gpr_idx_idx %[w0]\n v_pk_add_f32 v[96:97], v[96:97], v[32:33]\n"     \
    "s_lshr_b32 %[t], %[w0], 8\n s_set_gpr_idx_idx %[t]\n v_pk_add_f32 v[98:99], v[98:99], v[32:33]\n" \
    "s_lshr_b32 %[t], %[w0], 16\n s_set_gpr_idx_idx %[t]\n v_pk_add_f32 v[96:97], v[96:97], v[32:33]\n" \
    "s_lshr_b32 %[t], %[w0], 24\n s_set_gpr_idx_idx %[t]\n v_pk_add_f32 v[98:99], v[98:99], v[32:33]\n" \
    "s_set_gpr_idx_idx %[w1]\n v_pk_add_f32 v[96:97], v[96:97], v[32:33]\n"     \
    "s_lshr_b32 %[t], %[w1], 8\n s_set_gpr_idx_idx %[t]\n v_pk_add_f32 v[98:99], v[98:99], v[32:33]\n" \
    "s_lshr_b32 %[t], %[w1], 16\n s_set_gpr_idx_idx %[t]\n v_pk_add_f32 v[96:97], v[96:97], v[32:33]\n" \
    "s_lshr_b32 %[t], %[w1], 24\n s_set_gpr_idx_idx %[t]\n v_pk_add_f32 v[98:99], v[98:99], v[32:33]\n"
#define PLAIN8                                                                 \
    "v_pk_add_f32 v[96:97], v[96:97], v[40:41]\n"                              \
    "v_pk_add_f32 v[98:99], v[98:99], v[42:43]\n"                              \
    "v_pk_add_f32 v[96:97], v[96:97], v[44:45]\n"                              \
    "v_pk_add_f32 v[98:99], v[98:99], v[46:47]\n"                              \
    "v_pk_add_f32 v[96:97], v[96:97], v[48:49]\n"                              \
    "v_pk_add_f32 v[98:99], v[98:99], v[50:51]\n"                              \
    "v_pk_add_f32 v[96:97], v[96:97], v[52:53]\n"                              \
    "v_pk_add_f32 v[98:99], v[98:99], v[54:55]\n"

template <int MODE>
__global__ __launch_bounds__(1024, 1) void kern(float *out, int iters, uint32_t p0, uint32_t p1)
{
    const int tid = threadIdx.x, lane = tid & 63;
    X32 x, y;
#pragma unroll
    for (int k = 0; k < 32; k++) {
        x[k] = (float)(k * 0.5f + lane * 0.03125f);
        y[k] = (float)((k + 32) * 0.5f + lane * 0.03125f);
    }
    F4 acc = {0.f, 0.f, 0.f, 0.f};
    // indices (2*k, k in 0..31) from the packed words: byte b of p0/p1
    uint32_t i0 = p0 & 0xff, i1 = (p0 >> 8) & 0xff, i2 = (p0 >> 16) & 0xff, i3 = p0 >> 24;
    uint32_t i4 = p1 & 0xff, i5 = (p1 >> 8) & 0xff, i6 = (p1 >> 16) & 0xff, i7 = p1 >> 24;
    uint32_t t, n = iters;
    if (MODE == 0) {
        asm volatile("s_set_gpr_idx_on %[i0], gpr_idx(SRC1)\n"
                     ".Ll%=:\n" IDX8 IDX8 IDX8 IDX8
                     "s_sub_u32 %[n], %[n], 1\n s_cmp_lg_u32 %[n], 0\n s_cbranch_scc1 .Ll%=\n"
                     "s_set_gpr_idx_off\n"
                     : "+{v[32:63]}"(x), "+{v[64:95]}"(y), "+{v[96:99]}"(acc), [n] "+s"(n)
                     : [i0] "s"(i0), [i1] "s"(i1), [i2] "s"(i2), [i3] "s"(i3), [i4] "s"(i4),
                       [i5] "s"(i5), [i6] "s"(i6), [i7] "s"(i7)
                     : "scc");
    } else if (MODE == 1) {
        asm volatile("s_set_gpr_idx_on %[w0], gpr_idx(SRC1)\n"
                     ".Ll%=:\n" IDX8S IDX8S IDX8S IDX8S
                     "s_sub_u32 %[n], %[n], 1\n s_cmp_lg_u32 %[n], 0\n s_cbranch_scc1 .Ll%=\n"
                     "s_set_gpr_idx_off\n"
                     : "+{v[32:63]}"(x), "+{v[64:95]}"(y), "+{v[96:99]}"(acc), [n] "+s"(n), [t] "=&s"(t)
                     : [w0] "s"(p0), [w1] "s"(p1)
                     : "scc");
    } else {
        asm volatile(".Ll%=:\n" PLAIN8 PLAIN8 PLAIN8 PLAIN8
                     "s_sub_u32 %[n], %[n], 1\n s_cmp_lg_u32 %[n], 0\n s_cbranch_scc1 .Ll%=\n"
                     : "+{v[32:63]}"(x), "+{v[64:95]}"(y), "+{v[96:99]}"(acc), [n] "+s"(n)
                     :
                     : "scc");
    }
    float *o = out + ((size_t)blockIdx.x * 1024 + tid) * 4;
    o[0] = acc[0];
    o[1] = acc[1];
    o[2] = acc[2];
    o[3] = acc[3];
}

template <int MODE>
int run(int blocks, int iters, uint32_t p0, uint32_t p1, float *dout, std::vector<float> &h)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(1024), 0, 0, dout, iters, p0, p1);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(1024), 0, 0, dout, iters, p0, p1);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double adds = (double)blocks * 16 * iters * 32;  // wave-level pk_adds
    printf("mode %d blocks %d iters %d: %.3f ms, %.3f pk_add/clk/CU (2.4 GHz, 256 CUs)\n", MODE, blocks,
           iters, ms, adds / (ms * 1e-3) / 2.4e9 / 256);
    h.resize((size_t)blocks * 1024 * 4);
    CHECK(hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost));
    return 0;
}

int main()
{
    float *dout;
    CHECK(hipMalloc(&dout, (size_t)1024 * 1024 * 4 * 4));
    // indices 2*k for k = 3, 17, 0, 31, 8, 9, 22, 5
    const uint32_t p0 = (6u) | (34u << 8) | (0u << 16) | (62u << 24);
    const uint32_t p1 = (16u) | (18u << 8) | (44u << 16) | (10u << 24);
    std::vector<float> h;
    // correctness: 1 iteration, 1 block; 32 adds: chain A gets idx i0,i2,i4,i6 x4, chain B i1,i3,i5,i7 x4
    for (int mode = 0; mode < 2; mode++) {
        if ((mode == 0 ? run<0>(1, 1, p0, p1, dout, h) : run<1>(1, 1, p0, p1, dout, h))) return 1;
        const int ks[8] = {3, 17, 0, 31, 8, 9, 22, 5};
        int bad = 0;
        for (int lane = 0; lane < 64; lane++) {
            float a0 = 0, a1 = 0, b0 = 0, b1 = 0;
            for (int rep = 0; rep < 4; rep++)
                for (int j = 0; j < 8; j++) {
                    const int k = ks[j];
                    const float v0 = (float)((2 * k) * 0.5f + lane * 0.03125f);
                    const float v1 = (float)((2 * k + 1) * 0.5f + lane * 0.03125f);
                    if (j % 2 == 0) { a0 += v0; a1 += v1; } else { b0 += v0; b1 += v1; }
                }
            const float *g = &h[(size_t)lane * 4];
            if (g[0] != a0 || g[1] != a1 || g[2] != b0 || g[3] != b1) {
                if (bad < 3) printf("mode %d lane %d: got %g %g %g %g want %g %g %g %g\n", mode, lane, g[0], g[1],
                                    g[2], g[3], a0, a1, b0, b1);
                bad++;
            }
        }
        printf("mode %d correctness: %s\n", mode, bad ? "MISMATCH" : "ok");
    }
    for (int blocks : {256, 1024}) {
        if (run<0>(blocks, 20000, p0, p1, dout, h)) return 1;
        if (run<1>(blocks, 20000, p0, p1, dout, h)) return 1;
        if (run<2>(blocks, 20000, p0, p1, dout, h)) return 1;
    }
    return 0;
}
