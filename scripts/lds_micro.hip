// LDS gather micro-benchmark (diagnostic, not part of the product): how fast
// can a CU serve the stream kernel's access pattern -- wave-uniform entry
// byte -> v_perm address -> ds_read_b64 of one 256-B row per half-wave?
// Variants (template MODE):
//   0: perm + read + pk_add chain, lgkmcnt(13) pipeline (the flat kernel)
//   1: reads only (addresses precomputed, no VALU), lgkmcnt(13)
//   2: perm + read, no adds
//   3: as 0 but 2 independent chains
// Build: hipcc --offload-arch=gfx950 -O3 scripts/lds_micro.hip -o /tmp/lds_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(1024, 1) void kern(const uint32_t *__restrict__ words, int iters, float *out)
{
    __shared__ __attribute__((aligned(16))) char lds[131072];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 131072 / 4; i += 1024) reinterpret_cast<float *>(lds)[i] = (float)(i & 7);
    __syncthreads();
    const uint32_t lanec = ((uint32_t)(lane & 31) << 3) | ((uint32_t)(lane >> 5) << 16);
    const int wave = tid >> 6;
    float2 a = make_float2(0.f, 0.f), b = make_float2(0.f, 0.f);
    uint32_t w = words[(blockIdx.x * 16 + wave) & 255];
    for (int it = 0; it < iters; it++) {
        // 8 dwords per iteration, each 4 entries
#pragma unroll
        for (int d = 0; d < 8; d++) {
            w = w * 1664525u + 1013904223u;  // uniform pseudo-random entry bytes (SALU-able)
            const uint32_t ww = __builtin_amdgcn_readfirstlane(w);
            uint32_t ad[4];
            if (MODE == 1) {
#pragma unroll
                for (int e = 0; e < 4; e++) ad[e] = lanec + ((e * 37 + d * 11) & 127) * 256;
            } else {
                ad[0] = __builtin_amdgcn_perm(ww, lanec, 0x0C020400u | (4u << 8));
                ad[1] = __builtin_amdgcn_perm(ww, lanec, 0x0C020400u | (5u << 8));
                ad[2] = __builtin_amdgcn_perm(ww, lanec, 0x0C020400u | (6u << 8));
                ad[3] = __builtin_amdgcn_perm(ww, lanec, 0x0C020400u | (7u << 8));
            }
            float2 x[4];
#pragma unroll
            for (int e = 0; e < 4; e++) x[e] = *reinterpret_cast<const float2 *>(lds + ad[e]);
            if (MODE == 2) {
                a.x += x[0].x; a.y += x[3].y;
            } else if (MODE == 3) {
                a.x += x[0].x; a.y += x[0].y; b.x += x[1].x; b.y += x[1].y;
                a.x += x[2].x; a.y += x[2].y; b.x += x[3].x; b.y += x[3].y;
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++) { a.x += x[e].x; a.y += x[e].y; }
            }
        }
    }
    out[blockIdx.x * 1024 + tid] = a.x + a.y + b.x + b.y;
}

template <int MODE>
int run(int blocks, int iters, const uint32_t *dw, float *dout)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(1024), 0, 0, dw, iters, dout);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(1024), 0, 0, dw, iters, dout);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double reads = (double)blocks * 16 * iters * 32;  // wave-instructions
    const double bytes = reads * 512;
    printf("mode %d blocks %d: %.3f ms  %.1f TB/s  (%.1f B/clk/CU at 2.4GHz, 256 CUs)\n", MODE, blocks, ms,
           bytes / ms / 1e9, bytes / (ms * 1e-3) / 2.4e9 / 256);
    return 0;
}

int main()
{
    std::vector<uint32_t> w(256);
    for (int i = 0; i < 256; i++) w[i] = 0x9E3779B9u * (i + 1);
    uint32_t *dw;
    float *dout;
    CHECK(hipMalloc(&dw, 256 * 4));
    CHECK(hipMalloc(&dout, 4096 * 1024 * 4));
    CHECK(hipMemcpy(dw, w.data(), 1024, hipMemcpyHostToDevice));
    const int iters = 2000;
    for (int blocks : {256, 1024}) {
        if (run<0>(blocks, iters, dw, dout)) return 1;
        if (run<1>(blocks, iters, dw, dout)) return 1;
        if (run<2>(blocks, iters, dw, dout)) return 1;
        if (run<3>(blocks, iters, dw, dout)) return 1;
    }
    return 0;
}
