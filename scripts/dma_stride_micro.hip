// LDS-DMA staging cost by source pattern (round 5, configs[1] / small M):
// the 64-row image stages 48 KiB X chunks into a 3-buffer LDS ring, 6
// global_load_lds_dwordx4 pieces per wave per step, one barrier per step --
// either from the staged copy (every piece 1 KiB contiguous) or straight
// from row-major X ("direct": a piece = PR rows x 1024/PR bytes, rows ld
// bytes apart).  This kernel does ONLY that staging (no reads, no adds), for
// 2 passes over the chunks (BaseTCSC's +1 then -1 pass), on a one-round grid
// of 256 workgroups, and times it per pattern and row pitch: does the
// row-strided pattern cost more, and does it come from the 16-KiB pitch
// (K = 4096) that maps every row of a piece to the same cache channel?
//   hipcc --offload-arch=gfx950 -O3 scripts/dma_stride_micro.hip -o scripts/dma_stride_micro.bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr int kBuf = 48 * 1024;
constexpr int kBufA = 49 * 1024;  // ring buffer pitch (49 pieces for the aligned row runs)

__global__ __launch_bounds__(512, 1) void stage(const char *__restrict__ x, int mode, int pr, uint32_t ld,
                                               int nch, int steps, int mtiles, uint32_t *sink)
{
    __shared__ __attribute__((aligned(16))) char lds[3 * kBufA];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int mt = blockIdx.x % mtiles;
    asm volatile("; lds %0" ::"v"(lds));
    for (int q = 0; q < steps; q++) {
        const int c = q % nch, buf = q % 3;
#pragma unroll
        for (int i = 0; i < 7; i++) {
            if (i == 6 && mode != 3) continue;
            const int p = wave * 6 + i;
            uint64_t off;
            if (mode == 0) {  // staged copy: piece (c, mt, p) = 1 KiB contiguous
                off = ((uint64_t)(c * mtiles + mt) * 48 + p) * 1024 + lane * 16;
            } else if (mode == 2) {  // row runs: LDS rows of 47 quads (752 B), lane slot p*64+lane
                if (p >= 47) continue;
                const int slot = p * 64 + lane, row = mt * 64 + slot / 47, quad = slot % 47;
                off = (uint64_t)row * ld + (uint64_t)c * 752 + quad * 16;
            } else if (mode == 3) {  // aligned row runs: 48 quads (768 B = 12 lines) per row from
                // 64-B aligned chunk starts, LDS rows of 49 quads (the 49th a pad: its lane
                // re-reads the row's last quad); 49 pieces per chunk (6 or 7 per wave)
                if (i == 6 && wave >= 1) continue;  // 8 waves x 6 + wave 0's 7th = 49 pieces
                const int pp = i == 6 ? 48 : p;
                const int slot = pp * 64 + lane, row = mt * 64 + slot / 49, q = slot % 49, quad = q < 48 ? q : 47;
                off = (uint64_t)row * ld + (uint64_t)c * 768 + quad * 16;
            } else {  // direct: PR rows x (64 / PR) quads of row-major X
                const int rgs = 64 / pr;
                const int row = mt * 64 + (p % rgs) * pr + lane % pr;
                const int quad = (p / rgs) * rgs + lane / pr;
                off = (uint64_t)row * ld + (uint64_t)c * 768 + quad * 16;
            }
            const char *g = x + off;
            const int pl = mode == 3 && i == 6 ? 48 : p;  // LDS piece slot
            const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(buf * kBufA + pl * 1024));
            asm volatile("s_mov_b32 m0, %0\n\t"
                         "s_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, off"
                         :
                         : "s"(m0), "v"(g)
                         : "memory", "m0");
        }
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (tid == 0 && sink) sink[blockIdx.x] = *(volatile uint32_t *)lds;
}

int main(int argc, char **argv)
{
    const int M = argc > 1 ? atoi(argv[1]) : 512;
    const int K = argc > 2 ? atoi(argv[2]) : 4096;
    const int grid = argc > 3 ? atoi(argv[3]) : 256;
    const int mtiles = M / 64, nch = K / 192, steps = 2 * nch;  // (row runs: 188-row chunks, same count)
    const size_t maxbytes = (size_t)M * (K * 4 + 4096) + (size_t)nch * mtiles * kBuf + 4096;
    char *x;
    uint32_t *sink;
    hipMalloc(&x, maxbytes);
    hipMemset(x, 1, maxbytes);
    hipMalloc(&sink, 4 * grid);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Case {
        const char *name;
        int mode, pr;
        uint32_t pad;
    } cases[] = {{"staged (1 KiB contiguous pieces)", 0, 16, 0},
                 {"direct PR=16, pitch K*4", 1, 16, 0},
                 {"direct PR=8,  pitch K*4", 1, 8, 0},
                 {"direct PR=16, pitch K*4+128", 1, 16, 128},
                 {"direct PR=16, pitch K*4+256", 1, 16, 256},
                 {"direct PR=16, pitch K*4+1024", 1, 16, 1024},
                 {"direct PR=8,  pitch K*4+128", 1, 8, 128},
                 {"direct PR=8,  pitch K*4+256", 1, 8, 256},
                 {"row runs (47-quad rows), pitch K*4", 2, 0, 0},
                 {"row runs (47-quad rows), pitch K*4+256", 2, 0, 256},
                 {"aligned row runs (48 of 49 quads)", 3, 0, 0}};
    printf("M=%d K=%d grid=%d mtiles=%d chunks=%d steps=%d (48 KiB per step per workgroup)\n", M, K, grid, mtiles, nch,
           steps);
    for (int rep = 0; rep < 2; rep++)
        for (const Case &cs : cases) {
            const uint32_t ld = (uint32_t)K * 4 + cs.pad;
            for (int w = 0; w < 20; w++)
                stage<<<grid, 512>>>(x, cs.mode, cs.pr, ld, nch, steps, mtiles, sink);
            const int iters = 50;
            hipEventRecord(e0);
            for (int it = 0; it < iters; it++)
                stage<<<grid, 512>>>(x, cs.mode, cs.pr, ld, nch, steps, mtiles, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / iters;
            const double bytes = (double)grid * steps * kBuf;
            printf("%-36s %8.2f us/launch  %6.2f us/step  %7.1f GB/s LDS-DMA (%.1f B/clk/CU at 2.1 GHz)\n", cs.name, us,
                   us / steps, bytes / (us * 1e-6) / 1e9, bytes / grid / (us * 1e-6 * 2.1e9) * (grid > 256 ? (double)grid / 256 : 1));
        }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
