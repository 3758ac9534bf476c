// tsg_jit_kernel.hip -- dispatcher of the weight-compiled ("jit") TCSC kernel.
//
// Built as a standalone gfx950 code object (lib/tsg_jit.co), NOT into the
// shared library: at registration tsg_jit.cpp appends the machine code it
// generates from the TCSC arrays as an extra PT_LOAD segment and loads the
// result with hipModuleLoadData, so the loader maps that code executable
// together with this kernel.
//
// Why compile W into code: the BaseTCSC chain (comp.h:37-63)
// is one dependent fp32 add per nonzero, and a walk that READS the entry
// indices at run time pays, per nonzero, for the index (LDS gather or
// register-indexed add) and per column for a data-dependent branch -- the
// measured cost of the register-X walk was 2-3x its adds.  Here every nonzero
// of a wave's 32 columns is a v_pk_add_f32 pair whose X register (a row of
// the current X^T block, loaded by ds_read_b128) and accumulator are encoded
// in the instruction: no index traffic, no SALU, no branch.  The same code
// serves every 256-row M tile.
//
// Workgroup: 256 M rows (4 per lane) x 8 waves x 32 columns, 512 threads, one
// per CU (2 waves per SIMD).  Step q = p*nch + j (p = 0: +1 entries, p = 1:
// -1 entries; chunk j of 64 K rows): the chunk is in LDS buffer q&1 (staged
// by LDS-DMA during step q-1), the wave calls its generated section for step
// q, then the workgroup barriers.  Register contract with the generator
// (tsg_jit.cpp): v[8:103] X slots (24 rows x 4 M rows), v104/v105 LDS byte
// address of lane row 0 in buffer 0/1, v[112:239] accumulators (column c of
// the wave at v[112+4c : 115+4c]), s[92:93] code pointer, s[94:95] return
// address.  A section ends with `s_getpc_b64 s[92:93]; s_setpc_b64 s[94:95]`,
// so the next section starts 4 bytes past the returned pointer.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kJWaves = 8;
constexpr int kJNW = 32;
constexpr int kJTileM = 256;
constexpr int kJChunk = 64;
constexpr uint32_t kJMagic0 = 0x7453474a, kJMagic1 = 0x314a4954;  // region header

__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_dst)
{
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
}

// X^T chunk j (64 rows x 256 M) -> LDS buffer buf: one 1 KiB row per
// wave-instruction, 8 per wave.
__device__ __forceinline__ void stage(const float *__restrict__ XT, int Mp, int m0, int j, int buf, int wave,
                                      int lane)
{
#pragma unroll
    for (int i = 0; i < kJChunk / kJWaves; i++) {
        const int r = wave * (kJChunk / kJWaves) + i;
        glds16(XT + (size_t)(j * kJChunk + r) * Mp + m0 + 4 * lane, (uint32_t)(buf * 65536 + r * 1024));
    }
}

typedef float F32x32 __attribute__((ext_vector_type(32)));

#define TSG_JIT_CLOBBERS                                                                          \
    "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", \
        "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34",  \
        "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47",  \
        "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60",  \
        "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73",  \
        "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86",  \
        "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99",  \
        "v100", "v101", "v102", "v103", "s94", "s95", "scc", "memory"

}  // namespace

extern "C" __global__ __launch_bounds__(512, 1) void tsg_jit_kernel(
    const float *__restrict__ XT, int Mp, const uint32_t *__restrict__ wcode,
    const float *__restrict__ b, const float *__restrict__ alpha, float *__restrict__ Y, int M, int N,
    int nch, int mtiles, int ntiles, int prelu, uint32_t *__restrict__ status)
{
    __shared__ __attribute__((aligned(16))) char lds[2 * 65536];
    const int tid = threadIdx.x, lane = tid & 63;
    // LDS is only addressed from asm, at absolute offsets from 0 (the only
    // LDS object): this use keeps the allocation in the kernel descriptor
    asm volatile("; lds %0" ::"v"(lds));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // Base of the generated region: s_getpc + a literal that the loader-side
    // patcher (tsg_jit.cpp) sets to (region vaddr - vaddr of the s_add).
    uint64_t base;
    asm volatile("s_getpc_b64 s[92:93]\n\t"
                 "s_add_u32 s92, s92, 0x7a5e1234\n\t"
                 "s_addc_u32 s93, s93, 0"
                 : "={s[92:93]}"(base)
                 :
                 : "scc");
    // never jump into a region that is not ours
    const uint32_t *hdr = reinterpret_cast<const uint32_t *>(base);
    if (hdr[0] != kJMagic0 || hdr[1] != kJMagic1) {
        if (blockIdx.x == 0 && tid == 0) status[0] = 1u;
        return;
    }

    // XCD-aware bijective remap (as the rx kernel): each XCD gets a contiguous
    // n-tile-major run, so the 16 M tiles of a column tile run together on one
    // XCD and share its code (and entry-free X^T slab) through that XCD's L2.
    const int T = mtiles * ntiles, L = blockIdx.x;
    const int xcd = L & 7, slot = L >> 3, q8 = T >> 3, r8 = T & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
    const int nt = wg / mtiles, mt = wg - nt * mtiles;
    const int m0 = mt * kJTileM;
    const int ncol0 = nt * (kJWaves * kJNW) + wave * kJNW;

    uint64_t cp = base + __builtin_amdgcn_readfirstlane(wcode[(size_t)nt * kJWaves + wave]);
    const uint32_t lb0 = (uint32_t)lane * 16u, lb1 = 65536u + (uint32_t)lane * 16u;

    stage(XT, Mp, m0, 0, 0, wave, lane);
    F32x32 a0 = {}, a1 = {}, a2 = {}, a3 = {};  // comp.h:41
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int steps = 2 * nch;
    for (int q = 0; q < steps; q++) {
        if (q + 1 < steps) stage(XT, Mp, m0, (q + 1) % nch, (q + 1) & 1, wave, lane);
        asm volatile("s_getpc_b64 s[94:95]\n"
                     ".Ljr%=:\n\t"
                     "s_add_u32 s94, s94, (.Ljb%= - .Ljr%=)\n\t"
                     "s_addc_u32 s95, s95, 0\n\t"
                     "s_setpc_b64 s[92:93]\n"
                     ".Ljb%=:\n\t"
                     "s_add_u32 s92, s92, 4\n\t"
                     "s_addc_u32 s93, s93, 0"
                     : "+{v[112:143]}"(a0), "+{v[144:175]}"(a1), "+{v[176:207]}"(a2), "+{v[208:239]}"(a3),
                       "+{s[92:93]}"(cp)
                     : "{v104}"(lb0), "{v105}"(lb1)
                     : TSG_JIT_CLOBBERS);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA for q+1 landed
        __syncthreads();                                   // ... and every other wave's
    }

    if (ncol0 >= N) return;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int m = m0 + 4 * lane + r;
        if (m >= M) continue;
        float *yrow = Y + (size_t)m * N + ncol0;
        float v[kJNW];
#pragma unroll
        for (int c = 0; c < kJNW; c++) {
            const int n = ncol0 + c < N ? ncol0 + c : N - 1;
            const float acc = c < 8 ? a0[4 * (c & 7) + r] : c < 16 ? a1[4 * (c & 7) + r]
                             : c < 24 ? a2[4 * (c & 7) + r] : a3[4 * (c & 7) + r];
            float y = acc + b[n];                        // comp.h:63
            if (prelu) y = (y > 0) ? y : alpha[n] * y;   // comp_prelu.h:57-67
            v[c] = y;
        }
        if (ncol0 + kJNW <= N && ((((size_t)m * N + ncol0) & 3) == 0)) {
#pragma unroll
            for (int c = 0; c < kJNW; c += 4)
                *reinterpret_cast<float4 *>(yrow + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
        } else {
#pragma unroll
            for (int c = 0; c < kJNW; c++)
                if (ncol0 + c < N) yrow[c] = v[c];
        }
    }
}
