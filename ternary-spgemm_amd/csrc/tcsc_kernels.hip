// tcsc_kernels.hip -- the compiled-in gfx950 kernels of libternary_spgemm.so
// (the default weight-compiled kernel is a separate code object,
// tsg_jit_kernel.hip + tsg_jit.cpp).
//
// Arithmetic contract (cpp_impl/comp.h:37-63, BaseTCSC<float>): every output
// Y[m,n] is ONE serial fp32 chain  0 + x_p1 + ... + x_pP - x_n1 - ... - x_nQ,
// then + b[n], with the +1 run and the -1 run each in ascending k.  No output
// is ever split across lanes/waves: parallelism is over (m, n) pairs only.
//
// tsg_transpose_kernel / tsg_transpose4_kernel (K % 4 == 0):
//   X [M][K] -> X^T [Kp][Mp], zero padded.  HBM-bound copy (2 * 4 * M * K bytes).
// tsg_tcsc_rx_kernel: the register-X walk, the fallback when a W is too large
//   for one weight-compiled image (> ~300 M nonzeros on one handle) or the
//   generated image cannot be loaded (tsg_capi.cpp create_impl).
#include <hip/hip_runtime.h>

#include "tsg_internal.h"

namespace tsg {

// ------------------------------------------------------------------ kernel 1 --
__global__ __launch_bounds__(256) void tsg_transpose_kernel(const float *__restrict__ X,
                                                            float *__restrict__ XT, int M, int K,
                                                            int Mp, int Kp)
{
    __shared__ float tile[64][65];
    const int k0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int m = m0 + ty + 4 * i, k = k0 + tx;
        tile[ty + 4 * i][tx] = (m < M && k < K) ? X[(size_t)m * K + k] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int k = k0 + ty + 4 * i, m = m0 + tx;
        if (k < Kp) XT[(size_t)k * Mp + m] = tile[tx][ty + 4 * i];
    }
}

// Same transpose with 16-byte accesses on both sides (K % 4 == 0 and X 16-byte
// aligned): each lane loads 4 consecutive k of one m row and stores 4
// consecutive m of one X^T row -- a quarter of the memory instructions.
__global__ __launch_bounds__(256) void tsg_transpose4_kernel(const float *__restrict__ X,
                                                             float *__restrict__ XT, int M, int K,
                                                             int Mp, int Kp)
{
    __shared__ float tile[64][65];
    const int k0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
    const int c4 = (threadIdx.x & 15) * 4, r = threadIdx.x >> 4;  // 16 x 16
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int ml = r + 16 * i, m = m0 + ml, k = k0 + c4;
        float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (m < M && k < K) v = *reinterpret_cast<const float4 *>(X + (size_t)m * K + k);  // K % 4 == 0
        tile[ml][c4] = v.x;
        tile[ml][c4 + 1] = v.y;
        tile[ml][c4 + 2] = v.z;
        tile[ml][c4 + 3] = v.w;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int kl = r + 16 * i, k = k0 + kl;
        if (k < Kp)
            *reinterpret_cast<float4 *>(XT + (size_t)k * Mp + m0 + c4) =
                make_float4(tile[c4][kl], tile[c4 + 1][kl], tile[c4 + 2][kl], tile[c4 + 3][kl]);
    }
}

// X [M][K] -> the k-pair layout of the jit kernel (tsg_internal.h): for k-row
// pair p and M-row pair mp the 16 bytes at (p * Mp/2 + mp) * 16 hold
// X[2mp][2p], X[2mp+1][2p], X[2mp][2p+1], X[2mp+1][2p+1]; zero outside M x K.
// A 64 (m) x 64 (k) tile goes through LDS: loads along k (16 B per lane when
// VEC: K % 4 == 0 and X 16-byte aligned), stores 16 B per lane, consecutive
// lanes on consecutive mp (coalesced 512-B runs per pair row).  HBM-bound:
// 8 * M * K bytes.
template <bool VEC>
__global__ __launch_bounds__(256) void tsg_transpose_pairs_kernel(const float *__restrict__ X,
                                                                  float *__restrict__ XP, int M, int K,
                                                                  int Mp, int Kp)
{
    __shared__ float tile[64][65];  // [m][k]
    const int k0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
    if (VEC) {
        const int c4 = (threadIdx.x & 15) * 4, r = threadIdx.x >> 4;  // 16 x 16
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int ml = r + 16 * i, m = m0 + ml, k = k0 + c4;
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (m < M && k < K) v = *reinterpret_cast<const float4 *>(X + (size_t)m * K + k);  // K % 4 == 0
            tile[ml][c4] = v.x;
            tile[ml][c4 + 1] = v.y;
            tile[ml][c4 + 2] = v.z;
            tile[ml][c4 + 3] = v.w;
        }
    } else {
        const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int m = m0 + ty + 4 * i, k = k0 + tx;
            tile[ty + 4 * i][tx] = (m < M && k < K) ? X[(size_t)m * K + k] : 0.0f;
        }
    }
    __syncthreads();
    // 32 pairs x 32 M pairs of float4 per tile: 4 per thread
    const int mpl = threadIdx.x & 31, pl0 = threadIdx.x >> 5;  // 32 x 8
    const size_t half_mp = (size_t)Mp / 2;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int pl = pl0 + 8 * i, p = (k0 >> 1) + pl;
        if (2 * p >= Kp) continue;
        const int a = 2 * mpl, kk = 2 * pl;
        *reinterpret_cast<float4 *>(XP + ((size_t)p * half_mp + (size_t)(m0 >> 1) + mpl) * 4) =
            make_float4(tile[a][kk], tile[a + 1][kk], tile[a][kk + 1], tile[a + 1][kk + 1]);
    }
}

// X [M][K] -> the blocked k-quad layout of the 64-row image (tsg_internal.h),
// PR rows per piece (16 or 8) and Q = 64 / PR quads: the 1-KiB piece pr = Q qg
// + rg of (chunk c, M tile t) at ((c * Mt + t) * U + pr) KiB (U = 48 units per
// chunk, 24 for the half ring) holds, in 16-B
// lane slot j, X[64 t + PR rg + j % PR][4 (48 c + Q qg + j / PR) .. +3] -- zero
// past M or K -- so the kernel's DMA pieces are coalesced 1-KiB reads.  Every
// slot is 16 contiguous bytes of a row of X, so this is a gather-copy, not a
// transpose: one wave writes one whole piece (1 KiB, one store per lane) from
// PR row segments of 1024 / PR bytes (the other half of a PR = 16 segment's
// 128-B line is the next piece's, copied by the neighbouring workgroup); no
// LDS, no barrier.  A workgroup copies 4 consecutive pieces of one (chunk, M
// tile).  HBM-bound: 8 * Mp * Kp bytes.
template <bool VEC, int PR>
__global__ __launch_bounds__(256) void tsg_transpose_quads_kernel(const float *__restrict__ X,
                                                                  float *__restrict__ XQ, int M, int K,
                                                                  int Mp, int Kp, int units)
{
    // units: 1-KiB pieces per (chunk, M tile) -- 48, or 24 for the half ring
    constexpr int Q = 64 / PR;
    const int Mt = Mp >> 6, nch = Kp / (4 * units), groups = units / 4;
    // workgroup order (M tile * nch + chunk) * 12 + piece group: the workgroups
    // in flight read a few M tiles' rows end to end (long runs of each row), not
    // one chunk of every row
    const int blk = blockIdx.x;
    const int tc = blk / groups, pr = (blk % groups) * 4 + (threadIdx.x >> 6);
    const int t = tc / nch, c = tc % nch, j = threadIdx.x & 63;
    const int ct = c * Mt + t;
    const int qg = pr / Q, rg = pr % Q;
    const int m = 64 * t + PR * rg + (j % PR);
    const int k = 4 * (units * c + Q * qg + j / PR);
    float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (m < M) {
        const float *row = X + (size_t)m * K;
        if (VEC) {
            if (k < K) v = *reinterpret_cast<const float4 *>(row + k);  // K % 4 == 0: whole quad inside
        } else {
            if (k < K) v.x = row[k];
            if (k + 1 < K) v.y = row[k + 1];
            if (k + 2 < K) v.z = row[k + 2];
            if (k + 3 < K) v.w = row[k + 3];
        }
    }
    *reinterpret_cast<float4 *>(XQ + ((size_t)ct * units + pr) * 256 + (size_t)j * 4) = v;
}

// X [M][K] -> the staged copy of the 64-row image's ROW layout
// (tsg_internal.h kJit64RowFlag): (chunk c, M tile t) is 47 KiB at (c * Mt +
// t) * 47 KiB, rows of 47 quads (752 B) -- row r holds X[64 t + r][kb .. kb +
// 187], kb = c * 188 (the last chunk: K - 188 when K >= 188 and K % 4 == 0,
// jit64_row_kbase), zero past M and K.  Each 16-B slot is 16 contiguous bytes
// of a row of X, so this is a gather-copy of row runs (no transpose): reads
// and writes both run along rows.  Four workgroups per (chunk, M tile), 752
// slots each.  HBM-bound: 2 * 4 * Mp * Kp bytes.
template <bool VEC>
__global__ __launch_bounds__(256) void tsg_transpose_rows_kernel(const float *__restrict__ X,
                                                                 float *__restrict__ XR, int M, int K, int Mp,
                                                                 int nch)
{
    constexpr int kQ = 47, kSlots = 64 * kQ, kPer = kSlots / 4;  // 752 slots per workgroup
    const int Mt = Mp >> 6;
    const int blk = blockIdx.x, part = blk & 3, tc = blk >> 2;
    // workgroup order (M tile * nch + chunk) * 4 + part: the workgroups in
    // flight read a few M tiles' rows end to end
    const int t = tc / nch, c = tc % nch;
    const int kb = (c == nch - 1 && K >= 4 * kQ && (K & 3) == 0) ? K - 4 * kQ : c * 4 * kQ;
    float *dst = XR + ((size_t)c * Mt + t) * (kSlots * 4);
    for (int i = threadIdx.x; i < kPer; i += 256) {
        const int slot = part * kPer + i, r = slot / kQ, q = slot % kQ;
        const int m = 64 * t + r, k = kb + 4 * q;
        float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (m < M) {
            const float *row = X + (size_t)m * K;
            if (VEC) {
                if (k < K) v = *reinterpret_cast<const float4 *>(row + k);  // K % 4 == 0: whole quad inside
            } else {
                if (k < K) v.x = row[k];
                if (k + 1 < K) v.y = row[k + 1];
                if (k + 2 < K) v.z = row[k + 2];
                if (k + 3 < K) v.w = row[k + 3];
            }
        }
        *reinterpret_cast<float4 *>(dst + (size_t)slot * 4) = v;
    }
}

// One LDS-DMA piece: 64 lanes x 16 B from per-lane global addresses to LDS
// [lds_dst, lds_dst + 1 KiB).  Inline asm on purpose: hipcc cannot prove that
// later ds_reads do not alias an in-flight LDS-DMA and would put
// `s_waitcnt vmcnt(0)` in front of the first one (serialising the prefetch).
// The kernel waits for these itself (vmcnt(0) before each step's barrier);
// M0 is set and restored inside the statement (cdna_hip_programming.md 5.7).
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


// ------------------------------------------------------------ rx kernel --
// Register-X walk (see tsg_internal.h "rx"): the block's X rows live in
// VGPRs and each entry is a SRC1-relative v_pk_add pair; no LDS read per
// entry.  The block loop is generated inline asm (gen_rx_asm.py).
#ifdef TSG_RX_INC
#include TSG_RX_INC  // diagnostic variant of the generated walk
#else
#include "tsg_rx_asm.inc"
#endif
#define TSG_RX_CAT2(a, b) a##b
#define TSG_RX_CAT(a, b) TSG_RX_CAT2(a, b)

typedef float F32x32 __attribute__((ext_vector_type(32)));

template <bool NEG>
__device__ __forceinline__ void rx_walk(F32x32 &a0, F32x32 &a1, F32x32 &a2, F32x32 &a3,
                                        const uint32_t *base, uint32_t &off, uint32_t &hdr,
                                        uint32_t xb)
{
    uint32_t t, nhdr, m0s;
    if constexpr (NEG)
        asm volatile(TSG_RX_CAT(TSG_RX_WALK_NEG_R, TSG_RX_ROWS)
                     : "+{v[112:143]}"(a0), "+{v[144:175]}"(a1), "+{v[176:207]}"(a2),
                       "+{v[208:239]}"(a3), [off] "+s"(off), [hdr] "+s"(hdr), [t] "=&s"(t),
                       [nhdr] "=&s"(nhdr), [m0s] "=&s"(m0s)
                     : [base] "s"(base), [xb] "v"(xb)
                     : TSG_RX_CAT(TSG_RX_CLOBBERS_R, TSG_RX_ROWS));
    else
        asm volatile(TSG_RX_CAT(TSG_RX_WALK_POS_R, TSG_RX_ROWS)
                     : "+{v[112:143]}"(a0), "+{v[144:175]}"(a1), "+{v[176:207]}"(a2),
                       "+{v[208:239]}"(a3), [off] "+s"(off), [hdr] "+s"(hdr), [t] "=&s"(t),
                       [nhdr] "=&s"(nhdr), [m0s] "=&s"(m0s)
                     : [base] "s"(base), [xb] "v"(xb)
                     : TSG_RX_CAT(TSG_RX_CLOBBERS_R, TSG_RX_ROWS));
}

// X^T chunk j (kRxChunk rows x 256 M) -> LDS buffer buf: one 1 KiB row per
// wave-instruction, 8 per wave.
__device__ __forceinline__ void rx_stage(const float *__restrict__ XT, int Mp, int m0, int j, int buf,
                                         int wave, int lane)
{
#pragma unroll
    for (int i = 0; i < kRxChunk / kRxWaves; i++) {
        const int r = wave * (kRxChunk / kRxWaves) + i;
        glds16(XT + (size_t)(j * kRxChunk + r) * Mp + m0 + 4 * lane, (uint32_t)(buf * kRxChunkBytes + r * 1024));
    }
}

template <bool PRELU>
__global__ __launch_bounds__(kRxWaves * 64, 8 / kRxWaves) void tsg_tcsc_rx_kernel(
    const float *__restrict__ XT, int Mp, const uint32_t *__restrict__ wstart,
    const uint32_t *__restrict__ ent, const float *__restrict__ b, const float *__restrict__ alpha,
    float *__restrict__ Y, int M, int N, int nch, int mtiles, int ntiles)
{
    __shared__ __attribute__((aligned(16))) char lds[kRxLdsBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    // LDS is only touched from asm (LDS-DMA, ds_read_b128 at absolute offsets
    // from 0): a never-taken C++ store keeps the allocation in the kernel
    if (M < 0) lds[tid] = 0;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // XCD-aware bijective remap: each XCD gets a contiguous run of workgroups
    const int T = mtiles * ntiles, L = blockIdx.x;
    const int xcd = L & 7, slot = L >> 3, q8 = T >> 3, r8 = T & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
    // n-tile-major: the concurrent workgroups of an XCD share few column
    // tiles, so their entry streams (latency-critical scalar loads) stay in
    // that XCD's L2; X^T chunks arrive by LDS-DMA a whole step ahead.
    const int nt = wg / mtiles, mt = wg - nt * mtiles;
    const int m0 = mt * kRxTileM;
    const int ncol0 = nt * kRxTileCols + wave * kRxNW;

    // the walk addresses its stream as ent + off (bytes; SMEM base + SGPR offset)
    uint32_t off = 4u * __builtin_amdgcn_readfirstlane(wstart[(size_t)nt * kRxWaves + wave]);
    uint32_t hdr = __builtin_amdgcn_readfirstlane(ent[off / 4]);
    rx_stage(XT, Mp, m0, 0, 0, wave, lane);
    F32x32 a0 = {}, a1 = {}, a2 = {}, a3 = {};  // comp.h:41
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // two loops (not one with a branch per step: a uniform if/else between
    // the two walks trips hipcc's SGPR-copy fixup on the asm operands)
    const int steps = 2 * nch;
    for (int q = 0; q < nch; q++) {  // +1 runs, ascending K
        if (q + 1 < steps) rx_stage(XT, Mp, m0, (q + 1) % nch, (q + 1) & 1, wave, lane);
        rx_walk<false>(a0, a1, a2, a3, ent, off, hdr, (uint32_t)(q & 1) * (uint32_t)kRxChunkBytes + (uint32_t)lane * 16u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    for (int q = nch; q < steps; q++) {  // -1 runs, ascending K
        if (q + 1 < steps) rx_stage(XT, Mp, m0, (q + 1) % nch, (q + 1) & 1, wave, lane);
        rx_walk<true>(a0, a1, a2, a3, ent, off, hdr, (uint32_t)(q & 1) * (uint32_t)kRxChunkBytes + (uint32_t)lane * 16u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (ncol0 >= N) return;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int m = m0 + 4 * lane + r;
        if (m >= M) continue;
        float *yrow = Y + (size_t)m * N + ncol0;
        float v[kRxNW];
#pragma unroll
        for (int c = 0; c < kRxNW; c++) {
            const int n = ncol0 + c < N ? ncol0 + c : N - 1;
            const float acc = c < 8 ? a0[4 * (c & 7) + r] : c < 16 ? a1[4 * (c & 7) + r]
                             : c < 24 ? a2[4 * (c & 7) + r] : a3[4 * (c & 7) + r];
            float y = acc + b[n];                       // comp.h:63
            if (PRELU) y = (y > 0) ? y : alpha[n] * y;  // comp_prelu.h:57-67
            v[c] = y;
        }
        if (ncol0 + kRxNW <= N && (((uintptr_t)yrow & 15) == 0)) {  // float4 stores need 16-B alignment
#pragma unroll
            for (int c = 0; c < kRxNW; c += 4)
                *reinterpret_cast<float4 *>(yrow + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
        } else {
#pragma unroll
            for (int c = 0; c < kRxNW; c++)
                if (ncol0 + c < N) yrow[c] = v[c];
        }
    }
}

// ---------------------------------------------------------------- launchers --
int launch_transpose(const float *X, float *XT, int M, int K, int Mp, int Kp, void *stream)
{
    dim3 grid((unsigned)((Kp + 63) / 64), (unsigned)(Mp / 64));
    if (K % 4 == 0 && ((uintptr_t)X & 15) == 0)
        hipLaunchKernelGGL(tsg_transpose4_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, XT, M, K, Mp, Kp);
    else
        hipLaunchKernelGGL(tsg_transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, XT, M, K, Mp, Kp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}


int launch_transpose_pairs(const float *X, float *XP, int M, int K, int Mp, int Kp, void *stream)
{
    // Mp is a multiple of 128 (the jit M tile) and Kp of 96: the 64 x 64 tiles
    // cover [0, Kp) x [0, Mp) exactly in m and up to 32 pad rows in k
    dim3 grid((unsigned)((Kp + 63) / 64), (unsigned)(Mp / 64));
    if (K % 4 == 0 && ((uintptr_t)X & 15) == 0)
        hipLaunchKernelGGL(tsg_transpose_pairs_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, X, XP, M, K,
                           Mp, Kp);
    else
        hipLaunchKernelGGL(tsg_transpose_pairs_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, X, XP, M, K,
                           Mp, Kp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_transpose_quads(const float *X, float *XQ, int M, int K, int Mp, int Kp, int piece_rows, void *stream,
                           int chunk)
{
    hipStream_t s = (hipStream_t)stream;
    const bool vec = K % 4 == 0 && ((uintptr_t)X & 15) == 0;
    if (piece_rows == 0) {  // the row layout: 188-row chunks, 47 KiB per (chunk, M tile)
        if (chunk != 188 || Mp % 64 || Kp % 188) return -1;
        const int nch = Kp / 188;
        const int64_t blocks = (int64_t)nch * (Mp / 64) * 4;
        if (blocks >= ((int64_t)1 << 31)) return -1;
        if (vec) hipLaunchKernelGGL(tsg_transpose_rows_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, X, XQ, M, K, Mp, nch);
        else hipLaunchKernelGGL(tsg_transpose_rows_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, X, XQ, M, K, Mp, nch);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    // Mp is a multiple of 64 (the 64-row image's M tile) and Kp of 192 (its
    // chunk): the pieces cover [0, Kp) x [0, Mp) exactly
    if ((chunk != 192 && chunk != 96) || Mp % 64 || Kp % chunk) return -1;
    // chunk / 16 workgroups of 4 pieces per (chunk, M tile)
    const int units = chunk / 4;
    const int64_t blocks = (int64_t)(Kp / chunk) * (Mp / 64) * (units / 4);
    if (blocks >= ((int64_t)1 << 31)) return -1;
    dim3 grid((unsigned)blocks);
    if (piece_rows == 16) {
        if (vec) hipLaunchKernelGGL((tsg_transpose_quads_kernel<true, 16>), grid, dim3(256), 0, s, X, XQ, M, K, Mp, Kp, units);
        else hipLaunchKernelGGL((tsg_transpose_quads_kernel<false, 16>), grid, dim3(256), 0, s, X, XQ, M, K, Mp, Kp, units);
    } else if (piece_rows == 8) {
        if (vec) hipLaunchKernelGGL((tsg_transpose_quads_kernel<true, 8>), grid, dim3(256), 0, s, X, XQ, M, K, Mp, Kp, units);
        else hipLaunchKernelGGL((tsg_transpose_quads_kernel<false, 8>), grid, dim3(256), 0, s, X, XQ, M, K, Mp, Kp, units);
    } else {
        return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_tcsc_rx(const float *XT, int Mp, const uint32_t *wstart, const uint32_t *ent,
                   const float *b, const float *alpha, float *Y, int M, int N, int Npad, int nch,
                   int prelu, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    const int mtiles = Mp / kRxTileM, ntiles = Npad / kRxTileCols;
    const dim3 grid((unsigned)(mtiles * ntiles)), block(kRxWaves * kLanes);
    if (prelu)
        hipLaunchKernelGGL((tsg_tcsc_rx_kernel<true>), grid, block, 0, s, XT, Mp, wstart, ent, b, alpha, Y, M,
                           N, nch, mtiles, ntiles);
    else
        hipLaunchKernelGGL((tsg_tcsc_rx_kernel<false>), grid, block, 0, s, XT, Mp, wstart, ent, b, alpha, Y, M,
                           N, nch, mtiles, ntiles);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tsg
