// tcsc_kernels.hip -- gfx950 kernels for Y = X * W + b with W ternary (TCSC).
//
// Arithmetic contract (cpp_impl/comp.h:37-63, BaseTCSC<float>): every output
// Y[m,n] is ONE serial fp32 chain  0 + x_p1 + ... + x_pP - x_n1 - ... - x_nQ,
// then + b[n], with the +1 run and the -1 run each in ascending k.  Therefore
// no output is ever split across lanes/waves: parallelism is over (m, n)
// pairs only.  Lanes own M rows, a wave walks one column at a time (its k is
// wave-uniform, so the index stream rides the scalar unit), waves and
// workgroups own columns.
//
// Kernel 1 (tsg_transpose_kernel): X [M][K] -> X^T [Kp][Mp], zero padded.
//   HBM-bound copy (2 * 4 * M * K bytes).
// Kernel 2 (tsg_tcsc_lds_kernel): per workgroup a 128-row M tile x
//   (4 waves * NW) column tile.  For pass p in {+1 run, -1 run}, for each
//   128-row K chunk: stage X^T[chunk][tile] (64 KiB) in LDS, then each wave
//   walks, for each of its NW columns, the column's entries in the chunk
//   (uint8 row-in-chunk, 4 per dword, scalar loads), one ds_read_b64 per
//   entry (2 rows per lane), one v_pk_add/sub per entry.  Chunks are walked
//   in ascending k, pass +1 fully before pass -1, so each accumulator sees
//   exactly the reference's order.  Index groups are padded with an LDS row
//   of +0.0f: y + 0 == y and y - 0 == y bit-exactly, because the chain never
//   holds -0 (it starts at +0 and RN never yields -0 from it).
//   Roofline: LDS bandwidth (8 B of LDS read per 2 adds), see DESIGN.md.
#include <hip/hip_runtime.h>

#include "tsg_internal.h"

namespace tsg {

// ------------------------------------------------------------------ kernel 1 --
__global__ __launch_bounds__(256) void tsg_transpose_kernel(const float *__restrict__ X,
                                                            float *__restrict__ XT, int M, int K,
                                                            int Mp)
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
        XT[(size_t)k * Mp + m] = tile[tx][ty + 4 * i];
    }
}

// ------------------------------------------------------------------ kernel 2 --
template <bool NEG>
__device__ __forceinline__ float2 chain_step(float2 a, float2 x)
{
    // y += x  /  y -= x, one IEEE op per row (comp.h:48 / :58)
    if (NEG) return make_float2(a.x - x.x, a.y - x.y);
    return make_float2(a.x + x.x, a.y + x.y);
}

template <bool NEG>
__device__ __forceinline__ float2 walk_segment(float2 a, const uint32_t *__restrict__ ent,
                                               uint32_t d0, uint32_t d1,
                                               const float2 *__restrict__ lds, int lane)
{
    for (uint32_t d = d0; d < d1; d++) {
        const uint32_t w = ent[d];  // wave-uniform -> s_load_dword
        const float2 x0 = lds[((w >> 0) & 0xffu) * kLanes + lane];
        const float2 x1 = lds[((w >> 8) & 0xffu) * kLanes + lane];
        const float2 x2 = lds[((w >> 16) & 0xffu) * kLanes + lane];
        const float2 x3 = lds[((w >> 24) & 0xffu) * kLanes + lane];
        a = chain_step<NEG>(a, x0);
        a = chain_step<NEG>(a, x1);
        a = chain_step<NEG>(a, x2);
        a = chain_step<NEG>(a, x3);
    }
    return a;
}

template <int NW, bool NEG>
__device__ __forceinline__ void run_pass(float2 (&acc)[NW], const float *__restrict__ XT, int Mp,
                                         int m0, const uint32_t *__restrict__ seg,
                                         const uint32_t *__restrict__ ent, int ncol0, int nch,
                                         float2 *lds)
{
    float4 *lds4 = reinterpret_cast<float4 *>(lds);
    const int tid = threadIdx.x, lane = tid & 63;
    const int p = NEG ? 1 : 0;
    for (int j = 0; j < nch; j++) {
        __syncthreads();  // previous chunk fully consumed
        // stage X^T[j*KC .. +KC][m0 .. m0+128): 128 rows x 32 float4
#pragma unroll
        for (int t = 0; t < (kChunkK * kTileM / 4) / 256; t++) {
            const int i = tid + 256 * t;
            const int r = i >> 5, c4 = i & 31;
            lds4[i] = *reinterpret_cast<const float4 *>(XT + (size_t)(j * kChunkK + r) * Mp + m0 + 4 * c4);
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NW; c++) {
            const uint32_t *sp = seg + ((size_t)(ncol0 + c) * 2 + p) * (nch + 1) + j;
            acc[c] = walk_segment<NEG>(acc[c], ent, sp[0], sp[1], lds, lane);
        }
    }
}

template <int NW, bool PRELU>
__global__ __launch_bounds__(256, 2) void tsg_tcsc_lds_kernel(
    const float *__restrict__ XT, int Mp, const uint32_t *__restrict__ seg,
    const uint32_t *__restrict__ ent, const float *__restrict__ b,
    const float *__restrict__ alpha, float *__restrict__ Y, int M, int N, int nch)
{
    __shared__ float2 lds[(kChunkK + 1) * kLanes];  // row kZeroRow = +0.0f
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m0 = blockIdx.x * kTileM;
    const int ncol0 = blockIdx.y * (kWaves * NW) + wave * NW;

    if (threadIdx.x < kLanes) lds[kZeroRow * kLanes + threadIdx.x] = make_float2(0.0f, 0.0f);

    float2 acc[NW];
#pragma unroll
    for (int c = 0; c < NW; c++) acc[c] = make_float2(0.0f, 0.0f);  // comp.h:41

    run_pass<NW, false>(acc, XT, Mp, m0, seg, ent, ncol0, nch, lds);  // +1 run, all K
    run_pass<NW, true>(acc, XT, Mp, m0, seg, ent, ncol0, nch, lds);   // -1 run, all K

    if (ncol0 >= N) return;
    // epilogue: Y[m, n] = y + b[n] (comp.h:63) [PReLU: comp_prelu.h:50-67].
    // Lane owns rows m0+2*lane+{0,1}; its NW columns are contiguous in a row.
#pragma unroll
    for (int r = 0; r < kRowsPerLane; r++) {
        const int m = m0 + kRowsPerLane * lane + r;
        if (m >= M) continue;
        float *yrow = Y + (size_t)m * N + ncol0;
        float v[NW];
#pragma unroll
        for (int c = 0; c < NW; c++) {
            const int n = ncol0 + c < N ? ncol0 + c : N - 1;
            float y = (r == 0 ? acc[c].x : acc[c].y) + b[n];
            if (PRELU) y = (y > 0) ? y : alpha[n] * y;
            v[c] = y;
        }
        if (ncol0 + NW <= N && ((((size_t)m * N + ncol0) & 3) == 0)) {
#pragma unroll
            for (int c = 0; c < NW; c += 4)
                *reinterpret_cast<float4 *>(yrow + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
        } else {
#pragma unroll
            for (int c = 0; c < NW; c++)
                if (ncol0 + c < N) yrow[c] = v[c];
        }
    }
}

// ------------------------------------------------------------------ kernel 3 --
// tsg_tcsc_stream_kernel: one 1024-thread workgroup per CU (128 KiB LDS),
// 16 waves x NW columns, 128 M rows.  Double-buffered X^T chunks of 127 K rows.
// Each wave walks ONE linear entry stream (see StreamImage) with scalar loads
// (two dwords = 8 entries per s_load, prefetched one step ahead so the SMEM
// latency hides under the previous step's LDS reads), and one v_perm_b32 per
// entry turns the packed byte into the ds_read_b64 address: per entry the
// vector ALU does 2 instructions (perm + pk_add/sub), the scalar ALU none.

// address of entry I (0..3) of packed dword w: byte1 <- entry, bytes 0/2 <- lane constant
template <int I>
__device__ __forceinline__ uint32_t entry_addr(uint32_t w, uint32_t lanec)
{
    return __builtin_amdgcn_perm(w, lanec, 0x0C020400u | ((4u + I) << 8));
}

__device__ __forceinline__ float2 lds_f2(const char *lds, uint32_t a)
{
    return *reinterpret_cast<const float2 *>(lds + a);
}

template <bool NEG>
__device__ __forceinline__ float2 walk_column(float2 a, const uint32_t *__restrict__ p, uint32_t cnt,
                                              uint32_t lanec, const char *lds)
{
    if (cnt == 0) return a;
    uint2 w = *reinterpret_cast<const uint2 *>(p);  // segment starts are 8-byte aligned
    uint32_t i = 0;
    for (; i + 2 <= cnt; i += 2) {
        const uint2 nx = *reinterpret_cast<const uint2 *>(p + i + 2);  // prefetch (tail padded)
        const float2 x0 = lds_f2(lds, entry_addr<0>(w.x, lanec));
        const float2 x1 = lds_f2(lds, entry_addr<1>(w.x, lanec));
        const float2 x2 = lds_f2(lds, entry_addr<2>(w.x, lanec));
        const float2 x3 = lds_f2(lds, entry_addr<3>(w.x, lanec));
        const float2 x4 = lds_f2(lds, entry_addr<0>(w.y, lanec));
        const float2 x5 = lds_f2(lds, entry_addr<1>(w.y, lanec));
        const float2 x6 = lds_f2(lds, entry_addr<2>(w.y, lanec));
        const float2 x7 = lds_f2(lds, entry_addr<3>(w.y, lanec));
        a = chain_step<NEG>(a, x0);
        a = chain_step<NEG>(a, x1);
        a = chain_step<NEG>(a, x2);
        a = chain_step<NEG>(a, x3);
        a = chain_step<NEG>(a, x4);
        a = chain_step<NEG>(a, x5);
        a = chain_step<NEG>(a, x6);
        a = chain_step<NEG>(a, x7);
        w = nx;
    }
    if (i < cnt) {
        const float2 x0 = lds_f2(lds, entry_addr<0>(w.x, lanec));
        const float2 x1 = lds_f2(lds, entry_addr<1>(w.x, lanec));
        const float2 x2 = lds_f2(lds, entry_addr<2>(w.x, lanec));
        const float2 x3 = lds_f2(lds, entry_addr<3>(w.x, lanec));
        a = chain_step<NEG>(a, x0);
        a = chain_step<NEG>(a, x1);
        a = chain_step<NEG>(a, x2);
        a = chain_step<NEG>(a, x3);
    }
    return a;
}

// One chunk step of one wave: header (NW dword counts, NW/4 dwords), then the
// NW segments, each starting on an even dword.  Returns the next step's start.
template <int NW, bool NEG>
__device__ __forceinline__ const uint32_t *walk_chunk(float2 (&acc)[NW], const uint32_t *__restrict__ p,
                                                      uint32_t lanec, const char *lds)
{
    uint32_t hdr[NW / 4];
#pragma unroll
    for (int i = 0; i < NW / 4; i++) hdr[i] = p[i];
    p += NW / 4;
#pragma unroll
    for (int c = 0; c < NW; c++) {
        const uint32_t cnt = (hdr[c / 4] >> (8 * (c % 4))) & 0xffu;
        acc[c] = walk_column<NEG>(acc[c], p, cnt, lanec, lds);
        p += (cnt + 1) & ~1u;
    }
    return p;
}

// X^T chunk (127 rows x 128 M) -> registers (4 float4 per thread)
struct ChunkRegs {
    float4 v[4];
};

__device__ __forceinline__ void load_chunk(ChunkRegs &r, const float *__restrict__ XT, int Mp,
                                           int m0, int j, int tid)
{
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int i = tid + 1024 * t;  // < 127*32 = 4064 valid
        const int row = i >> 5, c4 = i & 31;
        if (row < kSChunk)
            r.v[t] = *reinterpret_cast<const float4 *>(XT + (size_t)(j * kSChunk + row) * Mp + m0 + 4 * c4);
    }
}

__device__ __forceinline__ void store_chunk(const ChunkRegs &r, char *lds, int buf, int tid)
{
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int i = tid + 1024 * t;
        const int row = i >> 5, c4 = i & 31;
        if (row < kSChunk) {
            const uint32_t a = (uint32_t)((c4 >> 4) * 65536 + buf * 32768 + row * 256 + (c4 & 15) * 16);
            *reinterpret_cast<float4 *>(lds + a) = r.v[t];
        }
    }
}

template <int NW, bool PRELU>
__global__ __launch_bounds__(1024, 1) void tsg_tcsc_stream_kernel(
    const float *__restrict__ XT, int Mp, const uint32_t *__restrict__ wstart,
    const uint32_t *__restrict__ ent, const float *__restrict__ b,
    const float *__restrict__ alpha, float *__restrict__ Y, int M, int N, int nch, int mtiles,
    int ntiles)
{
    __shared__ __attribute__((aligned(16))) char lds[kSLdsBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // XCD-aware bijective remap: blocks b and b+8 share an XCD (observed
    // round-robin dispatch); give each XCD a contiguous run of m-tile-major
    // tiles so its concurrent workgroups share the X^T slab in L2.  Speed only.
    const int T = mtiles * ntiles, L = blockIdx.x;
    const int xcd = L & 7, slot = L >> 3, q8 = T >> 3, r8 = T & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
    const int mt = wg / ntiles, nt = wg - mt * ntiles;
    const int m0 = mt * kTileM;
    const int ncol0 = nt * (kSWaves * NW) + wave * NW;

    const uint32_t lanec = ((uint32_t)(lane & 31) << 3) | ((uint32_t)(lane >> 5) << 16);

    // zero rows: row 127 of both buffers and both halves (4 x 256 B)
    if (tid < 256) {
        const int h = tid >> 7, bf = (tid >> 6) & 1, x = tid & 63;
        reinterpret_cast<float *>(lds + h * 65536 + bf * 32768 + kSZeroRow * 256)[x] = 0.0f;
    }
    ChunkRegs cr;
    load_chunk(cr, XT, Mp, m0, 0, tid);
    store_chunk(cr, lds, 0, tid);

    const uint32_t *sp = ent + wstart[(size_t)nt * kSWaves + wave];

    float2 acc[NW];
#pragma unroll
    for (int c = 0; c < NW; c++) acc[c] = make_float2(0.0f, 0.0f);  // comp.h:41
    __syncthreads();

    const int steps = 2 * nch;
    for (int q = 0; q < steps; q++) {
        const bool more = q + 1 < steps;
        if (more) load_chunk(cr, XT, Mp, m0, (q + 1) % nch, tid);
        // the entry bytes carry the buffer bit, so both buffers share one base
        if (q < nch) sp = walk_chunk<NW, false>(acc, sp, lanec, lds);  // +1 runs, ascending K
        else sp = walk_chunk<NW, true>(acc, sp, lanec, lds);           // -1 runs, ascending K
        if (more) store_chunk(cr, lds, (q + 1) & 1, tid);
        __syncthreads();
    }

    if (ncol0 >= N) return;
#pragma unroll
    for (int r = 0; r < kRowsPerLane; r++) {
        const int m = m0 + kRowsPerLane * lane + r;
        if (m >= M) continue;
        float *yrow = Y + (size_t)m * N + ncol0;
        float v[NW];
#pragma unroll
        for (int c = 0; c < NW; c++) {
            const int n = ncol0 + c < N ? ncol0 + c : N - 1;
            float y = (r == 0 ? acc[c].x : acc[c].y) + b[n];  // comp.h:63
            if (PRELU) y = (y > 0) ? y : alpha[n] * y;         // comp_prelu.h:57-67
            v[c] = y;
        }
        if (ncol0 + NW <= N && ((((size_t)m * N + ncol0) & 3) == 0)) {
#pragma unroll
            for (int c = 0; c < NW; c += 4)
                *reinterpret_cast<float4 *>(yrow + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
        } else {
#pragma unroll
            for (int c = 0; c < NW; c++)
                if (ncol0 + c < N) yrow[c] = v[c];
        }
    }
}

// ---------------------------------------------------------------- launchers --
int launch_transpose(const float *X, float *XT, int M, int K, int Mp, int Kp, void *stream)
{
    dim3 grid((unsigned)(Kp / 64), (unsigned)(Mp / 64));
    hipLaunchKernelGGL(tsg_transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, XT, M, K, Mp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int NW, bool PRELU>
static void launch_nw(const float *XT, int Mp, const uint32_t *seg, const uint32_t *ent,
                      const float *b, const float *alpha, float *Y, int M, int N, int Npad, int nch,
                      hipStream_t s)
{
    dim3 grid((unsigned)(Mp / kTileM), (unsigned)(Npad / (kWaves * NW)));
    hipLaunchKernelGGL((tsg_tcsc_lds_kernel<NW, PRELU>), grid, dim3(256), 0, s, XT, Mp, seg, ent, b,
                       alpha, Y, M, N, nch);
}

int launch_tcsc(const float *XT, int Mp, const uint32_t *seg, const uint32_t *ent,
                const float *b, const float *alpha, float *Y, int M, int N, int Npad, int nch,
                int tile_cols, int prelu, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    const int nw = tile_cols / kWaves;
    if (nw == 32) {
        if (prelu) launch_nw<32, true>(XT, Mp, seg, ent, b, alpha, Y, M, N, Npad, nch, s);
        else launch_nw<32, false>(XT, Mp, seg, ent, b, alpha, Y, M, N, Npad, nch, s);
    } else if (nw == 16) {
        if (prelu) launch_nw<16, true>(XT, Mp, seg, ent, b, alpha, Y, M, N, Npad, nch, s);
        else launch_nw<16, false>(XT, Mp, seg, ent, b, alpha, Y, M, N, Npad, nch, s);
    } else {
        return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int NW, bool PRELU>
static void launch_stream_nw(const float *XT, int Mp, const uint32_t *wstart, const uint32_t *ent,
                             const float *b, const float *alpha, float *Y, int M, int N, int Npad,
                             int nch, hipStream_t s)
{
    const int mtiles = Mp / kTileM, ntiles = Npad / (kSWaves * NW);
    hipLaunchKernelGGL((tsg_tcsc_stream_kernel<NW, PRELU>), dim3((unsigned)(mtiles * ntiles)),
                       dim3(1024), 0, s, XT, Mp, wstart, ent, b, alpha, Y, M, N, nch, mtiles, ntiles);
}

int launch_tcsc_stream(const float *XT, int Mp, const uint32_t *wstart, const uint32_t *ent,
                       const float *b, const float *alpha, float *Y, int M, int N, int Npad,
                       int nch, int nw, int prelu, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    if (nw == 16) {
        if (prelu) launch_stream_nw<16, true>(XT, Mp, wstart, ent, b, alpha, Y, M, N, Npad, nch, s);
        else launch_stream_nw<16, false>(XT, Mp, wstart, ent, b, alpha, Y, M, N, Npad, nch, s);
    } else if (nw == 8) {
        if (prelu) launch_stream_nw<8, true>(XT, Mp, wstart, ent, b, alpha, Y, M, N, Npad, nch, s);
        else launch_stream_nw<8, false>(XT, Mp, wstart, ent, b, alpha, Y, M, N, Npad, nch, s);
    } else {
        return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tsg
