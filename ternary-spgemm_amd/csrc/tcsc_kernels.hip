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
// tsg_tcsc_stream_kernel (default).  One 1024-thread workgroup per CU, the
// whole 160 KiB LDS:
//   [0, 128 KiB)      X^T chunk (127 K rows x 128 M rows), double buffered,
//                     byte(buf, half, row, l) = half*65536 + buf*32768 + row*256 + l*8;
//   [128, 160 KiB)    per wave, double buffered, 1 KiB of its entry stream.
// Step q (= p*nch + j: the +1 runs over all K chunks, then the -1 runs) is
// staged during step q-1 by LDS-DMA (global_load_lds_dwordx4, no VGPRs): the
// X^T chunk (4 pieces of 1 KiB per wave) and each wave's sub-stream (1 piece).
// A wave then walks its NW column segments; an entry byte e = row | buf<<7 is
// byte 1 of its LDS address, so one v_perm_b32 with the lane constant
// (bytes 0 and 2) forms each ds_read_b64 address.  Per entry: v_perm,
// ds_read_b64, v_pk_add/sub; per 8 entries one broadcast ds_read_b64 of
// index bytes.  Bound: LDS read bandwidth.

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
__device__ __forceinline__ float2 walk_quad(float2 a, uint32_t w, uint32_t lanec, const char *lds)
{
    const float2 x0 = lds_f2(lds, entry_addr<0>(w, lanec));
    const float2 x1 = lds_f2(lds, entry_addr<1>(w, lanec));
    const float2 x2 = lds_f2(lds, entry_addr<2>(w, lanec));
    const float2 x3 = lds_f2(lds, entry_addr<3>(w, lanec));
    a = chain_step<NEG>(a, x0);
    a = chain_step<NEG>(a, x1);
    a = chain_step<NEG>(a, x2);
    a = chain_step<NEG>(a, x3);
    return a;
}

// Tail of a segment: 1..3 entries of the dword at `ipos` (no padded reads).
template <bool NEG>
__device__ __forceinline__ float2 walk_tail(float2 a, uint32_t ipos, uint32_t t, uint32_t lanec,
                                            const char *lds)
{
    const uint32_t w = *reinterpret_cast<const uint32_t *>(lds + ipos);  // broadcast read
    const float2 x0 = lds_f2(lds, entry_addr<0>(w, lanec));
    a = chain_step<NEG>(a, x0);
    if (t > 1) {
        const float2 x1 = lds_f2(lds, entry_addr<1>(w, lanec));
        a = chain_step<NEG>(a, x1);
        if (t > 2) {
            const float2 x2 = lds_f2(lds, entry_addr<2>(w, lanec));
            a = chain_step<NEG>(a, x2);
        }
    }
    return a;
}

// Segment of `ne` entries (ne/4 full dwords + a tail) at LDS byte `ipos`
// (8-byte aligned), starting at full dword `i0`.
// Tails: by default the last dword of a segment is walked whole (its pad
// entries read the +0.0f row: ~10% more LDS reads, no branches); with
// TSG_EXACT_TAIL the 1-3 real entries are read one by one.
#ifdef TSG_EXACT_TAIL
constexpr bool kExactTail = true;
#else
constexpr bool kExactTail = false;
#endif
__device__ __forceinline__ uint32_t full_dwords(uint32_t ne) { return kExactTail ? ne >> 2 : (ne + 3) >> 2; }

template <bool NEG>
__device__ __forceinline__ float2 walk_column(float2 a, uint32_t ipos, uint32_t ne, uint32_t i0,
                                              uint32_t lanec, const char *lds)
{
    const uint32_t full = full_dwords(ne);
    uint32_t i = i0;
    if (i + 2 <= full) {
        uint2 w = *reinterpret_cast<const uint2 *>(lds + ipos + 4 * i);  // broadcast read
        for (; i + 2 <= full; i += 2) {
            const uint2 nx = *reinterpret_cast<const uint2 *>(lds + ipos + 4 * (i + 2));  // prefetch
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
    }
    if (i < full) {
        const uint32_t w = *reinterpret_cast<const uint32_t *>(lds + ipos + 4 * i);
        a = walk_quad<NEG>(a, w, lanec, lds);
        i++;
    }
    if (kExactTail) {
        const uint32_t t = ne & 3u;
        if (t) a = walk_tail<NEG>(a, ipos + 4 * i, t, lanec, lds);
    }
    return a;
}

// Two columns walked in lockstep for min(ca, cb) dwords: two independent
// chains per wave interleave their LDS latency; each chain keeps its own
// order.  The longer column finishes alone.
template <bool NEG>
__device__ __forceinline__ void walk_pair(float2 &acc_a, float2 &acc_b, uint32_t pa, uint32_t ea,
                                          uint32_t pb, uint32_t eb, uint32_t lanec, const char *lds)
{
    const uint32_t ca = full_dwords(ea), cb = full_dwords(eb);
    const uint32_t joint = ca < cb ? ca : cb;
    float2 a = acc_a, b = acc_b;
    uint32_t i = 0;
    if (joint >= 2) {
        uint2 wa = *reinterpret_cast<const uint2 *>(lds + pa);
        uint2 wb = *reinterpret_cast<const uint2 *>(lds + pb);
        for (; i + 2 <= joint; i += 2) {
            const uint2 na = *reinterpret_cast<const uint2 *>(lds + pa + 4 * (i + 2));
            const uint2 nb = *reinterpret_cast<const uint2 *>(lds + pb + 4 * (i + 2));
            const float2 x0 = lds_f2(lds, entry_addr<0>(wa.x, lanec));
            const float2 y0 = lds_f2(lds, entry_addr<0>(wb.x, lanec));
            const float2 x1 = lds_f2(lds, entry_addr<1>(wa.x, lanec));
            const float2 y1 = lds_f2(lds, entry_addr<1>(wb.x, lanec));
            const float2 x2 = lds_f2(lds, entry_addr<2>(wa.x, lanec));
            const float2 y2 = lds_f2(lds, entry_addr<2>(wb.x, lanec));
            const float2 x3 = lds_f2(lds, entry_addr<3>(wa.x, lanec));
            const float2 y3 = lds_f2(lds, entry_addr<3>(wb.x, lanec));
            const float2 x4 = lds_f2(lds, entry_addr<0>(wa.y, lanec));
            const float2 y4 = lds_f2(lds, entry_addr<0>(wb.y, lanec));
            const float2 x5 = lds_f2(lds, entry_addr<1>(wa.y, lanec));
            const float2 y5 = lds_f2(lds, entry_addr<1>(wb.y, lanec));
            const float2 x6 = lds_f2(lds, entry_addr<2>(wa.y, lanec));
            const float2 y6 = lds_f2(lds, entry_addr<2>(wb.y, lanec));
            const float2 x7 = lds_f2(lds, entry_addr<3>(wa.y, lanec));
            const float2 y7 = lds_f2(lds, entry_addr<3>(wb.y, lanec));
            a = chain_step<NEG>(a, x0);
            b = chain_step<NEG>(b, y0);
            a = chain_step<NEG>(a, x1);
            b = chain_step<NEG>(b, y1);
            a = chain_step<NEG>(a, x2);
            b = chain_step<NEG>(b, y2);
            a = chain_step<NEG>(a, x3);
            b = chain_step<NEG>(b, y3);
            a = chain_step<NEG>(a, x4);
            b = chain_step<NEG>(b, y4);
            a = chain_step<NEG>(a, x5);
            b = chain_step<NEG>(b, y5);
            a = chain_step<NEG>(a, x6);
            b = chain_step<NEG>(b, y6);
            a = chain_step<NEG>(a, x7);
            b = chain_step<NEG>(b, y7);
            wa = na;
            wb = nb;
        }
    }
    acc_a = walk_column<NEG>(a, pa, ea, i, lanec, lds);
    acc_b = walk_column<NEG>(b, pb, eb, i, lanec, lds);
}

template <int NW>
struct StreamHeader {
    static constexpr int kWords = ((1 + NW / 4) + 1) & ~1;  // len + counts, even
};

template <int NW, bool NEG>
__device__ __forceinline__ void walk_chunk(float2 (&acc)[NW], const uint32_t (&cw)[NW / 4],
                                           uint32_t ibase, uint32_t lanec, const char *lds)
{
    uint32_t pos[NW], cnt[NW];
    uint32_t ipos = ibase + 4u * StreamHeader<NW>::kWords;
#pragma unroll
    for (int c = 0; c < NW; c++) {
        cnt[c] = (cw[c / 4] >> (8 * (c % 4))) & 0xffu;  // entries (exact)
        pos[c] = ipos;
        ipos += 4u * ((((cnt[c] + 3) >> 2) + 1) & ~1u);   // dwords, even-aligned
    }
#pragma unroll
    for (int c = 0; c < NW; c += 2) {
#ifndef TSG_NO_PRIO
        // progress-based priority: a wave that is further through its chunk
        // yields the issue ports to waves that lag, so the 16 waves reach
        // the step barrier together instead of leaving a latency-bound tail
        if (c == NW / 4) __builtin_amdgcn_s_setprio(2);
        if (c == NW / 2) __builtin_amdgcn_s_setprio(1);
        if (c == 3 * NW / 4) __builtin_amdgcn_s_setprio(0);
#endif
        walk_pair<NEG>(acc[c], acc[c + 1], pos[c], cnt[c], pos[c + 1], cnt[c + 1], lanec, lds);
    }
}

// ------------------------------------------------------------ flat walk --
// The wave's step is ONE dword stream (segments back to back).  Accumulators
// live in a register vector indexed by the current column (hipcc lowers the
// uniform dynamic index to s_set_gpr_idx register moves at segment
// boundaries only).  The loop is software-pipelined by one dword pair: the
// 8 ds_reads of pair p+1 are in flight while the adds of pair p run, so each
// wave always keeps LDS busy; every chain still adds in stream order.
template <int NW>
struct AccVec {
    typedef float type __attribute__((ext_vector_type(2 * NW)));
};

template <int NW>
struct ColCursor {
    uint64_t lo, hi;   // remaining per-column dword counts, 8 bits each, LSB first
    int cur;           // current column
    uint32_t rem;      // dwords left in the current column
    __device__ __forceinline__ void advance()
    {
        do {
            cur++;
            rem = (uint32_t)(lo & 0xffu);
            lo = (lo >> 8) | (hi << 56);
            hi >>= 8;
        } while (rem == 0 && cur < NW - 1);
    }
};

template <int NW, bool NEG>
__device__ __forceinline__ void flat_quad(float2 &work, const float2 (&x)[4], ColCursor<NW> &cc,
                                          typename AccVec<NW>::type &acc)
{
    work = chain_step<NEG>(work, x[0]);
    work = chain_step<NEG>(work, x[1]);
    work = chain_step<NEG>(work, x[2]);
    work = chain_step<NEG>(work, x[3]);
    if (--cc.rem == 0) {  // segment boundary (wave-uniform, ~1 in 4 dwords)
        acc[2 * cc.cur] = work.x;
        acc[2 * cc.cur + 1] = work.y;
        if (cc.cur < NW - 1) {
            cc.advance();
            work = make_float2(acc[2 * cc.cur], acc[2 * cc.cur + 1]);
        }
    }
}

__device__ __forceinline__ void flat_reads(float2 (&x)[4], uint32_t w, uint32_t lanec, const char *lds)
{
    x[0] = lds_f2(lds, entry_addr<0>(w, lanec));
    x[1] = lds_f2(lds, entry_addr<1>(w, lanec));
    x[2] = lds_f2(lds, entry_addr<2>(w, lanec));
    x[3] = lds_f2(lds, entry_addr<3>(w, lanec));
}

template <int NW, bool NEG>
__device__ __forceinline__ void flat_pair(float2 &work, const float2 (&x)[8], ColCursor<NW> &cc,
                                          typename AccVec<NW>::type &acc)
{
    const float2 lo[4] = {x[0], x[1], x[2], x[3]};
    const float2 hi[4] = {x[4], x[5], x[6], x[7]};
    flat_quad<NW, NEG>(work, lo, cc, acc);
    flat_quad<NW, NEG>(work, hi, cc, acc);
}

__device__ __forceinline__ void flat_reads8(float2 (&x)[8], uint2 w, uint32_t lanec, const char *lds)
{
    x[0] = lds_f2(lds, entry_addr<0>(w.x, lanec));
    x[1] = lds_f2(lds, entry_addr<1>(w.x, lanec));
    x[2] = lds_f2(lds, entry_addr<2>(w.x, lanec));
    x[3] = lds_f2(lds, entry_addr<3>(w.x, lanec));
    x[4] = lds_f2(lds, entry_addr<0>(w.y, lanec));
    x[5] = lds_f2(lds, entry_addr<1>(w.y, lanec));
    x[6] = lds_f2(lds, entry_addr<2>(w.y, lanec));
    x[7] = lds_f2(lds, entry_addr<3>(w.y, lanec));
}

__device__ __forceinline__ uint2 idx_pair(const char *lds, uint32_t pd, uint32_t p)
{
    return *reinterpret_cast<const uint2 *>(lds + pd + 8u * p);  // broadcast read
}

// Pipeline.  LDS returns in order, so the index pair of dword pair p+2 is
// fetched BEFORE the 8 data reads of pair p+1 (a later wait on it then does
// not drain those reads); the adds of pair p run while pair p+1 is in
// flight.  Reads past the step's data are harmless: any entry byte maps into
// the X^T region.
template <int NW, bool NEG>
__device__ __forceinline__ void walk_chunk_flat(typename AccVec<NW>::type &acc, const uint32_t (&hw)[8],
                                                uint32_t ib, uint32_t lanec, const char *lds)
{
    const uint32_t npairs = hw[1] >> 1;
    if (npairs == 0) return;
    ColCursor<NW> cc;
    cc.lo = (uint64_t)hw[2] | ((uint64_t)hw[3] << 32);
    cc.hi = (uint64_t)hw[4] | ((uint64_t)hw[5] << 32);
    cc.cur = -1;
    cc.advance();
    float2 work = make_float2(acc[2 * cc.cur], acc[2 * cc.cur + 1]);
    const uint32_t pd = ib + 4u * kSFlatHdrWords;
    uint2 w = idx_pair(lds, pd, 0);
    uint2 wn = idx_pair(lds, pd, 1);
    float2 xa[4], xb[4];
    flat_reads(xa, w.x, lanec, lds);
    flat_reads(xb, w.y, lanec, lds);
    for (uint32_t p = 1; p < npairs; p++) {
        w = wn;
        wn = idx_pair(lds, pd, p + 1);      // 2 pairs ahead of the adds
        float2 ya[4], yb[4];
        flat_reads(ya, w.x, lanec, lds);    // pair p in flight ...
        flat_reads(yb, w.y, lanec, lds);
        flat_quad<NW, NEG>(work, xa, cc, acc);  // ... while pair p-1 is added
        flat_quad<NW, NEG>(work, xb, cc, acc);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            xa[i] = ya[i];
            xb[i] = yb[i];
        }
    }
    flat_quad<NW, NEG>(work, xa, cc, acc);
    flat_quad<NW, NEG>(work, xb, cc, acc);
}

// LDS-DMA of X^T chunk j (127 rows x 128 M) into buffer `buf`: 64 pieces of
// 1 KiB (4 rows of one half), 4 per wave; row 127 (the zero row) is sourced
// from a zeroed global buffer so every refill also re-zeroes it.
__device__ __forceinline__ void stage_x(const float *__restrict__ XT, const float *__restrict__ zero,
                                        int Mp, int m0, int j, int buf, int wave, int lane)
{
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int p = wave * 4 + i;
        const int h = p >> 5, r0 = (p & 31) * 4, rr = r0 + (lane >> 4), mo = (lane & 15) * 4;
        const float *src = rr < kSChunk ? XT + (size_t)(j * kSChunk + rr) * Mp + m0 + 64 * h + mo
                                        : zero + mo;
        glds16(src, (uint32_t)(h * 65536 + buf * 32768 + r0 * 256));
    }
}

__device__ __forceinline__ void stage_idx(const uint32_t *__restrict__ ent, uint32_t base,
                                          uint32_t dst, int lane)
{
    glds16(ent + base + 4 * lane, dst);
}

// STAMP: diagnostic build only (TSG_STAMPS=1): per wave, s_memtime cycles
// spent walking vs. waiting at the step barrier, written to `stamps`.
template <int NW, bool PRELU, bool STAMP, bool FLAT>
__global__ __launch_bounds__(1024, 1) void tsg_tcsc_stream_kernel(
    const float *__restrict__ XT, int Mp, const uint32_t *__restrict__ wstart,
    const uint32_t *__restrict__ ent, const float *__restrict__ zero, const float *__restrict__ b,
    const float *__restrict__ alpha, float *__restrict__ Y, int M, int N, int nch, int mtiles,
    int ntiles, unsigned long long *__restrict__ stamps)
{
    unsigned long long st_work = 0, st_wait = 0, st_t0 = 0;
    if (STAMP) st_t0 = __builtin_amdgcn_s_memtime();
    __shared__ __attribute__((aligned(16))) char lds[kSLdsBytes + kSIdxBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // XCD-aware bijective remap: blocks b and b+8 share an XCD (observed
    // round-robin dispatch); each XCD gets a contiguous, m-tile-major run of
    // tiles so its concurrent workgroups share the X^T slab in L2.  Speed only.
    const int T = mtiles * ntiles, L = blockIdx.x;
    const int xcd = L & 7, slot = L >> 3, q8 = T >> 3, r8 = T & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
    const int mt = wg / ntiles, nt = wg - mt * ntiles;
    const int m0 = mt * kTileM;
    const int ncol0 = nt * (kSWaves * NW) + wave * NW;

    const uint32_t lanec = ((uint32_t)(lane & 31) << 3) | ((uint32_t)(lane >> 5) << 16);
    const uint32_t ireg = (uint32_t)kSLdsBytes + (uint32_t)wave * 2u * kSIdxWaveBytes;  // + buf*1KiB

    uint32_t sbase = wstart[(size_t)nt * kSWaves + wave];
    stage_x(XT, zero, Mp, m0, 0, 0, wave, lane);
    stage_idx(ent, sbase, ireg, lane);

    float2 acc[NW];
#pragma unroll
    for (int c = 0; c < NW; c++) acc[c] = make_float2(0.0f, 0.0f);  // comp.h:41
    typename AccVec<NW>::type accv = {};                            // FLAT: same, as a vector

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int steps = 2 * nch;
    for (int q = 0; q < steps; q++) {
        unsigned long long ta = 0, tb = 0;
        if (STAMP) ta = __builtin_amdgcn_s_memtime();
        const uint32_t ib = ireg + (uint32_t)(q & 1) * kSIdxWaveBytes;
#ifndef TSG_NO_PRIO
        __builtin_amdgcn_s_setprio(3);
#endif
        // header of this step: [len][NW count bytes] / FLAT: [len][D][NW dword-count bytes]
        constexpr int kHW = FLAT ? kSFlatHdrWords : StreamHeader<NW>::kWords;
        uint32_t hw[kHW > 8 ? kHW : 8] = {};
#pragma unroll
        for (int i = 0; i < kHW; i += 2) {
            const uint2 v = *reinterpret_cast<const uint2 *>(lds + ib + 4 * i);
            hw[i] = __builtin_amdgcn_readfirstlane(v.x);
            hw[i + 1] = __builtin_amdgcn_readfirstlane(v.y);
        }
        if (q + 1 < steps) {  // stage step q+1 into the other buffers
            sbase += hw[0];
            stage_x(XT, zero, Mp, m0, (q + 1) % nch, (q + 1) & 1, wave, lane);
            stage_idx(ent, sbase, ireg + (uint32_t)((q + 1) & 1) * kSIdxWaveBytes, lane);
        }
        if (FLAT) {
            uint32_t h8[8];
#pragma unroll
            for (int i = 0; i < 8; i++) h8[i] = hw[i];
            if (q < nch) walk_chunk_flat<NW, false>(accv, h8, ib, lanec, lds);  // +1 runs
            else walk_chunk_flat<NW, true>(accv, h8, ib, lanec, lds);           // -1 runs
        } else {
            uint32_t cw[NW / 4];
#pragma unroll
            for (int i = 0; i < NW / 4; i++) cw[i] = hw[1 + i];
            if (q < nch) walk_chunk<NW, false>(acc, cw, ib, lanec, lds);  // +1 runs, ascending K
            else walk_chunk<NW, true>(acc, cw, ib, lanec, lds);           // -1 runs, ascending K
        }
        if (STAMP) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            tb = __builtin_amdgcn_s_memtime();
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA for q+1 landed
        __syncthreads();                                   // ... and every other wave's
        if (STAMP) {
            const unsigned long long tc = __builtin_amdgcn_s_memtime();
            st_work += tb - ta;
            st_wait += tc - tb;
        }
    }
    if (STAMP && lane == 0) {
        unsigned long long *o = stamps + ((size_t)blockIdx.x * kSWaves + wave) * 4;
        o[0] = st_work;
        o[1] = st_wait;
        o[2] = __builtin_amdgcn_s_memtime() - st_t0;
        o[3] = (unsigned long long)((nt << 16) | mt);
    }

    if (FLAT) {
#pragma unroll
        for (int c = 0; c < NW; c++) acc[c] = make_float2(accv[2 * c], accv[2 * c + 1]);
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
    dim3 grid((unsigned)((Kp + 63) / 64), (unsigned)(Mp / 64));
    hipLaunchKernelGGL(tsg_transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream, X, XT, M, K, Mp, Kp);
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

template <int NW, bool PRELU, bool STAMP>
static void launch_stream_nw(const float *XT, int Mp, const uint32_t *wstart, const uint32_t *ent,
                             const float *zero, const float *b, const float *alpha, float *Y, int M,
                             int N, int Npad, int nch, unsigned long long *stamps, bool flat,
                             hipStream_t s)
{
    const int mtiles = Mp / kTileM, ntiles = Npad / (kSWaves * NW);
    if (flat)
        hipLaunchKernelGGL((tsg_tcsc_stream_kernel<NW, PRELU, STAMP, true>),
                           dim3((unsigned)(mtiles * ntiles)), dim3(1024), 0, s, XT, Mp, wstart, ent,
                           zero, b, alpha, Y, M, N, nch, mtiles, ntiles, stamps);
    else
        hipLaunchKernelGGL((tsg_tcsc_stream_kernel<NW, PRELU, STAMP, false>),
                           dim3((unsigned)(mtiles * ntiles)), dim3(1024), 0, s, XT, Mp, wstart, ent,
                           zero, b, alpha, Y, M, N, nch, mtiles, ntiles, stamps);
}

int launch_tcsc_stream(const float *XT, int Mp, const uint32_t *wstart, const uint32_t *ent,
                       const float *zero, const float *b, const float *alpha, float *Y, int M,
                       int N, int Npad, int nch, int nw, int prelu, unsigned long long *stamps,
                       bool flat, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
#define TSG_NW(NWV)                                                                               \
    if (nw == NWV) {                                                                              \
        if (stamps) launch_stream_nw<NWV, false, true>(XT, Mp, wstart, ent, zero, b, alpha, Y, M, N, Npad, nch, stamps, flat, s); \
        else if (prelu) launch_stream_nw<NWV, true, false>(XT, Mp, wstart, ent, zero, b, alpha, Y, M, N, Npad, nch, nullptr, flat, s); \
        else launch_stream_nw<NWV, false, false>(XT, Mp, wstart, ent, zero, b, alpha, Y, M, N, Npad, nch, nullptr, flat, s); \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                          \
    }
    TSG_NW(16)
    TSG_NW(8)
    TSG_NW(4)
#undef TSG_NW
    return -2;
}

}  // namespace tsg
