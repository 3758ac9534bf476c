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
// Kernel 1 (tsg_transpose_kernel, tsg_transpose4_kernel when K % 4 == 0):
//   X [M][K] -> X^T [Kp][Mp], zero padded.  HBM-bound copy (2 * 4 * M * K bytes).
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
            asm volatile("" ::: "memory");  // keep the prefetch (see walk_pair)
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
//
// Software pipeline (default; -DTSG_NO_PIPE for the plain loop): the 8 reads
// of the next dword are in flight while the current dword's 8 adds run, and
// the index words of the next 2-dword block are read BEFORE those data reads
// (LDS returns in order, so waiting for them never drains the data in
// flight).  sched_barrier pins that issue order against the scheduler.
#ifdef TSG_NO_PIPE
constexpr bool kPipe = false;
#else
constexpr bool kPipe = true;
#endif

struct Quad2 { float2 a[4], b[4]; };

__device__ __forceinline__ void pair_reads(Quad2 &q, uint32_t wa, uint32_t wb, uint32_t lanec,
                                           const char *lds)
{
    q.a[0] = lds_f2(lds, entry_addr<0>(wa, lanec));
    q.b[0] = lds_f2(lds, entry_addr<0>(wb, lanec));
    q.a[1] = lds_f2(lds, entry_addr<1>(wa, lanec));
    q.b[1] = lds_f2(lds, entry_addr<1>(wb, lanec));
    q.a[2] = lds_f2(lds, entry_addr<2>(wa, lanec));
    q.b[2] = lds_f2(lds, entry_addr<2>(wb, lanec));
    q.a[3] = lds_f2(lds, entry_addr<3>(wa, lanec));
    q.b[3] = lds_f2(lds, entry_addr<3>(wb, lanec));
}

template <bool NEG>
__device__ __forceinline__ void pair_adds(float2 &a, float2 &b, const Quad2 &q)
{
#pragma unroll
    for (int e = 0; e < 4; e++) {
        a = chain_step<NEG>(a, q.a[e]);
        b = chain_step<NEG>(b, q.b[e]);
    }
}

__device__ __forceinline__ uint2 lds_u2(const char *lds, uint32_t a)
{
    return *reinterpret_cast<const uint2 *>(lds + a);
}

template <bool NEG>
__device__ __forceinline__ void walk_pair(float2 &acc_a, float2 &acc_b, uint32_t pa, uint32_t ea,
                                          uint32_t pb, uint32_t eb, uint32_t lanec, const char *lds)
{
    const uint32_t ca = full_dwords(ea), cb = full_dwords(eb);
    const uint32_t joint = ca < cb ? ca : cb;
    float2 a = acc_a, b = acc_b;
    uint32_t i = 0;
    if (kPipe) {
        const uint32_t nblk = joint >> 1;
        if (nblk) {
            uint2 wa = lds_u2(lds, pa), wb = lds_u2(lds, pb);
            Quad2 qa, qb;
            pair_reads(qa, wa.x, wb.x, lanec, lds);
            // branch-free body (a mid-loop exit gets tail-merged with the
            // adds, which then need lgkmcnt(0) and register copies)
            for (uint32_t blk = 1; blk < nblk; blk++) {
                const uint2 na = lds_u2(lds, pa + 8u * blk), nb = lds_u2(lds, pb + 8u * blk);
                __builtin_amdgcn_sched_barrier(0);
                pair_reads(qb, wa.y, wb.y, lanec, lds);
                __builtin_amdgcn_sched_barrier(0);
                pair_adds<NEG>(a, b, qa);
                __builtin_amdgcn_sched_barrier(0);
                pair_reads(qa, na.x, nb.x, lanec, lds);
                __builtin_amdgcn_sched_barrier(0);
                pair_adds<NEG>(a, b, qb);
                __builtin_amdgcn_sched_barrier(0);
                wa = na;
                wb = nb;
            }
            pair_reads(qb, wa.y, wb.y, lanec, lds);
            pair_adds<NEG>(a, b, qa);
            pair_adds<NEG>(a, b, qb);
            i = 2 * nblk;
        }
    } else if (joint >= 2) {
        uint2 wa = lds_u2(lds, pa);
        uint2 wb = lds_u2(lds, pb);
        for (; i + 2 <= joint; i += 2) {
            const uint2 na = lds_u2(lds, pa + 4 * (i + 2));
            const uint2 nb = lds_u2(lds, pb + 4 * (i + 2));
            Quad2 q0, q1;
            pair_reads(q0, wa.x, wb.x, lanec, lds);
            pair_reads(q1, wa.y, wb.y, lanec, lds);
            pair_adds<NEG>(a, b, q0);
            pair_adds<NEG>(a, b, q1);
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
// The wave's step is ONE dword stream: the column segments back to back, D
// dwords (a multiple of 4), per-column dword counts in the header.  The walk
// is a hand-scheduled software pipeline in inline asm (the compiler's
// scheduler and register allocator otherwise re-serialise it: see
// DESIGN.md, perf log):
//   * the 4 reads of dword d+3 are issued before the 4 adds of dword d, so
//     every wave keeps 12 LDS reads in flight through the whole step, across
//     column boundaries;
//   * index words come 4 at a time (ds_read_b128, broadcast) one batch ahead,
//     issued after the data reads they must not delay; every wait is one
//     counted lgkmcnt(13) (LDS returns in order);
//   * the chain being extended lives in v[50:51]; at a segment boundary
//     (a SALU counter carries out) it is written back to the accumulator
//     vector and the next column's accumulator fetched with
//     s_set_gpr_idx relative moves: the adds never branch.
// Every chain still adds its entries in stream order (BaseTCSC order).
// Fixed registers: v50-v95 (work, addresses, index batches, 4 data slots),
// the accumulators at the top of the VGPR file, counts in s[88:91].
template <int NW>
struct AccVec {
    typedef float type __attribute__((ext_vector_type(2 * NW)));
};
typedef uint32_t U32x4 __attribute__((ext_vector_type(4)));

#define TSG_S0_0 "v[64:65]"
#define TSG_S0_1 "v[66:67]"
#define TSG_S0_2 "v[68:69]"
#define TSG_S0_3 "v[70:71]"
#define TSG_S1_0 "v[72:73]"
#define TSG_S1_1 "v[74:75]"
#define TSG_S1_2 "v[76:77]"
#define TSG_S1_3 "v[78:79]"
#define TSG_S2_0 "v[80:81]"
#define TSG_S2_1 "v[82:83]"
#define TSG_S2_2 "v[84:85]"
#define TSG_S2_3 "v[86:87]"
#define TSG_S3_0 "v[88:89]"
#define TSG_S3_1 "v[90:91]"
#define TSG_S3_2 "v[92:93]"
#define TSG_S3_3 "v[94:95]"

// 4 entry addresses of index word I, 4 reads into data slot K
#define TSG_READS(I, K)                                                        \
    "v_perm_b32 v52, " I ", %[lanec], %[s0]\n"                                 \
    "v_perm_b32 v53, " I ", %[lanec], %[s1]\n"                                 \
    "v_perm_b32 v54, " I ", %[lanec], %[s2]\n"                                 \
    "v_perm_b32 v55, " I ", %[lanec], %[s3]\n"                                 \
    "ds_read_b64 " TSG_S##K##_0 ", v52\n"                                      \
    "ds_read_b64 " TSG_S##K##_1 ", v53\n"                                      \
    "ds_read_b64 " TSG_S##K##_2 ", v54\n"                                      \
    "ds_read_b64 " TSG_S##K##_3 ", v55\n"

// wait for slot K (13 younger LDS ops may stay in flight), 4 chained adds
#define TSG_ADDS(NEGM, K)                                                      \
    "s_waitcnt lgkmcnt(13)\n"                                                  \
    "v_pk_add_f32 v[50:51], v[50:51], " TSG_S##K##_0 NEGM "\n"                 \
    "v_pk_add_f32 v[50:51], v[50:51], " TSG_S##K##_1 NEGM "\n"                 \
    "v_pk_add_f32 v[50:51], v[50:51], " TSG_S##K##_2 NEGM "\n"                 \
    "v_pk_add_f32 v[50:51], v[50:51], " TSG_S##K##_3 NEGM "\n"

// one dword: reads of d+3 into slot RS, optional index batch, adds of d
// from slot AS, boundary check (branch to the out-of-line stub T)
#define TSG_STEP(T, I, RS, IDXOP, NEGM, AS)                                    \
    TSG_READS(I, RS) IDXOP TSG_ADDS(NEGM, AS)                                  \
    "s_add_u32 %[nrem], %[nrem], 1\n"                                          \
    "s_cbranch_scc1 .Lb" #T "_%=\n"                                            \
    ".Lr" #T "_%=:\n"

#define TSG_ADVANCE                                                            \
    "s_add_u32 %[cur], %[cur], 1\n"                                            \
    "s_lshr_b64 s[88:89], s[88:89], 8\n"                                       \
    "s_lshl_b32 %[t], s90, 24\n"                                               \
    "s_or_b32 s89, s89, %[t]\n"                                                \
    "s_lshr_b64 s[90:91], s[90:91], 8\n"                                       \
    "s_and_b32 %[t], s88, 0xff\n"

// segment boundary after step T: write the chain back (column `own`), find
// the next non-empty column, fetch its accumulator (s_set_gpr_idx relative
// moves).  Past the last column the counter is parked (never carries
// again) and `own` keeps the finished column, so the final write-back
// repeats the same value.
#define TSG_PUT(ACC0, ACC1)                                                    \
    "s_set_gpr_idx_on %[own], gpr_idx(DST)\n"                                  \
    "v_mov_b32 " ACC0 ", v50\n"                                                \
    "v_mov_b32 " ACC1 ", v51\n"                                                \
    "s_set_gpr_idx_off\n"
#define TSG_GET(ACC0, ACC1)                                                    \
    "s_lshl_b32 %[own], %[cur], 1\n"                                           \
    "s_set_gpr_idx_on %[own], gpr_idx(SRC0)\n"                                 \
    "v_mov_b32 v50, " ACC0 "\n"                                                \
    "v_mov_b32 v51, " ACC1 "\n"                                                \
    "s_set_gpr_idx_off\n"
#define TSG_STUB(T, ACC0, ACC1, NWM1)                                          \
    ".Lb" #T "_%=:\n"                                                          \
    TSG_PUT(ACC0, ACC1)                                                        \
    ".La" #T "_%=:\n"                                                          \
    "s_cmp_ge_u32 %[cur], " NWM1 "\n"                                          \
    "s_cbranch_scc1 .Lx" #T "_%=\n"                                            \
    TSG_ADVANCE                                                                \
    "s_cmp_eq_u32 %[t], 0\n"                                                   \
    "s_cbranch_scc1 .La" #T "_%=\n"                                            \
    "s_sub_u32 %[nrem], 0, %[t]\n"                                             \
    TSG_GET(ACC0, ACC1)                                                        \
    "s_branch .Lr" #T "_%=\n"                                                  \
    ".Lx" #T "_%=:\n"                                                          \
    "s_brev_b32 %[nrem], 1\n"                                                  \
    "s_branch .Lr" #T "_%=\n"

#define TSG_IDX_A "ds_read_b128 v[56:59], %[vidx] offset:32\n"
#define TSG_IDX_B "ds_read_b128 v[60:63], %[vidx] offset:48\n"

#define TSG_FLAT_ASM(NEGM, ACC0, ACC1, NWM1)                                   \
    "s_mov_b32 %[m0s], m0\n"                                                   \
    "s_mov_b32 %[cur], 0\n"                                                    \
    "s_and_b32 %[t], s88, 0xff\n"                                              \
    "s_cmp_eq_u32 %[t], 0\n"                                                   \
    "s_cbranch_scc0 .Li_%=\n"                                                  \
    ".Lia_%=:\n" TSG_ADVANCE                                                   \
    "s_cmp_eq_u32 %[t], 0\n"                                                   \
    "s_cbranch_scc1 .Lia_%=\n"                                                 \
    ".Li_%=:\n"                                                                \
    "s_sub_u32 %[nrem], 0, %[t]\n"                                             \
    TSG_GET(ACC0, ACC1)                                                        \
    "ds_read_b128 v[56:59], %[vidx]\n"                                         \
    "ds_read_b128 v[60:63], %[vidx] offset:16\n"                               \
    "s_waitcnt lgkmcnt(0)\n"                                                   \
    TSG_READS("v56", 0) TSG_READS("v57", 1)                    \
    TSG_READS("v58", 2)                                                \
    ".Lloop_%=:\n"                                                             \
    TSG_STEP(0, "v59", 3, TSG_IDX_A, NEGM, 0)                  \
    TSG_STEP(1, "v60", 0, "", NEGM, 1)                         \
    TSG_STEP(2, "v61", 1, "", NEGM, 2)                         \
    TSG_STEP(3, "v62", 2, "", NEGM, 3)                         \
    "s_cmp_le_i32 %[left], 4\n"                                                \
    "s_cbranch_scc1 .Lexit_%=\n"                                               \
    TSG_STEP(4, "v63", 3, TSG_IDX_B, NEGM, 0)                  \
    TSG_STEP(5, "v56", 0, "", NEGM, 1)                         \
    TSG_STEP(6, "v57", 1, "", NEGM, 2)                         \
    TSG_STEP(7, "v58", 2, "", NEGM, 3)                         \
    "v_add_u32 %[vidx], 32, %[vidx]\n"                                         \
    "s_sub_u32 %[left], %[left], 8\n"                                          \
    "s_cmp_gt_i32 %[left], 0\n"                                                \
    "s_cbranch_scc1 .Lloop_%=\n"                                               \
    ".Lexit_%=:\n"                                                             \
    "s_waitcnt lgkmcnt(0)\n"                                                   \
    TSG_PUT(ACC0, ACC1)                                                        \
    "s_branch .Lend_%=\n"                                                      \
    TSG_STUB(0, ACC0, ACC1, NWM1) TSG_STUB(1, ACC0, ACC1, NWM1)                \
    TSG_STUB(2, ACC0, ACC1, NWM1) TSG_STUB(3, ACC0, ACC1, NWM1)                \
    TSG_STUB(4, ACC0, ACC1, NWM1) TSG_STUB(5, ACC0, ACC1, NWM1)                \
    TSG_STUB(6, ACC0, ACC1, NWM1) TSG_STUB(7, ACC0, ACC1, NWM1)                \
    ".Lend_%=:\n"                                                               \
    "s_mov_b32 m0, %[m0s]\n"

#define TSG_NEG_MOD " neg_lo:[0,1] neg_hi:[0,1]"

#define TSG_FLAT_CLOBBERS                                                      \
    "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59",      \
    "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69",      \
    "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79",      \
    "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89",      \
    "v90", "v91", "v92", "v93", "v94", "v95", "scc", "memory"

#define TSG_FLAT_CALL(NEGM, ACCC, ACC0, ACC1, NWM1)                            \
    asm volatile(TSG_FLAT_ASM(NEGM, ACC0, ACC1, NWM1)                          \
                 : [acc] ACCC(acc), [cnt] "+{s[88:91]}"(cnt), [vidx] "+v"(vidx), \
                   [cur] "=&s"(cur), [nrem] "=&s"(nrem), [t] "=&s"(t), [own] "=&s"(own), [m0s] "=&s"(m0s), \
                   [left] "+s"(left)                                           \
                 : [lanec] "v"(lanec), [s0] "s"(0x0C020400u | (4u << 8)),      \
                   [s1] "s"(0x0C020400u | (5u << 8)), [s2] "s"(0x0C020400u | (6u << 8)), \
                   [s3] "s"(0x0C020400u | (7u << 8))                           \
                 : TSG_FLAT_CLOBBERS)

template <int NW, bool NEG>
__device__ __forceinline__ void walk_chunk_flat(typename AccVec<NW>::type &acc, const uint32_t (&hw)[8],
                                                uint32_t ib, uint32_t lanec)
{
    uint32_t left = hw[1];  // D, a multiple of 4
    if (left == 0) return;
    U32x4 cnt = {hw[2], hw[3], hw[4], hw[5]};
    uint32_t vidx = ib + 4u * kSFlatHdrWords;
    uint32_t cur, nrem, t, own, m0s;  // m0s: M0 (gpr_idx state) saved around
    if constexpr (NW == 16) {
        if constexpr (NEG) TSG_FLAT_CALL(TSG_NEG_MOD, "+{v[96:127]}", "v96", "v97", "15");
        else TSG_FLAT_CALL("", "+{v[96:127]}", "v96", "v97", "15");
    } else if constexpr (NW == 8) {
        if constexpr (NEG) TSG_FLAT_CALL(TSG_NEG_MOD, "+{v[112:127]}", "v112", "v113", "7");
        else TSG_FLAT_CALL("", "+{v[112:127]}", "v112", "v113", "7");
    } else {
        static_assert(NW == 4, "NW");
        if constexpr (NEG) TSG_FLAT_CALL(TSG_NEG_MOD, "+{v[120:127]}", "v120", "v121", "3");
        else TSG_FLAT_CALL("", "+{v[120:127]}", "v120", "v121", "3");
    }
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
            if (q < nch) walk_chunk_flat<NW, false>(accv, h8, ib, lanec);  // +1 runs
            else walk_chunk_flat<NW, true>(accv, h8, ib, lanec);           // -1 runs
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

// TSG_RX_DIAG_NOSYNC: diagnostic build only -- no chunk staging and no step
// barriers (results are WRONG; times the bare block walk).
#ifdef TSG_RX_DIAG_NOSYNC
constexpr bool kRxDiagNoSync = true;
#else
constexpr bool kRxDiagNoSync = false;
#endif

template <bool PRELU, bool STAMP>
__global__ __launch_bounds__(kRxWaves * 64, 8 / kRxWaves) void tsg_tcsc_rx_kernel(
    const float *__restrict__ XT, int Mp, const uint32_t *__restrict__ wstart,
    const uint32_t *__restrict__ ent, const float *__restrict__ b, const float *__restrict__ alpha,
    float *__restrict__ Y, int M, int N, int nch, int mtiles, int ntiles,
    unsigned long long *__restrict__ stamps)
{
    unsigned long long st_work = 0, st_wait = 0, st_t0 = 0;
    if (STAMP) st_t0 = __builtin_amdgcn_s_memtime();
    __shared__ __attribute__((aligned(16))) char lds[kRxLdsBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    // LDS is only touched from asm (LDS-DMA, ds_read_b128 at absolute offsets
    // from 0): a never-taken C++ store keeps the allocation in the kernel
    if (M < 0) lds[tid] = 0;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // XCD-aware bijective remap, as in the stream kernel
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
        if (!kRxDiagNoSync && q + 1 < steps) rx_stage(XT, Mp, m0, (q + 1) % nch, (q + 1) & 1, wave, lane);
        const unsigned long long ta = STAMP ? __builtin_amdgcn_s_memtime() : 0;
        rx_walk<false>(a0, a1, a2, a3, ent, off, hdr, (uint32_t)(q & 1) * (uint32_t)kRxChunkBytes + (uint32_t)lane * 16u);
        const unsigned long long tb = STAMP ? __builtin_amdgcn_s_memtime() : 0;
        if (!kRxDiagNoSync) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (STAMP) {
            const unsigned long long tc = __builtin_amdgcn_s_memtime();
            st_work += tb - ta;
            st_wait += tc - tb;
        }
    }
    for (int q = nch; q < steps; q++) {  // -1 runs, ascending K
        if (!kRxDiagNoSync && q + 1 < steps) rx_stage(XT, Mp, m0, (q + 1) % nch, (q + 1) & 1, wave, lane);
        const unsigned long long ta = STAMP ? __builtin_amdgcn_s_memtime() : 0;
        rx_walk<true>(a0, a1, a2, a3, ent, off, hdr, (uint32_t)(q & 1) * (uint32_t)kRxChunkBytes + (uint32_t)lane * 16u);
        const unsigned long long tb = STAMP ? __builtin_amdgcn_s_memtime() : 0;
        if (!kRxDiagNoSync) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (STAMP) {
            const unsigned long long tc = __builtin_amdgcn_s_memtime();
            st_work += tb - ta;
            st_wait += tc - tb;
        }
    }
    if (STAMP && lane == 0) {
        unsigned long long *o = stamps + ((size_t)blockIdx.x * kRxWaves + wave) * 4;
        o[0] = st_work;
        o[1] = st_wait;
        o[2] = __builtin_amdgcn_s_memtime() - st_t0;
        o[3] = (unsigned long long)((nt << 16) | mt);
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
        if (ncol0 + kRxNW <= N && ((((size_t)m * N + ncol0) & 3) == 0)) {
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

int launch_tcsc_rx(const float *XT, int Mp, const uint32_t *wstart, const uint32_t *ent,
                   const float *b, const float *alpha, float *Y, int M, int N, int Npad, int nch,
                   int prelu, unsigned long long *stamps, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    const int mtiles = Mp / kRxTileM, ntiles = Npad / kRxTileCols;
    const dim3 grid((unsigned)(mtiles * ntiles)), block(kRxWaves * kLanes);
    if (stamps)
        hipLaunchKernelGGL((tsg_tcsc_rx_kernel<false, true>), grid, block, 0, s, XT, Mp, wstart, ent, b,
                           alpha, Y, M, N, nch, mtiles, ntiles, stamps);
    else if (prelu)
        hipLaunchKernelGGL((tsg_tcsc_rx_kernel<true, false>), grid, block, 0, s, XT, Mp, wstart, ent, b,
                           alpha, Y, M, N, nch, mtiles, ntiles, nullptr);
    else
        hipLaunchKernelGGL((tsg_tcsc_rx_kernel<false, false>), grid, block, 0, s, XT, Mp, wstart, ent, b,
                           alpha, Y, M, N, nch, mtiles, ntiles, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tsg
