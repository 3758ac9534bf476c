// tsg_ell.hip -- the small-M TCSC kernel (tsg_tcsc_ell_kernel): an
// index-reading walk for GEMV-like calls (M up to a few dozen rows), where the
// weight-compiled kernel has too few M tiles to fill the GPU and would stream
// a code image 2.5x the size of the TCSC.
//
// Format ("sliced ELL", built from the TCSC arrays by tsg::build_ell_image,
// tsg_host.cpp, for one M tile size MT): columns in slices of 16; K in chunks
// of C rows.  Per (slice, step) each column's entries in ascending k as the
// uint16 float index (k - chunk * C) * MT of its row in the LDS chunk, padded
// to the slice's longest list (rounded up to 8) with C * MT: the LDS row C is
// all +0.0f, and y +- 0 == y bit for bit because the chain never holds -0 (it
// starts at +0 and RN gives -0 only from (-0) + (-0)).  When K fits one chunk
// a step holds the +1 blocks and then the -1 blocks of the slice (ONE stream
// per column); else there is a step per (pass, chunk) -- BaseTCSC's order,
// comp.h:37-63, either way.  Storage: 256-B blocks = [16 columns][8 entries];
// a lane loads its column's 8 entries with one 16-byte load (the 16 lanes of a
// slice read 256 contiguous bytes).  tab[slice * steps + step] = {offset in
// blocks, n8 | n8pos << 16}: blocks below n8pos add, the rest subtract.  Block
// 0 of the image is all padding: a lane past its list's end reads it.
//
// Kernel (template LG lanes per column, RPL M rows per lane, WPG waves per
// workgroup): a wave owns 64 / LG columns, the LG consecutive lanes of a
// column its MT = LG * RPL rows (so the lanes of a column read one contiguous
// LDS run per entry, and small M still gives N * LG / 64 waves); a workgroup
// owns an M tile and WPG * 64 / LG columns.  Per step: the step's index blocks
// are requested first (kDepth deep), then X^T[chunk][MT] is staged in LDS
// straight from the row-major X (no transpose kernel) while they are in
// flight; then every lane walks its column's stream -- blocks of a group
// straight-line, the LDS reads of block d + 1 issued before the adds of block
// d, each block refilled kDepth ahead -- one LDS read of its RPL rows per
// entry (v_mad_u32_u16 forms the address from either half of an index word)
// and per row y = fma(x, +-1, y), which IS y + x / y - x bit for bit (x * -1 is
// exact, one rounding).  So each Y[m,n] is ONE serial fp32 chain
// 0 + x_p1 + ... - x_n1 - ... in the reference's order, then + b[n]
// (comp.h:63) and the PReLU epilogue (comp_prelu.h:57-67).  The walk is
// bound by the per-wave issue of that chain (DESIGN.md 4 "Small M").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "tsg_internal.h"

namespace tsg {

namespace {

typedef __attribute__((address_space(3))) const float lds_f;
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const v2f lds_f2;
typedef __attribute__((address_space(3))) const v4f lds_f4;

// LDS byte address of an entry: its uint16 float index (the low or the high
// half of a word) * 4 + the lane's row base, in one VALU op
__device__ __forceinline__ uint32_t ent_addr_lo(uint32_t w, uint32_t base)
{
    uint32_t r;
    asm("v_mad_u32_u16 %0, %1, 4, %2" : "=v"(r) : "v"(w), "v"(base));
    return r;
}
__device__ __forceinline__ uint32_t ent_addr_hi(uint32_t w, uint32_t base)
{
    uint32_t r;
    asm("v_mad_u32_u16 %0, %1, 4, %2 op_sel:[1,0,0,0]" : "=v"(r) : "v"(w), "v"(base));
    return r;
}

// Index blocks (8 entries each) in flight per lane: deep enough to cover the
// HBM latency of the entry stream at one wave per SIMD, within the VGPRs the
// workgroup size leaves (256 up to 4 waves, 128 at 16) without spilling
// (checked with -Rpass-analysis=kernel-resource-usage).
template <int WPG, int RPL>
constexpr int ell_depth() { return WPG >= 16 ? (RPL >= 2 ? 4 : 8) : (RPL >= 4 ? 8 : 32); }

// One 16-byte index block = 8 entries: their X values (RPL rows each) from LDS.
template <int RPL>
__device__ __forceinline__ void ell_load(float (&x)[8][RPL], const uint4 e, uint32_t base)
{
    const uint32_t w[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
    for (int h = 0; h < 8; h++) {
        const uint32_t a = (h & 1) ? ent_addr_hi(w[h >> 1], base) : ent_addr_lo(w[h >> 1], base);
        if constexpr (RPL % 4 == 0) {
#pragma unroll
            for (int q = 0; q < RPL; q += 4) {
                const v4f v = *(lds_f4 *)(uintptr_t)(a + 4 * q);
                x[h][q] = v.x; x[h][q + 1] = v.y; x[h][q + 2] = v.z; x[h][q + 3] = v.w;
            }
        } else if constexpr (RPL == 2) {
            const v2f v = *(lds_f2 *)(uintptr_t)a;
            x[h][0] = v.x; x[h][1] = v.y;
        } else {
#pragma unroll
            for (int q = 0; q < RPL; q++) x[h][q] = *(lds_f *)(uintptr_t)(a + 4 * q);
        }
    }
}

// ... and their adds in entry order (comp.h:44-61): sg = +1 / -1
template <int RPL>
__device__ __forceinline__ void ell_add(float (&y)[RPL], const float (&x)[8][RPL], float sg)
{
#pragma unroll
    for (int h = 0; h < 8; h++)
#pragma unroll
        for (int r = 0; r < RPL; r++) y[r] = __builtin_fmaf(x[h][r], sg, y[r]);
}

// The walk of one step's stream: blocks [0, n8) of the lane's column (e0 +
// (off + i) * 16), blocks past n8 read as block 0 (padding), bound by the
// wave's longest list nmax (uniform).  q holds blocks 0..D-1 on entry.  Whole
// groups of D blocks refill their slots D blocks ahead and have no exit
// branch; the last nmax % D blocks are then already in q and run with an
// early exit and no loads (a load ahead of an exit branch would be sunk past
// it by the compiler, exposing one memory latency per group).
// LA: LDS lookahead in blocks -- the reads of block d + LA go out before the
// adds of block d (LA + 1 register sets of 8 x RPL values).
template <int RPL, int D, int LA>
__device__ __forceinline__ void ell_walk(float (&y)[RPL], uint4 (&q)[D], const uint4 *__restrict__ e0, uint32_t off,
                                         uint32_t n8, uint32_t n8pos, uint32_t nmax, uint32_t base)
{
    static_assert(LA >= 1 && LA < D, "lookahead");
    constexpr int NS = LA + 1;  // register sets
    uint32_t g = 0;
    for (; g + D <= nmax; g += D) {
        float x[NS][8][RPL];
#pragma unroll
        for (int a = 0; a < LA; a++) ell_load<RPL>(x[a], q[a], base);
#pragma unroll
        for (int d = 0; d < D; d++) {
            if (d + LA < D) ell_load<RPL>(x[(d + LA) % NS], q[d + LA], base);
            // the reads of block d + LA stay ahead of the adds of block d
            __builtin_amdgcn_sched_barrier(0);
            ell_add<RPL>(y, x[d % NS], g + d < n8pos ? 1.0f : -1.0f);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t nb = g + D + d;  // refill: D blocks ahead, padding past the end
            q[d] = e0[nb < n8 ? (off + nb) * 16 : 0];
        }
    }
    const uint32_t rest = nmax - g;  // < D, uniform
    if (rest == 0) return;
    float x[NS][8][RPL];
#pragma unroll
    for (int a = 0; a < LA; a++) ell_load<RPL>(x[a], q[a], base);
#pragma unroll
    for (int d = 0; d < D; d++) {
        if (d + LA < D) ell_load<RPL>(x[(d + LA) % NS], q[d + LA], base);
        __builtin_amdgcn_sched_barrier(0);
        ell_add<RPL>(y, x[d % NS], g + d < n8pos ? 1.0f : -1.0f);
        __builtin_amdgcn_sched_barrier(0);
        if ((uint32_t)d + 1 >= rest) return;
    }
}

// the largest of n over the lanes of the wave (lanes of one slice agree)
template <int LG>
__device__ __forceinline__ uint32_t wave_max(uint32_t n)
{
    if constexpr (16 * LG < 64) {
#pragma unroll
        for (int o = 16 * LG; o < 64; o *= 2) n = max(n, (uint32_t)__shfl_xor((int)n, o));
    }
    return __builtin_amdgcn_readfirstlane(n);
}

// Stage X^T[chunk at kc][MT rows from m0] into xs ([C][MT], row-major by k)
// with NT threads: a thread loads 4 consecutive k of one row m (16 B when
// aligned) and writes them to 4 LDS rows; consecutive threads take
// consecutive m, so the LDS writes hit consecutive banks.  SB unconditional
// loads from clamped in-range addresses go out before their masked stores
// (no branch between them, so no wait per load).  Rows past M and k past K
// are +0.
template <int MT, int NT, int SB>
__device__ __forceinline__ void ell_stage(float *xs, const float *__restrict__ X, int M, int K, int m0, int kc, int C,
                                          int tid, bool vec, int xb)
{
    const int per = C / 4 * MT;
    if (vec) {
        for (int i0 = tid; i0 < per; i0 += SB * NT) {
            float4 v[SB];
#pragma unroll
            for (int u = 0; u < SB; u++) {
                const int i = i0 + u * NT;
                const int mm = i % MT, r4 = (i / MT) * 4, m = m0 + mm, k = kc + r4;
                const bool in = i < per && m < M && k + 3 < K;
                v[u] = *reinterpret_cast<const float4 *>(X + (in ? (size_t)m * K + k : 0));
            }
#pragma unroll
            for (int u = 0; u < SB; u++) {
                const int i = i0 + u * NT;
                const int mm = i % MT, r4 = (i / MT) * 4, m = m0 + mm, k = kc + r4;
                const bool in = i < per && m < M && k + 3 < K;
                const float4 w = in ? v[u] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (i < per) {
                    xs[(r4 + 0) * MT + mm] = w.x;
                    xs[(r4 + 1) * MT + mm] = w.y;
                    xs[(r4 + 2) * MT + mm] = w.z;
                    xs[(r4 + 3) * MT + mm] = w.w;
                    if (xb) {  // the second copy (tsg_host.cpp build_ell_image)
                        xs[xb + (r4 + 0) * MT + mm] = w.x;
                        xs[xb + (r4 + 1) * MT + mm] = w.y;
                        xs[xb + (r4 + 2) * MT + mm] = w.z;
                        xs[xb + (r4 + 3) * MT + mm] = w.w;
                    }
                }
            }
        }
    } else {
        for (int i = tid; i < per; i += NT) {
            const int mm = i % MT, r4 = (i / MT) * 4, m = m0 + mm, k = kc + r4;
            float4 w = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (m < M) {
                const float *xr = X + (size_t)m * K + k;
                if (k < K) w.x = xr[0];
                if (k + 1 < K) w.y = xr[1];
                if (k + 2 < K) w.z = xr[2];
                if (k + 3 < K) w.w = xr[3];
            }
            xs[(r4 + 0) * MT + mm] = w.x;
            xs[(r4 + 1) * MT + mm] = w.y;
            xs[(r4 + 2) * MT + mm] = w.z;
            xs[(r4 + 3) * MT + mm] = w.w;
            if (xb) {
                xs[xb + (r4 + 0) * MT + mm] = w.x;
                xs[xb + (r4 + 1) * MT + mm] = w.y;
                xs[xb + (r4 + 2) * MT + mm] = w.z;
                xs[xb + (r4 + 3) * MT + mm] = w.w;
            }
        }
    }
}

}  // namespace

template <int LG, int RPL, int WPG, int LA, bool PRELU>
__global__ __launch_bounds__(WPG * 64) void tsg_tcsc_ell_kernel(
    const float *__restrict__ X, const uint4 *__restrict__ ent, const uint2 *__restrict__ tab,
    const float *__restrict__ b, const float *__restrict__ alpha, float *__restrict__ Y, int M, int N, int K,
    int C, int nch, int steps, int nsg, int xb, int zr)
{
    constexpr int MT = LG * RPL;                     // M rows of the tile
    constexpr int CPW = 64 / LG;                     // columns per wave
    constexpr int D = ell_depth<WPG, RPL>();
    constexpr int SB = WPG >= 8 ? 8 : 16;           // staging loads in flight per thread
    extern __shared__ __attribute__((aligned(16))) float xs[];  // [(C + 1)][MT]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cw = lane / LG, g = lane % LG;         // the lane's column in the wave, its row group
    const int sg = blockIdx.x % nsg, mt = blockIdx.x / nsg;
    const int n = (sg * WPG + wave) * CPW + cw;      // the lane's column
    const int slice = n >> 4, c = n & 15;
    const int m0 = mt * MT;
    const int nslices = (N + 15) / 16;
    const bool vec = K >= 4 && (K & 3) == 0 && ((((uintptr_t)X) & 15) == 0);  // X[0..3] exists
    const uint4 *e0 = ent + c;                       // the lane's column in block 0
    const uint32_t base = (uint32_t)(uintptr_t)(lds_f *)xs + (uint32_t)(g * RPL * 4);

    float y[RPL];
#pragma unroll
    for (int r = 0; r < RPL; r++) y[r] = 0.0f;  // comp.h:41

    // the zero row (padding entries point at it); and the second copy's
    for (int i = tid; i < zr * MT; i += WPG * 64) {
        xs[C * MT + i] = 0.0f;
        if (xb && i < MT) xs[xb + C * MT + i] = 0.0f;
    }

    for (int step = 0; step < steps; step++) {
        // the step's entry stream first: its blocks travel while X is staged
        uint32_t off = 0, n8 = 0, n8pos = 0;
        if (slice < nslices) {
            const uint2 t = tab[(size_t)slice * steps + step];
            off = t.x;
            n8 = t.y & 0xffffu;
            n8pos = t.y >> 16;
        }
        if constexpr (CPW == 16) {
            // the wave is one slice: its stream offset, list length and sign
            // split are uniform -- in SGPRs the refill addresses and the
            // block signs need no per-lane compare / select
            off = __builtin_amdgcn_readfirstlane(off);
            n8 = __builtin_amdgcn_readfirstlane(n8);
            n8pos = __builtin_amdgcn_readfirstlane(n8pos);
        }
        uint4 q[D];
#pragma unroll
        for (int d = 0; d < D; d++) q[d] = e0[(uint32_t)d < n8 ? (off + d) * 16 : 0];
        const uint32_t nmax = wave_max<LG>(n8);

        const int j = steps == 1 ? 0 : step % nch, kc = j * C;
        if (step == 0 || steps > 1) {
            __syncthreads();  // previous chunk's reads are done
            ell_stage<MT, WPG * 64, SB>(xs, X, M, K, m0, kc, C, tid, vec, xb);
            __syncthreads();
        }
        ell_walk<RPL, D, LA>(y, q, e0, off, n8, n8pos, nmax, base);
    }
    if (slice >= nslices || n >= N) return;
    const float bn = b[n];
    const float an = PRELU ? alpha[n] : 0.0f;
#pragma unroll
    for (int r = 0; r < RPL; r++) {
        const int m = m0 + g * RPL + r;
        if (m >= M) break;
        float v = y[r] + bn;                         // comp.h:63
        if (PRELU) v = (v > 0) ? v : an * v;         // comp_prelu.h:57-67
        Y[(size_t)m * N + n] = v;
    }
}


// ---------------------------------------------------------------------------
// tsg_tcsc_ell_pc_kernel: the same image and order for very few chains (M = 1,
// K in one LDS chunk), where each Y[m,n] chain's latency, not throughput,
// bounds the walk (~26 cycles per entry for a wave that also gathers; a lone
// dependent fma chain fed by ds_read_b128 runs at ~7, profiles/r02q_ell_micro.txt).  A workgroup owns 64 columns x MT rows = 64 MT chains and
// splits the work: MT consumer waves (a lane = a chain) do nothing but the
// chain -- y = fma(x, +-1, y), x read 4 at a time with ds_read_b128 one phase
// ahead -- while MT * E / 8 producer waves (a lane = one chain's index block
// of a phase) gather the next phases' X values (v_mad_u32_u16 address, one LDS
// read per entry) into a 3-slot LDS ring laid out in chain order.  A phase =
// E entries of every chain; one LDS-only barrier per phase (index-block loads
// stay in flight across it).  Slot ph % 3 holds phase ph: producers fill phase
// k + 2 while the consumers add phase k and read phase k + 1.
namespace {

__device__ __forceinline__ void lds_barrier()
{
    // nothing moves across it: the scheduler would otherwise hoist later
    // phases' address math (and with it the waits for their index blocks)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    __builtin_amdgcn_sched_barrier(0);
}

template <int MT, int E>
struct PcShape {
    static constexpr int CH = 64 * MT;  // chains: 64 columns x MT rows (chain = column * MT + row)
    static constexpr int CW = MT;       // consumer waves
    static constexpr int NB = E / 8;    // index blocks per column per phase
    static constexpr int PW = NB;       // producer waves (a lane = a column's block: all MT rows)
    static constexpr int NT = 64 * (CW + PW);
    static constexpr int D = 16;        // phases of index blocks in flight per producer lane
};

}  // namespace

template <int MT, int E, bool PRELU>
__global__ __launch_bounds__(64 * (MT + E / 8)) void tsg_tcsc_ell_pc_kernel(
    const float *__restrict__ X, const uint4 *__restrict__ ent, const uint2 *__restrict__ tab,
    const float *__restrict__ b, const float *__restrict__ alpha, float *__restrict__ Y, int M, int N, int K,
    int C, int nsg)
{
    using S = PcShape<MT, E>;
    static_assert(S::NT == 64 * (MT + E / 8), "launch bounds");
    constexpr int CH = S::CH, CW = S::CW, NB = S::NB, D = S::D;
    extern __shared__ __attribute__((aligned(16))) float xs[];  // [(C + 1)][MT], then float4 ring[3][E / 4][CH]
    float4 *ring = reinterpret_cast<float4 *>(xs + ((C + 1) * MT + 3) / 4 * 4);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sg = blockIdx.x % nsg, mt = blockIdx.x / nsg;
    const int m0 = mt * MT;
    const int nslices = (N + 15) / 16;
    const bool consumer = wave < CW;
    const int pj = consumer ? 0 : wave - CW;          // a producer's block within the phase
    const int ch = consumer ? wave * 64 + lane : 0;   // a consumer lane's chain
    const int n = sg * 64 + (consumer ? ch / MT : lane), r = consumer ? ch % MT : 0;  // its column (and row)
    const int slice = n >> 4;
    uint32_t off = 0, n8 = 0, n8pos = 0;
    if (slice < nslices) {
        const uint2 t = tab[slice];
        off = t.x;
        n8 = t.y & 0xffffu;
        n8pos = t.y >> 16;
    }
    // phases: the longest list of the workgroup's 4 slices, in blocks of NB
    uint32_t nmax = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int sl = sg * 4 + i;
        if (sl < nslices) nmax = max(nmax, tab[sl].y & 0xffffu);
    }
    const int nph = (int)((nmax + NB - 1) / NB);
    const uint4 *e0 = ent + (n & 15);

    // a producer's index blocks first (they travel while X is staged)
    uint4 q[D];
    auto load = [&](int ph) {
        const uint32_t bl = (uint32_t)(ph * NB + pj);
        return e0[bl < n8 ? (off + bl) * 16 : 0];
    };
    if (!consumer) {
#pragma unroll
        for (int d = 0; d < D; d++) q[d] = load(d);
    }
    for (int i = tid; i < MT; i += S::NT) xs[C * MT + i] = 0.0f;  // the zero row
    const bool vec = K >= 4 && (K & 3) == 0 && ((((uintptr_t)X) & 15) == 0);
    ell_stage<MT, S::NT, 8>(xs, X, M, K, m0, 0, C, tid, vec, 0);
    lds_barrier();

    if (consumer) {
        __builtin_amdgcn_s_setprio(3);  // the chain is the critical path
        float y = 0.0f;                 // comp.h:41
        float4 va[E / 4], vb[E / 4];
        auto read = [&](float4(&v)[E / 4], int ph) {
            const float4 *src = ring + (size_t)(ph % 3) * (E / 4) * CH + ch;
#pragma unroll
            for (int q4 = 0; q4 < E / 4; q4++) v[q4] = src[q4 * CH];
        };
        auto chain = [&](const float4(&v)[E / 4], int ph) {
#pragma unroll
            for (int q4 = 0; q4 < E / 4; q4++) {
                const float sg1 = (uint32_t)(ph * NB + q4 / 2) < n8pos ? 1.0f : -1.0f;  // +1 / -1 block
                y = __builtin_fmaf(v[q4].x, sg1, y);
                y = __builtin_fmaf(v[q4].y, sg1, y);
                y = __builtin_fmaf(v[q4].z, sg1, y);
                y = __builtin_fmaf(v[q4].w, sg1, y);
            }
        };
        lds_barrier();  // phases 0 and 1 are in the ring
        read(va, 0);
        for (int k = 0; k < nph; k += 2) {
            read(vb, k + 1);
            chain(va, k);
            lds_barrier();
            if (k + 1 >= nph) break;
            read(va, k + 2);
            chain(vb, k + 1);
            lds_barrier();
        }
        if (n >= N || m0 + r >= M) return;
        float v = y + b[n];                          // comp.h:63
        if (PRELU) v = (v > 0) ? v : alpha[n] * v;   // comp_prelu.h:57-67
        Y[(size_t)(m0 + r) * N + n] = v;
    } else {
        const uint32_t base = (uint32_t)(uintptr_t)(lds_f *)xs;
        // A block's 8 entries, all MT rows each (one LDS read per entry), are
        // gathered into registers one interval before they are written to the
        // ring as 4-entry runs of each of the column's MT chains: in interval
        // k a producer writes phase k + 2 (gathered in interval k - 1), waits
        // for those writes only, then issues the gathers of phase k + 3 and
        // meets the barrier without waiting for them, so the gathers' latency
        // and the LDS burst they cause overlap the barrier and the next
        // interval instead of lengthening this one.
        auto gather = [&](const uint4 e, float (&x)[8][MT]) {
            const uint32_t w[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
            for (int h = 0; h < 8; h++) {
                const uint32_t a = (h & 1) ? ent_addr_hi(w[h >> 1], base) : ent_addr_lo(w[h >> 1], base);
                if constexpr (MT == 4) {
                    const v4f v = *(lds_f4 *)(uintptr_t)a;
                    x[h][0] = v.x; x[h][1] = v.y; x[h][2] = v.z; x[h][3] = v.w;
                } else {
                    x[h][0] = *(lds_f *)(uintptr_t)a;
                }
            }
        };
        auto put = [&](int ph, const float (&x)[8][MT]) {
            float4 *dst = ring + ((size_t)(ph % 3) * (E / 4) + 2 * pj) * CH + lane * MT;
#pragma unroll
            for (int rr = 0; rr < MT; rr++) {
                dst[rr] = make_float4(x[0][rr], x[1][rr], x[2][rr], x[3][rr]);
                dst[CH + rr] = make_float4(x[4][rr], x[5][rr], x[6][rr], x[7][rr]);
            }
        };
        // after a put: its ring writes complete (s_waitcnt lgkmcnt(0) with
        // vmcnt/expcnt not waited: the index loads stay in flight); the
        // gathers issued after it read only the X chunk, so the interval's
        // barrier does not wait for them
        auto writes_done = [&]() {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_sched_barrier(0);
        };
        auto end_interval = [&]() {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
        };
        float xa[8][MT], xb[8][MT];
        gather(q[0], xa);
        put(0, xa);
        q[0] = load(D);
        gather(q[1], xb);
        put(1, xb);
        q[1] = load(D + 1);
        gather(q[2], xa);  // phase 2, written in interval 0
        q[2] = load(D + 2);
        lds_barrier();     // phases 0 and 1 are in the ring (full wait: the gathers of phase 2 included)
        // interval k: put phase k + 2 (in x[k % 2]), gather phase k + 3 into
        // x[(k + 1) % 2]; whole groups of D refill their index slots (no exit
        // branch between a load and its use), the rest runs without loads
        int k = 0;
        for (; k + D <= nph; k += D) {
#pragma unroll
            for (int d = 0; d < D; d++) {
                if (d % 2 == 0) {
                    put(k + d + 2, xa);
                    writes_done();
                    gather(q[(d + 3) % D], xb);
                } else {
                    put(k + d + 2, xb);
                    writes_done();
                    gather(q[(d + 3) % D], xa);
                }
                q[(d + 3) % D] = load(k + d + 3 + D);
                end_interval();
            }
        }
#pragma unroll
        for (int d = 0; d < D; d++) {
            if (k + d >= nph) break;
            if (d % 2 == 0) {
                put(k + d + 2, xa);
                writes_done();
                gather(q[(d + 3) % D], xb);
            } else {
                put(k + d + 2, xb);
                writes_done();
                gather(q[(d + 3) % D], xa);
            }
            end_interval();
        }
    }
}

namespace {

template <int LG, int RPL, int WPG, int LA>
int launch_ell_la(const float *X, const uint4 *ent, const uint2 *tab, const float *b, const float *alpha, float *Y,
                  int M, int N, int K, int C, int nch, int xb, int zr, int prelu, hipStream_t s)
{
    constexpr int MT = LG * RPL, CPW = 64 / LG;
    const int nsg = (N + WPG * CPW - 1) / (WPG * CPW);
    const int mtiles = (M + MT - 1) / MT;
    const int steps = nch == 1 ? 1 : 2 * nch;
    const size_t lds = ell_lds_floats(C, MT, xb, zr) * sizeof(float);
    const dim3 grid((unsigned)(nsg * mtiles)), block(WPG * 64);
    if (prelu)
        hipLaunchKernelGGL((tsg_tcsc_ell_kernel<LG, RPL, WPG, LA, true>), grid, block, lds, s, X, ent, tab, b, alpha,
                           Y, M, N, K, C, nch, steps, nsg, xb, zr);
    else
        hipLaunchKernelGGL((tsg_tcsc_ell_kernel<LG, RPL, WPG, LA, false>), grid, block, lds, s, X, ent, tab, b, alpha,
                           Y, M, N, K, C, nch, steps, nsg, xb, zr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// LDS lookahead of the walk (ell_walk): LA_DEFAULT, or TSG_ELL_LA=1/2 (A/B)
int pick_la()
{
    static const int env = [] {
        const char *v = knob_value("TSG_ELL_LA");
        const int x = v ? atoi(v) : 0;
        return x == 1 || x == 2 ? x : 0;
    }();
    return env ? env : 1;
}

template <int LG, int RPL, int WPG>
int launch_ell_t(const float *X, const uint4 *ent, const uint2 *tab, const float *b, const float *alpha, float *Y,
                 int M, int N, int K, int C, int nch, int xb, int zr, int prelu, hipStream_t s)
{
    if (pick_la() == 2)
        return launch_ell_la<LG, RPL, WPG, 2>(X, ent, tab, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
    return launch_ell_la<LG, RPL, WPG, 1>(X, ent, tab, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
}

}  // namespace

namespace {

// Waves per workgroup: 16 or 8 when the grid is then one round that still
// gives (nearly) every CU a workgroup (kEllWideWgs ... 256 x the workgroups
// per CU the LDS chunk allows; (24, 4096, 16384) at 8 waves would take two
// rounds: 60.8 vs 52.5 us at 16) -- a workgroup stages its X chunk once for
// all its columns, so fewer, wider workgroups stage less (round 5,
// profiles/r05t_ell_wpg_ab.jsonl, kernel us: (32, 2048, 8192) 21.2 vs 29.0 at
// 4 waves; (16, 2048, 16384) 21.1 vs 29.7; (32, 2048, 16384) 31.2 vs 38.2 at
// 4, 37.9 at 8), else the fewest (4, 8, 16) that keep every wave resident in
// one round, given the workgroups per CU the LDS chunk allows ((16, 1024,
// 4096) 11.7 at 4 vs 13.6 at 8); 8 and 16 only while a lane holds at most 2
// rows (more spill at 8 and 16 waves).  TSG_ELL_WPG=4/8/16 forces one (A/B).
constexpr int64_t kEllWideWgs = 224;  // 7/8 of the CUs

template <int LG, int RPL>
int launch_lg(const float *X, const uint4 *e, const uint2 *t, const float *b, const float *alpha, float *Y, int M,
              int N, int K, int C, int nch, int xb, int zr, int prelu, hipStream_t s)
{
    constexpr int MT = LG * RPL, CPW = 64 / LG;
    const int64_t waves = (int64_t)((N + CPW - 1) / CPW) * ((M + MT - 1) / MT);
    const int64_t per_cu = std::max<int64_t>(1, 163840 / ((int64_t)ell_lds_floats(C, MT, xb, zr) * 4));
    static const int env_wpg = [] {  // TSG_ELL_WPG=4/8/16: waves per workgroup (A/B)
        const char *v = knob_value("TSG_ELL_WPG");
        return v ? atoi(v) : 0;
    }();
    if (env_wpg == 4) return launch_ell_t<LG, RPL, 4>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
    if constexpr (RPL <= 2) {
        if (env_wpg == 8) return launch_ell_t<LG, RPL, 8>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
        if (env_wpg == 16) return launch_ell_t<LG, RPL, 16>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
    }
    if constexpr (RPL <= 2) {
        auto one_round = [&](int64_t wpg) {  // >= 7/8 of the CUs busy, no second round
            const int64_t wgs = (waves + wpg - 1) / wpg;
            return wgs >= kEllWideWgs && wgs <= 256 * per_cu;
        };
        if (one_round(16)) return launch_ell_t<LG, RPL, 16>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
        if (one_round(8)) return launch_ell_t<LG, RPL, 8>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
        if (waves > 256 * per_cu * 8)
            return launch_ell_t<LG, RPL, 16>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
        if (waves > 256 * per_cu * 4)
            return launch_ell_t<LG, RPL, 8>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
    }
    return launch_ell_t<LG, RPL, 4>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);
}

// lanes per column of an M tile: the default, or TSG_ELL_LG (diagnostic sweeps)
int pick_lg(int dflt)
{
    static const int env = [] {
        const char *v = knob_value("TSG_ELL_LG");
        return v ? atoi(v) : 0;
    }();
    return env > 0 ? env : dflt;
}

template <int MT, int E>
constexpr size_t pc_lds(int C)
{
    return ((size_t)((C + 1) * MT + 3) / 4 * 4) * sizeof(float) + (size_t)3 * (E / 4) * PcShape<MT, E>::CH * 16;
}

template <int MT, int E>
int launch_pc_t(const float *X, const uint4 *ent, const uint2 *tab, const float *b, const float *alpha, float *Y,
                int M, int N, int K, int C, int prelu, hipStream_t s)
{
    using S = PcShape<MT, E>;
    const int nsg = (N + 63) / 64;
    const int mtiles = (M + MT - 1) / MT;
    const size_t lds = pc_lds<MT, E>(C);
    const dim3 grid((unsigned)(nsg * mtiles)), block(S::NT);
    if (prelu)
        hipLaunchKernelGGL((tsg_tcsc_ell_pc_kernel<MT, E, true>), grid, block, lds, s, X, ent, tab, b, alpha, Y, M, N,
                           K, C, nsg);
    else
        hipLaunchKernelGGL((tsg_tcsc_ell_pc_kernel<MT, E, false>), grid, block, lds, s, X, ent, tab, b, alpha, Y, M, N,
                           K, C, nsg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

namespace {

// Phase length E (entries of every chain per barrier).  64 while every
// workgroup is resident at once (M * ceil(N / 64) <= 256: one per CU), the
// chains are long (K >= 2048; at K = 512-1024 the 9-wave workgroup costs more
// than it saves: (1, 512, 2048) 6.5 vs 7.1 us, profiles/r02_ref_cases_final.jsonl)
// and its larger ring fits beside the X chunk: half the barriers, and the wider
// producer set keeps more gathers in flight (M = 1: K = N = 16384 37.7 vs
// 42.2 us, K = N = 4096 13.5 vs 14.2 us); else 32 (M = 2 at N = 16384, 512
// workgroups: 20.0 vs 26.4 us with E = 64; profiles/r02_pc_phase_ab.txt).
// TSG_ELL_PC_E=16/32/64 forces one (A/B sweeps; 32 when the forced ring does
// not fit).  Availability (tsg_capi.cpp ell_pc_available) is judged at E = 32.
int pc_phase(int M, int N, int C)
{
    static const int env = [] {
        const char *v = knob_value("TSG_ELL_PC_E");
        const int x = v ? atoi(v) : 0;
        return x == 16 || x == 32 || x == 64 ? x : 0;
    }();
    const bool fits64 = pc_lds<1, 64>(C) <= kLdsBytes, fits16 = pc_lds<1, 16>(C) <= kLdsBytes;
    if (env == 64) return fits64 ? 64 : 32;
    if (env) return env == 16 && fits16 ? 16 : 32;
    const int64_t wgs = (int64_t)M * ((N + 63) / 64);
    return wgs <= 256 && C >= 2048 && fits64 ? 64 : 32;
}

}  // namespace

// 1-row tiles only: with 4 rows the ring's extra write and read of every row
// value make the walk LDS-bound (39 vs 22.5 us at M = 4, K = 4096, N = 16384;
// profiles/r02x_ell_pc.txt)
size_t ell_pc_lds_bytes(int variant, int C)
{
    return variant == 0 ? pc_lds<1, 32>(C) : 0;
}

int launch_tcsc_ell_pc(int variant, const float *X, const uint32_t *ent, const uint32_t *tab, const float *b,
                       const float *alpha, float *Y, int M, int N, int K, int C, int nch, int prelu, void *stream)
{
    // one stream per column, X chunk + ring within a workgroup's LDS
    if (nch != 1 || ell_pc_lds_bytes(variant, C) == 0 || ell_pc_lds_bytes(variant, C) > kLdsBytes) return -2;
    hipStream_t s = (hipStream_t)stream;
    const uint4 *e = reinterpret_cast<const uint4 *>(ent);
    const uint2 *t = reinterpret_cast<const uint2 *>(tab);
    switch (pc_phase(M, N, C)) {
    case 16: return launch_pc_t<1, 16>(X, e, t, b, alpha, Y, M, N, K, C, prelu, s);
    case 64: return launch_pc_t<1, 64>(X, e, t, b, alpha, Y, M, N, K, C, prelu, s);
    default: return launch_pc_t<1, 32>(X, e, t, b, alpha, Y, M, N, K, C, prelu, s);  // 1 consumer + 4 producer waves
    }
}

int launch_tcsc_ell(int variant, const float *X, const uint32_t *ent, const uint32_t *tab, const float *b,
                    const float *alpha, float *Y, int M, int N, int K, int C, int nch, int xb, int zr, int prelu,
                    void *stream)
{
    // the second X^T copy and the bank-window schedule serve the 8-row tile's
    // 4-lane columns only (tsg_host.cpp build_ell_image)
    if ((xb || zr != 1) && (variant != 2 || pick_lg(4) != 4)) return -2;
    hipStream_t s = (hipStream_t)stream;
    const uint4 *e = reinterpret_cast<const uint4 *>(ent);
    const uint2 *t = reinterpret_cast<const uint2 *>(tab);
#define TSG_ELL_LG(lg, rpl) \
    case lg: return launch_lg<lg, rpl>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s)
    switch (variant) {
    case 0: return launch_ell_t<1, 1, 1>(X, e, t, b, alpha, Y, M, N, K, C, nch, xb, zr, prelu, s);  // MT = 1
    case 1:                                                                                   // MT = 4
        switch (pick_lg(4)) {
            TSG_ELL_LG(4, 1);
            TSG_ELL_LG(2, 2);
        default: return -2;
        }
    case 2:                                                                                   // MT = 8
        switch (pick_lg(4)) {
            TSG_ELL_LG(8, 1);
            TSG_ELL_LG(4, 2);
            TSG_ELL_LG(2, 4);
        default: return -2;
        }
    case 3:                                                                                   // MT = 16
        switch (pick_lg(8)) {
            TSG_ELL_LG(8, 2);
            TSG_ELL_LG(16, 1);
        default: return -2;
        }
    case 4:                                                                                   // MT = 32
        switch (pick_lg(16)) {
            TSG_ELL_LG(16, 2);
        default: return -2;
        }
    default: return -2;
    }
#undef TSG_ELL_LG
}

}  // namespace tsg
