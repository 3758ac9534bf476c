// tsg_ell.hip -- the small-M TCSC kernel (tsg_tcsc_ell_kernel): an
// index-reading walk for GEMV-like calls (M up to a few dozen rows), where the
// weight-compiled kernel has too few M tiles to fill the GPU and would stream
// a code image 2.5x the size of the TCSC.
//
// Format ("sliced ELL", built from the TCSC arrays by tsg::build_ell_image,
// tsg_host.cpp, for one M tile size MT): columns in slices of 16; K in chunks
// of C rows; for every (slice, step) with step = pass * nch + chunk (pass 0:
// the +1 entries, pass 1: the -1 entries -- BaseTCSC's order, comp.h:37-63)
// each column's entries of that chunk and pass, ascending k, as the uint16
// float index (k - chunk * C) * MT of the row in the LDS chunk, padded to the
// slice's longest list (rounded up to 8) with C * MT: the LDS row C is all +0.0f,
// and y +- 0 == y bit for bit because the chain never holds -0 (it starts at
// +0 and RN gives -0 only from (-0) + (-0)).  Storage: per (slice, step) n8
// blocks of 256 B = [16 columns][8 entries]; a lane loads its column's 8
// entries with one 16-byte load (the 16 lanes of a slice read 256 contiguous
// bytes).  tab[slice * steps + step] = {offset in 256-B units, n8}.
//
// Kernel (template LG lanes per column, RPL M rows per lane, WPG waves per
// workgroup): a wave owns 64 / LG columns, the LG consecutive lanes of a
// column its MT = LG * RPL rows (so the lanes of a column read one contiguous
// LDS run per entry, and small M still gives N * LG / 64 waves); a workgroup
// owns an M tile and WPG * 64 / LG columns (WPG = 16 when that still gives
// >= 256 workgroups, else 4: the chunk staging is shared by more columns).  Per step it stages
// X^T[chunk][MT] (+ the zero row) in LDS straight from the row-major X (no
// transpose kernel), then every lane walks its column's list -- index blocks
// prefetched kEllDepth deep, the blocks of a group unrolled straight-line so
// the LDS reads of later blocks overlap the adds of earlier ones (one chain
// per (row, column): the walk is latency-bound otherwise) -- per entry one LDS
// read of its RPL rows and RPL adds (subtractions in the -1 pass), so each
// Y[m,n] is ONE serial fp32 chain 0 + x_p1 + ... - x_n1 - ... in the
// reference's order, then + b[n] (comp.h:63) and the PReLU epilogue
// (comp_prelu.h:57-67).  Roofline: HBM (the entry stream, read once per M
// tile) at M = 1, LDS gathers above (DESIGN.md 4 "Small M").
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tsg_internal.h"

namespace tsg {

// Index blocks (8 entries each) in flight per lane.  The walk is bound by the
// memory-level parallelism of the entry stream (Little's law: ~30 KiB in
// flight per CU for ~5 TB/s at ~1.5 us latency), not by its bandwidth.
// 32 blocks with at most 4 waves per workgroup and one row per lane (a wave
// may use 256 VGPRs), fewer where the registers run out (no scratch spills:
// checked with -Rpass-analysis=kernel-resource-usage).
template <int WPG, int RPL>
constexpr int ell_depth() { return WPG >= 16 ? (RPL >= 2 ? 4 : 8) : (RPL >= 2 ? 12 : 32); }

// One 16-byte index block = 8 entries: their X values (RPL rows each) from LDS.
template <int RPL>
__device__ __forceinline__ void ell_load(float (&x)[8][RPL], const uint4 e, const float *xb)
{
    const uint32_t w[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
    for (int h = 0; h < 8; h++) {
        const float *xp = xb + ((w[h >> 1] >> (16 * (h & 1))) & 0xffffu);
        if constexpr (RPL % 4 == 0) {
#pragma unroll
            for (int q = 0; q < RPL; q += 4) {
                const float4 v = *reinterpret_cast<const float4 *>(xp + q);
                x[h][q] = v.x; x[h][q + 1] = v.y; x[h][q + 2] = v.z; x[h][q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < RPL; q++) x[h][q] = xp[q];
        }
    }
}

// ... and their adds, in entry order (comp.h:44-61)
template <int RPL, bool NEG>
__device__ __forceinline__ void ell_add(float (&y)[RPL], const float (&x)[8][RPL])
{
#pragma unroll
    for (int h = 0; h < 8; h++)
#pragma unroll
        for (int r = 0; r < RPL; r++) y[r] = NEG ? y[r] - x[h][r] : y[r] + x[h][r];
}

// Entry h of a block: the LDS read of the NEXT block's entry h interleaved with
// the add of this block's entry h -- a lane's adds form one dependent chain,
// so the independent address/read work fills the VALU latency between them.
template <int RPL, bool NEG>
__device__ __forceinline__ void ell_add_load(float (&y)[RPL], const float (&x)[8][RPL], float (&xn)[8][RPL],
                                             const uint4 en, const float *xb)
{
    const uint32_t w[4] = {en.x, en.y, en.z, en.w};
#pragma unroll
    for (int h = 0; h < 8; h++) {
        const float *xp = xb + ((w[h >> 1] >> (16 * (h & 1))) & 0xffffu);
        if constexpr (RPL % 4 == 0) {
#pragma unroll
            for (int q = 0; q < RPL; q += 4) {
                const float4 v = *reinterpret_cast<const float4 *>(xp + q);
                xn[h][q] = v.x; xn[h][q + 1] = v.y; xn[h][q + 2] = v.z; xn[h][q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < RPL; q++) xn[h][q] = xp[q];
        }
#pragma unroll
        for (int r = 0; r < RPL; r++) y[r] = NEG ? y[r] - x[h][r] : y[r] + x[h][r];
    }
}

template <int RPL, bool NEG, int kEllDepth>
__device__ __forceinline__ void ell_walk(float (&y)[RPL], const uint4 *__restrict__ p, uint32_t n8, const float *xb)
{
    if (n8 == 0) return;
    // Every prefetch load is unconditional (the block index clamped to the
    // last block): branches between them would make the compiler wait with
    // vmcnt(0) instead of counting the loads still in flight.
    const uint32_t last = n8 - 1;
    uint4 q[kEllDepth];
#pragma unroll
    for (int d = 0; d < kEllDepth; d++) q[d] = p[(size_t)min((uint32_t)d, last) * 16];
    uint32_t i = 0;
    // whole groups of kEllDepth blocks, straight-line: the LDS reads of block
    // d + 1 are issued before the adds of block d (a lane's adds are one
    // dependent chain, so the read latency would otherwise be exposed per
    // block), and slot d is refilled kEllDepth blocks ahead after its use
    for (; i + kEllDepth <= n8; i += kEllDepth) {
        float x0[8][RPL], x1[8][RPL];
        ell_load<RPL>(x0, q[0], xb);
#pragma unroll
        for (int d = 0; d < kEllDepth; d++) {
            if (d + 1 == kEllDepth) ell_add<RPL, NEG>(y, d % 2 == 0 ? x0 : x1);
            else if (d % 2 == 0) ell_add_load<RPL, NEG>(y, x0, x1, q[d + 1], xb);
            else ell_add_load<RPL, NEG>(y, x1, x0, q[d + 1], xb);
            q[d] = p[(size_t)min(i + kEllDepth + d, last) * 16];  // prefetch
        }
    }
#pragma unroll
    for (int d = 0; d < kEllDepth; d++)  // the rest (< kEllDepth blocks, already loaded)
        if (i + d < n8) {
            float x[8][RPL];
            ell_load<RPL>(x, q[d], xb);
            ell_add<RPL, NEG>(y, x);
        }
}

template <int LG, int RPL, int WPG, bool PRELU>
__global__ __launch_bounds__(WPG * 64) void tsg_tcsc_ell_kernel(
    const float *__restrict__ X, const uint4 *__restrict__ ent, const uint2 *__restrict__ tab,
    const float *__restrict__ b, const float *__restrict__ alpha, float *__restrict__ Y, int M, int N, int K,
    int C, int nch, int nsg)
{
    constexpr int MT = LG * RPL;                     // M rows of the tile
    constexpr int CPW = 64 / LG;                     // columns per wave
    extern __shared__ __attribute__((aligned(16))) float xs[];  // [(C + 1)][MT]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cw = lane / LG, g = lane % LG;         // the lane's column in the wave, its row group
    const int sg = blockIdx.x % nsg, mt = blockIdx.x / nsg;
    const int n = (sg * WPG + wave) * CPW + cw;      // the lane's column
    const int slice = n >> 4, c = n & 15;
    const int m0 = mt * MT;
    const int steps = 2 * nch;
    const int nslices = (N + 15) / 16;
    const bool vec = K >= 4 && (K & 3) == 0 && ((((uintptr_t)X) & 15) == 0);  // X[0..3] exists

    float y[RPL];
#pragma unroll
    for (int r = 0; r < RPL; r++) y[r] = 0.0f;  // comp.h:41

    // the zero row (padding entries point at it)
    for (int i = tid; i < MT; i += WPG * 64) xs[C * MT + i] = 0.0f;

    for (int step = 0; step < steps; step++) {
        const int j = step % nch, kc = j * C;
        if (step == 0 || nch > 1) {
            __syncthreads();  // previous chunk's reads are done
            // stage X^T[chunk j] -- a thread loads 4 consecutive k of one row m
            // (16 B when aligned) and writes them to 4 LDS rows; consecutive
            // threads take consecutive m, so the LDS writes hit consecutive
            // banks.  8 loads are issued before their LDS writes (a loop of
            // load-then-store would wait out one memory latency per float4).
            const int per = C / 4 * MT;
            for (int i0 = tid; i0 < per; i0 += 8 * WPG * 64) {
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int i = i0 + u * WPG * 64;
                    const int mm = i % MT, r4 = (i / MT) * 4, m = m0 + mm, k = kc + r4;
                    v[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    if (vec) {
                        // unconditional load from a clamped in-range address, then masked
                        const bool in = i < per && m < M && k + 3 < K;
                        const size_t at = in ? (size_t)m * K + k : 0;
                        const float4 q = *reinterpret_cast<const float4 *>(X + at);
                        if (in) v[u] = q;
                    } else if (i < per && m < M) {
                        const float *xr = X + (size_t)m * K + k;
                        if (k < K) v[u].x = xr[0];
                        if (k + 1 < K) v[u].y = xr[1];
                        if (k + 2 < K) v[u].z = xr[2];
                        if (k + 3 < K) v[u].w = xr[3];
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int i = i0 + u * WPG * 64;
                    if (i >= per) break;
                    const int mm = i % MT, r4 = (i / MT) * 4;
                    xs[(r4 + 0) * MT + mm] = v[u].x;
                    xs[(r4 + 1) * MT + mm] = v[u].y;
                    xs[(r4 + 2) * MT + mm] = v[u].z;
                    xs[(r4 + 3) * MT + mm] = v[u].w;
                }
            }
            __syncthreads();
        }
        if (slice >= nslices) continue;
        const uint2 t = tab[(size_t)slice * steps + step];
        const uint4 *p = ent + (size_t)t.x * 16 + c;
        const float *xb = xs + g * RPL;
        if (step < nch) ell_walk<RPL, false, ell_depth<WPG, RPL>()>(y, p, t.y, xb);   // +1 entries
        else ell_walk<RPL, true, ell_depth<WPG, RPL>()>(y, p, t.y, xb);               // -1 entries
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

namespace {

template <int LG, int RPL, int WPG>
int launch_ell_t(const float *X, const uint4 *ent, const uint2 *tab, const float *b, const float *alpha, float *Y,
                 int M, int N, int K, int C, int nch, int prelu, hipStream_t s)
{
    constexpr int MT = LG * RPL, CPW = 64 / LG;
    const int nsg = (N + WPG * CPW - 1) / (WPG * CPW);
    const int mtiles = (M + MT - 1) / MT;
    const size_t lds = (size_t)(C + 1) * MT * sizeof(float);
    const dim3 grid((unsigned)(nsg * mtiles)), block(WPG * 64);
    if (prelu)
        hipLaunchKernelGGL((tsg_tcsc_ell_kernel<LG, RPL, WPG, true>), grid, block, lds, s, X, ent, tab, b, alpha, Y,
                           M, N, K, C, nch, nsg);
    else
        hipLaunchKernelGGL((tsg_tcsc_ell_kernel<LG, RPL, WPG, false>), grid, block, lds, s, X, ent, tab, b, alpha, Y,
                           M, N, K, C, nch, nsg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

int launch_tcsc_ell(int variant, const float *X, const uint32_t *ent, const uint32_t *tab, const float *b,
                    const float *alpha, float *Y, int M, int N, int K, int C, int nch, int prelu, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    const uint4 *e = reinterpret_cast<const uint4 *>(ent);
    const uint2 *t = reinterpret_cast<const uint2 *>(tab);
    // 16-wave workgroups (one chunk staging shared by 16x the columns) when the
    // grid still has >= 256 of them, else 4 waves
    auto big = [&](int lg, int mt) {
        const int cols = 16 * 64 / lg;
        return (int64_t)((N + cols - 1) / cols) * ((M + mt - 1) / mt) >= 256;
    };
    switch (variant) {
    case 0: return launch_ell_t<1, 1, 1>(X, e, t, b, alpha, Y, M, N, K, C, nch, prelu, s);  // MT = 1
    case 1:                                                                                   // MT = 4
        return big(4, 4) ? launch_ell_t<4, 1, 16>(X, e, t, b, alpha, Y, M, N, K, C, nch, prelu, s)
                         : launch_ell_t<4, 1, 4>(X, e, t, b, alpha, Y, M, N, K, C, nch, prelu, s);
    case 2:                                                                                   // MT = 16
        return big(16, 16) ? launch_ell_t<16, 1, 16>(X, e, t, b, alpha, Y, M, N, K, C, nch, prelu, s)
                           : launch_ell_t<16, 1, 4>(X, e, t, b, alpha, Y, M, N, K, C, nch, prelu, s);
    case 3:                                                                                   // MT = 32
        return big(16, 32) ? launch_ell_t<16, 2, 16>(X, e, t, b, alpha, Y, M, N, K, C, nch, prelu, s)
                           : launch_ell_t<16, 2, 4>(X, e, t, b, alpha, Y, M, N, K, C, nch, prelu, s);
    default: return -2;
    }
}

}  // namespace tsg
