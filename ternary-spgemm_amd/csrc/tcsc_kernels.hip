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

}  // namespace tsg
