// tsg_encode.hip -- GPU-side TCSC encoder: dense row-major K x N ternary W
// (device memory) -> col_start_pos / col_start_neg / row_index_pos /
// row_index_neg (device memory), exactly the TCSC constructor
// (data_structures/TCSC.h:13-41): column by column, the rows holding +1 (and,
// separately, -1) in ascending k; col_start[n] = entries of the columns < n;
// any value other than +1 / -1 is a zero.
//
// Three passes, all HBM-bound (the dense W of config 5 is
// 2 GiB, seconds on the host):
//   1. count: one thread per column walks k (consecutive threads read
//      consecutive columns of a row: coalesced), counts +1 and -1;
//   2. exclusive scan of the counts (hipCUB) -> col_start, total in [N];
//   3. fill: the same walk writes the row indices at col_start[n].
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>

#include "tsg_internal.h"

namespace tsg {

namespace {

__global__ __launch_bounds__(256) void tsg_encode_count_kernel(const int32_t *__restrict__ W, int K, int N,
                                                                int32_t *__restrict__ cnt_pos,
                                                                int32_t *__restrict__ cnt_neg)
{
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    int p = 0, q = 0;
    for (int k = 0; k < K; k++) {
        const int32_t v = W[(size_t)k * N + n];
        p += v == 1;
        q += v == -1;
    }
    cnt_pos[n] = p;
    cnt_neg[n] = q;
}

__global__ __launch_bounds__(256) void tsg_encode_fill_kernel(const int32_t *__restrict__ W, int K, int N,
                                                               const int32_t *__restrict__ csp,
                                                               const int32_t *__restrict__ csn,
                                                               int32_t *__restrict__ rip, int32_t *__restrict__ rin)
{
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    int32_t p = csp[n], q = csn[n];
    for (int k = 0; k < K; k++) {
        const int32_t v = W[(size_t)k * N + n];
        if (v == 1) rip[p++] = k;
        else if (v == -1) rin[q++] = k;
    }
}

}  // namespace

int encode_count(const int32_t *dW, int K, int N, int32_t *d_csp, int32_t *d_csn, void *d_tmp, size_t *tmp_bytes,
                 void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    // scan workspace query
    size_t need = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, need, d_csp, d_csp, N + 1, s) != hipSuccess) return -1;
    if (!d_tmp) {
        *tmp_bytes = need;
        return 0;
    }
    if (*tmp_bytes < need) return -2;
    // counts into [0, N), 0 at [N]; the exclusive scan makes col_start with the total at [N]
    if (N > 0)
        hipLaunchKernelGGL(tsg_encode_count_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, dW, K, N,
                           d_csp, d_csn);
    if (hipMemsetAsync(d_csp + N, 0, sizeof(int32_t), s) != hipSuccess ||
        hipMemsetAsync(d_csn + N, 0, sizeof(int32_t), s) != hipSuccess)
        return -1;
    size_t t = *tmp_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(d_tmp, t, d_csp, d_csp, N + 1, s) != hipSuccess) return -1;
    t = *tmp_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(d_tmp, t, d_csn, d_csn, N + 1, s) != hipSuccess) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int encode_fill(const int32_t *dW, int K, int N, const int32_t *d_csp, const int32_t *d_csn, int32_t *d_rip,
                int32_t *d_rin, void *stream)
{
    if (N > 0)
        hipLaunchKernelGGL(tsg_encode_fill_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, dW, K, N, d_csp, d_csn, d_rip, d_rin);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tsg
