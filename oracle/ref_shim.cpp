// ref_shim.cpp -- extern "C" shim over the reference's OWN headers, compiled
// unmodified from /root/reference (never copied): cpp_impl/data_structures/TCSC.h,
// cpp_impl/data_structures/BlockedTCSC.h and cpp_impl/sparseUtils.h.
//
// TEST INFRASTRUCTURE ONLY: built into oracle/_ref/libref.so by oracle/Makefile
// when /root/reference is present; used by tests/golden/make_golden.py to
// generate golden vectors and by tests/test_oracle.py to pin the restatement.
// comp.h (BaseTCSC) is NOT built: it includes <arm_neon.h> unconditionally
// (comp.h:6) and the x86 image has no such header.
#include <cstdint>
#include <cstring>
#include <vector>

#include "data_structures/TCSC.h"
#include "data_structures/BlockedTCSC.h"
#include "sparseUtils.h"

template <int B>
static void blocked(const int32_t *W, int K, int N, int64_t *np, int64_t *nn, int32_t *csp,
                    int32_t *csn, int32_t *rip, int32_t *rin)
{
    BlockedTCSC<B> t(const_cast<int *>(W), K, N);
    *np = (int64_t)t.row_index_pos.size();
    *nn = (int64_t)t.row_index_neg.size();
    if (csp) std::memcpy(csp, t.col_start_pos.data(), sizeof(int) * t.col_start_pos.size());
    if (csn) std::memcpy(csn, t.col_start_neg.data(), sizeof(int) * t.col_start_neg.size());
    if (rip) std::memcpy(rip, t.row_index_pos.data(), sizeof(int) * t.row_index_pos.size());
    if (rin) std::memcpy(rin, t.row_index_neg.data(), sizeof(int) * t.row_index_neg.size());
}

extern "C" {

// generateSparseMatrix<int>(K, N, s, false, seed) (sparseUtils.h:25-90).
void ref_generate_sparse(int K, int N, int s, int seed, int32_t *W)
{
    std::vector<int> w = generateSparseMatrix<int>(K, N, s, false, seed);
    std::memcpy(W, w.data(), sizeof(int) * (size_t)K * N);
}

// class TCSC ctor (TCSC.h:13-41).  Returns nnz_pos / nnz_neg; arrays copied
// out when the destination pointers are non-null (call twice: size, then fill).
void ref_tcsc_encode(const int32_t *W, int K, int N, int64_t *nnz_pos, int64_t *nnz_neg,
                     int32_t *csp, int32_t *csn, int32_t *rip, int32_t *rin, int64_t *ds_bytes)
{
    TCSC t(W, K, N);
    *nnz_pos = (int64_t)t.row_index_pos.size();
    *nnz_neg = (int64_t)t.row_index_neg.size();
    *ds_bytes = (int64_t)t.getDataStructureSize();
    if (csp) std::memcpy(csp, t.col_start_pos.data(), sizeof(int) * t.col_start_pos.size());
    if (csn) std::memcpy(csn, t.col_start_neg.data(), sizeof(int) * t.col_start_neg.size());
    if (rip) std::memcpy(rip, t.row_index_pos.data(), sizeof(int) * t.row_index_pos.size());
    if (rin) std::memcpy(rin, t.row_index_neg.data(), sizeof(int) * t.row_index_neg.size());
}

// BlockedTCSC<B> ctor (BlockedTCSC.h:15-41) for the block sizes the tests use.
int ref_blocked_tcsc_encode(const int32_t *W, int K, int N, int B, int64_t *np, int64_t *nn,
                            int32_t *csp, int32_t *csn, int32_t *rip, int32_t *rin)
{
    switch (B) {
    case 2: blocked<2>(W, K, N, np, nn, csp, csn, rip, rin); return 0;
    case 4: blocked<4>(W, K, N, np, nn, csp, csn, rip, rin); return 0;
    case 64: blocked<64>(W, K, N, np, nn, csp, csn, rip, rin); return 0;
    case 512: blocked<512>(W, K, N, np, nn, csp, csn, rip, rin); return 0;
    default: return -1;
    }
}

// GEMM<float> (sparseUtils.h:92-108) -- the reference's correctness oracle.
void ref_gemm(float *X, float *W, float *b, float *Y, int M, int N, int K)
{
    GEMM<float>(X, W, b, Y, M, N, K);
}

// GEMM_PreLU<float> (sparseUtils.h:110-137).
void ref_gemm_prelu(float *X, float *W, float *b, float *alpha, float *Y, int M, int N, int K)
{
    GEMM_PreLU<float>(X, W, b, alpha, Y, M, N, K);
}

// compare_results<float> (sparseUtils.h:139-156): 1 = pass (abs tol 10e-6).
int ref_compare_results(float *result, float *truth, int H, int W)
{
    return compare_results<float>(result, truth, H, W) ? 1 : 0;
}

} // extern "C"
