/*
 * ternary_spgemm.h -- C-ABI of the MI355X-native ternary TCSC spGEMM.
 *
 *     Y[m,n] = ( sum_{k in P(n)} X[m,k]  -  sum_{k in N(n)} X[m,k] ) + b[n]
 *
 * with W in {-1,0,+1}^{K x N} given in the reference's TCSC layout
 * (col_start_pos/neg: N+1 ints; row_index_pos/neg: ascending k per column).
 * Results are bit-identical to the reference CPU kernel BaseTCSC<float>
 * (cpp_impl/comp.h:25-69): every output is ONE serial fp32 chain
 * 0 + x_p1 + ... + x_pP - x_n1 - ... - x_nQ, then + b[n].
 *
 * This header is the drop-in surface (registration, the comp_func calls,
 * introspection, host helpers).  Tuning and test hooks of the same library
 * (stream widths, kernel and image choices, the generated code for CPU
 * emulation) are declared in ternary_spgemm_test.h.
 *
 * Plain pointers and sizes only; no torch or HIP types.  Every function
 * returns TSG_OK (0) or a TSG_ERR_* code; tcsc_hip_last_error() gives text.
 * Reference interfaces each entry point replaces are cited as
 * path:line relative to alessiomelone/Ternary-spGEMM.
 */
#ifndef TERNARY_SPGEMM_H
#define TERNARY_SPGEMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSG_ABI_VERSION 1

enum tsg_status {
    TSG_OK = 0,
    TSG_ERR_ARG = 1,     /* bad argument: null pointer, shape mismatch, malformed TCSC */
    TSG_ERR_HIP = 2,     /* HIP runtime / launch failure */
    TSG_ERR_NOMEM = 3,   /* device or host allocation failed */
    TSG_ERR_NODEV = 4,   /* no usable gfx950 device */
    TSG_ERR_RANGE = 5    /* size exceeds a supported limit */
};

/* Opaque handle: one TCSC weight matrix resident on one device (the device
 * image built from the TCSC arrays at registration, plus a work buffer). */
typedef struct tsg_tcsc tsg_tcsc;

/* ---- registration ---------------------------------------------------------
 * Replaces `std::make_shared<TCSC>(W_raw, K, N)` + capture in the
 * add_function lambda (cpp_impl/main.cpp:63,76-81; TCSC.h:13-41): the format
 * is built/uploaded ONCE, before any call.  Arrays are copied; the caller
 * keeps ownership.  device < 0 selects the current HIP device.
 * On failure *out is NULL and the status says why. */
int tcsc_hip_create(const int32_t *col_start_pos, const int32_t *col_start_neg,
                    const int32_t *row_index_pos, const int32_t *row_index_neg,
                    int K, int N, int device, tsg_tcsc **out);

/* Same, from a dense row-major K x N ternary matrix (TCSC ctor semantics,
 * TCSC.h:13-41; any value other than +1/-1 is treated as 0, as there). */
int tcsc_hip_create_dense(const int32_t *W, int K, int N, int device, tsg_tcsc **out);

/* GPU-side TCSC encoder (the TCSC ctor, TCSC.h:13-41, on the device): dW is a
 * dense row-major K x N int32 ternary matrix in device memory; d_csp / d_csn
 * (int32[N+1], caller-allocated device arrays) receive the column starts and
 * *nnz_pos / *nnz_neg the entry counts (the call synchronises `stream` to
 * return them).  When d_rip and d_rin are non-NULL (device arrays of at least
 * rip_cap >= nnz_pos and rin_cap >= nnz_neg int32s) the row indices are filled
 * too; call first with NULLs to size them.  Same arrays as tcsc_hip_create_dense
 * builds on the host, bit for bit. */
int tcsc_hip_encode_dense_dev(const int32_t *dW, int K, int N, int32_t *d_csp, int32_t *d_csn,
                              int32_t *d_rip, int64_t rip_cap, int32_t *d_rin, int64_t rin_cap,
                              int64_t *nnz_pos, int64_t *nnz_neg, void *stream);

/* Same, from "CSC with compressed values vector (1s and -1s, 8 bits for 5
 * values)" (readme.md:111, the reference's optimisation idea 2): col_ptr
 * int32[N+1], row_idx int32[nnz] (ascending k per column), values base-3
 * packed 5 per byte in CSC order, digit = v + 1.  Results are the same
 * BaseTCSC chains (+1 entries, then -1 entries, each ascending). */
int tcsc_hip_create_csc_packed(const int32_t *col_ptr, const int32_t *row_idx,
                               const uint8_t *packed, int K, int N, int device, tsg_tcsc **out);

/* BlockedTCSC<B> registration (data_structures/BlockedTCSC.h:5-49; the
 * reference's main.cpp:69 builds it with B = BLOCK_SIZE = 512): col_start_pos /
 * col_start_neg have (K/B)*N + 1 entries, slot kb*N + n listing column n's
 * +1 / -1 rows of block kb ([kb*B, kb*B + B), ascending); rows past (K/B)*B
 * are not part of the format.  Calls through the handle then compute
 * BaseBlockedTCSC<float> (comp.h:607-658): per block y = 0 + pos - neg, Y += y
 * block by block, then + b -- bit for bit, in that order.  Runs on the
 * weight-compiled kernel only (TSG_KERNEL must be unset or "jit"). */
int tcsc_hip_create_blocked(const int32_t *col_start_pos, const int32_t *col_start_neg,
                            const int32_t *row_index_pos, const int32_t *row_index_neg,
                            int K, int N, int B, int device, tsg_tcsc **out);

/* Releases every device/host resource of the handle (NULL is a no-op). */
void tcsc_hip_destroy(tsg_tcsc *h);

/* ---- compute --------------------------------------------------------------
 * Replaces one call of the registered comp_func
 *   using comp_func = std::function<void(float*X, float*B, float*Y, int M, int N, int K)>
 * (cpp_impl/common.h:12) bound to BaseTCSC<float> (comp.h:25-69).
 * Argument order M, N, K as there.  HOST pointers: X is M x K row-major,
 * b has N floats, Y is M x N row-major and is fully overwritten.
 * Synchronous: Y is valid on return (main.cpp:214-216, perf.cpp:62-66).
 * Host threads sharing a handle run their host-pointer calls one at a time
 * (the handle's staging buffers and streams).
 * A large call is pipelined by M chunks (tcsc_hip_host_chunk_rows): X chunk
 * i+1 travels in while chunk i computes and chunk i-1's Y travels out, on
 * three streams of the handle plus one helper thread for the Y copies; the
 * result is the unchunked one bit for bit (rows are independent). */
int tcsc_hip_gemm(tsg_tcsc *h, const float *X, const float *b, float *Y, int M, int N, int K);

/* Optional page-locking of a host buffer the caller passes to repeated
 * host-pointer calls (e.g. the X and Y of a benchmark loop, perf.cpp:37-71):
 * the call's copies then DMA directly instead of through the runtime's
 * pin-on-the-fly staging.  The buffer must stay allocated until
 * tcsc_hip_host_unregister.  Unregistered (pageable) buffers keep working.
 * Extension: no reference counterpart. */
int tcsc_hip_host_register(void *p, size_t bytes);
int tcsc_hip_host_unregister(void *p);

/* DEVICE pointers (on the handle's device), enqueued on `stream`
 * (a hipStream_t; NULL = legacy default stream); returns without waiting.
 * Streams: calls on one handle are serialised on the host (a mutex) and share
 * the handle's X^T work buffer; a call on a different stream than the
 * previous call waits (hipStreamWaitEvent) for the previous call's kernel
 * before it overwrites that buffer, so calls from several streams / threads
 * on one handle are safe (and run one after the other on the device).
 * The first call whose M picks a code image or work-buffer size the handle
 * has not prepared yet compiles / allocates it and synchronises `stream`
 * (the image's probe launch); tcsc_hip_reserve(h, max_M) is the place to do
 * that ahead of time.
 * Graph capture: after tcsc_hip_reserve(h, max_M), calls with M <= max_M
 * allocate, compile and synchronise nothing and can be captured; a captured
 * call reuses the work buffer when replayed, so a replay must not overlap
 * other calls on the same handle issued on other streams (a capture does not
 * change what uncaptured calls on other streams wait for). */
int tcsc_hip_gemm_dev(tsg_tcsc *h, const float *dX, const float *db, float *dY,
                      int M, int N, int K, void *stream);

/* PReLU twin: comp_func_prelu (common.h:13) bound to BaseTCSC_PreLU<float>
 * (comp_prelu.h:12-70): y = chain + b[n]; Y = y > 0 ? y : alpha[n]*y. */
int tcsc_hip_gemm_prelu(tsg_tcsc *h, const float *X, const float *b, const float *alpha,
                        float *Y, int M, int N, int K);
int tcsc_hip_gemm_prelu_dev(tsg_tcsc *h, const float *dX, const float *db, const float *dalpha,
                            float *dY, int M, int N, int K, void *stream);

/* Pre-allocates the per-handle work buffer for row counts up to max_M and, on
 * the weight-compiled kernel, compiles every code image a call with M <= max_M
 * rows runs (and the small-M images), so no later such call allocates or
 * compiles (graph capture).  It covers the host-pointer pipeline's M chunks
 * too (each chunk is a call with fewer rows). */
int tcsc_hip_reserve(tsg_tcsc *h, int max_M);

/* ---- introspection ------------------------------------------------------- */
typedef struct tsg_info {
    int32_t K, N, device, abi_version;
    int64_t nnz_pos, nnz_neg;
    int64_t tcsc_bytes;     /* TCSC::getDataStructureSize() (TCSC.h:43-49) */
    int64_t image_bytes;    /* bytes of the device image (segments + entries) */
    int64_t work_bytes;     /* current work-buffer size */
    int32_t chunk_rows;     /* K rows per LDS chunk of the image registration loaded
                               (the 64-row image's 128 x 8 shape when it could, else the
                               128-row image's 64 x 8, or rx); calls may compile others */
    int32_t tile_rows;      /* M rows per workgroup (same image) */
    int32_t tile_cols;      /* N columns per workgroup (same image) */
    int32_t reserved;
} tsg_info;
int tcsc_hip_info(const tsg_tcsc *h, tsg_info *out);

/* DataStructureInterface::getVectorRepresentation (DataStructureInterface.hpp:13)
 * for the registered matrix: dense K x N row-major ternary ints. */
int tcsc_hip_to_dense(const tsg_tcsc *h, int32_t *W, int K, int N);

/* Kernel timing: when enabled, HIP events bracket every launch of the main
 * (dominant) kernel on its own stream; totals accumulate until reset. */
int tcsc_hip_set_timing(tsg_tcsc *h, int enable);
int tcsc_hip_kernel_time(tsg_tcsc *h, double *total_ms, int64_t *launches, int reset);

/* Name of the device kernel this handle launches (the one timed above):
 * "tsg_jit_kernel" (default: W compiled into gfx950 code at registration) or
 * "tsg_tcsc_rx_kernel" (the register-X walk: W too large for one compiled
 * image, a generated image the loader refused -- logged on stderr -- or
 * TSG_KERNEL=rx at registration). */
const char *tcsc_hip_kernel_name(const tsg_tcsc *h);

/* The device kernel a call with M rows launches on this handle (calls pick
 * per M): "tsg_jit64_kernel" (the weight-compiled 64-row image:
 * one M row per lane; the default for M <= 512 and for configs[2]),
 * "tsg_jit_kernel" (the weight-compiled 128-row image; also what a call runs
 * after the image it picked could not be loaded -- logged on stderr),
 * "tsg_tcsc_ell_kernel" / "tsg_tcsc_ell_pc_kernel" (the small-M walks) or
 * "tsg_tcsc_rx_kernel". */
const char *tcsc_hip_call_kernel(const tsg_tcsc *h, int M);

const char *tcsc_hip_last_error(void);
int tcsc_hip_device_count(int *count);

/* ---- host-side helpers (no GPU needed) -------------------------------------
 * Column slice [n0, n1) of a TCSC, rebased to start at 0: the shard a rank
 * owns when W's columns are split across GPUs (Y[:,n] depends only on
 * column n).  Pass NULL outputs to query nnz_pos/nnz_neg of the slice. */
int tsg_tcsc_slice(const int32_t *col_start_pos, const int32_t *col_start_neg,
                   const int32_t *row_index_pos, const int32_t *row_index_neg, int N,
                   int n0, int n1, int32_t *out_csp, int32_t *out_csn,
                   int32_t *out_rip, int32_t *out_rin, int64_t *nnz_pos, int64_t *nnz_neg);

/* Checks the TCSC invariants the kernels rely on: monotone col_start of
 * length N+1 starting at 0, 0 <= k < K, strictly ascending k per column, no
 * k both +1 and -1 in a column.  TSG_OK or TSG_ERR_ARG (with message). */
int tsg_tcsc_validate(const int32_t *col_start_pos, const int32_t *col_start_neg,
                      const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N);

/* Synthetic W with the distribution of generateSparseMatrix
 * (cpp_impl/sparseUtils.h:52-87), emitted directly as TCSC restricted to the
 * columns [n0, n1) (rebased).  Deterministic in `seed` (splitmix64 stream,
 * the same draw sequence as the test oracle's dense generator).  Call with
 * NULL arrays to get nnz_pos/nnz_neg, then again to fill. */
int tsg_gen_tcsc(int K, int N, int s, uint64_t seed, int n0, int n1,
                 int32_t *csp, int32_t *csn, int32_t *rip, int32_t *rin,
                 int64_t *nnz_pos, int64_t *nnz_neg);

/* Format conversions between TCSC and CSC + base-3 packed values (see
 * tcsc_hip_create_csc_packed).  NULL outputs query the sizes only.
 * packed has ceil(nnz/5) bytes. */
int tsg_tcsc_to_csc_packed(const int32_t *col_start_pos, const int32_t *col_start_neg,
                           const int32_t *row_index_pos, const int32_t *row_index_neg, int N,
                           int32_t *col_ptr, int32_t *row_idx, uint8_t *packed, int64_t *nnz);
int tsg_csc_packed_to_tcsc(const int32_t *col_ptr, const int32_t *row_idx, const uint8_t *packed,
                           int N, int32_t *col_start_pos, int32_t *col_start_neg,
                           int32_t *row_index_pos, int32_t *row_index_neg, int64_t *nnz_pos,
                           int64_t *nnz_neg);

/* Checks BlockedTCSC<B> arrays (layout as tcsc_hip_create_blocked): monotone
 * column starts, every row inside its block, ascending, no row both +1 and -1. */
int tsg_blocked_tcsc_validate(const int32_t *col_start_pos, const int32_t *col_start_neg,
                              const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N,
                              int B);

/* X[i] = integer-valued fp32 U{-range..range} (initX, sparseUtils.h:6-23). */
int tsg_gen_x(int64_t len, int range, uint64_t seed, float *X);

#ifdef __cplusplus
}
#endif
#endif /* TERNARY_SPGEMM_H */
