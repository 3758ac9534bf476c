/*
 * ternary_spgemm_test.h -- tuning and test hooks of libternary_spgemm.so.
 *
 * Not needed to use the library as a drop-in (include/ternary_spgemm.h is
 * that surface).  These entry points pin or report the
 * per-call choices the library makes automatically, expose the
 * generated gfx950 code and the small-M image for CPU emulation in tests/,
 * and check the environment knobs.  None of them changes a result: every
 * choice they force is bit-identical to the automatic one.
 */
#ifndef TERNARY_SPGEMM_TEST_H
#define TERNARY_SPGEMM_TEST_H

#include "ternary_spgemm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Host-pointer pipeline chunks: 0 = automatic (one per ~16 MiB of Y, at most
 * 16, >= 256 rows, multiples of 128; small-M calls whole), or force n chunks
 * (1 = no pipeline; tests and A/B).  tcsc_hip_host_chunk_rows: rows per chunk
 * a call with M rows uses (M = unchunked).  Extension: no reference
 * counterpart. */
int tcsc_hip_set_host_chunks(tsg_tcsc *h, int chunks);
int tcsc_hip_host_chunk_rows(tsg_tcsc *h, int M);

/* Bytes of the device image a call with M rows reads: the small-M kernel's
 * sliced-ELL image, or the weight-compiled code (+ stream table) of the width
 * that call runs; 0 if that image is not built yet (tcsc_hip_reserve builds
 * it).  For reporting the bytes a launch moves besides X and Y.  Extension. */
int64_t tcsc_hip_call_image_bytes(tsg_tcsc *h, int M);

/* Weight-compiled kernel: columns per generated stream (a wave's columns).
 * 64 is the default; small-M calls use narrower streams (32, 16, 8) so more
 * workgroups fill the GPU -- each width is its own code image, compiled on the
 * first call (or tcsc_hip_reserve) that picks it.  Same results bit for bit.
 * tcsc_hip_jit_width: the width a call with M rows runs (0: not a jit handle).
 * tcsc_hip_set_jit_width: 0 = automatic (default), or pin 64/32/16/8, or
 * 128 (the 64-row image only: pinning it selects that image; BlockedTCSC: 64
 * only).  Extension: no reference counterpart. */
int tcsc_hip_jit_width(const tsg_tcsc *h, int M);
int tcsc_hip_set_jit_width(tsg_tcsc *h, int width);
/* Waves per workgroup of that call's image: 8, or 4 (narrow widths at mid M:
 * twice the workgroups of the same width). */
int tcsc_hip_jit_waves(const tsg_tcsc *h, int M);

/* Small-M kernel (no reference counterpart; DESIGN.md 4 "Small M"): calls
 * with few rows (GEMV-like: M <= 32 when K fits an 8-row LDS chunk -- up to
 * 128 for a small W, M x nnz <= 420 M -- else M <= 16, and grids the jit
 * kernel cannot fill) on a plain-TCSC handle run an index-reading sliced-ELL walk
 * (tsg_tcsc_ell_kernel; tsg_tcsc_ell_pc_kernel, a producer/consumer split of
 * it, for M = 1) that reads X in place and streams its entry stream from HBM
 * once per M tile, instead of the weight-compiled kernel.  Same results bit
 * for bit.  mode: 0 = automatic (default), 1 = never, 2 = every call, 3 =
 * every call without the producer/consumer split (tests).  The image is built
 * on the first call that needs it (or tcsc_hip_reserve). */
int tcsc_hip_set_small_m(tsg_tcsc *h, int mode);

/* Far-X^T code image (no reference counterpart; DESIGN.md 4.1 "Long K"):
 * calls that run the 64-wide weight-compiled kernel on its long-stream tile
 * map (K >= 8192, density > 3/16) with an X^T far larger than the 256 MiB
 * Infinity Cache (4 * M * K >= 768 MiB) and a code image that fits in it
 * (8 * nnz <= 160 MiB) run a second image of the same code without
 * code touches and with X^T staged by non-temporal loads, so the X^T stream
 * does not evict the code the other column tiles re-read.  Same results bit
 * for bit.  mode: 0 = automatic (default), 1 = never, 2 = every 64-wide call
 * (tests).  Compiled on the first call that picks it (or tcsc_hip_reserve).
 * tcsc_hip_call_far: 1 if a call with M rows runs it. */
int tcsc_hip_set_far(tsg_tcsc *h, int mode);
int tcsc_hip_call_far(const tsg_tcsc *h, int M);

/* The automatic per-call plan (host only, no GPU) of a plain-TCSC handle with
 * K, N and nnz nonzeros for a call with M rows -- the rules calls follow
 * (DESIGN.md 4): *kernel 0 = weight-compiled, 1 = small-M walk, 2 = its
 * producer/consumer form; for the weight-compiled kernel the stream width and
 * waves per workgroup, the far-X^T image (0/1), the tile-map groups
 * (gn column tiles x gm M tiles) and the code-touch mask. */
int tsg_call_plan(int K, int N, int64_t nnz, int M, int *kernel, int *width, int *waves, int *far,
                  int *gn, int *gm, int *tmask);

/* Whether that call spreads the generated code's per-group code touches over
 * the stream's lines (1) or points them at one line (0) -- round 6, DESIGN.md
 * 4.3 "Code touches"; host only.  < 0: TSG_ERR_ARG. */
int tsg_call_xtouch(int K, int N, int64_t nnz, int M);

/* Machine code of the weight-compiled kernel (TSG_KERNEL=jit) for a TCSC:
 * the generated gfx950 region (uint32 words; region byte offset 0 = word 0)
 * and, per (256-column tile, wave), the byte offset of that wave's stream.
 * Host only (no GPU): lets tests decode and emulate the code the device will
 * run.  NULL buffers query the lengths (in elements). */
int tsg_jit_codegen(const int32_t *col_start_pos, const int32_t *col_start_neg,
                    const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N,
                    uint32_t *code, int64_t code_cap, int64_t *code_len,
                    uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len);
/* Same for BlockedTCSC<B> arrays (tcsc_hip_create_blocked); B = 0 is plain TCSC. */
int tsg_jit_codegen_blocked(const int32_t *col_start_pos, const int32_t *col_start_neg,
                            const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N,
                            int B, uint32_t *code, int64_t code_cap, int64_t *code_len,
                            uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len);

/* Same with an explicit stream width (64, 32, 16, 8; BlockedTCSC: 64). */
int tsg_jit_codegen_w(const int32_t *col_start_pos, const int32_t *col_start_neg,
                      const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N,
                      int B, int width, uint32_t *code, int64_t code_cap, int64_t *code_len,
                      uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len);

/* ... and waves per workgroup (8; 4 for widths 32, 16, 8: the mid-M shapes). */
int tsg_jit_codegen_wv(const int32_t *col_start_pos, const int32_t *col_start_neg,
                       const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N,
                       int B, int width, int waves, uint32_t *code, int64_t code_cap, int64_t *code_len,
                       uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len);

/* The far-X^T image (tcsc_hip_set_far) of the 64-wide plain-TCSC code: no
 * code touches, non-temporal LDS-DMA; region header word 7 bit 17 set. */
int tsg_jit_codegen_far(const int32_t *col_start_pos, const int32_t *col_start_neg,
                        const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N,
                        uint32_t *code, int64_t code_cap, int64_t *code_len,
                        uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len);

/* The weight-compiled kernel's tile map (tsg_jit_map.h): workgroup id L of a
 * grid of mtiles x ntiles -> (column tile *nt, M tile *mt) for groups of gn
 * column tiles x gm M tiles per XCD.  Host only (tests check it is a
 * bijection for every shape the library launches). */
int tsg_jit_tile_map(int L, int mtiles, int ntiles, int gn, int gm, int *nt, int *mt);

/* The small-M kernel's sliced-ELL image for an M tile of MT rows and K chunks
 * of at most Cmax rows (tsg_ell.hip header): entry words (2 uint16 LDS float
 * indices each) and per (16-column slice, step) {offset in 256-B units,
 * 8-entry blocks}; *C, *nch: chunk rows and chunks.  copies = 2 (MT = 8
 * only; 1 otherwise): two X^T copies in LDS, the second at float *xb, each
 * entry pointing at one of them (tsg_internal.h ell_copy_offset); *xb = 0
 * with one copy.  copies = 3 (MT = 8): one copy with the bank-window schedule
 * (tsg_internal.h kEllSchedZeroRows), *xb = minus its zero rows after the
 * chunk.  Host only; NULL buffers query the lengths (in uint32). */
int tsg_ell_build(const int32_t *col_start_pos, const int32_t *col_start_neg, const int32_t *row_index_pos,
                  const int32_t *row_index_neg, int K, int N, int Cmax, int MT, int copies, uint32_t *ent,
                  int64_t ent_cap, int64_t *ent_len, uint32_t *tab, int64_t tab_cap, int64_t *tab_len, int32_t *C,
                  int32_t *nch, int32_t *xb);

/* The 64-row image (no reference counterpart): one M row per
 * lane, 64-row M tiles, every nonzero one 4-byte VOP2 v_add_f32 / v_sub_f32,
 * X^T in the k-quad layout.  Same results bit for bit.  rows: 0 = automatic
 * (default), 64 = the 64-row image, 128 = the 128-row image (v_pk_add_f32) for
 * every weight-compiled call (plain TCSC only).  tcsc_hip_call_tile_rows: the
 * M tile (64 / 128) of a call with M rows, 0 if it runs a small-M walk.
 * (The 128-row image's v_pk_add_f32 stream slows on full-mantissa X more than
 * the 64-row image's VOP2 stream) */
int tcsc_hip_set_tile_rows(tsg_tcsc *h, int rows);
int tcsc_hip_call_tile_rows(const tsg_tcsc *h, int M);

/* Device kernels a device-pointer call with M rows and this X launches: 1
 * when the kernel reads X itself (the small-M walks; the 64-row image's
 * direct X), 2 when an X^T staging kernel runs first.  bench.py
 * times such a one-launch step's stream as the kernel's duration. */
int tcsc_hip_call_launches(const tsg_tcsc *h, const float *dX, int M);

/* The 64-row image's machine code (layout as tsg_jit_codegen; region header
 * word 7 format 3, the k-quad layout): width 128 / 64 / 32 / 16 / 8, waves 8
 * (or 4 for widths 32, 16, 8). */
int tsg_jit_codegen64(const int32_t *col_start_pos, const int32_t *col_start_neg,
                      const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N,
                      int width, int waves, uint32_t *code, int64_t code_cap, int64_t *code_len,
                      uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len);
/* Its half ring (4-wave workgroups, widths 32 / 16 / 8; 96-row chunks, a
 * 72-KiB ring so two workgroups share a CU; region header word 7 bit 19;
 * TSG_JIT_HALF=1 selects it for the 4-wave calls, A/B). */
int tsg_jit_codegen64h(const int32_t *col_start_pos, const int32_t *col_start_neg,
                       const int32_t *row_index_pos, const int32_t *row_index_neg, int K, int N,
                       int width, uint32_t *code, int64_t code_cap, int64_t *code_len,
                       uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len);

/* The environment knobs (csrc/tsg_knobs.cpp): "" when every set TSG_* knob
 * has an accepted value, else the error registration reports (a set
 * TSG_JIT_DIAG is an error in the product build: its code variants give
 * wrong results and exist only in lib/libternary_spgemm_diag.so).  Host only. */
const char *tsg_knob_check(void);

#ifdef __cplusplus
}
#endif
#endif /* TERNARY_SPGEMM_TEST_H */
