// tsg_internal.h -- shared between the host planner, the C-ABI and the HIP
// kernels.  Not part of the public ABI (that is include/ternary_spgemm.h).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace tsg {

constexpr int kLanes = 64;                     // wavefront width (CDNA)

// ---------------------------------------------------------------------------
// "rx" (register-X) kernel (tsg_tcsc_rx_kernel)
//
// Workgroup: 256 M rows (4 per lane) x 8 waves x 32 columns, 512 threads,
// 256 VGPRs per wave.  X^T chunks of kRxChunk rows are staged in LDS (1 KiB
// per row, double buffered); a wave walks its columns in BLOCKS of at most
// kRxBlockRows consecutive K rows: the block's X rows are loaded into VGPRs
// (ds_read_b128) and every entry is one s_set_gpr_idx_idx (SRC1-relative
// X slot) + two v_pk_add_f32 -- no LDS traffic per entry.  A block holds at
// most kRxCap entries per column (the builder cuts blocks so it does).
// Variant knobs (compile-time, -DTSG_RX_*): waves per workgroup (4: two
// workgroups share a CU so one's barrier/latency stalls are covered by the
// other; 8: one per CU), K rows per LDS chunk, K rows per register block.
#ifndef TSG_RX_WAVES
#define TSG_RX_WAVES 8
#endif
#ifndef TSG_RX_CHUNK
#define TSG_RX_CHUNK 64
#endif
#ifndef TSG_RX_ROWS
#define TSG_RX_ROWS 24
#endif
constexpr int kRxTileM = 256;
constexpr int kRxWaves = TSG_RX_WAVES;
constexpr int kRxNW = 32;
constexpr int kRxTileCols = kRxWaves * kRxNW;
constexpr int kRxChunk = TSG_RX_CHUNK;         // K rows per LDS chunk
constexpr int kRxChunkBytes = kRxChunk * 1024;
constexpr int kRxBlockRows = TSG_RX_ROWS;
constexpr int kRxCap = 8;
constexpr int kRxBlockWords = 2 + 2 * kRxNW;  // [hdr][0][column c: 2 dwords of entry bytes]
// 2 chunks + the over-read of a block that starts on a chunk's last row
constexpr int kRxLdsBytes = 2 * kRxChunkBytes + (kRxBlockRows - 1) * 1024;
static_assert(kRxChunk % kRxWaves == 0, "chunk rows split over waves");
static_assert(kRxLdsBytes * (8 / kRxWaves) <= 160 * 1024, "workgroups per CU must fit the 160 KiB LDS");

// Stream of one wave: for every step q = p*nch + j (p = 0: +1 entries, p = 1:
// -1 entries; chunk j) one or more blocks of kRxBlockWords dwords:
//   hdr = (k0 - j*kRxChunk) * 1024 | (last block of the step) << 31
//   column c: 8 bytes, entry byte 4*(k - k0 + 1) for its entries of the
//   block, ascending k, then 0 bytes (0 = "empty": the kernel adds X slot 0,
//   which is +0.0f).
struct RxImage {
    int K = 0, N = 0, Npad = 0, nch = 0;
    std::vector<uint32_t> wstart;   // per (column tile, wave): first dword of its stream
    std::vector<uint32_t> ent;
};
void build_rx_image(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                    const int32_t *rin, int K, int N, RxImage &img);

// ---------------------------------------------------------------------------
// "jit" (weight-compiled) kernel: dispatcher tsg_jit_kernel (tsg_jit_kernel.hip,
// built as the code object lib/tsg_jit.co) + machine code generated from the
// TCSC arrays (tsg_jit.cpp).  A workgroup covers kJitTileM = 128 M rows (2 per
// lane) x kJitTileCols columns: 8 waves, each running the generated stream of
// kJitNW columns; X^T chunks of kJitChunk K rows in a ring of kJitRing LDS
// buffers (3 x 48 KiB), staged by LDS-DMA two steps ahead.
//
// X^T layout ("k-pair" layout, written by tsg_transpose_pairs_kernel): rows
// come in pairs p = (2p, 2p+1), and for M row pair mp = (2mp, 2mp+1) the 16
// bytes at ((p * Mp/2) + mp) * 16 hold
//     X[2mp][2p], X[2mp+1][2p], X[2mp][2p+1], X[2mp+1][2p+1]
// so one ds_read_b128 of lane l (M rows m0 + 2l, m0 + 2l + 1) loads BOTH k
// rows of a pair into a 4-VGPR X slot: row 2p in v[s:s+1], row 2p+1 in
// v[s+2:s+3] (a pair with one used row is read with ds_read_b64 into v[s:s+1]).
// An M tile's slice of a pair row is 64 lanes x 16 B = 1 KiB: one LDS-DMA piece.
constexpr int kJitTileM = 128;
constexpr int kJitWaves = 8;
constexpr int kJitMSplit = 1;
constexpr int kJitStreams = kJitWaves / kJitMSplit;     // streams per column tile
constexpr int kJitNW = 64;
constexpr int kJitTileCols = kJitStreams * kJitNW;
constexpr int kJitRing = 3;
constexpr int kJitChunk = 96;                           // K rows per chunk (48 pairs)
constexpr int kJitXRegs = 96;                           // X slot registers v[8 : 8 + 96)
constexpr int kJitSlotRegs = 4;                         // one X slot = one k-row pair (2 x 2 M rows)
constexpr int kJitSlots = kJitXRegs / kJitSlotRegs;     // 24 X slots
constexpr uint32_t kJitMagic0 = 0x7453474a, kJitMagic1 = 0x314a4954;
constexpr uint32_t kJitFormat = 2;                      // region header word 7 bits 8-15: k-pair layout
// region header word 7 bit 16: the DMA pieces take their in-group offset from
// the instruction offset field (one M0 per 4 pieces); the dispatcher then
// subtracts (piece & 3) KiB from its per-piece global offsets
constexpr uint32_t kJitM0kFlag = 1u << 16;
// region header word 7 bit 17: the far-X^T image -- no code touches, X^T
// staged with non-temporal loads (tsg_capi.cpp far_xt)
constexpr uint32_t kJitFarFlag = 1u << 17;

// The 64-row image (round 4): one M row per lane, 64-row M
// tiles, every nonzero one 4-byte VOP2 `v_add_f32 acc, acc, x` (+1) or
// `v_sub_f32 acc, acc, x` (-1) on one accumulator VGPR per column -- half the
// code bytes per useful add of the 128-row image when M <= 64 (whose
// v_pk_add_f32 then works on 64 padding rows).  On gfx950 a wave64 VALU op
// issues over 2 cycles (32 lanes per cycle), so with two waves per SIMD the
// VOP2 add retires as many adds per clock as v_pk_add_f32.
//
// Blocked k-quad layout: a lane's unit is a quad, the 16 B X[m][4q .. 4q+3]
// (contiguous in row-major X).  An M tile's chunk (64 rows x 192 K rows = 48
// quads, 48 KiB) is 48 pieces of 1 KiB; piece pr = 8 qg + rg holds row group
// rg (rows 8 rg .. 8 rg + 7) x quad group qg (quads 8 qg .. 8 qg + 7: one
// 128-B line of each row) with DMA lane j carrying row 8 rg + j % 8, quad
// 8 qg + j / 8.  So in LDS the quad q of row r sits at (q / 8) * 8 KiB +
// (r / 8) * 1 KiB + (q % 8) * 128 + (r % 8) * 16: a lane's base (r / 8) * 1 KiB
// + (r % 8) * 16 plus a uniform offset per quad (one ds_read_b128 loads four
// k rows of its row; b64 / b32 for quads with 2 / 1 used rows), each 8 lanes
// reading 128 contiguous bytes (no bank conflict).  The DMA pieces read
// either a staged copy in the same order (tsg_transpose_quads_kernel: piece
// (chunk c, M tile t, pr) is the 1 KiB at ((c * Mt + t) * 48 + pr) KiB,
// coalesced) or row-major X itself ("direct X": 8 whole 128-B lines per
// piece, no X^T pass).  The ring, the DMA issue and the register contract are
// the 128-row image's.
// Dispatchers lib/tsg_jit64_w<nw>[_4w].co (kernel tsg_jit64_kernel).
constexpr int kJit64TileM = 64;
constexpr int kJit64Chunk = 192;
constexpr uint32_t kJit64Format = 3;                    // region header word 7 bits 8-15: blocked k-quad layout
// region header word 7 bit 18 (64-row image): pieces of 16 rows x 4 quads
// (row base (r / 16) KiB + (r % 16) * 16: every ds_read_b128 lane group on 16
// distinct 16-B slots, no bank conflict; direct-X pieces read 64 B of each
// row) instead of 8 rows x 8 quads (whole 128-B lines per row; 2-way bank
// conflicts on ds_read_b128).  TSG_JIT_QBLOCK=16|8 picks (A/B).
constexpr uint32_t kJit64R16Flag = 1u << 18;
// Row layout (round 5, the default; region header word 7 bit 20): the LDS
// buffer holds the tile's 64 rows row-major, 47 quads (188 K rows, 752 B) per
// row -- quad q of row r at r * 752 + q * 16.  752 / 4 = 188 = -4 (mod 64), so
// the 16 lanes of every ds_read_b128 lane group (rows r, distinct r mod 16)
// read 16 distinct 16-B bank slots: conflict-free (ds_read_b64 / b32 as the
// blocked layout).  A lane's base is r * 752 plus one uniform offset q * 16
// per quad.  The chunk is 47 KiB = pieces 0 .. 46 of the 48-KiB ring buffer;
// DMA lane j of piece pr carries slot 64 pr + j = (row, quad) = divmod(., 47),
// so a piece reads one to three runs of contiguous row bytes: straight from
// row-major X ("direct X") as fast as from a staged copy
// (profiles/r05_dma_stride_micro.txt: 0.81 vs 0.85 us per 48-KiB step, against
// 1.55 for the blocked layout's 16-row x 64-B pieces).  The last chunk starts
// at K - 188 (when K >= 188 and K % 4 == 0; jit64_row_kbase), so direct X
// never reads past a row's end; the staged copy (tsg_transpose_rows_kernel)
// holds the same bytes.
constexpr uint32_t kJit64RowFlag = 1u << 20;
constexpr int kJit64RowQuads = 47;
constexpr int kJit64RowChunk = 4 * kJit64RowQuads;           // 188 K rows
constexpr int kJit64RowPitch = 16 * kJit64RowQuads;          // 752 B per M row in LDS
// first K row of chunk c of nch (row layout): c * 188, the last chunk K - 188
inline int jit64_row_kbase(int K, int nch, int c)
{
    const bool shift = c == nch - 1 && K >= kJit64RowChunk && K % 4 == 0;
    return shift ? K - kJit64RowChunk : c * kJit64RowChunk;
}
// rows per DMA piece of the blocked layout (16, 8: TSG_JIT_QBLOCK), or 0: the
// row layout (default); tsg_jit.cpp
int jit64_piece_rows();
// K rows per chunk of the 64-row image: the row layout 188, the blocked
// layout 192, the half ring 96
inline int jit64_chunk(bool half) { return half ? 96 : jit64_piece_rows() ? 192 : kJit64RowChunk; }
// Half ring (64-row image, 4-wave workgroups only; region header word 7 bit
// 19): 96-row chunks of 24 pieces (24 KiB), a 72-KiB ring, so two workgroups
// share a CU and each SIMD runs two waves (a lone wave issues its VOP2 adds
// at half rate); the 8-wave register contract (6 pieces per wave).  Staged
// copy: piece (chunk c, M tile t, pr) at ((c * Mt + t) * 24 + pr) KiB.
// Dispatchers lib/tsg_jit64h_w<nw>.co (TSG_JIT_HALF=1).
constexpr int kJit64HalfChunk = 96;
constexpr uint32_t kJit64HalfFlag = 1u << 19;

// Stream width: columns per generated stream.  kJitNW (64) is the default;
// narrower streams (32, 16, 8: same register contract, fewer accumulators,
// dispatcher lib/tsg_jit_w<nw>.co) give small-M calls more workgroups
// (tsg_capi.cpp pick_jit_width).  BlockedTCSC runs at kJitNW only.
constexpr int kJitWidths[] = {kJitNW, 32, 16, 8};
inline bool jit_width_ok(int nw) { return nw == kJitNW || nw == 32 || nw == 16 || nw == 8; }
// waves per workgroup: 8, or 4 for the narrow widths (lib/tsg_jit_w<nw>_4w.co):
// the same 48 KiB chunks staged by 4 waves (12 DMA pieces each), half the
// columns per workgroup -> twice the workgroups at mid M
inline bool jit_waves_ok(int nw, int waves) { return waves == kJitWaves || (waves == 4 && nw < kJitNW); }
// The 64-row image also runs 128 columns per wave (8 waves; one accumulator
// VGPR per column, v116..v243; lib/tsg_jit64_w128.co): twice the adds per
// staged chunk and per X read of its 64-wide stream
constexpr int kJit64WideNW = 128;
constexpr int kJit64Widths[] = {kJit64WideNW, kJitNW, 32, 16, 8};
inline bool jit64_width_ok(int nw) { return jit_width_ok(nw) || nw == kJit64WideNW; }

// words of padding after the last stream (the code prefetch reads ahead)
constexpr int kJitTailPadWords = 32768 + 1024;

struct JitImage {
    int K = 0, N = 0, Npad = 0, nch = 0, B = 0, nw = 0, waves = kJitWaves;
    int tile_m = kJitTileM, chunk = kJitChunk;  // 64 / kJit64Chunk for the 64-row image
    int piece_rows = 0;                          // 64-row image: rows per DMA piece (16 or 8; 0 = row layout)
    bool half = false;                           // 64-row image: the half ring (kJit64HalfChunk)
    std::vector<uint32_t> code;    // region: [magic x2][0][0] then one stream per (tile, wave)
    std::vector<uint32_t> wcode;   // per (column tile, stream): byte offset of the stream
};
// B = 0: BaseTCSC order (comp.h:25-69); B > 0: BaseBlockedTCSC<B> order
// (comp.h:607-658) from BlockedTCSC<B> arrays
// rows64: the 64-row image (plain TCSC only; BaseTCSC order, VOP2 adds)
void build_jit_code(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                    const int32_t *rin, int K, int N, int B, JitImage &img, int nw = kJitNW,
                    int waves = kJitWaves, bool far = false, bool rows64 = false, bool half = false);

struct JitModule {
    void *module = nullptr;        // hipModule_t
    void *function = nullptr;      // hipFunction_t of tsg_jit_kernel
    void *probe = nullptr;         // hipFunction_t of tsg_jit_probe (region check, at load)
    // pair: the 64-row image's 4-wave streams run by 8-wave workgroups of
    // half-masked wave pairs (lib/tsg_jit64p_w<nw>.co; launch 8 waves)
    std::string load(const std::vector<uint32_t> &code, int nw = kJitNW, int waves = kJitWaves,
                     bool rows64 = false, bool half = false, bool pair = false);  // "" on success
    void unload();
};
// xrow > 0: the 64-row image stages straight from X (xrow floats per row);
// lastadj: bytes the row layout's last chunk starts below its slot (direct X);
// xtouch: the per-group code touches (v[lane128 + 1]) spread over the lines;
// tnear: the code touches' window starts at the step's own position
int launch_tcsc_jit(const JitModule &jm, const float *XT, int Mp, const uint32_t *wcode,
                    const float *b, const float *alpha, float *Y, int M, int N, int Npad, int nch,
                    int prelu, uint32_t *status, int tile_cols, int waves, int gn, int gm, int tmask,
                    void *stream, int tile_m = kJitTileM, int xrow = 0, int lastadj = 0, int xtouch = 0,
                    int tnear = 0);
int launch_jit_probe(const JitModule &jm, uint32_t *status, void *stream);

// ---------------------------------------------------------------------------
// "ell" small-M kernel (tsg_tcsc_ell_kernel, tsg_ell.hip): sliced-ELL entry
// stream, see the header of tsg_ell.hip.  Variants = M tiles (the image
// depends on the tile only; lanes per column x rows per lane are a launch
// choice, tsg_ell.hip launch_tcsc_ell), with the K rows per LDS chunk C each
// allows: (C + 1) * tile floats <= 160 KiB of LDS, float indices C * tile
// < 65536.  K <= C runs as ONE stream per column (no restaging).
//   0: M tile 1,  C <= 40956      1: M tile 4,  C <= 10236
//   2: M tile 8,  C <= 5116       3: M tile 16, C <= 2556
//   4: M tile 32, C <= 1276
constexpr int kEllVariants = 5;
constexpr int kEllTileM[kEllVariants] = {1, 4, 8, 16, 32};
constexpr int kEllMaxC[kEllVariants] = {40956, 10236, 5116, 2556, 1276};
struct EllImage {
    int C = 0, nch = 0, steps = 0, nslices = 0;
    int xb = 0;                  // float offset of the second X^T copy (0: one copy)
    int zr = 1;                  // zero rows after the chunk (8: the bank-window schedule)
    std::vector<uint32_t> ent;   // uint16 entries, 2 per word (256-B blocks)
    std::vector<uint32_t> tab;   // per (slice, step): {offset in 256-B units, 8-entry blocks}
};
// Two X^T copies (round 5, the 8-row tile's 4-lane columns: a ds_read_b64 lane
// group = 8 columns, each reading an 8-float row = 8 of the 64 LDS banks, so
// random k collide on 8 bank windows): copy B starts 32 banks off copy A's
// window of the same row, and the image points each entry at the copy that
// balances its lane group's windows (tsg_host.cpp build_ell_image).
// LDS floats of a chunk of C rows (+ the zero row) of an MT-row tile: one copy,
// or copy B at xb (a multiple of 64 floats + 32 past copy A)
constexpr int ell_copy_offset(int C, int MT) { return ((C + 1) * MT + 63) / 64 * 64 + 32; }
__host__ __device__ constexpr int ell_lds_floats(int C, int MT, int xb, int zr = 1)
{
    return xb ? xb + (C + 1) * MT : (C + zr) * MT;
}
// Bank-window schedule (round 5, the 8-row tile's 4-lane columns): per
// ds_read_b64 lane group of 8 columns and entry position, only columns whose
// next row lies in a window no other column of the group reads there advance;
// the others read a zero row (8 of them after the chunk, one per window; all
// such pads of a position read the same one), so every gather is
// conflict-free, at ~1.5x the positions (tsg_host.cpp build_ell_image)
constexpr int kEllSchedZeroRows = 8;
void build_ell_image(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin, int K, int N,
                     int Cmax, int MT, EllImage &img, int copies = 1, bool sched = false);
int launch_tcsc_ell(int variant, const float *X, const uint32_t *ent, const uint32_t *tab, const float *b,
                    const float *alpha, float *Y, int M, int N, int K, int C, int nch, int xb, int zr, int prelu,
                    void *stream);
// the producer/consumer walk (tsg_tcsc_ell_pc_kernel) of variant 0 (M = 1) when
// K fits one chunk and the chunk plus its LDS ring fit kLdsBytes
// (ell_pc_lds_bytes; 0 = no such variant); -2 = not available for this image
constexpr size_t kLdsBytes = 160 * 1024;
size_t ell_pc_lds_bytes(int variant, int C);
int launch_tcsc_ell_pc(int variant, const float *X, const uint32_t *ent, const uint32_t *tab, const float *b,
                       const float *alpha, float *Y, int M, int N, int K, int C, int nch, int prelu, void *stream);

// Environment knobs (csrc/tsg_knobs.cpp): A/B studies and tests, none of
// which changes a result.  knob_check: "" when every set knob has an
// accepted value, else the first error (registration and the host codegen
// entry points refuse it); in the product build a set TSG_JIT_DIAG is an
// error (its code variants give wrong results: diagnostic build only).
// knob_value: the text of a set, valid knob, else nullptr.
std::string knob_check();
const char *knob_value(const char *name);
bool diag_build();

// B = 0: plain TCSC; B > 0: BlockedTCSC<B> arrays ((K/B)*N + 1 column starts)
std::string validate_tcsc(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                          const int32_t *rin, int K, int N, int B = 0);

// GPU-side TCSC encoder (csrc/tsg_encode.hip).  encode_count: column starts
// into d_csp/d_csn (N+1 each); with d_tmp == nullptr it only returns the scan
// workspace size in *tmp_bytes.  encode_fill: row indices.
int encode_count(const int32_t *dW, int K, int N, int32_t *d_csp, int32_t *d_csn, void *d_tmp, size_t *tmp_bytes,
                 void *stream);
int encode_fill(const int32_t *dW, int K, int N, const int32_t *d_csp, const int32_t *d_csn, int32_t *d_rip,
                int32_t *d_rin, void *stream);

// Kernel launchers (csrc/tcsc_kernels.hip).  All enqueue on `stream`.
int launch_transpose(const float *X, float *XT, int M, int K, int Mp, int Kp, void *stream);
// X [M][K] -> X^T in the k-pair layout of the jit kernel (Kp even, Mp even)
int launch_transpose_pairs(const float *X, float *XP, int M, int K, int Mp, int Kp, void *stream);
// X [M][K] -> the blocked k-quad layout of the 64-row image (Mp % 64 == 0, Kp % 192 == 0;
// piece_rows 16 or 8, kJit64R16Flag), or with piece_rows 0 its row layout's
// staged copy (kJit64RowFlag; Kp % 188 == 0)
int launch_transpose_quads(const float *X, float *XQ, int M, int K, int Mp, int Kp, int piece_rows, void *stream,
                           int chunk = kJit64Chunk);
int launch_tcsc_rx(const float *XT, int Mp, const uint32_t *wstart, const uint32_t *ent,
                   const float *b, const float *alpha, float *Y, int M, int N, int Npad, int nch,
                   int prelu, void *stream);

}  // namespace tsg
