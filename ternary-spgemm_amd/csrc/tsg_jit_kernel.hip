// tsg_jit_kernel.hip -- dispatcher of the weight-compiled ("jit") TCSC kernel.
//
// Built as a standalone gfx950 code object (lib/tsg_jit.co), NOT into the
// shared library: at registration tsg_jit.cpp appends the machine code it
// generates from the TCSC arrays as an extra PT_LOAD segment and loads the
// result with hipModuleLoadData, so the loader maps that code executable
// together with this kernel.
//
// Why compile W into code: the BaseTCSC chain (comp.h:37-63)
// is one dependent fp32 add per nonzero, and a walk that READS the entry
// indices at run time pays, per nonzero, for the index (LDS gather or
// register-indexed add) and per column for a data-dependent branch -- the
// measured cost of the register-X walk was 2-3x its adds.  Here every nonzero
// of a wave's columns is one v_pk_add_f32 (2 M rows per lane) whose X
// register (a row of the current X^T chunk, loaded from LDS) and accumulator
// are encoded in the instruction: no index traffic, no SALU, no branch.  The
// same code serves every 128-row M tile.
//
// Workgroup: 128 M rows x (8 waves x kJNW columns), one per CU; a wave owns 2
// M rows per lane and the kJNW columns of its stream (2 waves per SIMD, 244
// VGPRs).  The dispatcher sets up registers and calls the wave's generated
// stream ONCE; the stream runs the whole K loop: X^T chunks of 96 K rows (48
// k-row pairs, tsg_internal.h "k-pair layout") in a ring of 3 LDS buffers,
// each staged by LDS-DMA two steps ahead (6 pair rows of 1 KiB per wave), one
// `s_waitcnt vmcnt(0); s_barrier` per step (step q = pass p * nch + chunk j:
// p = 0 the +1 entries, p = 1 the -1 entries), X pairs read with ds_read_b128
// (both k rows at once), the next step's first reads issued before the
// barrier, the stream's own code touched ahead (L2 prefetch).
// Register contract (tsg_jit.cpp), 8 waves (4 waves: 12 pieces v108-119,
// lane*128 v120, accumulators from v122):
//   v[8:104)   24 X slots of 4 VGPRs (k-row pair: row 2p in v[s:s+1], 2p+1 in v[s+2:s+3])
//   v104-106   LDS byte address of lane*16 in ring buffer 0..2
//   v107       code-prefetch sink
//   v108-113   per-lane byte offsets (from the chunk base) of this wave's 6 LDS-DMA pieces
//   v114       lane * 128 (code prefetch)
//   v115       lane * 128 or 0 (the per-group code touches, per call; 4 waves: v121)
//   v[116:244) accumulators, column c at v116 + 2c (rows 2l, 2l+1 of the lane)
//   s[80:81] X^T base, s82 chunk stride in bytes, s83 LDS byte offset of this
//   wave's first DMA piece, s[84:85] chunk base (stream),
//   s86 saved M0, s87 bytes the 64-row row layout's last chunk starts below
//   its slot (direct X; else 0), s[88:89] prefetch address (stream),
//   s[90:91] code-touch base (region base, or 8 KiB below it per call),
//   s[92:93] region base, s[94:95] return address.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tsg_jit_map.h"

namespace {

// TSG_JIT_NW: a narrower stream width (32, 16 or 8 columns per wave;
// lib/tsg_jit_w<NW>.co) -- more workgroups for small M, same registers.
// TSG_JIT_WAVES=4 (narrow widths, lib/tsg_jit_w<NW>_4w.co): 4-wave workgroups,
// twice the workgroups again; each wave stages 12 of the chunk's 48 pair
// rows, so the piece offsets take v108-119, lane*128 v120, accumulators from v122.
#ifndef TSG_JIT_NW
#define TSG_JIT_NW 64
#endif
#ifndef TSG_JIT_WAVES
#define TSG_JIT_WAVES 8
#endif
// TSG_JIT_ROWS64=1: the 64-row image's dispatcher (lib/tsg_jit64_w<NW>[_4w].co,
// kernel tsg_jit64_kernel; tsg_internal.h): one M row per lane, 64-row M
// tiles, one accumulator VGPR per column, X^T in the k-quad layout, 192-row
// chunks (48 quads) -- the same ring, DMA pieces and register contract
#ifndef TSG_JIT_ROWS64
#define TSG_JIT_ROWS64 0
#endif
// TSG_JIT_HALF=1 (64-row image, 4 waves; lib/tsg_jit64h_w<NW>.co): the half
// ring -- 96-row chunks of 24 pieces, 3 x 24 KiB of LDS, two workgroups per
// CU -- with the 8-wave register contract (6 pieces per wave)
#ifndef TSG_JIT_HALF
#define TSG_JIT_HALF 0
#endif
// TSG_JIT_PAIR=1 (64-row image, 4-wave streams; lib/tsg_jit64p_w<NW>.co): an
// 8-wave workgroup runs the 4-wave image -- waves w and w + 4 (one SIMD) run
// stream w, each on one half of the tile's rows (exec = lanes 0-31, resp.
// 32-63).  A lone wave per SIMD issues a VOP2 only every ~5.5 cycles; two
// half-masked waves keep the SIMD issuing.  Together the pair stages the
// stream's 12 DMA pieces (each wave its lanes' halves: the LDS-DMA address is
// per lane), reads and touches what the 4-wave wave would; each wave stores
// its half of the rows.
#ifndef TSG_JIT_PAIR
#define TSG_JIT_PAIR 0
#endif
constexpr int kJWaves = TSG_JIT_WAVES;
constexpr int kJNW = TSG_JIT_NW;
constexpr bool kJRows64 = TSG_JIT_ROWS64 != 0;
constexpr bool kJHalf = TSG_JIT_HALF != 0;
constexpr bool kJPair = TSG_JIT_PAIR != 0;
static_assert(!kJHalf || (kJRows64 && TSG_JIT_WAVES == 4), "the half ring is a 4-wave 64-row image");
static_assert(!kJPair || (kJRows64 && TSG_JIT_WAVES == 4 && !kJHalf), "wave pairs run the 4-wave 64-row image");
static_assert(kJNW == 64 || kJNW == 32 || kJNW == 16 || kJNW == 8 || (kJRows64 && kJNW == 128), "stream width");
static_assert(kJWaves == 8 || (kJWaves == 4 && kJNW < 64), "waves per workgroup");
constexpr int kJTileM = kJRows64 ? 64 : 128;
constexpr int kJRowsPerLane = kJTileM / 64;
constexpr int kJTileCols = kJWaves * kJNW;
constexpr int kJThreads = (kJPair ? 2 : 1) * kJWaves * 64;  // workgroup size (wave pairs: 8 waves, 4 streams)
constexpr int kJRing = 3;                            // LDS buffers in the X^T ring (tsg_internal.h)
constexpr int kJChunk = kJRows64 ? (kJHalf ? 96 : 192) : 96;  // K rows per chunk = 48 (half ring 24) quads / pairs
constexpr int kJUnits = kJRows64 ? kJChunk / 4 : kJChunk / 2;  // 1-KiB LDS units per chunk
constexpr int kJBufBytes = kJChunk * kJTileM * 4;    // 48 KiB
constexpr int kJPieces = kJUnits / kJWaves;          // LDS-DMA pieces (1-KiB unit rows) per wave per chunk
static_assert(kJBufBytes == kJUnits * 1024, "one LDS-DMA piece per unit row");
static_assert(kJPieces == 6 || (kJWaves == 4 && kJPieces == 12), "register contract: 6 pieces (v108-113) or 12");
constexpr uint32_t kJMagic0 = 0x7453474a, kJMagic1 = 0x314a4954;  // region header
constexpr uint32_t kJM0kFlag = 1u << 16;  // header word 7: piece offsets in the DMA instruction (tsg_internal.h)
constexpr uint32_t kJFormat = kJRows64 ? 3u : 2u;  // header word 7 bits 8-15: the X^T layout the code expects
constexpr uint32_t kJR16Flag = 1u << 18;            // header word 7: 64-row image pieces of 16 rows x 4 quads
constexpr uint32_t kJHalfFlag = 1u << 19;           // header word 7: the half ring
constexpr uint32_t kJRowFlag = 1u << 20;            // header word 7: the 64-row image's row layout (188-row chunks)
#if TSG_JIT_ROWS64
#define TSG_JIT_KERNEL_NAME tsg_jit64_kernel
#else
#define TSG_JIT_KERNEL_NAME tsg_jit_kernel
#endif

typedef float F32x32 __attribute__((ext_vector_type(32)));
typedef float F32x16 __attribute__((ext_vector_type(16)));
typedef float F32x8 __attribute__((ext_vector_type(8)));

#if TSG_JIT_WAVES == 8 || TSG_JIT_HALF  // 6 DMA pieces per wave
#define TSG_JIT_IN                                                                                  \
    "{v104}"(lb0), "{v105}"(lb1), "{v106}"(lb2), "{v108}"(off[0]), "{v109}"(off[1]),             \
        "{v110}"(off[2]), "{v111}"(off[3]), "{v112}"(off[4]), "{v113}"(off[5]), "{v114}"(l128), "{v115}"(l128x)
#else
#define TSG_JIT_IN                                                                                  \
    "{v104}"(lb0), "{v105}"(lb1), "{v106}"(lb2), "{v108}"(off[0]), "{v109}"(off[1]),             \
        "{v110}"(off[2]), "{v111}"(off[3]), "{v112}"(off[4]), "{v113}"(off[5]), "{v114}"(off[6]), \
        "{v115}"(off[7]), "{v116}"(off[8]), "{v117}"(off[9]), "{v118}"(off[10]), "{v119}"(off[11]), \
        "{v120}"(l128), "{v121}"(l128x)
#endif

#define TSG_JIT_CLOBBERS \
    "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", \
        "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", \
        "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", \
        "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", \
        "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", \
        "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", \
        "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", \
        "v100", "v101", "v102", "v103", "v107", "s84", "s85", "s86", "s88", "s89", "s94", "s95", \
        "scc", "memory"

}  // namespace

// Probe (tsg_capi.cpp ensure_jit_variant, once per loaded image, never in a
// call): the same region-base computation as tsg_jit_kernel -- its own
// s_getpc + literal, patched by the loader like the kernel's -- and the magic
// check; status[1] = magic when the generated region is where the kernel
// will jump.  A separate kernel so that traces of tsg_jit_kernel hold calls only.
extern "C" __global__ __launch_bounds__(64) void tsg_jit_probe(uint32_t *__restrict__ status)
{
    uint64_t base;
    asm volatile("s_getpc_b64 s[92:93]\n\t"
                 "s_add_u32 s92, s92, 0x7a5e1234\n\t"
                 "s_addc_u32 s93, s93, 0"
                 : "={s[92:93]}"(base)
                 :
                 : "scc");
    const uint32_t *hdr = reinterpret_cast<const uint32_t *>(base);
    if (threadIdx.x == 0) {
        // the region is ours and laid out for this dispatcher (the kernel makes
        // the same check per launch, where a mismatch could only zero-exit)
        const bool ok = hdr[0] == kJMagic0 && hdr[1] == kJMagic1 && ((hdr[7] >> 8) & 0xffu) == kJFormat &&
                        ((hdr[7] & kJHalfFlag) != 0) == kJHalf;
        status[0] = ok ? 0u : 1u;
        status[1] = ok ? kJMagic0 : 0u;
    }
}

// (the half ring: two workgroups per CU, so at most 256 VGPRs -- two waves per SIMD)
extern "C" __global__ __launch_bounds__(kJThreads, kJHalf ? 2 : 1) void TSG_JIT_KERNEL_NAME(
    const float *__restrict__ XT, int Mp, const uint32_t *__restrict__ wcode,
    const float *__restrict__ b, const float *__restrict__ alpha, float *__restrict__ Y, int M, int N,
    int nch, int mtiles, int ntiles, int prelu, uint32_t *__restrict__ status, int gn, int gm,
    int tmask, int xrow, int lastadj, int xtouch, int tnear)
{
    __shared__ __attribute__((aligned(16))) char lds[kJRing * kJBufBytes];
    const int tid = threadIdx.x, lane = tid & 63;
    // LDS is only addressed from the generated code, at absolute offsets from
    // 0 (the only LDS object): this use keeps the allocation in the descriptor
    asm volatile("; lds %0" ::"v"(lds));
    // the wave's stream index (wave pairs: waves w and w + 4 share stream w)
    // and, for a pair, which half of the rows it runs
    const int wraw = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wave = kJPair ? (wraw & 3) : wraw;
    const int rhalf = kJPair ? (wraw >> 2) : 0;

    // Base of the generated region: s_getpc + a literal that the loader-side
    // patcher (tsg_jit.cpp) sets to (region vaddr - vaddr of the s_add).
    uint64_t base;
    asm volatile("s_getpc_b64 s[92:93]\n\t"
                 "s_add_u32 s92, s92, 0x7a5e1234\n\t"
                 "s_addc_u32 s93, s93, 0"
                 : "={s[92:93]}"(base)
                 :
                 : "scc");
    // never jump into a region that is not ours (or laid out for the other image)
    const uint32_t *hdr = reinterpret_cast<const uint32_t *>(base);
    if (hdr[0] != kJMagic0 || hdr[1] != kJMagic1 || ((hdr[7] >> 8) & 0xffu) != kJFormat ||
        ((hdr[7] & kJHalfFlag) != 0) != kJHalf) {
        if (blockIdx.x == 0 && tid == 0) status[0] = 1u;
        return;
    }

    // tile map (tsg_jit_map.h): gn column tiles x gm M tiles per XCD group,
    // chosen per call by the host (tsg_capi.cpp pick_jit_map)
    int nt, mt;
    tsg_jit_tile(blockIdx.x, mtiles, ntiles, gn, gm, nt, mt);
    const int m0 = mt * kJTileM;
    const int stream = wave;  // the wave's column stream
    const int ncol0 = nt * kJTileCols + stream * kJNW;
    const uint64_t cp = base + __builtin_amdgcn_readfirstlane(wcode[(size_t)nt * kJWaves + stream]);
    // the lane's LDS base in ring buffer 0 (64-row image, blocked k-quad
    // layout, PR rows per piece: row r at (r / PR) KiB + (r % PR) * 16;
    // tsg_internal.h)
    const uint32_t pr_rows = (hdr[7] & kJR16Flag) ? 16u : 8u;
    // row layout (tsg_internal.h kJit64RowFlag): row r at r * 752 B
    // (uniform: the SGPR stride and chunk adjustment below depend on it)
    const bool rowlay = kJRows64 && !kJHalf && (__builtin_amdgcn_readfirstlane(hdr[7]) & kJRowFlag) != 0;
    const uint32_t lb0 = rowlay   ? (uint32_t)lane * 752u
                         : kJRows64 ? ((uint32_t)lane / pr_rows) * 1024u + ((uint32_t)lane % pr_rows) * 16u
                                    : (uint32_t)lane * 16u;
    const uint32_t lb1 = lb0 + kJBufBytes, lb2 = lb0 + 2 * kJBufBytes;
    // LDS-DMA piece i of this wave = pair row pr = wave * P + i of the chunk: the
    // lane's 16 B at ((pr * Mp/2) + m0/2 + lane) * 16 from the chunk base (64-row
    // image: quad row pr, ((pr * Mp) + m0 + lane) * 16).  With
    // the header's m0k flag the generated code adds (i & 3) KiB through the
    // instruction offset (to the LDS and the global address alike): subtracted
    // here (never negative: pr >= i and a pair row of X^T is >= 1 KiB)
    const uint32_t m0k = (hdr[7] & kJM0kFlag) ? 1u : 0u;
    uint32_t off[kJPieces];
    // 64-row image (blocked k-quad layout, tsg_internal.h): piece pr = (64 /
    // PR) qg + rg, DMA lane j carries row PR rg + j % PR, quad (64 / PR) qg + j
    // / PR.  Staged:
    // the piece is the 1 KiB at ((chunk * Mt + mt) * 48 + pr) KiB of the
    // staged copy.  Direct X (xrow > 0 floats per row): the quad X[m][4q ..
    // 4q+3] is 16 contiguous bytes of row-major X, so the pieces stage straight
    // from X -- no X^T pass; rows past M read row M-1 (their results are never
    // stored), pieces at or past K are never staged (the generated code omits
    // them; K % (256 / PR) == 0), and the chunk base starts 3 KiB below X so that
    // off[i] stays non-negative after the m0k subtraction.
    const bool direct = kJRows64 && xrow > 0;
    const uint32_t xrow_b = (uint32_t)xrow * 4u;
#pragma unroll
    for (int i = 0; i < kJPieces; i++) {
        const uint32_t pr = (uint32_t)(wave * kJPieces + i);
        uint32_t o;
        if (!kJRows64) {
            o = (pr * ((uint32_t)Mp / 2u) + (uint32_t)m0 / 2u + (uint32_t)lane) * 16u;
        } else if (rowlay) {
            // slot 64 pr + lane = (row, quad) of the 64 x 47-quad chunk; pieces
            // pr >= 47 are never staged (their offset only has to be valid)
            const uint32_t slot = min(pr * 64u + (uint32_t)lane, 64u * 47u - 1u);
            const uint32_t row = slot / 47u, quad = slot % 47u;
            o = direct ? (uint32_t)min(m0 + (int)row, M - 1) * xrow_b + quad * 16u + 3072u
                       : ((uint32_t)mt * 47u + pr) * 1024u + (uint32_t)lane * 16u;
        } else if (direct) {
            const uint32_t rgs = 64u / pr_rows;  // row groups per tile = quads per piece
            const uint32_t row = (uint32_t)min(m0 + (int)((pr % rgs) * pr_rows + (uint32_t)lane % pr_rows), M - 1);
            o = row * xrow_b + ((pr / rgs) * rgs + (uint32_t)lane / pr_rows) * 16u + 3072u;
        } else {
            o = ((uint32_t)mt * (uint32_t)kJUnits + pr) * 1024u + (uint32_t)lane * 16u;
        }
        off[i] = o - m0k * (uint32_t)(i & 3) * 1024u;
    }
    const uint64_t xbase = (uint64_t)(uintptr_t)XT - (direct ? 3072u : 0u);
    const uint32_t wb = (uint32_t)(wave * kJPieces) * 1024u;  // s83
    // code touch (one dword per 128-B line of the stream ahead, into L2): only
    // workgroups with (mt & tmask) == 0 spread it over the lines; the others
    // load one line 64 times (one request) -- the M tiles that run the same
    // stream share what one of them touched (tsg_capi.cpp pick_jit_map)
    const uint32_t l128 = (mt & tmask) == 0 ? (uint32_t)lane * 128u : 0u;
    // the generated code's per-group touches (round 6) use v[lane128 + 1]:
    // the same lines where the call wants them (xtouch), else one line
    const uint32_t l128x = xtouch ? l128 : 0u;
    // the code touches' base (s[90:91]): the region base, or 8 KiB below it
    // for calls whose touch window should start at the step's own position
    // (tnear; the generated code never touches less than 8 KiB ahead of its
    // position relative to this base, so the window stays inside the region)
    const uint64_t tbase = base - (tnear ? 8192u : 0u);
    // chunk stride: kJChunk K rows of X^T (both staged layouts: Mp * chunk * 4
    // bytes), or of one row-major X row (direct)
    // (row layout: 188-row chunks; the staged copy holds 47 KiB per (chunk, M tile))
    const uint32_t chunk_rows = rowlay ? 188u : (uint32_t)kJChunk;
    const uint32_t stride = direct ? chunk_rows * 4u : chunk_rows * (uint32_t)Mp * 4u;
    // row layout, direct X: the last chunk starts lastadj bytes below its slot (K - 188)
    const uint32_t adj = direct ? (uint32_t)lastadj : 0u;

#if TSG_JIT_PAIR
    // wave pairs: the stream runs with exec = the wave's half of the lanes;
    // exec is saved around it (the dispatcher itself runs on all 64 lanes)
    const uint64_t emask = rhalf ? 0xffffffff00000000ull : 0x00000000ffffffffull;
    uint64_t esave;
#define TSG_JIT_EXEC_IN "s_mov_b64 %[es], exec\n\ts_mov_b64 exec, %[em]\n\t"
#define TSG_JIT_EXEC_OUT "\n\ts_mov_b64 exec, %[es]"
#define TSG_JIT_EXEC_OPS , [es] "=&s"(esave)
#define TSG_JIT_EXEC_INS , [em] "s"(emask)
#else
#define TSG_JIT_EXEC_IN ""
#define TSG_JIT_EXEC_OUT ""
#define TSG_JIT_EXEC_OPS
#define TSG_JIT_EXEC_INS
#endif
#define TSG_JIT_CALL(...)                                                                           \
    asm volatile(TSG_JIT_EXEC_IN                                                                    \
                 "s_getpc_b64 s[94:95]\n"                                                           \
                 ".Ljr%=:\n\t"                                                                      \
                 "s_add_u32 s94, s94, (.Ljb%= - .Ljr%=)\n\t"                                        \
                 "s_addc_u32 s95, s95, 0\n\t"                                                       \
                 "s_setpc_b64 %[cp]\n"                                                              \
                 ".Ljb%=:" TSG_JIT_EXEC_OUT                                                         \
                 : __VA_ARGS__ TSG_JIT_EXEC_OPS                                                     \
                 : [cp] "s"(cp), "{s[92:93]}"(base), "{s[90:91]}"(tbase), "{s[80:81]}"(xbase), "{s82}"(stride),  \
                   "{s83}"(wb), "{s87}"(adj),                                                          \
                   TSG_JIT_IN TSG_JIT_EXEC_INS                                                      \
                 : TSG_JIT_CLOBBERS)
#if TSG_JIT_ROWS64  // one accumulator VGPR per column (acc0 = v116; 4 waves: v122, half ring v116)
#if TSG_JIT_WAVES == 8 || TSG_JIT_HALF
#define TSG_JIT_A0 "v[116:147]"
#define TSG_JIT_A1 "v[148:179]"
#define TSG_JIT_A16 "v[116:131]"
#define TSG_JIT_A8 "v[116:123]"
#else
#define TSG_JIT_A0 "v[122:153]"
#define TSG_JIT_A16 "v[122:137]"
#define TSG_JIT_A8 "v[122:129]"
#endif
#if TSG_JIT_NW == 128  // 8 waves only: v[116:244)
    F32x32 a0 = {}, a1 = {}, a2 = {}, a3 = {};  // comp.h:41
    TSG_JIT_CALL("+{v[116:147]}"(a0), "+{v[148:179]}"(a1), "+{v[180:211]}"(a2), "+{v[212:243]}"(a3));
    auto acc_of = [&](int c, int) { return c < 32 ? a0[c] : c < 64 ? a1[c - 32] : c < 96 ? a2[c - 64] : a3[c - 96]; };
#elif TSG_JIT_NW == 64
    F32x32 a0 = {}, a1 = {};  // comp.h:41
    TSG_JIT_CALL("+{" TSG_JIT_A0 "}"(a0), "+{" TSG_JIT_A1 "}"(a1));
    auto acc_of = [&](int c, int) { return c < 32 ? a0[c] : a1[c - 32]; };
#elif TSG_JIT_NW == 32
    F32x32 a0 = {};  // comp.h:41
    TSG_JIT_CALL("+{" TSG_JIT_A0 "}"(a0));
    auto acc_of = [&](int c, int) { return a0[c]; };
#elif TSG_JIT_NW == 16
    F32x16 a0 = {};  // comp.h:41
    TSG_JIT_CALL("+{" TSG_JIT_A16 "}"(a0));
    auto acc_of = [&](int c, int) { return a0[c]; };
#else
    F32x8 a0 = {};  // comp.h:41
    TSG_JIT_CALL("+{" TSG_JIT_A8 "}"(a0));
    auto acc_of = [&](int c, int) { return a0[c]; };
#endif
#elif TSG_JIT_WAVES == 8 && TSG_JIT_NW == 64
    F32x32 a0 = {}, a1 = {}, a2 = {}, a3 = {};  // comp.h:41
    TSG_JIT_CALL("+{v[116:147]}"(a0), "+{v[148:179]}"(a1), "+{v[180:211]}"(a2), "+{v[212:243]}"(a3));
    auto acc_of = [&](int c, int r) {
        return c < 16 ? a0[2 * (c & 15) + r] : c < 32 ? a1[2 * (c & 15) + r]
             : c < 48 ? a2[2 * (c & 15) + r] : a3[2 * (c & 15) + r];
    };
#elif TSG_JIT_WAVES == 8 && TSG_JIT_NW == 32
    F32x32 a0 = {}, a1 = {};  // comp.h:41
    TSG_JIT_CALL("+{v[116:147]}"(a0), "+{v[148:179]}"(a1));
    auto acc_of = [&](int c, int r) { return c < 16 ? a0[2 * (c & 15) + r] : a1[2 * (c & 15) + r]; };
#elif TSG_JIT_WAVES == 8 && TSG_JIT_NW == 16
    F32x32 a0 = {};  // comp.h:41
    TSG_JIT_CALL("+{v[116:147]}"(a0));
    auto acc_of = [&](int c, int r) { return a0[2 * c + r]; };
#elif TSG_JIT_WAVES == 8
    F32x16 a0 = {};  // comp.h:41
    TSG_JIT_CALL("+{v[116:131]}"(a0));
    auto acc_of = [&](int c, int r) { return a0[2 * c + r]; };
#elif TSG_JIT_NW == 32  // 4 waves: accumulators from v122
    F32x32 a0 = {}, a1 = {};  // comp.h:41
    TSG_JIT_CALL("+{v[122:153]}"(a0), "+{v[154:185]}"(a1));
    auto acc_of = [&](int c, int r) { return c < 16 ? a0[2 * (c & 15) + r] : a1[2 * (c & 15) + r]; };
#elif TSG_JIT_NW == 16
    F32x32 a0 = {};  // comp.h:41
    TSG_JIT_CALL("+{v[122:153]}"(a0));
    auto acc_of = [&](int c, int r) { return a0[2 * c + r]; };
#else
    F32x16 a0 = {};  // comp.h:41
    TSG_JIT_CALL("+{v[122:137]}"(a0));
    auto acc_of = [&](int c, int r) { return a0[2 * c + r]; };
#endif
#undef TSG_JIT_CALL

    if (ncol0 >= N) return;
    if (kJPair && (lane >> 5) != rhalf) return;  // the pair's other wave holds these rows
#pragma unroll
    for (int r = 0; r < kJRowsPerLane; r++) {
        const int m = m0 + kJRowsPerLane * lane + r;
        if (m >= M) continue;
        float *yrow = Y + (size_t)m * N + ncol0;
        float v[kJNW];
#pragma unroll
        for (int c = 0; c < kJNW; c++) {
            const int n = ncol0 + c < N ? ncol0 + c : N - 1;
            const float acc = acc_of(c, r);
            float y = acc + b[n];                        // comp.h:63
            if (prelu) y = (y > 0) ? y : alpha[n] * y;   // comp_prelu.h:57-67
            v[c] = y;
        }
        if (ncol0 + kJNW <= N && (((uintptr_t)yrow & 15) == 0)) {  // float4 stores need 16-B alignment
#pragma unroll
            for (int c = 0; c < kJNW; c += 4)
                *reinterpret_cast<float4 *>(yrow + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
        } else {
#pragma unroll
            for (int c = 0; c < kJNW; c++)
                if (ncol0 + c < N) yrow[c] = v[c];
        }
    }
}
