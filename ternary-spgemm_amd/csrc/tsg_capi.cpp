// tsg_capi.cpp -- the C-ABI (include/ternary_spgemm.h): handle lifetime,
// device image upload, work buffers, launches, host-pointer convenience path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <atomic>
#include <iterator>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ternary_spgemm_test.h"
#include "tsg_internal.h"

extern thread_local std::string g_tsg_host_err;  // one per-thread message for the whole ABI

static int fail(int code, const std::string &msg)
{
    g_tsg_host_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(TSG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));  \
    } while (0)

struct tsg_tcsc {
    int K = 0, N = 0, device = 0;
    int B = 0;                            // BlockedTCSC<B> block size (0: plain TCSC)
    int64_t nnz_pos = 0, nnz_neg = 0;
    // kernel family: jit (weight-compiled, default) or rx (register-X walk:
    // images too large for 32-bit stream offsets, a failed image load, or
    // TSG_KERNEL=rx)
    enum Kind { kRx, kJit } kind = kJit;
    tsg::RxImage rimg;                    // device image of the rx kernel
    // jit kernel: one compiled image per (stream width, waves per workgroup)
    // (shape_index): the default shape at registration, others on the first
    // call with an M that picks them (or tcsc_hip_reserve)
    struct JitVariant {
        int nw = 0, waves = 0, Npad = 0;
        int piece_rows = 0;               // 64-row image: rows per DMA piece (its X^T layout; 0 = row layout)
        bool pair = false;                // 64-row 4-wave streams run by 8-wave workgroups of wave pairs
        int nch = 0, chunk = 0;           // X^T chunks of the image and K rows per chunk
        tsg::JitModule mod;               // dispatcher + generated code, loaded
        uint32_t *d_wcode = nullptr;      // per (column tile, stream): byte offset of its code
        int64_t code_bytes = 0, wcode_words = 0;
    };
    JitVariant jv[8];                     // 7: the 64 x 8 "far X^T" image (pick_jit_shape)
    JitVariant jv64[8];                   // the 64-row image (tsg_internal.h), shape_index 0..7
    JitVariant jv64h[3];                  // its half ring (kJit64HalfChunk): 4-wave widths 32, 16, 8
    int jit_nch = 0;                      // X^T chunks (all widths)
    int jit64_nch = 0;                    // X^T chunks of the 64-row image (192 rows each)
    int tile_rows = 0;                    // tcsc_hip_set_tile_rows: 0 auto, 128 or 64 (jit images)
    int jit_force = 0;                    // tcsc_hip_set_jit_width / TSG_JIT_NW: 0 = auto
    uint32_t *d_status = nullptr;         // jit dispatcher status word (nonzero: region check failed)
    // images that failed to load or probe at a call (bit variant_bit): calls
    // that pick them run the 128-row 64 x 8 image (loaded on that fallback)
    uint32_t bad_variants = 0;
    // small-M kernel (tsg_ell.hip): one sliced-ELL image per variant, built on
    // the first call (or tcsc_hip_reserve) that picks the variant
    struct EllVariant {
        tsg::EllImage img;                // host metadata (C, nch, ...); arrays freed after upload
        uint32_t *d_ent = nullptr, *d_tab = nullptr;
        int64_t bytes = 0;
        bool ready = false;
    };
    EllVariant ell[tsg::kEllVariants];
    int far_mode = 0;                     // tcsc_hip_set_far: 0 auto, 1 never, 2 always (64 x 8 calls)
    int small_m = 0;                      // tcsc_hip_set_small_m: 0 auto, 1 never, 2 always, 3 always w/o pc (plain TCSC only)
    std::vector<int32_t> csp, csn, rip, rin;  // host TCSC (getVectorRepresentation)
    uint32_t *d_seg = nullptr, *d_ent = nullptr;
    float *d_work = nullptr;              // X^T [Kp][Mp]
    size_t work_bytes = 0;
    // d_work is shared by every call on the handle: the last stream that read
    // it and an event recorded after that read; a call on another stream
    // waits for the event before it overwrites X^T (run_dev)
    hipStream_t work_stream = nullptr;
    hipEvent_t work_ev = nullptr;
    bool work_used = false;
    // host-pointer path staging (tcsc_hip_gemm): grow-only
    float *d_x = nullptr, *d_b = nullptr, *d_y = nullptr, *d_alpha = nullptr;
    size_t x_bytes = 0, y_bytes = 0;
    hipStream_t stream = nullptr;         // stream of the host-pointer path (compute)
    std::mutex host_mu;                   // one host-pointer call at a time (its staging buffers)
    // host-pointer pipeline (run_host): X chunks in on s_in, chunk compute on
    // `stream`, Y chunks out on s_out; one event pair per chunk
    static constexpr int kHostChunksMax = 16;
    hipStream_t s_in = nullptr, s_out = nullptr;
    hipEvent_t ev_in[kHostChunksMax] = {}, ev_c[kHostChunksMax] = {};
    int host_chunks = 0;                  // tcsc_hip_set_host_chunks: 0 = automatic
    // timing of the main kernel
    bool timing = false;
    static constexpr int kRing = 256;     // event pairs in flight before a harvest blocks
    hipEvent_t ev0[kRing] = {}, ev1[kRing] = {};
    int ring_head = 0, ring_count = 0;    // pending pairs: [head - count, head)
    double total_ms = 0.0;
    int64_t launches = 0;
    // run_dev, reserve and the setters write the plan state (bad_variants,
    // JitVariant, pins) under it; the const per-call queries read under it too
    mutable std::mutex mu;
};

namespace {

// Largest M the automatic choice sends to the small-M (ELL) kernel (see
// pick_ell_variant), the variant with 8-row tiles, and the M up to which
// 8-row tiles are used.
constexpr int kEllAutoMaxM = 32;
constexpr int kEllAutoMaxMChunked = 16;
constexpr int kEllTile8 = 2;
constexpr int kEllMidM = 32;
constexpr int64_t kEllPcRowsMaxMN = 32768;
constexpr int kEllStarvedMaxM = 1024;
constexpr int kEllSmallWMaxM = 128;          // small W: the walk up to this M ...
constexpr double kEllSmallWWork = 420e6;     // ... while M x nnz stays below this
// M up to which the automatic choice always takes the 64-row image, and the
// filled fraction of its last round below which the 128-row image's widest
// shape loses to it (pick_rows64)
constexpr int kRows64AutoMaxM = 512;
constexpr double kRows64FullRound = 0.9;
constexpr int64_t kJitFullWgs = 230;
constexpr int64_t kJitOneRoundWgs = 256;  // one jit workgroup per CU (144 KiB of LDS)
constexpr double kFarXtBytes = 768.0 * 1024 * 1024;  // X^T >= 3x the 256 MiB Infinity Cache
constexpr double kFarCodeBytes = 160.0 * 1024 * 1024;  // code image well inside it
constexpr double kFarKeepXtBytes = 1536.0 * 1024 * 1024;  // X^T >= 6x it: the far image beats the staged 64-row one
constexpr double kXDirectMinAddsPerRow = 32.0;  // 64-row image: direct X from width x density >= this
constexpr int64_t kEllStarvedWgs = 64;
constexpr double kXTouchMaxXBytes = 384.0 * 1024 * 1024;        // pick_xtouch
constexpr double kXTouchDenseMaxXBytes = 1024.0 * 1024 * 1024;  // (dense W)
// the 64-row image's step when it cannot read X directly: its X^T staging
// launch (tsg_transpose_rows_kernel) ahead of the image, at the walk's M
// (X <= 20 MB) -- r06_staged_floor_ab.jsonl
constexpr double kStagedXtUs = 5.0;
static_assert(tsg::kEllTileM[kEllTile8] == 8, "kEllTile8 is the 8-row tile");

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int check_device(int dev)
{
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return fail(TSG_ERR_NODEV, "hipGetDeviceProperties failed for device " + std::to_string(dev));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(TSG_ERR_NODEV, std::string("device is ") + prop.gcnArchName +
                                       "; this library is built for gfx950 (MI355X) only");
    return TSG_OK;
}

// X^T dimensions of a call with M rows: rows padded to the M tile, K to
// whole chunks (64-row image: k-quad layout, 64-row tiles, 192-row chunks)
int dims_for(const tsg_tcsc *h, int M, int &Mp, int &Kp, bool r64 = false, bool half = false)
{
    const bool jit = h->kind == tsg_tcsc::kJit;
    const int tm = !jit ? tsg::kRxTileM : r64 ? tsg::kJit64TileM : tsg::kJitTileM;
    Mp = ((std::max(M, 1) + tm - 1) / tm) * tm;
    const int c64 = tsg::jit64_chunk(half);
    const int nch64 = std::max(1, (h->K + c64 - 1) / c64);
    Kp = !jit ? h->rimg.nch * tsg::kRxChunk : r64 ? nch64 * c64 : h->jit_nch * tsg::kJitChunk;
    return TSG_OK;
}

// Grows the X^T work buffer (grow-only).  A grow frees the old buffer, so it
// first waits for every launch that may still read it; it cannot happen while
// a stream is being captured (tcsc_hip_reserve(max_M) before the capture).
int ensure_work(tsg_tcsc *h, int M, bool capturing, bool r64 = false, bool half = false)
{
    int Mp, Kp;
    dims_for(h, M, Mp, Kp, r64, half);
    const size_t need = (size_t)Mp * Kp * sizeof(float);
    if (need <= h->work_bytes) return TSG_OK;
    if (capturing)
        return fail(TSG_ERR_ARG, "M=" + std::to_string(M) + " needs a larger work buffer during stream capture; "
                                 "call tcsc_hip_reserve(h, max_M) before capturing");
    if (h->d_work) {
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipFree(h->d_work));
    }
    h->d_work = nullptr;
    h->work_bytes = 0;
    h->work_used = false;
    if (hipMalloc(&h->d_work, need) != hipSuccess)
        return fail(TSG_ERR_NOMEM, "hipMalloc of " + std::to_string(need) + " B work buffer failed");
    h->work_bytes = need;
    return TSG_OK;
}

// Folds finished event pairs into the totals.  `all` waits for every pending
// pair; otherwise only the oldest is waited for (ring full).
int harvest_timing(tsg_tcsc *h, bool all)
{
    int todo = all ? h->ring_count : (h->ring_count == tsg_tcsc::kRing ? 1 : 0);
    while (todo-- > 0) {
        const int i = (h->ring_head - h->ring_count + tsg_tcsc::kRing) % tsg_tcsc::kRing;
        HIP_TRY(hipEventSynchronize(h->ev1[i]));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, h->ev0[i], h->ev1[i]));
        h->total_ms += ms;
        h->launches += 1;
        h->ring_count--;
    }
    return TSG_OK;
}

int ensure_events(tsg_tcsc *h)
{
    if (h->ev0[0]) return TSG_OK;
    for (int i = 0; i < tsg_tcsc::kRing; i++) {
        HIP_TRY(hipEventCreate(&h->ev0[i]));
        HIP_TRY(hipEventCreate(&h->ev1[i]));
    }
    return TSG_OK;
}

int width_index(int nw)
{
    for (int i = 0; i < 4; i++)
        if (tsg::kJitWidths[i] == nw) return i;
    return -1;
}

// jv index of a (width, waves) shape: 8-wave widths 0..3, 4-wave widths
// 32/16/8 4..6, the 64 x 8 far-X^T image 7; jv64 (the 64-row image): the
// same 0..6 and 128 x 8 at 7
int shape_index(int nw, int waves, bool far = false)
{
    if (nw == tsg::kJit64WideNW) return waves == tsg::kJitWaves && !far ? 7 : -1;
    const int w = width_index(nw);
    if (w < 0 || !tsg::jit_waves_ok(nw, waves) || (far && (nw != tsg::kJitNW || waves != tsg::kJitWaves))) return -1;
    return far ? 7 : waves == tsg::kJitWaves ? w : 3 + w;
}

struct JitShape {
    int nw, waves;
    bool far = false;  // the far-X^T code image (tsg_jit.cpp build_jit_code)
    bool r64 = false;  // the 64-row image (tsg_internal.h)
    bool half = false; // its half ring (4-wave shapes; tsg_internal.h kJit64HalfChunk)
};
int shape_index(const JitShape &sh) { return shape_index(sh.nw, sh.waves, sh.far && !sh.r64); }

tsg_tcsc::JitVariant &variant_of(tsg_tcsc *h, const JitShape &sh)
{
    if (sh.r64 && sh.half) return h->jv64h[width_index(sh.nw) - 1];
    return sh.r64 ? h->jv64[shape_index(sh.nw, sh.waves)] : h->jv[shape_index(sh)];
}

// bit of a shape in tsg_tcsc::bad_variants: 128-row 0..7, 64-row 8..15, half ring 16..18
int variant_bit(const JitShape &sh)
{
    return sh.r64 && sh.half ? 16 + width_index(sh.nw) - 1 : (sh.r64 ? 8 : 0) + shape_index(sh);
}

// Shape (stream width x waves per workgroup) for a call with M rows.  Every
// shape walks the same X^T chunks; a wider stream reads fewer LDS bytes per
// add (32 / width: an X pair read feeds width x 2 rows x d adds), and a
// workgroup needs a CU.  Rule (measured, profiles/r02w4_waves_ab.txt,
// r02_ref_cases.jsonl): the widest stream among the shapes that still give
// >= 230 workgroups (~90% of the CUs: (16000, 1024, 1024) runs 64 x 8 on 250,
// 0.116 ms, not 32 x 8 on 500, 0.141 ms), 8 waves before 4 at equal width;
// if none does, the most workgroups.  configs[1]
// (M = 512, N = 4096): 16 columns x 4 waves, 0.105 ms (8 x 8: 0.120);
// M = 256, N = 16384: 32 x 4, 0.153 ms (16 x 8: 0.173); M >= 1024: 64 x 8.
// A pinned width (tcsc_hip_set_jit_width) runs 8 waves; TSG_JIT_WAVES=4 forces
// 4 waves for every narrow width (diagnostic).
// The far-X^T image (no code touches, non-temporal X^T staging) for 64-wide
// calls on the 1 x 32 tile map (long streams: K >= 8192, density > 3/16, more
// than 4 column and 8 M tiles, pick_jit_map) whose X^T is far larger than the
// 256 MiB Infinity Cache while the code fits in it: the X^T stream then no
// longer evicts the code that every M tile of the XCD re-reads
// (profiles/r03e_far_ab.txt, r03e_long_k_ab.txt, r03e_big_ab.txt, kernel ms):
// (64000, 16384, 4096) s = 4 25.3-26.2 -> 21.6-22.2, (32000, 16384, 4096)
// 12.3-12.4 -> 10.8-10.9, (16000, 16384, 4096) 5.9-6.1 -> 5.35-5.43,
// (64000, 8192, 4096) 11.4-11.8 -> 10.8-10.9; it loses where X^T fits the
// cache ((4096, 16384, 4096) 1.17 -> 1.50, (8192, ...) 2.63 -> 2.77), where
// the code does not (s = 2: 38.9 -> 42.0) and on sparse W (s = 8 / 16: 4.9-9%
// slower; those run the 4 x 8 map).  TSG_JIT_FAR=0/1 overrides.
bool far_xt(const tsg_tcsc *h, int M)
{
    static const int env = [] { const char *e = tsg::knob_value("TSG_JIT_FAR"); return e ? atoi(e) : -1; }();
    if (h->B || h->far_mode == 1) return false;
    if (h->far_mode == 2) return true;
    if (h->jit_force) return false;
    if (env >= 0) return env > 0;
    const double nnz = (double)(h->nnz_pos + h->nnz_neg), density = nnz / std::max(1.0, (double)h->K * h->N);
    const int64_t mtiles = ((int64_t)M + tsg::kJitTileM - 1) / tsg::kJitTileM,
                  ntiles = ((int64_t)h->N + tsg::kJitTileCols - 1) / tsg::kJitTileCols;
    const bool long_map = h->K >= 8192 && density > 0.1875 && ntiles > 4 && mtiles > 8;
    return long_map && 4.0 * (double)M * (double)h->K >= kFarXtBytes && 8.0 * nnz <= kFarCodeBytes;
}

// The 64-row image can stage its pieces straight from row-major X (PR rows x
// 1024 / PR contiguous bytes each; tsg_internal.h) when rows start 16-B
// aligned (X 16-B aligned, K % 4 == 0), no piece straddles K (K % (256 / PR)
// == 0: pieces at or past K are omitted, so nothing reads past a row's end)
// and the per-lane offsets fit 32 bits.  Every workgroup of an M tile then
// gathers the same rows, 4K bytes apart, chunk after chunk: that costs more
// than the X^T pass unless a step's work is long enough to hide it -- so
// automatic only for streams of >= 32 adds per k row per wave (width x
// density: 128 columns at s <= 4, 64 at s <= 2).  Measured (kernel / step
// us): configs[2] on 128 x 8 1231.4 / 1239.4 direct vs 1230.4 / 1273.0 staged
// (profiles/r04z_direct_big_ab.jsonl); but s = 16 on 128 x 8 530.7 / 539.5 vs
// 463.3 / 505.8, configs[1] on 16 x 8 94.3 / 101.0 vs 68.5 / 84.3, and K =
// 4096, N = 16384: M = 64 (16 x 4) 85.2-85.7 / 91.6-92.4 vs 65.5-65.9 /
// 78.9-79.5, M = 512 (64 x 8, s = 4) 208-209 / 215 vs 202-205 / 217-220
// (r04f_shape_ab.jsonl, r04g_bound_ab.jsonl).  TSG_JIT_XDIRECT=1 / 0 forces it
// on (where possible) / off, read per call (A/B).
// Row layout (round 5, tsg_internal.h kJit64RowFlag): its pieces read runs of
// contiguous row bytes, as fast from X as from the staged copy
// (profiles/r05_dma_stride_micro.txt), so every call that can reads X
// directly (K >= 188, K % 4 == 0, X 16-B aligned): no X^T pass, no work
// buffer.  The blocked layout keeps the round-4 rule above.
bool x_direct_auto(const tsg_tcsc *h, int nw, int piece_rows)
{
    if (piece_rows == 0) return true;
    const double density = (double)(h->nnz_pos + h->nnz_neg) / std::max(1.0, (double)h->K * (double)h->N);
    return (double)nw * density >= kXDirectMinAddsPerRow;
}

// K (and X) allow direct X for a 64-row image with this piece shape
bool x_direct_shape_ok(int K, int piece_rows)
{
    return piece_rows == 0 ? K >= tsg::kJit64RowChunk && K % 4 == 0 : K > 0 && K % (256 / piece_rows) == 0;
}

// the dispatcher's per-lane X offsets are 32-bit
bool x_direct_offsets_ok(int M, int K) { return (int64_t)M * K * 4 + 4096 < ((int64_t)1 << 32); }

bool x_direct(const tsg_tcsc *h, const float *dX, int M, int K, const tsg_tcsc::JitVariant &jv)
{
    const char *e = tsg::knob_value("TSG_JIT_XDIRECT");
    const bool on = e ? e[0] == '1' : x_direct_auto(h, jv.nw, jv.piece_rows);
    return on && x_direct_shape_ok(K, jv.piece_rows) && ((uintptr_t)dX & 15) == 0 && x_direct_offsets_ok(M, K);
}

JitShape pick_jit_shape(const tsg_tcsc *h, int M, bool r64 = false);

// The 64-row image (VOP2 adds, one M row per lane) or the 128-row one
// (v_pk_add_f32, two rows per lane) for a call with M rows (that the small-M
// walk does not take); BlockedTCSC runs the 128-row image only.  Measured
// (profiles/r04f_shape_ab.jsonl, r04g_bound_ab.jsonl, r04h_big_ab.jsonl; step
// us, X staged for both): the 64-row image wins at every M <= 512 (K = 4096,
// N = 16384: M = 64 79 vs 121, M = 192 130 vs 163, M = 512 217 vs 243;
// configs[1] 108 vs 116) and above that wherever the 128-row image's shape is
// narrower than 64 x 8 or leaves a round partly empty (N = 16384: M = 640 336
// vs 385, M = 1536 547 vs 617; N = 8192, M = 1024 204 vs 236; N = 4096, M =
// 2048 224 vs 245; K = 16384, N = 4096, M = 2048 806 vs 973); the 128-row
// image keeps the calls its widest shape fills in whole rounds (configs[2]
// 1360 vs 1437, N = 16384 M = 1024 339 vs 358, N = 8192 M = 4096 686 vs 708,
// s = 8 / 16 862 / 637 vs 880 / 661) -- against its 64-wide streams.  At 128
// columns per wave (round 4, profiles/r04l_w128_ab.jsonl, kernel / step us)
// the 64-row image wins those too wherever that shape is its modelled best:
// configs[2] 1286 / 1329 vs 1350 / 1387, s = 8 748 / 790 vs 841 / 886, s = 16
// 500 / 542 vs 609 / 651, N = 16384 M = 1024 320 / 337 vs 331 / 347, M =
// 2048 643 / 664 vs 660 / 685, N = 8192 M = 4096 623 vs 655, configs[2] s = 2
// 2403 vs 2465, (16000, 8192, 2048) 1219 vs 1302, (8192, 16384, 4096) 2467
// vs 2833, (64000, 16384, 4096) s = 8 / 16 11.2 / 7.2 vs 14.3 / 8.7 ms (one
// loss: M = N = K = 4096 361 vs 353); the far-X^T image and dense W over
// long K stay 128-row.
// tcsc_hip_set_tile_rows pins one; TSG_JIT_ROWS64_MAXM replaces the rule by
// M <= its value (A/B).
bool pick_rows64(const tsg_tcsc *h, int M)
{
    static const int env_max = [] {
        const char *e = tsg::knob_value("TSG_JIT_ROWS64_MAXM");
        return e ? atoi(e) : -1;
    }();
    if (h->B || h->kind != tsg_tcsc::kJit) return false;
    if (h->tile_rows) return h->tile_rows == 64;
    if (h->jit_force == tsg::kJit64WideNW) return true;  // only the 64-row image has that width
    if (env_max >= 0) return M <= env_max;
    if (M <= kRows64AutoMaxM) return true;
    const JitShape s = pick_jit_shape(h, M, false);
    // Round 4 kept two regimes on the 128-row image: the far-X^T image where
    // X^T is >= 8x the Infinity Cache ((64000, 16384, 4096) s = 4 22.1 vs 24.3
    // ms) and dense W over long K ((64000, 16384, 4096) s = 2 39.0 vs 50.6,
    // profiles/r04p_far_ab.jsonl, r04m_w128_big.jsonl).  Round 5's 64-row
    // image reads X directly and takes the long-stream map there too
    // (pick_jit_map), and wins both (step ms, each image in its own process,
    // r05z_longk_maps_ab.jsonl, r05z_longk_maps2_ab.jsonl): (64000, 16384,
    // 4096) s = 4 18.87-19.00 vs 23.37-23.93, s = 2 37.99 vs 39.57; (32000,
    // ...) s = 4 9.40-9.49 vs 12.05-12.15; (8192, ...) s = 2 4.76 vs 4.94.
    const double density = (double)(h->nnz_pos + h->nnz_neg) / std::max(1.0, (double)h->K * (double)h->N);
    // 128 columns per wave fill whole rounds: twice the adds per staged chunk
    // and per X read of either 64-wide stream (profiles/r04l_w128_ab.jsonl,
    // r04m_w128_big.jsonl) -- for sparse W or long K, and for dense W over
    // short K when its stream reads X directly (x_direct): there the kernels
    // depend on the data (r04o_xdata_ab.jsonl, kernel us: with bench.py's
    // small-integer X the 128-row image runs configs[2] in 1197 vs 1232, with
    // full-mantissa X 1277 vs 1252 -- v_pk_add_f32 slows on high-entropy data,
    // the VOP2 stream hardly), and the 64-row image's step saves the X^T pass:
    // configs[2] 1239.4 vs 1248.8 us per step with integer X
    // (r04z_direct_big_ab.jsonl); the sparse end is the 64-row image's either
    // way (s = 16: 468 vs 569 int, 496 vs 600 frac).
    // x_direct's own limits that M and K decide (the 32-bit per-lane offsets:
    // X below 4 GiB); X's alignment is checked per call
    const bool direct_capable = x_direct_shape_ok(h->K, tsg::jit64_piece_rows()) &&
                                x_direct_auto(h, tsg::kJit64WideNW, tsg::jit64_piece_rows()) &&
                                x_direct_offsets_ok(M, h->K);
    // round 5: whenever the 64-row image reads X directly (the row layout: K
    // >= 188, K % 4 == 0) its call is one launch, while the 128-row image's
    // step adds its X^T pass -- the 128-row image's whole-round shapes below
    // lose their step too (r05z_n512_ab.jsonl, step us, M = 64000, N = 512:
    // K = 4096 s = 4 693 vs 1093, K = 16384 2690 vs 4244, K = 1024 s = 16 170
    // vs 261)
    if (direct_capable) return true;
    // X past the 32-bit offsets: both images stage X, as in round
    // 4, whose two rules for that regime stand -- the far-X^T image (128-row
    // only) where X^T is >= 6x the Infinity Cache ((64000, 16384, 4096) 22.1
    // vs 24.3 ms for the 64-row 128 x 8, profiles/r04p_far_ab.jsonl), and the
    // 128-row long-stream map for dense W over long K with few columns
    // ((64000, 16384, 4096) s = 2 39.0 vs 50.6 ms, r04m_w128_big.jsonl)
    if (x_direct_shape_ok(h->K, tsg::jit64_piece_rows()) && !x_direct_offsets_ok(M, h->K)) {
        if (s.far && 4.0 * (double)M * (double)h->K >= kFarKeepXtBytes) return false;
        if (h->K >= 16384 && h->N <= 8192 && density > 0.375) return false;
    }
    if ((density <= 0.1875 || h->K >= 8192) && pick_jit_shape(h, M, true).nw == tsg::kJit64WideNW) return true;
    if (s.nw != tsg::kJitNW || s.waves != tsg::kJitWaves) return true;
    const int64_t wgs = (int64_t)((M + tsg::kJitTileM - 1) / tsg::kJitTileM) *
                        ((h->N + (int64_t)s.waves * s.nw - 1) / ((int64_t)s.waves * s.nw));
    const int64_t rounds = (wgs + kJitOneRoundWgs - 1) / kJitOneRoundWgs;
    return (double)wgs < kRows64FullRound * (double)(rounds * kJitOneRoundWgs);
}

JitShape pick_jit_shape(const tsg_tcsc *h, int M, bool r64)
{
    static const int env_waves = [] {
        const char *e = tsg::knob_value("TSG_JIT_WAVES");
        return e ? atoi(e) : 0;
    }();
    if (h->B) return {tsg::kJitNW, tsg::kJitWaves};
    // the 64-row image's half ring for its 4-wave shapes (TSG_JIT_HALF=1, read per call: A/B)
    const char *hv = r64 ? tsg::knob_value("TSG_JIT_HALF") : nullptr;
    const bool half_on = hv && hv[0] == '1';
    if (h->jit_force) {
        const int f = !r64 && h->jit_force == tsg::kJit64WideNW ? tsg::kJitNW : h->jit_force;
        const int w = env_waves == 4 && tsg::jit_waves_ok(f, 4) ? 4 : tsg::kJitWaves;
        return {f, w, !r64 && f == tsg::kJitNW && w == tsg::kJitWaves && far_xt(h, M), r64, r64 && w == 4 && half_on};
    }
    const int tile_m = r64 ? tsg::kJit64TileM : tsg::kJitTileM;
    const int64_t mt = (std::max(M, 1) + tile_m - 1) / tile_m;
    const double image8 = (r64 ? 4.0 : 8.0) * (double)(h->nnz_pos + h->nnz_neg);
    if (r64) {
        // 64-row image: the shape with the least modelled time = rounds of
        // one-workgroup-per-CU x the time of a workgroup, which grows with the
        // columns a SIMD carries (width x waves / 4) scaled by density, over a
        // fixed part (the K sweep's staging and barriers).  A lone wave per
        // SIMD (4-wave workgroups) issues its VOP2 adds at half the rate of a
        // pair, and 8-column streams feed few adds per X read.  Fitted on
        // one-round grids at K = 4096, s = 4 with X staged
        // (profiles/r04j_waves_ab.jsonl, kernel us): configs[1] 16 x 8 79.6 vs
        // 32 x 4 92.8; M = 128, N = 16384: 16 x 8 87.1 vs 32 x 4 91.3-96.7;
        // M = 64: 16 x 4 66.2 vs 8 x 8 76.0; M = 256, N = 4096: 16 x 4
        // 56.1-58.9 vs 8 x 8 59.3.  A fractional round costs a whole one
        // (M = 192: 32 x 4 on 384 workgroups 178 us; one round of 32 x 8 123).
        // Ties go to the wider stream (fewer LDS reads per add).
        const double dens4 = 4.0 * (double)(h->nnz_pos + h->nnz_neg) / std::max(1.0, (double)h->K * (double)h->N);
        JitShape pick{tsg::kJitNW, tsg::kJitWaves, false, true};
        double best_cost = 0.0;
        bool any = false;
        for (int nw : tsg::kJit64Widths)
            for (int waves : {tsg::kJitWaves, 4}) {
                if (!tsg::jit_waves_ok(nw, waves)) continue;
                if (env_waves == 4 && nw < tsg::kJitNW && waves != 4) continue;
                const int64_t ntile = (h->N + (int64_t)waves * nw - 1) / ((int64_t)waves * nw), wgs = mt * ntile;
                const double image = image8 + (double)ntile * waves * h->jit_nch * 2 * (160.0 + 8.0 * tsg::kJitChunk);
                if (nw != tsg::kJitNW && image > 2.0 * (double)(1ull << 30)) continue;
                const double rounds = (double)((wgs + kJitOneRoundWgs - 1) / kJitOneRoundWgs);
                const double adds = (double)nw * waves / 4.0 * dens4 * (waves == 4 ? 1.35 : 1.0);
                const double cost = rounds * (48.0 + adds + (nw == 8 ? 10.0 : 0.0));
                if (!any || cost < best_cost) {
                    any = true;
                    best_cost = cost;
                    pick = {nw, waves, false, true};
                }
            }
        pick.half = pick.waves == 4 && half_on;
        return pick;
    }
    JitShape best{tsg::kJitNW, tsg::kJitWaves}, most{tsg::kJitNW, tsg::kJitWaves};
    int64_t most_wgs = -1;
    bool full = false;
    for (int nw : tsg::kJitWidths) {
        for (int waves : {tsg::kJitWaves, 4}) {
            if (!tsg::jit_waves_ok(nw, waves)) continue;
            if (env_waves == 4 && nw != tsg::kJitNW && waves != 4) continue;
            const int64_t ntile = (h->N + (int64_t)waves * nw - 1) / ((int64_t)waves * nw), wgs = mt * ntile;
            // narrow streams repeat the reads and step scaffolding per stream:
            // keep the image inside the 32-bit stream offsets
            const double image = image8 + (double)ntile * waves * h->jit_nch * 2 * (160.0 + 8.0 * tsg::kJitChunk);
            if (nw != tsg::kJitNW && image > 2.0 * (double)(1ull << 30)) continue;
            if (!full && wgs >= kJitFullWgs) {  // widths come widest first
                best = {nw, waves};
                full = true;
            }
            if (wgs > most_wgs) {
                most_wgs = wgs;
                most = {nw, waves};
            }
        }
    }
    JitShape sh = full ? best : most;
    sh.far = !r64 && sh.nw == tsg::kJitNW && sh.waves == tsg::kJitWaves && far_xt(h, M);
    sh.r64 = r64;
    return sh;
}

// The image and shape a jit call with M rows runs: the automatic (or pinned)
// pick, unless that image failed to load at an earlier call -- then the
// 128-row 64 x 8 image (run_dev's fallback, which loads it).
// A call may fall back from an image that cannot be loaded to the 128-row
// 64 x 8 image when nothing pinned its image or shape (a pinned request fails
// loudly instead: TSG_ERR_HIP).
bool may_fall_back(const tsg_tcsc *h, const JitShape &sh)
{
    const bool is_default = !sh.r64 && !sh.far && sh.nw == tsg::kJitNW && sh.waves == tsg::kJitWaves;
    return !is_default && !h->tile_rows && !h->jit_force && h->far_mode != 2 &&
           !tsg::knob_value("TSG_JIT_ROWS64_MAXM") && !tsg::knob_value("TSG_JIT_NW");
}

// The generated code's per-group code touches (tsg_jit.cpp, round 6: a 128-
// wide dense stream writes more code per step than the step's one 8-KiB
// touch covers) run where they were measured to pay: X of at most 384 MiB
// (~1.5x the Infinity Cache), and dense W (s <= 2: steps of ~25 KiB of code)
// with X up to 1 GiB.  With large X they cost more than they save
// (profiles/r06h_tgroup_longk_ab.jsonl, kernel us: (16000, 16384, 4096) s = 4
// 5221 vs 4727 off, (16000, 8192, 2048) s = 4 1371 vs 1203;
// r06i_xtouch_big_ab.jsonl: (64000, 16384, 4096) s = 2 34.2-46.5 ms, unsteady,
// vs 38.0-38.4 off) -- but (4096, 16384, 4096) 1115 vs 1192, configs[2] 1157
// vs 1221, (16000, 8192, 2048) s = 2 2152 vs 2394.  Elsewhere the dispatcher
// points them all at one line.  TSG_JIT_XTOUCH=0|1 forces it (A/B, per call).
bool pick_xtouch(const tsg_tcsc *h, int M)
{
    if (const char *e = tsg::knob_value("TSG_JIT_XTOUCH")) return e[0] == '1';
    const double density = (double)(h->nnz_pos + h->nnz_neg) / std::max(1.0, (double)h->K * (double)h->N);
    const double xbytes = 4.0 * (double)M * (double)h->K;
    return xbytes <= kXTouchMaxXBytes || (density > 0.375 && xbytes <= kXTouchDenseMaxXBytes);
}

// The code-touch window (tsg_jit.cpp: 8 KiB, from 8 KiB ahead of the step's
// position) starts at the step's own position instead -- the dispatcher
// moves the touch base back 8 KiB -- for 64-row calls with at most 2 M
// tiles, and on 4-wave workgroups: with few M tiles each code line is
// fetched by few workgroups, much of it straight from HBM, and the nearer
// window pays (profiles/r06j_touch_small_ab.jsonl, r06p_touch_8w_ab.jsonl,
// kernel us: M = 64 / 48, N = 16384 (16 x 4) 58.9 / 57.4 -> 51.7 / 50.0,
// M = 128 (16 x 8, 2 M tiles) 74.3 -> 64.4, (64, 2048, 8192) s = 2 32.1 ->
// 28.6, (1024, 4096, 1024) (16 x 4) 56.1 -> 54.9; M = 192 (3 tiles) -1%,
// configs[1] (8 tiles) +1%, (256, 4096, 8192) a tie).  TSG_JIT_TNEAR=0|1
// forces it (A/B, read per call).
bool pick_tnear(bool r64, int waves, int mtiles)
{
    if (const char *e = tsg::knob_value("TSG_JIT_TNEAR")) return e[0] == '1';
    return r64 && (mtiles <= 2 || waves == 4);
}

JitShape call_shape(const tsg_tcsc *h, int M)
{
    const JitShape sh = pick_jit_shape(h, M, pick_rows64(h, M));
    if (((h->bad_variants >> variant_bit(sh)) & 1u) && may_fall_back(h, sh)) return JitShape{tsg::kJitNW, tsg::kJitWaves};
    return sh;
}

// Tile map groups (tsg_jit_map.h) per call: gn column tiles x gm M tiles per
// XCD group, 32 workgroups (the XCD's CUs).  Measured
// (profiles/r03_map_density_ab.txt, r02_jit_map_bench_ab.txt):
//  * with at most 4 column tiles or 8 M tiles, 4 x 8: every column tile, or
//    every M tile, of the XCD's group shares its X^T chunks or code
//    ((16000, 8192, 2048) 1.19-1.21 vs 1.31-1.34 ms at 2 x 16);
//  * sparse W (density <= 3/16, s >= 8): 4 x 8 -- a column tile's code is
//    short, so sharing each X^T slab between more column tiles wins (s = 16:
//    0.565 vs 0.604 ms at 2 x 16; s = 8: 0.769 vs 0.792);
//  * long streams (K >= 8192, density > 3/32): 1 x 32, every CU of the XCD on
//    one column tile's code ((64000, 16384, 4096): 25.6 vs 26.8 ms; s = 8
//    13.7 vs 15.3-15.8 ms);
//  * otherwise 2 x 16: the CU pairs that share an instruction cache on one
//    code stream (configs[2] 1.212 ms vs 1.264 at 4 x 8; s = 2 2.554 vs 2.712).
// Code touches (tsg_jit_kernel.hip): only M tiles with (mt & tmask) == 0
// spread theirs over the stream's lines.  When the whole grid is resident at
// once (<= 256 workgroups: one per CU) and >= 4 M tiles share each stream,
// those M tiles run together, so one touch in four serves them (profiles/
// r03e_touch_ab.txt, r03e_long_k_ab.txt: configs[1] 0.0989-0.1013 -> 0.0931-
// 0.0938 ms, (1024, 4096, 1024) 0.0878 -> 0.0834, (1024, 16384, 1024) 0.317 ->
// 0.303); with several rounds the touching tile may not run beside the others
// (configs[2] +4%, s = 16 +15%), and with 2 M tiles per stream it loses too
// ((256, 4096, 16384) +7-17%, r03g_ref_cases.jsonl), so every tile touches.
// TSG_JIT_GN / TSG_JIT_GM / TSG_JIT_TMASK override (A/B).
void pick_jit_map(const tsg_tcsc *h, int mtiles, int ntiles, int &gn, int &gm, int &tmask, int nw = 0)
{
    static const int env_gn = [] { const char *e = tsg::knob_value("TSG_JIT_GN"); return e ? atoi(e) : 0; }();
    static const int env_gm = [] { const char *e = tsg::knob_value("TSG_JIT_GM"); return e ? atoi(e) : 0; }();
    static const int env_tm = [] { const char *e = tsg::knob_value("TSG_JIT_TMASK"); return e ? atoi(e) : -1; }();
    const double density = (double)(h->nnz_pos + h->nnz_neg) / std::max(1.0, (double)h->K * (double)h->N);
    // the 64-row image's 128-wide streams thin their touches over several
    // rounds too: configs[2] 1.2243-1.2252 vs 1.2315-1.2317 ms kernel, three
    // alternating bench runs each (profiles/r04t_tmask_bench_ab.txt); configs[3]
    // s = 8 / 16 680.6-681.2 / 444.3-448.1 vs 684.7-690.5 / 458.2-462.8 us
    // (r04t_tmask_sparse_ab.txt); (16000, 8192, 2048) s = 4 / 8 1227-1239 /
    // 729-735 vs 1248-1261 / 739-749 us (r04t_tmask_long_ab.txt; (8192, 16384,
    // 4096) within its run-to-run spread) -- but not for sparse W over long K
    // (round 5, direct X on the row layout, kernel us, r05p_tmask_long_ab.jsonl):
    // (64000, 16384, 4096) s = 8 / 16 14640 / 8310 thinned vs 10796 / 7020
    // with every tile touching, (16000, 8192, 2048) s = 8 / 16 799 / 532 vs
    // 726 / 494; (8192, 16384, 4096) s = 4 a tie (2359 vs 2355)
    const bool wide_short = nw == tsg::kJit64WideNW && (h->K < 8192 || density > 0.1875);
    tmask = env_tm >= 0 ? env_tm
                        : (((int64_t)mtiles * ntiles <= kJitOneRoundWgs || wide_short) && mtiles >= 4 ? 3 : 0);
    int n = 2, m = 16;
    // s = 8 over long K takes the long-stream map ((64000, 16384, 4096) s = 8:
    // 13.72-13.73 ms vs 15.3-15.8 at 4 x 8, profiles/r03f_sparse_big_ab.txt);
    // s = 16 stays on 4 x 8 (8.38-8.45 vs 11.66 at 1 x 32)
    const bool long_sparse = h->K >= 8192 && density > 0.09375;
    // round 5: the 64-row image's 128-wide streams over K >= 16384 with dense
    // W (s <= 4) take the long-stream map even on <= 4 column tiles -- an XCD
    // on one tile's code, 32 M tiles in step through it (profiles/
    // r05z_longk_maps_ab.jsonl, step ms, 1 x 32 vs 4 x 8: (64000, 16384,
    // 4096) s = 2 / 4 37.99 / 18.87 vs 50.15 / 24.71, (16000, ...) s = 4 4.73
    // vs 4.94, (8192, ...) s = 2 4.76 vs 4.92, s = 4 and (4096, ...) ties;
    // s = 8 stays 4 x 8: 10.90 vs 12.99; K = 8192, N = 2048 too: 1.19 vs 1.41)
    // (and K = 8192 with >= 4 column tiles: (64000, 8192, 4096) s = 4 10.91 vs
    // 12.86, (32000, 8192, 4096) s = 2 9.08 vs 12.20; with 2 column tiles 4 x 8
    // (gn = 2) stays: (64000, 8192, 2048) a tie, (16000, 8192, 2048) 1.19 vs
    // 1.41; r05z_k8192_maps_ab.jsonl)
    // The 64-row image takes the long-stream map only with >= 64-column
    // streams and >= 32 M tiles (a full group): narrower streams and half
    // groups run faster on 4 x 8 (r05z_midm_longk_maps_ab.jsonl, us, 4 x 8
    // vs 1 x 32 / 1 x 16: (1024, 16384, 4096) 32 x 8 374 vs 471, (2048, 8192,
    // 1024) s = 2 16 x 8 165 vs 210, (1024, 8192, 16384) 128 x 8 600 vs 630;
    // the long map (2048, 16384, 4096) 64 x 8 622 vs 709, (2048, 16384,
    // 16384) s = 2 4929 vs 6014)
    const bool long_ok = nw == 0 || (nw >= 64 && mtiles >= 32);
    const bool long_dense_wide = nw == tsg::kJit64WideNW && h->K >= 8192 && density > 0.1875 && mtiles >= 32 &&
                                 (h->K >= 16384 || ntiles >= 4);
    if (!long_dense_wide && (ntiles <= 4 || mtiles <= 8 || (density <= 0.1875 && !long_sparse))) {
        n = 4;
        m = 8;
    } else if (h->K >= 8192) {
        n = long_dense_wide || long_ok ? 1 : 4;
        m = long_dense_wide || long_ok ? 32 : 8;
    }
    gn = std::min(env_gn > 0 ? env_gn : n, std::max(ntiles, 1));  // a group never exceeds the grid
    gm = std::min(env_gm > 0 ? env_gm : m, std::max(mtiles, 1));
}

// The handle's own non-blocking stream (host-pointer calls, probes without a
// call stream): created once at registration (create_impl), so threads never
// race to create it.
int handle_stream(tsg_tcsc *h, hipStream_t &s)
{
    if (!h->stream) return fail(TSG_ERR_HIP, "handle has no stream (registration did not complete)");
    s = h->stream;
    return TSG_OK;
}

// Compiles and loads the image of one shape (registration, tcsc_hip_reserve,
// or the first call that picks it) and runs its probe on `s` -- the call's
// stream, or the handle's own non-blocking stream (nullptr) -- and
// synchronises that stream only.  Caller holds h->mu (or owns h exclusively).
int ensure_jit_variant(tsg_tcsc *h, int nw, int waves = tsg::kJitWaves, hipStream_t s = nullptr, bool far = false,
                       bool r64 = false, bool half = false)
{
    const int i = shape_index(nw, waves, far && !r64);
    if (i < 0 || !(r64 ? tsg::jit64_width_ok(nw) : tsg::jit_width_ok(nw)) || (r64 && (far || h->B)) ||
        (half && (!r64 || waves != 4 || nw >= tsg::kJitNW)))
        return fail(TSG_ERR_ARG, "unsupported jit stream width " + std::to_string(nw) + " x " + std::to_string(waves) +
                                 " waves" + (r64 ? (half ? " (64-row image, half ring)" : " (64-row image)") : ""));
    tsg_tcsc::JitVariant &v = half ? h->jv64h[width_index(nw) - 1] : r64 ? h->jv64[i] : h->jv[i];
    if (v.mod.function) return TSG_OK;
    tsg::JitImage img;
    tsg::build_jit_code(h->csp.data(), h->csn.data(), h->rip.empty() ? nullptr : h->rip.data(),
                        h->rin.empty() ? nullptr : h->rin.data(), h->K, h->N, h->B, img, nw, waves, far, r64, half);
    // stream offsets (wcode) and the dispatcher's region literal are 32-bit
    if ((uint64_t)img.code.size() * 4 >= (1ull << 32) - (1ull << 20))
        return fail(TSG_ERR_RANGE, "jit image of " + std::to_string((uint64_t)img.code.size() * 4) +
                                       " B exceeds the 32-bit stream offsets; shard W's columns");
#ifdef TSG_DIAG
    if (!h->B)
        if (const char *d = tsg::knob_value("TSG_JIT_DIAG")) {  // diagnostic code sharing (results WRONG)
            const size_t S = (size_t)waves;  // streams per column tile
            if (std::strstr(d, "simdpair"))  // waves w and w + S/2 (one SIMD) share w's stream
                for (size_t k = 0; k < img.wcode.size(); k++)
                    if (k % S >= S / 2) img.wcode[k] = img.wcode[k - S / 2];
            if (std::strstr(d, "samecode"))  // every column tile runs tile 0's streams
                for (size_t k = S; k < img.wcode.size(); k++) img.wcode[k] = img.wcode[k % S];
            if (std::strstr(d, "samewave"))  // every wave of a tile runs its wave 0's stream
                for (size_t k = 0; k < img.wcode.size(); k++) img.wcode[k] = img.wcode[k - k % S];
            if (std::strstr(d, "pairwave"))  // waves 2i and 2i+1 share a stream
                for (size_t k = 0; k < img.wcode.size(); k++) img.wcode[k] = img.wcode[k & ~(size_t)1];
        }
#endif
    DeviceGuard g(h->device);
    // the 64-row image's 4-wave streams: run by 8-wave workgroups of
    // half-masked wave pairs (TSG_JIT_PAIR=1, read at load: A/B)
    const char *pv = tsg::knob_value("TSG_JIT_PAIR");
    const bool pair = r64 && waves == 4 && !half && pv && pv[0] == '1';
    const std::string err = v.mod.load(img.code, nw, waves, r64, half, pair);
    if (!err.empty()) return fail(TSG_ERR_HIP, "jit kernel (width " + std::to_string(nw) + "): " + err);
    const size_t wb = img.wcode.size() * sizeof(uint32_t);
    if (hipMalloc(&v.d_wcode, std::max<size_t>(wb, 4)) != hipSuccess) {
        v.mod.unload();
        return fail(TSG_ERR_NOMEM, "hipMalloc of the jit stream table failed");
    }
    if (hipMemcpy(v.d_wcode, img.wcode.data(), wb, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(v.d_wcode);
        v.d_wcode = nullptr;
        v.mod.unload();
        return fail(TSG_ERR_HIP, "upload of the jit stream table failed");
    }
    // probe launch: the dispatcher checks that its patched literal reaches the
    // generated region (magic header) and reports it; nothing else runs.  Done
    // here, at registration / reserve, so calls never read the status back
    // (they stay asynchronous and graph-capturable).
    if (!h->d_status && hipMalloc(&h->d_status, 16) != hipSuccess) {
        (void)hipFree(v.d_wcode);
        v.d_wcode = nullptr;
        v.mod.unload();
        return fail(TSG_ERR_NOMEM, "hipMalloc of the jit status word failed");
    }
    uint32_t st[2] = {0xffffffffu, 0u};
    if (!s) {
        const int rs = handle_stream(h, s);
        if (rs) {
            (void)hipFree(v.d_wcode);
            v.d_wcode = nullptr;
            v.mod.unload();
            return rs;
        }
    }
    bool ok = hipMemsetAsync(h->d_status, 0, 16, s) == hipSuccess && tsg::launch_jit_probe(v.mod, h->d_status, s) == 0 &&
              hipMemcpyAsync(st, h->d_status, sizeof st, hipMemcpyDeviceToHost, s) == hipSuccess &&
              hipStreamSynchronize(s) == hipSuccess;
    if (!ok || st[0] != 0 || st[1] != tsg::kJitMagic0) {
        (void)hipFree(v.d_wcode);
        v.d_wcode = nullptr;
        v.mod.unload();
        return fail(TSG_ERR_HIP, "jit kernel (width " + std::to_string(nw) + "): probe launch did not find the "
                                 "generated code region (status " + std::to_string(st[0]) + ")");
    }
    v.nw = nw;
    v.waves = waves;
    v.pair = pair;
    v.Npad = img.Npad;
    v.piece_rows = img.piece_rows;
    v.nch = img.nch;
    v.chunk = img.chunk;
    v.code_bytes = (int64_t)img.code.size() * 4;
    v.wcode_words = (int64_t)img.wcode.size();
    if (!half) (r64 ? h->jit64_nch : h->jit_nch) = img.nch;
    return TSG_OK;
}

// The producer/consumer walk (tsg_tcsc_ell_pc_kernel) on 1-row tiles when K
// fits one chunk and the chunk plus its ring fit LDS: few chains, each
// latency-bound (M = 1: 15.6 vs 20.6 us at K = 4096, N = 16384;
// profiles/r02x_ell_pc.txt).  TSG_ELL_PC=0 turns it off (diagnostic A/B);
// tcsc_hip_set_small_m(h, 3) too.
bool ell_pc_available(const tsg_tcsc *h)
{
    static const bool on = [] {
        const char *e = tsg::knob_value("TSG_ELL_PC");
        return !(e && e[0] == '0');
    }();
    if (!on || h->small_m == 3 || h->K > tsg::kEllMaxC[0]) return false;
    const int C = std::min(tsg::kEllMaxC[0], std::max(4, (h->K + 3) / 4 * 4));  // build_ell_image's chunk
    const size_t lds = tsg::ell_pc_lds_bytes(0, C);
    return lds > 0 && lds <= tsg::kLdsBytes;
}

bool use_ell_pc(const tsg_tcsc *h, int v) { return v == 0 && ell_pc_available(h); }

// Small-M kernel choice (DESIGN.md 4 "Small M"): the sliced-ELL walk for a
// plain-TCSC weight-compiled handle when M is small enough that the jit
// kernel cannot fill the GPU; -1 = the jit (or rx) kernel.  Measured on
// configs[2]'s and configs[0]'s K, N (profiles/r02u_ell_lg.txt): up to M = 8
// the smallest M tile that holds M; up to M = 32 tiles of 8 (2 rows per lane:
// an 8-row chunk of K <= 5116 fits LDS, one stream per column); above that the
// largest tile whose chunk holds K.  Automatic (round 4, against the 64-row
// image, profiles/r04g_bound_ab.jsonl, step us) up to M = 32 while an 8-row
// chunk holds K (K = 4096, N = 16384: M = 32 56 vs 70, M = 48 101 vs 71), up to
// M = 16 when K is chunked (K = N = 16384: M = 16 184 vs 247, M = 32 310 vs
// 248; K = 16384, N = 4096: M = 16 178 vs 158, M = 32 281 vs 155); and, while
// an 8-row chunk holds K, up to M = 1024 when the jit kernel would have at
// most 64 workgroups (the reference's (1000, 2048, 512): 38 vs 52 us;
// (256, 4096, 1024): 41 vs 82; (256, 2048, 2048): 37 vs 47; at 128 workgroups
// the jit kernel wins: (1024, 1024, 1024) 43 vs 35).  With K chunked the
// starved grid goes to the 64-row image ((64, 16384, 4096): 266 vs 156 us).
int pick_ell_variant(const tsg_tcsc *h, int M)
{
    if (h->kind != tsg_tcsc::kJit || h->B || h->small_m == 1) return -1;
    const bool one8 = h->K <= tsg::kEllMaxC[kEllTile8];
    // the jit kernel's workgroups at its narrowest width (8 columns per wave)
    const int64_t jit_wgs = (int64_t)((M + tsg::kJitTileM - 1) / tsg::kJitTileM) *
                            ((h->N + 8 * tsg::kJitWaves - 1) / (8 * tsg::kJitWaves));
    const bool starved = one8 && M <= kEllStarvedMaxM && jit_wgs <= kEllStarvedWgs;
    static const int env_max = [] {  // TSG_ELL_MAXM: A/B of the small-M boundary (not of the small-W rule)
        const char *e = tsg::knob_value("TSG_ELL_MAXM");
        return e ? atoi(e) : -1;
    }();
    const int auto_max = env_max >= 0 ? env_max : kEllAutoMaxM;
    // a small W (M x nnz <= 420 M) keeps the walk up to M = 128 while K fits
    // one chunk: the 64-row image streams its whole code image and stages X
    // (~13 us of step overhead against ~6) whatever M is, the walk's cost
    // grows with M x nnz (profiles/r04r_sparse_small_ab.jsonl, step us:
    // (64, 2048, 8192) s = 8 26.6 vs 36.9, s = 16 21.7 vs 35.2, s = 4 35.9 vs
    // 41.0; (96, 4096, 16384) s = 16 61.3 vs 77.9; beyond it the image wins:
    // (128, 4096, 16384) s = 16 80.3 vs 76.1, (64, 4096, 16384) s = 8 66.2 vs
    // 63.0, s = 4 at M = 48 101 vs 71)
    const bool small_w = one8 && M <= kEllSmallWMaxM &&
                         (double)M * (double)(h->nnz_pos + h->nnz_neg) <= kEllSmallWWork;
    // ... unless the 64-row image (one launch, X read directly since round 5)
    // is faster there even at its floor: its K sweep costs ~0.9 us per step (2
    // passes over ceil(K / 188) chunks) + 1.4, the walk's chains ~9.9 +
    // 0.0143 us per entry of a column (K / s); profiles/r05z_walk_vs_image2.jsonl
    // (88 shapes with r05z_walk_vs_image_ab.jsonl: the round-4 rule picked the
    // slower kernel by > 3% on 21, this one on 4), step us: K = 1024, s = 4, M = 48 ... 1024, N = 512 / 1024 /
    // 4096 12.2-15.6 vs 13.6-18.8 (every M); s = 16 10.8-11.1 walk vs
    // 11.6-12.2; K = 2048 walk 17.2 vs 19.5 (M <= 256)
    // (this floor was measured with X read directly, one launch: with K % 4 !=
    // 0 or X past the 32-bit offsets the image's step also runs its X^T
    // staging kernel, priced here at kStagedXtUs -- ADVICE r05)
    const bool image_one_launch = x_direct_shape_ok(h->K, tsg::jit64_piece_rows()) && x_direct_offsets_ok(M, h->K);
    const double nnz_col = (double)(h->nnz_pos + h->nnz_neg) / std::max(1, h->N);
    const bool image_floor_lower = 0.9 * 2.0 * ((h->K + tsg::kJit64RowChunk - 1) / tsg::kJit64RowChunk) + 1.4 +
                                       (image_one_launch ? 0.0 : kStagedXtUs) <
                                   9.9 + 0.0143 * nnz_col;
    if (h->small_m < 2 && M > (one8 ? auto_max : std::min(auto_max, kEllAutoMaxMChunked)) &&
        ((!starved && !small_w) || image_floor_lower))
        return -1;
    // K in chunks (the 16-row tile, 8 columns per wave) at 8 < M <= 16: the
    // walk needs >= 2048 waves (N >= 16384) to beat the 64-row image
    // (r05z_walk_longk2_ab.jsonl, us, image vs walk: (16, 8192, 8192) 81.6 vs
    // 96.4, (12, 8192, 4096) 68.7 vs 91.3, (16, 16384, 4096) 131.7 vs 181.0,
    // (16, 8192, 2048) 66.3 vs 96.2; the walk (16, 16384, 16384) 170 vs 205,
    // and at M <= 8 (8, 8192, 4096) 61.5 vs 68.5, r05z_walk_longk_ab.jsonl)
    // (measured with direct X; the image's margin, 15-50 us, exceeds its X^T
    // pass at these M -- 16 x 8194 floats -- so the rule holds staged too)
    if (h->small_m < 2 && !one8 && M > 8 && h->N < 16384) return -1;
    int v = 0;
    if (one8 && M > tsg::kEllTileM[kEllTile8] && M <= kEllMidM) {
        v = kEllTile8;
    } else if (one8 && M > kEllMidM) {
        v = kEllTile8;
        for (int i = kEllTile8 + 1; i < tsg::kEllVariants; i++)
            if (h->K <= tsg::kEllMaxC[i]) v = i;
    } else {
        while (v + 1 < tsg::kEllVariants && M > tsg::kEllTileM[v]) v++;
    }
    // M rows as M 1-row producer/consumer tiles while the M index streams stay
    // small (M = 2 at N = 16384: 20.0 vs 22.9 us; M = 4 at N = 4096: 14.7 vs
    // 21.9 us; profiles/r02z2_pc_rows.txt)
    static const int64_t pc_rows_max_mn = [] {  // TSG_ELL_PC_MAXMN: A/B sweeps of the threshold
        const char *e = tsg::knob_value("TSG_ELL_PC_MAXMN");
        return e ? (int64_t)atoll(e) : kEllPcRowsMaxMN;
    }();
    if (M <= 4 && (int64_t)M * h->N <= pc_rows_max_mn && ell_pc_available(h)) v = 0;
    static const int force = [] {  // TSG_ELL_VARIANT: diagnostic sweeps only
        const char *e = tsg::knob_value("TSG_ELL_VARIANT");
        return e ? atoi(e) : -1;
    }();
    if (force >= 0 && force < tsg::kEllVariants) v = force;
    return v;
}

// Builds and uploads the ELL image of a variant.  Caller holds h->mu.
// X^T copies of a small-M image (tsg_internal.h ell_copy_offset): two for the
// 8-row tile's 4-lane columns when TSG_ELL_COPIES=2 (A/B), else one
int ell_copies(int v)
{
    static const int env = [] {
        const char *c = tsg::knob_value("TSG_ELL_COPIES");
        const char *lg = tsg::knob_value("TSG_ELL_LG");
        return c && c[0] == '2' && (!lg || std::atoi(lg) == 4) ? 2 : 1;
    }();
    return v == kEllTile8 ? env : 1;
}

// The bank-window schedule of the 8-row tile's image (tsg_internal.h
// kEllSchedZeroRows): TSG_ELL_SCHED=0 / 1 (A/B)
bool ell_sched(int v)
{
    static const int env = [] {
        const char *c = tsg::knob_value("TSG_ELL_SCHED");
        const char *lg = tsg::knob_value("TSG_ELL_LG");
        return c && c[0] == '1' && (!lg || std::atoi(lg) == 4) ? 1 : 0;
    }();
    return v == kEllTile8 && env && ell_copies(v) == 1;
}

int ensure_ell(tsg_tcsc *h, int v)
{
    tsg_tcsc::EllVariant &e = h->ell[v];
    if (e.ready) return TSG_OK;
    tsg::build_ell_image(h->csp.data(), h->csn.data(), h->rip.empty() ? nullptr : h->rip.data(),
                         h->rin.empty() ? nullptr : h->rin.data(), h->K, h->N, tsg::kEllMaxC[v], tsg::kEllTileM[v], e.img,
                         ell_copies(v), ell_sched(v));
    DeviceGuard g(h->device);
    const size_t eb = e.img.ent.size() * 4, tb = std::max<size_t>(e.img.tab.size() * 4, 8);
    // allocate and upload into locals; the variant owns them only once both
    // uploads succeeded (a failed attempt leaves nothing behind, a retry
    // starts clean)
    uint32_t *d_ent = nullptr, *d_tab = nullptr;
    auto drop = [&](int code, const char *msg) {
        if (d_ent) (void)hipFree(d_ent);
        if (d_tab) (void)hipFree(d_tab);
        return fail(code, msg);
    };
    if (hipMalloc(&d_ent, eb) != hipSuccess || hipMalloc(&d_tab, tb) != hipSuccess)
        return drop(TSG_ERR_NOMEM, "hipMalloc of the small-M (ELL) image failed");
    if (hipMemcpy(d_ent, e.img.ent.data(), eb, hipMemcpyHostToDevice) != hipSuccess ||
        (!e.img.tab.empty() && hipMemcpy(d_tab, e.img.tab.data(), e.img.tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
        return drop(TSG_ERR_HIP, "upload of the small-M (ELL) image failed");
    e.d_ent = d_ent;
    e.d_tab = d_tab;
    e.bytes = (int64_t)(eb + tb);
    std::vector<uint32_t>().swap(e.img.ent);
    std::vector<uint32_t>().swap(e.img.tab);
    e.ready = true;
    return TSG_OK;
}

int run_dev(tsg_tcsc *h, const float *dX, const float *db, const float *dalpha, float *dY, int M,
            int N, int K, hipStream_t s, bool prelu)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    if (N != h->N || K != h->K)
        return fail(TSG_ERR_ARG, "shape mismatch: handle has K=" + std::to_string(h->K) + " N=" +
                                     std::to_string(h->N) + ", call has K=" + std::to_string(K) +
                                     " N=" + std::to_string(N));
    if (M < 0) return fail(TSG_ERR_ARG, "M < 0");
    if (M == 0 || N == 0) return TSG_OK;
    if (!dY || !db || (K > 0 && !dX) || (prelu && !dalpha))
        return fail(TSG_ERR_ARG, "null device pointer");
    DeviceGuard g(h->device);
    // One call at a time per handle: the X^T work buffer, the jit images and
    // the timing ring are shared by every stream that uses the handle.
    std::lock_guard<std::mutex> lk(h->mu);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(s, &cap));
    const bool capturing = cap != hipStreamCaptureStatusNone;
    int rc;
    const int ev = pick_ell_variant(h, M);
    if (ev >= 0) {
        // small M: the ELL walk reads X in place (no X^T staging, no work buffer)
        if (!h->ell[ev].ready && capturing)
            return fail(TSG_ERR_ARG, "M=" + std::to_string(M) + " runs the small-M kernel, whose image is not "
                                     "built yet; call tcsc_hip_reserve before capturing");
        rc = ensure_ell(h, ev);
        if (rc) return rc;
        int slot = -1;
        if (h->timing && !capturing) {
            rc = harvest_timing(h, false);
            if (rc) return rc;
            slot = h->ring_head;
            HIP_TRY(hipEventRecord(h->ev0[slot], s));
        }
        const tsg_tcsc::EllVariant &e = h->ell[ev];
        const int lrc = use_ell_pc(h, ev) ? tsg::launch_tcsc_ell_pc(ev, dX, e.d_ent, e.d_tab, db, dalpha, dY, M, N, K,
                                                                    e.img.C, e.img.nch, prelu ? 1 : 0, s)
                                          : tsg::launch_tcsc_ell(ev, dX, e.d_ent, e.d_tab, db, dalpha, dY, M, N, K,
                                                                 e.img.C, e.img.nch, e.img.xb, e.img.zr, prelu ? 1 : 0, s);
        if (lrc != 0)
            return fail(TSG_ERR_HIP, std::string("small-M kernel launch: ") + hipGetErrorString(hipGetLastError()));
        if (slot >= 0) {
            HIP_TRY(hipEventRecord(h->ev1[slot], s));
            h->ring_head = (h->ring_head + 1) % tsg_tcsc::kRing;
            h->ring_count++;
        }
        return TSG_OK;
    }
    JitShape sh = h->kind == tsg_tcsc::kJit ? call_shape(h, M) : JitShape{0, 0};
    if (h->kind == tsg_tcsc::kJit && !variant_of(h, sh).mod.function) {
        if (capturing)
            return fail(TSG_ERR_ARG, "M=" + std::to_string(M) + " runs the width-" + std::to_string(sh.nw) +
                                         " image, which is not compiled yet; call tcsc_hip_reserve before capturing");
        rc = ensure_jit_variant(h, sh.nw, sh.waves, s, sh.far, sh.r64, sh.half);
        if (rc == TSG_ERR_HIP && may_fall_back(h, sh)) {
            // an image the loader refuses (or whose probe fails): this and later
            // calls that pick it run the 128-row 64 x 8 image -- same result
            // bit for bit, another speed
            std::fprintf(stderr, "[ternary_spgemm] warning: %s; running the 128-row 64 x 8 image instead\n",
                         g_tsg_host_err.c_str());
            h->bad_variants |= 1u << variant_bit(sh);
            sh = JitShape{tsg::kJitNW, tsg::kJitWaves};
            rc = ensure_jit_variant(h, sh.nw, sh.waves, s);
            if (rc) return rc;
        } else if (rc) {
            return rc;
        }
    }
    const bool r64 = sh.r64, half = sh.half;
    const int tile_m = r64 ? tsg::kJit64TileM : tsg::kJitTileM,
              chunk = r64 ? tsg::jit64_chunk(half) : tsg::kJitChunk;
    int Mp, Kp;
    dims_for(h, M, Mp, Kp, r64, half);
    tsg_tcsc::JitVariant *jv = nullptr;
    if (h->kind == tsg_tcsc::kJit) {
        jv = &variant_of(h, sh);
        // the stream steps through X^T chunks with a 32-bit stride, and the grid
        // (one workgroup per M tile x column tile) must stay under 2^32 threads
        const int64_t wgs = (int64_t)(Mp / tile_m) * (jv->Npad / (jv->nw * jv->waves));
        if ((int64_t)Mp * chunk * 4 >= (1ll << 31) || wgs * jv->waves * 64 >= (1ll << 32))
            return fail(TSG_ERR_ARG, "M=" + std::to_string(M) + " is too large for one jit launch; split the rows");
    }
    // the 64-row image stages straight from row-major X (no X^T pass, no work
    // buffer) when every row starts 16-B aligned and the offsets fit 32 bits
    const bool direct = r64 && x_direct(h, dX, M, K, *jv);
    if (r64 && jv->chunk != chunk)  // the image and this call's X^T dims must agree (TSG_JIT_QBLOCK read at both)
        return fail(TSG_ERR_ARG, "64-row image built for " + std::to_string(jv->chunk) + "-row chunks, call expects " +
                                     std::to_string(chunk) + " (TSG_JIT_QBLOCK changed after the image was built)");
    // row layout, direct X: the last chunk starts at K - 188, lastadj bytes
    // below its slot (tsg_internal.h jit64_row_kbase)
    const int lastadj = direct && jv->piece_rows == 0
                            ? 4 * ((jv->nch - 1) * tsg::kJit64RowChunk - tsg::jit64_row_kbase(K, jv->nch, jv->nch - 1))
                            : 0;
    if (!direct) {
        rc = ensure_work(h, M, capturing, r64, half);
        if (rc) return rc;
    }
    // X^T of the previous call may still be read by its kernel on another
    // stream: this call's staging waits for it (same stream: stream order)
    if (!direct && !capturing && h->work_used && h->work_stream != s) HIP_TRY(hipStreamWaitEvent(s, h->work_ev, 0));
    if (direct) {
        // no staging kernel: the dispatcher's DMA reads X itself
    } else if (K == 0) {
        // no X at all: chain is +0; X^T stays zero
        HIP_TRY(hipMemsetAsync(h->d_work, 0, (size_t)Mp * Kp * sizeof(float), s));
    } else if ((h->kind != tsg_tcsc::kJit ? tsg::launch_transpose(dX, h->d_work, M, K, Mp, Kp, s)
                : r64                      ? tsg::launch_transpose_quads(dX, h->d_work, M, K, Mp, Kp, jv->piece_rows, s,
                                                                         chunk)
                                           : tsg::launch_transpose_pairs(dX, h->d_work, M, K, Mp, Kp, s)) != 0) {
        return fail(TSG_ERR_HIP, std::string("transpose launch: ") + hipGetErrorString(hipGetLastError()));
    }
    int slot = -1;
    if (h->timing && !capturing) {
        rc = harvest_timing(h, false);
        if (rc) return rc;
        slot = h->ring_head;
        HIP_TRY(hipEventRecord(h->ev0[slot], s));
    }
    int gn = 2, gm = 16, tmask = 0;
    if (h->kind == tsg_tcsc::kJit)
        pick_jit_map(h, Mp / tile_m, jv->Npad / (jv->nw * jv->waves), gn, gm, tmask, r64 ? jv->nw : 0);
    // (jv is null on the rx kernel)
    const bool jit = h->kind == tsg_tcsc::kJit;
    const int xtouch = jit && pick_xtouch(h, M) ? 1 : 0;
    const int tnear = jit && pick_tnear(r64, jv->waves, Mp / tile_m) ? 1 : 0;
    const int lrc = h->kind == tsg_tcsc::kJit
        ? tsg::launch_tcsc_jit(jv->mod, direct ? dX : h->d_work, Mp, jv->d_wcode, db, dalpha, dY, M, N, jv->Npad,
                               jv->nch, prelu ? 1 : 0, h->d_status, jv->nw * jv->waves,
                               jv->pair ? 2 * jv->waves : jv->waves, gn, gm, tmask, s, tile_m, direct ? K : 0,
                               lastadj, xtouch, tnear)
        : tsg::launch_tcsc_rx(h->d_work, Mp, h->d_seg, h->d_ent, db, dalpha, dY, M, N, h->rimg.Npad,
                              h->rimg.nch, prelu ? 1 : 0, s);
    if (lrc != 0)
        return fail(TSG_ERR_HIP, std::string("tcsc launch: ") + hipGetErrorString(hipGetLastError()));
    if (slot >= 0) {
        HIP_TRY(hipEventRecord(h->ev1[slot], s));
        h->ring_head = (h->ring_head + 1) % tsg_tcsc::kRing;
        h->ring_count++;
    }
    if (!capturing && !direct) {
        // (a captured call's reads happen at replay time and are not tracked:
        // a replay must not overlap calls on other streams,
        // include/ternary_spgemm.h; the record of the last uncaptured call
        // stays, so the next uncaptured call still waits for it)
        HIP_TRY(hipEventRecord(h->work_ev, s));
        h->work_stream = s;
        h->work_used = true;
    }
    return TSG_OK;
}

// Chunks of the host-pointer pipeline: one per ~16 MiB of Y (the PCIe leg
// that binds: Y is the largest transfer), at most kHostChunksMax, each a whole
// number of 128-row M tiles and at least 256 rows; calls the small-M kernel
// takes run whole.  configs[2] (268 MB of Y): 16 chunks of 256 rows, 5.45 ms
// per call (8 chunks 5.50, 4 chunks 5.72, unchunked 7.38;
// profiles/r03b_host_pipe_ab.jsonl).
int host_chunk_rows(const tsg_tcsc *h, int M)
{
    const int64_t ybytes = (int64_t)M * h->N * 4;
    int n = h->host_chunks > 0 ? h->host_chunks : (int)std::min<int64_t>(ybytes >> 24, tsg_tcsc::kHostChunksMax);
    n = std::min(n, tsg_tcsc::kHostChunksMax);
    if (n <= 1 || (h->host_chunks <= 0 && pick_ell_variant(h, M) >= 0)) return M;
    int rows = (M + n - 1) / n;
    rows = (rows + tsg::kJitTileM - 1) / tsg::kJitTileM * tsg::kJitTileM;
    if (h->host_chunks <= 0) rows = std::max(rows, 256);
    return std::min(rows, M);
}

int host_pipe_ready(tsg_tcsc *h)
{
    if (h->s_in) return TSG_OK;
    HIP_TRY(hipStreamCreateWithFlags(&h->s_out, hipStreamNonBlocking));
    for (int i = 0; i < tsg_tcsc::kHostChunksMax; i++) {
        HIP_TRY(hipEventCreateWithFlags(&h->ev_in[i], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&h->ev_c[i], hipEventDisableTiming));
    }
    HIP_TRY(hipStreamCreateWithFlags(&h->s_in, hipStreamNonBlocking));  // last: marks the pipeline ready
    return TSG_OK;
}

// The comp_func call (main.cpp:214-216): host X, b, Y; synchronous.  Pipelined
// by M chunks over three streams: the calling thread copies X chunk i in
// (s_in) and enqueues its compute (the handle's stream, after chunk i's copy)
// while a helper thread copies the finished Y chunks out (s_out, after each
// chunk's compute), so the H2D of chunk i+1, the kernel of chunk i and the
// D2H of chunk i-1 overlap (PCIe is full duplex).  Rows are independent, so
// the chunked result is the unchunked one bit for bit.
int run_host_impl(tsg_tcsc *h, const float *X, const float *b, const float *alpha, float *Y, int M, int N, int K,
                  bool prelu);

// No exception crosses the extern "C" boundary: a std::bad_alloc or
// std::system_error (thread creation) inside the pipeline becomes a status.
int run_host(tsg_tcsc *h, const float *X, const float *b, const float *alpha, float *Y, int M, int N, int K,
             bool prelu)
{
    try {
        return run_host_impl(h, X, b, alpha, Y, M, N, K, prelu);
    } catch (const std::bad_alloc &) {
        return fail(TSG_ERR_NOMEM, "host-pointer call: out of host memory");
    } catch (const std::exception &e) {
        return fail(TSG_ERR_HIP, std::string("host-pointer call: ") + e.what());
    }
}

int run_host_impl(tsg_tcsc *h, const float *X, const float *b, const float *alpha, float *Y, int M, int N, int K,
                  bool prelu)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    if (N != h->N || K != h->K) return run_dev(h, nullptr, nullptr, nullptr, nullptr, M, N, K, nullptr, prelu);
    if (M < 0) return fail(TSG_ERR_ARG, "M < 0");
    if (M == 0 || N == 0) return TSG_OK;
    if (!Y || !b || (K > 0 && !X) || (prelu && !alpha)) return fail(TSG_ERR_ARG, "null host pointer");
    DeviceGuard g(h->device);
    // the staging buffers and the streams are the handle's: a second host
    // thread waits here until this call's Y is back (run_dev takes h->mu inside)
    std::lock_guard<std::mutex> lk(h->host_mu);
    const size_t xb = (size_t)M * K * sizeof(float), yb = (size_t)M * N * sizeof(float);
    if (xb > h->x_bytes) {
        if (h->d_x) HIP_TRY(hipFree(h->d_x));
        h->d_x = nullptr;
        h->x_bytes = 0;
        if (hipMalloc(&h->d_x, std::max<size_t>(xb, 4)) != hipSuccess) return fail(TSG_ERR_NOMEM, "hipMalloc X");
        h->x_bytes = xb;
    }
    if (yb > h->y_bytes) {
        if (h->d_y) HIP_TRY(hipFree(h->d_y));
        h->d_y = nullptr;
        h->y_bytes = 0;
        if (hipMalloc(&h->d_y, yb) != hipSuccess) return fail(TSG_ERR_NOMEM, "hipMalloc Y");
        h->y_bytes = yb;
    }
    hipStream_t s = nullptr;
    int rc = handle_stream(h, s);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(h->d_b, b, (size_t)N * sizeof(float), hipMemcpyHostToDevice, s));
    if (prelu) HIP_TRY(hipMemcpyAsync(h->d_alpha, alpha, (size_t)N * sizeof(float), hipMemcpyHostToDevice, s));
    const int rows = host_chunk_rows(h, M);
    if (rows >= M) {
        if (xb) HIP_TRY(hipMemcpyAsync(h->d_x, X, xb, hipMemcpyHostToDevice, s));
        rc = run_dev(h, h->d_x, h->d_b, h->d_alpha, h->d_y, M, N, K, s, prelu);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(Y, h->d_y, yb, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        return TSG_OK;
    }
    rc = host_pipe_ready(h);
    if (rc) return rc;
    const int nchunk = (M + rows - 1) / rows;
    // chunks enqueued by this thread (their ev_c recorded); -1 = stop (error)
    std::mutex m;
    std::condition_variable cv;
    int enq = 0;
    hipError_t out_err = hipSuccess;
    // joins the helper on every path out of this scope (an exception included)
    struct Joiner {
        std::thread &t;
        std::mutex &m;
        std::condition_variable &cv;
        int &enq;
        ~Joiner()
        {
            if (!t.joinable()) return;
            {
                std::lock_guard<std::mutex> gl(m);
                enq = -1;
            }
            cv.notify_all();
            t.join();
        }
    };
    std::thread out([&] {
        DeviceGuard tg(h->device);
        for (int i = 0; i < nchunk && out_err == hipSuccess; i++) {
            {
                std::unique_lock<std::mutex> ul(m);
                cv.wait(ul, [&] { return enq > i || enq < 0; });
                if (enq < 0) break;
            }
            const size_t r0 = (size_t)i * rows, nr = std::min<size_t>(rows, (size_t)M - r0);
            out_err = hipStreamWaitEvent(h->s_out, h->ev_c[i], 0);
            if (out_err == hipSuccess)
                out_err = hipMemcpyAsync(Y + r0 * N, h->d_y + r0 * N, nr * N * sizeof(float), hipMemcpyDeviceToHost,
                                         h->s_out);
        }
        const hipError_t e = hipStreamSynchronize(h->s_out);
        if (out_err == hipSuccess) out_err = e;
    });
    Joiner joiner{out, m, cv, enq};
    auto stop = [&](int code) {
        {
            std::lock_guard<std::mutex> gl(m);
            if (code) enq = -1;
        }
        cv.notify_all();
        out.join();
        // on an error, chunks already enqueued may still read d_x / write d_y:
        // drain them so the next call's copies cannot overtake them
        if (code) (void)hipStreamSynchronize(s);
        return code;
    };
    for (int i = 0; i < nchunk; i++) {
        const size_t r0 = (size_t)i * rows, nr = std::min<size_t>(rows, (size_t)M - r0);
        hipError_t e = hipSuccess;
        if (K > 0) e = hipMemcpyAsync(h->d_x + r0 * K, X + r0 * K, nr * K * sizeof(float), hipMemcpyHostToDevice, h->s_in);
        if (e == hipSuccess) e = hipEventRecord(h->ev_in[i], h->s_in);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, h->ev_in[i], 0);
        if (e != hipSuccess) return stop(fail(TSG_ERR_HIP, std::string("host pipeline (X chunk): ") + hipGetErrorString(e)));
        rc = run_dev(h, h->d_x + r0 * K, h->d_b, h->d_alpha, h->d_y + r0 * N, (int)nr, N, K, s, prelu);
        if (rc) return stop(rc);
        e = hipEventRecord(h->ev_c[i], s);
        if (e != hipSuccess) return stop(fail(TSG_ERR_HIP, std::string("host pipeline (event): ") + hipGetErrorString(e)));
        {
            std::lock_guard<std::mutex> gl(m);
            enq = i + 1;
        }
        cv.notify_all();
    }
    stop(0);
    if (out_err != hipSuccess) {
        // chunks still queued on the compute stream may read d_x / write d_y:
        // drain them before the next call's copies can overwrite d_x
        (void)hipStreamSynchronize(s);
        return fail(TSG_ERR_HIP, std::string("host pipeline (Y chunk): ") + hipGetErrorString(out_err));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return TSG_OK;
}

void free_handle(tsg_tcsc *h)
{
    if (!h) return;
    DeviceGuard g(h->device);
    if (h->ring_count) (void)hipDeviceSynchronize();
    if (h->work_ev) (void)hipEventDestroy(h->work_ev);
    for (void *p : {(void *)h->d_seg, (void *)h->d_ent, (void *)h->d_work, (void *)h->d_x,
                    (void *)h->d_b, (void *)h->d_y, (void *)h->d_alpha, (void *)h->d_status})
        if (p) (void)hipFree(p);
    for (auto *vs : {&h->jv[0], &h->jv64[0], &h->jv64h[0]})
        for (size_t i = 0; i < (vs == &h->jv[0] ? std::size(h->jv) : vs == &h->jv64[0] ? std::size(h->jv64)
                                                                                      : std::size(h->jv64h)); i++) {
            if (vs[i].d_wcode) (void)hipFree(vs[i].d_wcode);
            vs[i].mod.unload();
        }
    for (auto &e : h->ell) {
        if (e.d_ent) (void)hipFree(e.d_ent);
        if (e.d_tab) (void)hipFree(e.d_tab);
    }
    if (h->stream) (void)hipStreamDestroy(h->stream);
    if (h->s_in) (void)hipStreamDestroy(h->s_in);
    if (h->s_out) (void)hipStreamDestroy(h->s_out);
    for (int i = 0; i < tsg_tcsc::kHostChunksMax; i++) {
        if (h->ev_in[i]) (void)hipEventDestroy(h->ev_in[i]);
        if (h->ev_c[i]) (void)hipEventDestroy(h->ev_c[i]);
    }
    for (int i = 0; i < tsg_tcsc::kRing; i++) {
        if (h->ev0[i]) (void)hipEventDestroy(h->ev0[i]);
        if (h->ev1[i]) (void)hipEventDestroy(h->ev1[i]);
    }
    delete h;
}

}  // namespace

// ================================================================ C-ABI ==

extern "C" const char *tcsc_hip_last_error(void)
{
    return g_tsg_host_err.c_str();
}

extern "C" int tcsc_hip_device_count(int *count)
{
    if (!count) return fail(TSG_ERR_ARG, "null count");
    *count = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return fail(TSG_ERR_NODEV, "hipGetDeviceCount failed");
    *count = n;
    return TSG_OK;
}

namespace {

// Registration of TCSC (B = 0) or BlockedTCSC<B> arrays.
int create_impl(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin, int K, int N,
                int B, int device, tsg_tcsc **out)
{
    if (!out) return fail(TSG_ERR_ARG, "null out");
    *out = nullptr;
    if (B < 0) return fail(TSG_ERR_ARG, "negative block size");
    // a malformed environment knob (or, in the product build, the wrong-result
    // diagnostics of TSG_JIT_DIAG) is refused before anything else
    const std::string ke = tsg::knob_check();
    if (!ke.empty()) return fail(TSG_ERR_ARG, ke);
    std::string e = tsg::validate_tcsc(csp, csn, rip, rin, K, N, B);
    if (!e.empty()) return fail(TSG_ERR_ARG, std::string(B ? "malformed BlockedTCSC: " : "malformed TCSC: ") + e);
    if (B && (tsg::kJitXRegs - tsg::kJitNW) / tsg::kJitSlotRegs < 2)
        return fail(TSG_ERR_ARG, "BlockedTCSC: this jit kernel geometry has no registers for the block sums");
    const int64_t slots = (B ? (int64_t)(K / B) : 1) * N;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(TSG_ERR_NODEV, "no HIP device");
    if (device < 0) HIP_TRY(hipGetDevice(&device));
    if (device >= ndev) return fail(TSG_ERR_ARG, "device index out of range");
    int rc = check_device(device);
    if (rc) return rc;

    tsg_tcsc *h = new tsg_tcsc();
    h->K = K;
    h->N = N;
    h->B = B;
    h->device = device;
    {
        DeviceGuard g0(device);
        if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
            delete h;
            return fail(TSG_ERR_HIP, "hipStreamCreate of the handle's stream failed");
        }
    }
    h->nnz_pos = csp[slots];
    h->nnz_neg = csn[slots];
    h->csp.assign(csp, csp + slots + 1);
    h->csn.assign(csn, csn + slots + 1);
    if (h->nnz_pos) h->rip.assign(rip, rip + h->nnz_pos);
    if (h->nnz_neg) h->rin.assign(rin, rin + h->nnz_neg);
    // kernel family (default: the weight-compiled kernel); TSG_KERNEL selects
    // the others for A/B and their own tests
    const char *kenv = tsg::knob_value("TSG_KERNEL");
    // The weight-compiled image costs ~8 B per nonzero plus ~15% schedule code;
    // stream offsets are 32-bit, so a W whose image would pass ~3 GiB (e.g.
    // K=16384, N=131072, s=4 on ONE GPU -- shard columns instead)
    // defaults to the rx kernel.  Asking for jit explicitly is then an error.
    // A stream step (DMA, barrier, waits) costs ~256 B on top; BlockedTCSC walks
    // every block's chunks twice per column half.
    const int64_t nchk = std::max(1, (K + tsg::kJitChunk - 1) / tsg::kJitChunk);
    const int64_t steps = B ? 4 * (int64_t)(K / B) * ((B + tsg::kJitChunk - 1) / tsg::kJitChunk + 1) : 2 * nchk;
    const int64_t streams = (int64_t)((N + tsg::kJitTileCols - 1) / tsg::kJitTileCols) * tsg::kJitStreams;
    const double jit_est =
        8.0 * 1.25 * ((double)h->nnz_pos + (double)h->nnz_neg) + 256.0 * (double)steps * (double)streams;
    const bool jit_fits = jit_est < 3.0 * (double)(1ull << 30);
    const std::string kname = kenv ? kenv : (jit_fits ? "jit" : "rx");
    if (kname != "jit" && kname != "rx") {
        free_handle(h);  // destroys the handle's stream too
        return fail(TSG_ERR_ARG, "TSG_KERNEL=" + kname + ": expected jit or rx");
    }
    if (B && kname != "jit") {
        free_handle(h);
        return fail(TSG_ERR_ARG, "BlockedTCSC runs on the jit kernel only (TSG_KERNEL=" + kname + ")");
    }
    if ((kname == "jit" || B) && !jit_fits) {
        free_handle(h);
        return fail(TSG_ERR_ARG, "TSG_KERNEL=jit: W has too many nonzeros for one weight-compiled image "
                                 "(> ~300M); shard columns across handles or use TSG_KERNEL=rx");
    }
    h->kind = kname == "jit" ? tsg_tcsc::kJit : tsg_tcsc::kRx;
    if (h->kind == tsg_tcsc::kJit) {
        // TSG_JIT_NW=<64|32|16|8> pins the stream width (A/B); default: per call
        if (const char *wv = tsg::knob_value("TSG_JIT_NW")) {
            const int nw = std::atoi(wv);
            if (width_index(nw) < 0 || !tsg::jit_width_ok(nw) || (B && nw != tsg::kJitNW)) {
                free_handle(h);
                return fail(TSG_ERR_ARG, std::string("TSG_JIT_NW=") + wv + ": expected 64, 32, 16 or 8 (64 for BlockedTCSC)");
            }
            h->jit_force = nw;
        }
        // Registration compiles, loads and probes the image most calls run --
        // the 64-row image's 128 x 8 (configs[2] and the sparse end, M >= 1024
        // at N = 16384) -- so a handle does not also carry the 128-row image
        // (8 B per nonzero) unless a call picks it or falls back to it.  If the
        // 64-row image cannot load here, the 128-row 64 x 8 one is tried (calls
        // that pick a 64-row image then warn and fall back, run_dev), then rx.
        h->jit_nch = std::max(1, (K + tsg::kJitChunk - 1) / tsg::kJitChunk);
        int rc0 = !B && !h->jit_force && !tsg::knob_value("TSG_JIT_ROWS64_MAXM") ? ensure_jit_variant(h, tsg::kJit64WideNW, tsg::kJitWaves, nullptr, false, true)
                                                                                 : TSG_ERR_ARG;
        if (rc0) rc0 = ensure_jit_variant(h, h->jit_force ? h->jit_force : tsg::kJitNW);
        if (rc0) {
            // A generated image that the loader refuses (or whose probe launch
            // does not find its region) falls back to the rx kernel, unless jit
            // was asked for explicitly or the format needs it (BlockedTCSC).
            if ((rc0 != TSG_ERR_HIP && rc0 != TSG_ERR_RANGE) || kenv || B) {
                free_handle(h);
                return rc0;
            }
            std::fprintf(stderr, "[ternary_spgemm] warning: weight-compiled image unavailable (%s); "
                                 "falling back to the rx kernel\n", g_tsg_host_err.c_str());
            h->kind = tsg_tcsc::kRx;
        }
    }
    if (h->kind == tsg_tcsc::kRx) tsg::build_rx_image(csp, csn, rip, rin, K, N, h->rimg);
    static const std::vector<uint32_t> kNoEntries(1, 0u);
    const std::vector<uint32_t> *segv = h->kind == tsg_tcsc::kRx ? &h->rimg.wstart : &kNoEntries;
    const std::vector<uint32_t> *entv = h->kind == tsg_tcsc::kRx ? &h->rimg.ent : &kNoEntries;

    DeviceGuard g(device);
    const size_t sb = segv->size() * sizeof(uint32_t), eb = entv->size() * sizeof(uint32_t);
    if (hipMalloc(&h->d_seg, sb) != hipSuccess || hipMalloc(&h->d_ent, eb) != hipSuccess ||
        hipMalloc(&h->d_b, std::max<size_t>((size_t)N * sizeof(float), 4)) != hipSuccess ||
        hipMalloc(&h->d_alpha, std::max<size_t>((size_t)N * sizeof(float), 4)) != hipSuccess ||
        (!h->d_status && hipMalloc(&h->d_status, 16) != hipSuccess)) {
        free_handle(h);
        return fail(TSG_ERR_NOMEM, "hipMalloc of the device image failed");
    }
    if (hipEventCreateWithFlags(&h->work_ev, hipEventDisableTiming) != hipSuccess) {
        free_handle(h);
        return fail(TSG_ERR_HIP, "hipEventCreate of the work-buffer event failed");
    }
    if (hipMemset(h->d_status, 0, 16) != hipSuccess ||
        hipMemcpy(h->d_seg, segv->data(), sb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->d_ent, entv->data(), eb, hipMemcpyHostToDevice) != hipSuccess) {
        free_handle(h);
        return fail(TSG_ERR_HIP, "upload of the device image failed");
    }
    *out = h;
    return TSG_OK;
}

}  // namespace

extern "C" int tcsc_hip_create(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                               const int32_t *rin, int K, int N, int device, tsg_tcsc **out)
{
    return create_impl(csp, csn, rip, rin, K, N, 0, device, out);
}

extern "C" int tcsc_hip_create_blocked(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                                       const int32_t *rin, int K, int N, int B, int device, tsg_tcsc **out)
{
    if (B <= 0) {
        if (out) *out = nullptr;
        return fail(TSG_ERR_ARG, "block size must be positive");
    }
    return create_impl(csp, csn, rip, rin, K, N, B, device, out);
}

extern "C" int tcsc_hip_create_dense(const int32_t *W, int K, int N, int device, tsg_tcsc **out)
{
    if (!out) return fail(TSG_ERR_ARG, "null out");
    *out = nullptr;
    if (!W || K < 0 || N < 0) return fail(TSG_ERR_ARG, "bad dense matrix");
    // TCSC ctor (TCSC.h:13-41): column by column, +1 / -1 rows ascending
    std::vector<int32_t> csp, csn, rip, rin;
    csp.reserve((size_t)N + 1);
    csn.reserve((size_t)N + 1);
    for (int n = 0; n < N; n++) {
        csp.push_back((int32_t)rip.size());
        csn.push_back((int32_t)rin.size());
        for (int k = 0; k < K; k++) {
            const int32_t v = W[(size_t)k * N + n];
            if (v == 1) rip.push_back(k);
            else if (v == -1) rin.push_back(k);
        }
    }
    csp.push_back((int32_t)rip.size());
    csn.push_back((int32_t)rin.size());
    return tcsc_hip_create(csp.data(), csn.data(), rip.data(), rin.data(), K, N, device, out);
}

extern "C" int tcsc_hip_encode_dense_dev(const int32_t *dW, int K, int N, int32_t *d_csp, int32_t *d_csn,
                                         int32_t *d_rip, int64_t rip_cap, int32_t *d_rin, int64_t rin_cap,
                                         int64_t *nnz_pos, int64_t *nnz_neg, void *stream)
{
    if (K < 0 || N < 0 || !d_csp || !d_csn || !nnz_pos || !nnz_neg || (K > 0 && N > 0 && !dW))
        return fail(TSG_ERR_ARG, "tcsc_hip_encode_dense_dev: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    size_t tmp_bytes = 0;
    if (tsg::encode_count(dW, K, N, d_csp, d_csn, nullptr, &tmp_bytes, s) != 0)
        return fail(TSG_ERR_HIP, "tcsc_hip_encode_dense_dev: scan workspace query failed");
    void *tmp = nullptr;
    HIP_TRY(hipMallocAsync(&tmp, std::max<size_t>(tmp_bytes, 4), s));
    const int rc = tsg::encode_count(dW, K, N, d_csp, d_csn, tmp, &tmp_bytes, s);
    HIP_TRY(hipFreeAsync(tmp, s));
    if (rc != 0) return fail(TSG_ERR_HIP, std::string("tcsc_hip_encode_dense_dev: count/scan: ") +
                                              hipGetErrorString(hipGetLastError()));
    int32_t tot[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&tot[0], d_csp + N, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&tot[1], d_csn + N, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *nnz_pos = tot[0];
    *nnz_neg = tot[1];
    if (!d_rip || !d_rin) return TSG_OK;
    if (rip_cap < tot[0] || rin_cap < tot[1])
        return fail(TSG_ERR_ARG, "tcsc_hip_encode_dense_dev: row index arrays too small");
    if (tsg::encode_fill(dW, K, N, d_csp, d_csn, d_rip, d_rin, s) != 0)
        return fail(TSG_ERR_HIP, std::string("tcsc_hip_encode_dense_dev: fill: ") + hipGetErrorString(hipGetLastError()));
    return TSG_OK;
}

extern "C" int tcsc_hip_create_csc_packed(const int32_t *col_ptr, const int32_t *row_idx,
                                          const uint8_t *packed, int K, int N, int device,
                                          tsg_tcsc **out)
{
    if (!out) return fail(TSG_ERR_ARG, "null out");
    *out = nullptr;
    int64_t p = 0, q = 0;
    int rc = tsg_csc_packed_to_tcsc(col_ptr, row_idx, packed, N, nullptr, nullptr, nullptr,
                                    nullptr, &p, &q);
    if (rc) return rc;
    std::vector<int32_t> csp((size_t)N + 1), csn((size_t)N + 1), rip((size_t)std::max<int64_t>(p, 1)),
        rin((size_t)std::max<int64_t>(q, 1));
    rc = tsg_csc_packed_to_tcsc(col_ptr, row_idx, packed, N, csp.data(), csn.data(), rip.data(),
                                rin.data(), &p, &q);
    if (rc) return rc;
    return tcsc_hip_create(csp.data(), csn.data(), rip.data(), rin.data(), K, N, device, out);
}

extern "C" void tcsc_hip_destroy(tsg_tcsc *h) { free_handle(h); }

// Prepares every call with M <= max_M: the work buffer for max_M rows and the
// image of every shape such a call picks (pick_jit_shape depends on M
// only through the number of 128-row M tiles).  After it, calls with M <=
// max_M allocate and compile nothing, so they can be captured in a graph.
extern "C" int tcsc_hip_reserve(tsg_tcsc *h, int max_M)
{
    if (!h || max_M < 0) return fail(TSG_ERR_ARG, "bad reserve arguments");
    DeviceGuard g(h->device);
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = ensure_work(h, max_M, false);
    if (!rc) rc = ensure_work(h, max_M, false, true);  // the 64-row image's k-quad X^T (same bytes or fewer)
    if (rc || h->kind != tsg_tcsc::kJit) return rc;
    // the image choice and its shape depend on M only through the 64- / 128-row
    // M tiles (and the small-M rule): the first and last M of every 64-row
    // range cover every image a call with M <= max_M picks
    const int ranges = (std::max(max_M, 1) + tsg::kJit64TileM - 1) / tsg::kJit64TileM;
    for (int r = 1; r <= ranges; r++) {
        for (const int m : {(r - 1) * tsg::kJit64TileM + 1, std::min(std::max(max_M, 1), r * tsg::kJit64TileM)}) {
            if (pick_ell_variant(h, m) >= 0) continue;  // the small-M kernel (its images below)
            const JitShape sh = call_shape(h, m);
            rc = ensure_jit_variant(h, sh.nw, sh.waves, nullptr, sh.far, sh.r64, sh.half);
            if (rc == TSG_ERR_HIP && may_fall_back(h, sh)) {  // as run_dev
                std::fprintf(stderr, "[ternary_spgemm] warning: %s; running the 128-row 64 x 8 image instead\n",
                             g_tsg_host_err.c_str());
                h->bad_variants |= 1u << variant_bit(sh);
                rc = ensure_jit_variant(h, tsg::kJitNW);
            }
            if (rc) return rc;
        }
    }
    // the small-M images calls with M <= max_M run: the choice only changes
    // at M = 1..4 (1-row tiles by M * N), past an M tile or past kEllMidM, so
    // trying those covers them all
    for (int i = -4; i <= tsg::kEllVariants; i++) {
        const int m = i < 0 ? -i : i == tsg::kEllVariants ? kEllMidM + 1 : tsg::kEllTileM[i] + 1;
        const int v = m <= std::max(max_M, 1) ? pick_ell_variant(h, m) : -1;
        if (v >= 0) {
            rc = ensure_ell(h, v);
            if (rc) return rc;
        }
    }
    return TSG_OK;
}

extern "C" int tcsc_hip_set_jit_width(tsg_tcsc *h, int width)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    if (h->kind != tsg_tcsc::kJit) return fail(TSG_ERR_ARG, "tcsc_hip_set_jit_width: not a jit handle");
    if (width != 0 && (!tsg::jit64_width_ok(width) || (h->B && width != tsg::kJitNW)))
        return fail(TSG_ERR_ARG, "tcsc_hip_set_jit_width: expected 0 (auto), 128 (64-row image), 64, 32, 16 or 8 "
                                 "(64 for BlockedTCSC)");
    std::lock_guard<std::mutex> lk(h->mu);
    h->jit_force = width;
    return TSG_OK;
}

extern "C" int tcsc_hip_jit_width(const tsg_tcsc *h, int M)
{
    if (!h || h->kind != tsg_tcsc::kJit) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    return call_shape(h, M).nw;
}

extern "C" int tcsc_hip_jit_waves(const tsg_tcsc *h, int M)
{
    if (!h || h->kind != tsg_tcsc::kJit) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    return call_shape(h, M).waves;
}

extern "C" int tcsc_hip_set_tile_rows(tsg_tcsc *h, int rows)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    if (rows != 0 && rows != 64 && rows != 128) return fail(TSG_ERR_ARG, "tcsc_hip_set_tile_rows: expected 0 (auto), 64 or 128");
    if (rows == 64 && (h->kind != tsg_tcsc::kJit || h->B))
        return fail(TSG_ERR_ARG, "tcsc_hip_set_tile_rows: the 64-row image computes plain TCSC on the jit kernel only");
    std::lock_guard<std::mutex> lk(h->mu);
    h->tile_rows = rows;
    return TSG_OK;
}

extern "C" int tcsc_hip_call_launches(const tsg_tcsc *h, const float *dX, int M)
{
    if (!h || M <= 0) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    if (pick_ell_variant(h, M) >= 0) return 1;
    if (h->kind != tsg_tcsc::kJit) return 2;
    const JitShape sh = call_shape(h, M);
    if (!sh.r64) return 2;
    // the variant's width and layout as run_dev sees them (built or not yet)
    tsg_tcsc::JitVariant v = variant_of(const_cast<tsg_tcsc *>(h), sh);
    v.nw = sh.nw;
    if (!v.mod.function) v.piece_rows = sh.half ? (tsg::jit64_piece_rows() ? tsg::jit64_piece_rows() : 16)
                                                : tsg::jit64_piece_rows();
    return x_direct(h, dX, M, h->K, v) ? 1 : 2;
}

extern "C" int tcsc_hip_call_tile_rows(const tsg_tcsc *h, int M)
{
    if (!h) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->kind != tsg_tcsc::kJit || M <= 0 || pick_ell_variant(h, M) >= 0) return 0;
    return call_shape(h, M).r64 ? tsg::kJit64TileM : tsg::kJitTileM;
}

// Opt-in page-locking of a caller's host buffer (X or Y of repeated
// host-pointer calls): the copies of the pipeline then DMA straight from / to
// it instead of the runtime's pin-on-the-fly staging.  The caller keeps the
// buffer alive until tcsc_hip_host_unregister.
extern "C" int tcsc_hip_host_register(void *p, size_t bytes)
{
    if (!p || bytes == 0) return fail(TSG_ERR_ARG, "tcsc_hip_host_register: null pointer or zero size");
    HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterDefault));
    return TSG_OK;
}

extern "C" int tcsc_hip_host_unregister(void *p)
{
    if (!p) return fail(TSG_ERR_ARG, "tcsc_hip_host_unregister: null pointer");
    HIP_TRY(hipHostUnregister(p));
    return TSG_OK;
}

extern "C" int tcsc_hip_set_host_chunks(tsg_tcsc *h, int chunks)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    if (chunks < 0 || chunks > tsg_tcsc::kHostChunksMax)
        return fail(TSG_ERR_ARG, "tcsc_hip_set_host_chunks: expected 0 (auto) .. " +
                                     std::to_string(tsg_tcsc::kHostChunksMax));
    std::lock_guard<std::mutex> lk(h->host_mu);
    h->host_chunks = chunks;
    return TSG_OK;
}

extern "C" int tcsc_hip_host_chunk_rows(tsg_tcsc *h, int M)
{
    if (!h || M <= 0) return 0;
    std::lock_guard<std::mutex> lk(h->host_mu);
    return host_chunk_rows(h, M);
}

extern "C" int tcsc_hip_set_far(tsg_tcsc *h, int mode)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    if (mode < 0 || mode > 2) return fail(TSG_ERR_ARG, "tcsc_hip_set_far: expected 0 (auto), 1 (never) or 2 (always)");
    std::lock_guard<std::mutex> lk(h->mu);
    h->far_mode = mode;
    return TSG_OK;
}

extern "C" int tcsc_hip_call_far(const tsg_tcsc *h, int M)
{
    if (!h) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->kind != tsg_tcsc::kJit || M <= 0 || pick_ell_variant(h, M) >= 0) return 0;
    const JitShape sh = call_shape(h, M);
    return !sh.r64 && sh.far ? 1 : 0;
}

extern "C" int tcsc_hip_set_small_m(tsg_tcsc *h, int mode)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    if (mode < 0 || mode > 3)
        return fail(TSG_ERR_ARG, "tcsc_hip_set_small_m: expected 0 (auto), 1 (never), 2 (always) or 3 (always, "
                                 "without the producer/consumer walk)");
    if (mode >= 2 && (h->kind != tsg_tcsc::kJit || h->B))
        return fail(TSG_ERR_ARG, "tcsc_hip_set_small_m: the small-M kernel computes plain TCSC (BaseTCSC) only");
    std::lock_guard<std::mutex> lk(h->mu);
    h->small_m = mode;
    return TSG_OK;
}

// The automatic per-call plan of a plain-TCSC handle with K, N and nnz
// nonzeros at density split evenly (host only, no GPU: the same functions
// run_dev uses on a handle).  kernel: 0 weight-compiled (128-row image), 1
// ELL walk, 2 ELL producer/consumer walk, 3 weight-compiled 64-row image.
extern "C" int tsg_call_plan(int K, int N, int64_t nnz, int M, int *kernel, int *width, int *waves, int *far,
                             int *gn, int *gm, int *tmask)
{
    if (K < 0 || N <= 0 || nnz < 0 || nnz > (int64_t)K * N || M <= 0 || !kernel || !width || !waves || !far ||
        !gn || !gm || !tmask) {
        g_tsg_host_err = "tsg_call_plan: bad arguments";
        return TSG_ERR_ARG;
    }
    tsg_tcsc h;  // plain struct: nothing allocated, nothing on the device
    h.K = K;
    h.N = N;
    h.nnz_pos = nnz - nnz / 2;
    h.nnz_neg = nnz / 2;
    h.jit_nch = std::max(1, (K + tsg::kJitChunk - 1) / tsg::kJitChunk);
    const int ev = pick_ell_variant(&h, M);
    const bool r64 = ev < 0 && pick_rows64(&h, M);
    *kernel = ev >= 0 ? (use_ell_pc(&h, ev) ? 2 : 1) : r64 ? 3 : 0;
    *width = *waves = *far = *gn = *gm = *tmask = 0;
    if (ev < 0) {
        const JitShape sh = pick_jit_shape(&h, M, r64);
        const int tm = r64 ? tsg::kJit64TileM : tsg::kJitTileM;
        const int ntiles = (N + sh.nw * sh.waves - 1) / (sh.nw * sh.waves);
        *width = sh.nw;
        *waves = sh.waves;
        *far = sh.far ? 1 : 0;
        pick_jit_map(&h, (M + tm - 1) / tm, ntiles, *gn, *gm, *tmask, r64 ? sh.nw : 0);
    }
    return TSG_OK;
}

// Whether an M-row call of a plain-TCSC handle with K, N and nnz nonzeros
// spreads the generated code's per-group touches (pick_xtouch; host only).
extern "C" int tsg_call_xtouch(int K, int N, int64_t nnz, int M)
{
    if (K < 0 || N <= 0 || nnz < 0 || nnz > (int64_t)K * N || M <= 0) {
        g_tsg_host_err = "tsg_call_xtouch: bad arguments";
        return TSG_ERR_ARG;
    }
    tsg_tcsc h;
    h.K = K;
    h.N = N;
    h.nnz_pos = nnz - nnz / 2;
    h.nnz_neg = nnz / 2;
    return pick_xtouch(&h, M) ? 1 : 0;
}

extern "C" const char *tcsc_hip_call_kernel(const tsg_tcsc *h, int M)
{
    if (!h) return "";
    std::lock_guard<std::mutex> lk(h->mu);
    const int ev = pick_ell_variant(h, M);
    if (ev >= 0) return use_ell_pc(h, ev) ? "tsg_tcsc_ell_pc_kernel" : "tsg_tcsc_ell_kernel";
    if (h->kind == tsg_tcsc::kJit && call_shape(h, M).r64) return "tsg_jit64_kernel";
    return h->kind == tsg_tcsc::kJit ? "tsg_jit_kernel" : "tsg_tcsc_rx_kernel";
}

extern "C" int64_t tcsc_hip_call_image_bytes(tsg_tcsc *h, int M)
{
    if (!h || M <= 0) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    const int ev = pick_ell_variant(h, M);
    if (ev >= 0) return h->ell[ev].ready ? h->ell[ev].bytes : 0;
    if (h->kind != tsg_tcsc::kJit) return (int64_t)(h->rimg.wstart.size() + h->rimg.ent.size()) * 4;
    const tsg_tcsc::JitVariant &v = variant_of(h, call_shape(h, M));
    return v.mod.function ? v.code_bytes + v.wcode_words * 4 : 0;
}

extern "C" int tcsc_hip_gemm(tsg_tcsc *h, const float *X, const float *b, float *Y, int M, int N, int K)
{
    return run_host(h, X, b, nullptr, Y, M, N, K, false);
}

extern "C" int tcsc_hip_gemm_prelu(tsg_tcsc *h, const float *X, const float *b, const float *alpha,
                                   float *Y, int M, int N, int K)
{
    return run_host(h, X, b, alpha, Y, M, N, K, true);
}

extern "C" int tcsc_hip_gemm_dev(tsg_tcsc *h, const float *dX, const float *db, float *dY, int M,
                                 int N, int K, void *stream)
{
    return run_dev(h, dX, db, nullptr, dY, M, N, K, (hipStream_t)stream, false);
}

extern "C" int tcsc_hip_gemm_prelu_dev(tsg_tcsc *h, const float *dX, const float *db,
                                       const float *dalpha, float *dY, int M, int N, int K,
                                       void *stream)
{
    return run_dev(h, dX, db, dalpha, dY, M, N, K, (hipStream_t)stream, true);
}

extern "C" int tcsc_hip_info(const tsg_tcsc *h, tsg_info *o)
{
    if (!h || !o) return fail(TSG_ERR_ARG, "null argument");
    std::memset(o, 0, sizeof(*o));
    o->K = h->K;
    o->N = h->N;
    o->device = h->device;
    o->abi_version = TSG_ABI_VERSION;
    o->nnz_pos = h->nnz_pos;
    o->nnz_neg = h->nnz_neg;
    // TCSC / BlockedTCSC getDataStructureSize (TCSC.h:43-49, BlockedTCSC.h:43-47)
    o->tcsc_bytes = 4 * (2 * (int64_t)h->csp.size() + h->nnz_pos + h->nnz_neg);
    const bool jit = h->kind == tsg_tcsc::kJit;
    int64_t jit_bytes = 0;
    for (const auto &v : h->jv) jit_bytes += v.code_bytes + v.wcode_words * 4;
    for (const auto &v : h->jv64) jit_bytes += v.code_bytes + v.wcode_words * 4;
    for (const auto &v : h->jv64h) jit_bytes += v.code_bytes + v.wcode_words * 4;
    for (const auto &e : h->ell) jit_bytes += e.bytes;
    o->image_bytes = jit ? jit_bytes : (int64_t)(h->rimg.wstart.size() + h->rimg.ent.size()) * 4;
    o->work_bytes = (int64_t)h->work_bytes;
    // the image registration loaded: the 64-row image's 128 x 8 when it could
    // (create_impl), else the 128-row 64 x 8 one (or rx)
    const tsg_tcsc::JitVariant &r64 = h->jv64[shape_index(tsg::kJit64WideNW, tsg::kJitWaves, false)];
    const bool reg64 = jit && r64.mod.function;
    o->chunk_rows = reg64 ? r64.chunk : jit ? tsg::kJitChunk : tsg::kRxChunk;
    o->tile_rows = reg64 ? tsg::kJit64TileM : jit ? tsg::kJitTileM : tsg::kRxTileM;
    o->tile_cols = reg64 ? tsg::kJit64WideNW * tsg::kJitWaves : jit ? tsg::kJitTileCols : tsg::kRxTileCols;
    return TSG_OK;
}

extern "C" const char *tcsc_hip_kernel_name(const tsg_tcsc *h)
{
    if (!h) return "";
    return h->kind == tsg_tcsc::kJit ? "tsg_jit_kernel" : "tsg_tcsc_rx_kernel";
}

extern "C" int tcsc_hip_to_dense(const tsg_tcsc *h, int32_t *W, int K, int N)
{
    if (!h || !W || K != h->K || N != h->N) return fail(TSG_ERR_ARG, "bad to_dense arguments");
    std::memset(W, 0, sizeof(int32_t) * (size_t)K * N);
    const size_t slots = h->csp.size() - 1;  // N, or (K/B)*N for BlockedTCSC (slot s: column s % N)
    for (size_t s = 0; s < slots; s++) {
        const size_t n = s % (size_t)N;
        for (int32_t i = h->csp[s]; i < h->csp[s + 1]; i++) W[(size_t)h->rip[i] * N + n] = 1;
        for (int32_t i = h->csn[s]; i < h->csn[s + 1]; i++) W[(size_t)h->rin[i] * N + n] = -1;
    }
    return TSG_OK;
}

extern "C" int tcsc_hip_set_timing(tsg_tcsc *h, int enable)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    int rc = enable ? ensure_events(h) : harvest_timing(h, true);
    if (rc) return rc;
    h->timing = enable != 0;
    return TSG_OK;
}

extern "C" int tcsc_hip_kernel_time(tsg_tcsc *h, double *total_ms, int64_t *launches, int reset)
{
    if (!h) return fail(TSG_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard g(h->device);
    int rc = harvest_timing(h, true);
    if (rc) return rc;
    if (total_ms) *total_ms = h->total_ms;
    if (launches) *launches = h->launches;
    if (reset) {
        h->total_ms = 0.0;
        h->launches = 0;
    }
    return TSG_OK;
}
