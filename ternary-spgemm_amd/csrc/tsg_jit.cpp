// tsg_jit.cpp -- host side of the weight-compiled ("jit") TCSC kernel:
//   1. build_jit_code: turns the TCSC arrays into gfx950 machine code, one
//      straight-line stream per (column tile, wave) (register contract:
//      tsg_jit_kernel.hip header);
//   2. JitModule::load: appends that code to the dispatcher's code object
//      (lib/tsg_jit.co) as a PT_LOAD R|X segment, patches the dispatcher's
//      region-base literal, and loads the image with hipModuleLoadData.
//
// Order contract (cpp_impl/comp.h:37-63, BaseTCSC): for every column the
// generated adds are its +1 entries in ascending k over all chunks, then its
// -1 entries in ascending k, one v_pk_add_f32 pair per entry (two IEEE adds,
// rows 0-1 and 2-3 of the lane); the dispatcher adds b[n] last.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <elf.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>

#include "tsg_internal.h"
#include "tsg_jit_map.h"
#include "../../include/ternary_spgemm_test.h"

namespace tsg {

namespace {

// --- gfx950 encodings (checked against llvm-mc -mcpu=gfx950 -show-encoding) ---
struct Emit {
    std::vector<uint32_t> &c;
    bool pad8 = true;  // TSG_JIT_NOALIGN=1: A/B knob (results unchanged)
    // keep 8-byte instructions 8-byte aligned (hand-asm placement rule)
    void align8()
    {
        if (pad8 && (c.size() & 1)) c.push_back(0xbf800000u);  // s_nop 0
    }
    // v_pk_add_f32 v[d:d+1], v[d:d+1], v[x:x+1] [neg_lo:[0,1] neg_hi:[0,1]]  (VOP3P;
    // the two halves are rows 0 and 1 of the lane: two IEEE adds)
    void pk_add(uint32_t d, uint32_t x, bool neg)
    {
        align8();
        c.push_back(0xd3b24000u | d | (neg ? 0x200u : 0u));
        c.push_back((3u << 27) | ((256u + x) << 9) | (256u + d) | (neg ? (2u << 29) : 0u));
    }
    // v_pk_add_f32 v[d:d+1], [-]v[x:x+1], 0: the first entry of a BlockedTCSC
    // block, 0 + x (resp. 0 - x) as one IEEE add per half
    void pk_first(uint32_t d, uint32_t x, bool neg)
    {
        align8();
        c.push_back(0xd3b24000u | d | (neg ? 0x100u : 0u));
        c.push_back((3u << 27) | (128u << 9) | (256u + x) | (neg ? (1u << 29) : 0u));
    }
    // v_pk_add_f32 v[d:d+1], v[d:d+1], v[t:t+1]: Y += y of a finished block
    void pk_acc(uint32_t d, uint32_t t)
    {
        align8();
        c.push_back(0xd3b24000u | d);
        c.push_back((3u << 27) | ((256u + t) << 9) | (256u + d));
    }
    // 64-row image: v_add_f32 v[d], v[d], v[x] / v_sub_f32 v[d], v[d], v[x]
    // (VOP2, 4 bytes: d = d + x for a +1 entry, d = d - x for a -1 entry --
    // comp.h:47 `y += x` and comp.h:57 `y -= x` on one M row per lane)
    void v_addsub(uint32_t d, uint32_t x, bool neg)
    {
        c.push_back(((neg ? 2u : 1u) << 25) | (d << 17) | (x << 9) | (256u + d));
    }
    // ds_read_b32 v[d], v[a] offset:off
    void ds_read_b32(uint32_t d, uint32_t a, uint32_t off)
    {
        align8();
        c.push_back(0xd86c0000u | off);
        c.push_back((d << 24) | a);
    }
    // ds_read_b64 v[d:d+1], v[a] offset:off
    void ds_read_b64(uint32_t d, uint32_t a, uint32_t off)
    {
        align8();
        c.push_back(0xd8ec0000u | off);
        c.push_back((d << 24) | a);
    }
    // ds_read_b128 v[d:d+3], v[a] offset:off   (a k-row pair: both rows of the lane's 2 M rows)
    void ds_read_b128(uint32_t d, uint32_t a, uint32_t off)
    {
        align8();
        c.push_back(0xd9fe0000u | off);
        c.push_back((d << 24) | a);
    }
    // global_load_lds_dwordx4 v[voff], s[84:85] offset:off   (LDS-DMA: global
    // s[84:85] + v[voff] + off -> LDS M0 + off; the offset applies to BOTH
    // addresses on gfx950, scripts/glds_offset_micro.hip)
    uint32_t dma_cp = 0, touch_cp = 0;  // cache-policy bits (sc0 16, nt 17, sc1 25) of the DMA / touch loads
    void glds_x4(uint32_t voff, uint32_t off = 0)
    {
        align8();
        c.push_back(0xddf48000u | (off & 0xfffu) | dma_cp);
        c.push_back((84u << 16) | voff);
    }
    // global_load_dword v[sink], v[lane*128], s[88:89]   (code prefetch into L2)
    void code_touch(uint32_t sink, uint32_t l128)
    {
        align8();
        c.push_back(0xdc508000u | touch_cp);
        c.push_back((sink << 24) | (88u << 16) | l128);
    }
    void m0_wave(uint32_t v) { align8(); c.push_back(0x807cff53u); c.push_back(v); }  // s_add_u32 m0, s83, v
    void save_m0() { c.push_back(0xbed6007cu); }      // s_mov_b32 s86, m0
    void restore_m0() { c.push_back(0xbefc0056u); }   // s_mov_b32 m0, s86
    void base_reset() { c.push_back(0xbed40150u); }   // s_mov_b64 s[84:85], s[80:81]
    void base_next()                                  // s[84:85] += s82
    {
        c.push_back(0x80545254u);
        c.push_back(0x82558055u);
    }
    void base_last_adj()                              // s[84:85] -= s87 (row layout: the last chunk starts at K - 188)
    {
        c.push_back(0x80d45754u);
        c.push_back(0x82d58055u);
    }
    // s[88:89] = s[90:91] + off: s[90:91] is the touch base the dispatcher
    // sets per call -- the region base, or 8 KiB below it (the touches then
    // cover the code from the step's own position, tsg_capi.cpp tnear)
    void touch_addr(uint32_t region_off)
    {
        align8();
        c.push_back(0x8058ff5au);
        c.push_back(region_off);
        c.push_back(0x8259805bu);
    }
    void nop(uint32_t n = 0) { c.push_back(0xbf800000u | n); }
    void wait_lgkm(uint32_t n) { c.push_back(0xbf8cc07fu | (n << 8)); }  // s_waitcnt lgkmcnt(n), n <= 15
    void wait_vm0() { c.push_back(0xbf8c0f70u); }
    void wait_vm(uint32_t n) { c.push_back(0xbf8c0f70u | n); }            // s_waitcnt vmcnt(n), n <= 15
    void barrier() { c.push_back(0xbf8a0000u); }
    void setprio(uint32_t p) { c.push_back(0xbf8f0000u | p); }  // s_setprio p (issue arbitration between waves)
    void ret() { c.push_back(0xbe801d5eu); }         // s_setpc_b64 s[94:95]
    uint32_t pos_bytes() const { return (uint32_t)(c.size() * 4); }
};

// Register contract (tsg_jit_kernel.hip): X slots v[8 : 8 + 96) (24 slots of 4
// VGPRs: one k-row pair each), then kJitRing LDS buffer bases (buffer + lane *
// 16), the code-prefetch sink, the DMA piece offsets, lane*128, and the
// accumulators from the next even register.
constexpr uint32_t kPairBytes = kJitTileM * 8;            // one k-row pair (64-row image: quad) of the tile in LDS: 1 KiB
static_assert(kPairBytes == 1024, "one LDS-DMA piece (64 lanes x 16 B) is one pair row");
static_assert(kJit64HalfChunk / 4 % 4 == 0, "half ring: whole pieces per wave at 4 waves");
static_assert(kJit64TileM * 16 == (int)kPairBytes && kJit64Chunk / 4 == kJitChunk / 2,
              "64-row image: a quad row is one 1-KiB piece, 48 of them per chunk (the same ring)");
constexpr uint32_t kXSlot0 = 8;                            // slot s: v[8 + 4s : 11 + 4s]
constexpr uint32_t kLdsBaseV = kXSlot0 + kJitXRegs;        // + b: buffer b + lane * 16
constexpr uint32_t kSinkV = kLdsBaseV + kJitRing;
constexpr uint32_t kDmaOffV = kSinkV + 1;                  // + i: DMA piece i offsets
// then, by the waves W of the workgroup: chunk/2/W DMA piece offsets, lane*128,
// and the accumulators from the next even register (JitRegs)
struct JitRegs {
    int pieces;         // DMA pieces (pair rows) per wave per chunk
    uint32_t lane128;   // v[lane * 128]
    uint32_t acc0;      // column c: v[acc0 + 2c : acc0 + 2c + 1]
    explicit JitRegs(int waves, int units = kJitChunk / 2)  // units: 1-KiB pieces per chunk
        : pieces(units / waves), lane128(kDmaOffV + (uint32_t)(units / waves)),
          acc0((kDmaOffV + (uint32_t)(units / waves) + 2) & ~1u)
    {
    }
};
static_assert(((kDmaOffV + kJitChunk / 2 / kJitWaves + 2) & ~1u) + 2 * kJitNW <= 256u, "VGPR budget");
static_assert(((kDmaOffV + kJitChunk / 2 / 4 + 2) & ~1u) + 2 * 32 <= 256u, "VGPR budget, 4 waves");
static_assert(((kDmaOffV + kJitChunk / 2 / kJitWaves + 2) & ~1u) + kJit64WideNW <= 256u, "VGPR budget, 64-row x 128");
// narrower streams (jit width < kJitNW) use the same register contract, fewer accumulators
constexpr int kTailPad = kJitTailPadWords;  // words of padding after the last stream (code prefetch reads ahead)
static_assert((kJitChunk / 2 - 1) * kPairBytes + 8 < 65536, "ds_read offset field");

// One step's work for a wave: its X reads (k-row units of the chunk with an
// entry in the step, ascending: pairs, or quads in the 64-row image) and, per
// read, the columns with an entry in each row of the unit.
struct Section {
    struct Read {
        int pair = 0;                      // unit index in the chunk (pair / quad)
        int mask = 0;                      // bit r: row r of the unit used
        std::vector<uint8_t> cols[4];
    };
    std::vector<Read> reads;
};

// 64-row image: how a quad with used-row mask `mask` is read -- byte offset in
// the quad, VGPRs loaded and the first row they hold (ds_read_b32 / b64 for
// quads with one used row / rows only in one half, else ds_read_b128)
struct QuadRead {
    uint32_t off;
    int nreg, row0;
};
QuadRead quad_read(int mask)
{
    if (mask == 1 || mask == 2 || mask == 4 || mask == 8) {
        const int r = mask == 1 ? 0 : mask == 2 ? 1 : mask == 4 ? 2 : 3;
        return {(uint32_t)r * 4u, 1, r};
    }
    if ((mask & ~3) == 0) return {0u, 2, 0};
    if ((mask & 3) == 0) return {8u, 2, 2};
    return {0u, 4, 0};
}

// One step of a stream: the X^T chunk staged into LDS buffer q % kJitRing and which
// of its entries the step adds.
struct StepSpec {
    int chunk;       // X^T chunk (kJitChunk rows)
    int pass;        // 0: +1 entries, 1: -1 entries
    int c0, c1;      // the wave's columns [c0, c1)
    int klo, khi;    // rows the step consumes (a BlockedTCSC block may end inside the chunk)
    int64_t slot0;   // column n's entries are TCSC slot slot0 + n (BlockedTCSC: block * N)
    bool reset;      // first step of a (block, pass) run: the entry cursors restart at the slots
    bool flush;      // BlockedTCSC: the block's last step: Y += y for its columns
};

// BaseTCSC (comp.h:37-63): pass 0 over every chunk, then pass 1; the wave's
// columns accumulate in place.
// BaseBlockedTCSC (comp.h:620-646): per block y = 0 + pos - neg, then
// Y += y.  y of every column of a block is live across the block's chunks, so
// a wave runs its columns in two halves (y of half the columns in the upper
// X-slot registers); per half, block by block: pass 0 over the chunks the
// block touches, pass 1, then Y += y.
std::vector<StepSpec> plan_steps(int K, int N, int B, int nch, int nw, int C = kJitChunk)
{
    std::vector<StepSpec> plan;
    if (!B) {
        for (int p = 0; p < 2; p++)
            for (int j = 0; j < nch; j++) plan.push_back({j, p, 0, nw, j * C, j * C + C, 0, j == 0, false});
        return plan;
    }
    const int nb = K / B, half = nw / 2;  // rows past nb * B are not in the format (BlockedTCSC.h:17)
    for (int h = 0; h < 2; h++)
        for (int kb = 0; kb < nb; kb++) {
            const int r0 = kb * B, r1 = r0 + B, jlo = r0 / C, jhi = (r1 - 1) / C;
            for (int p = 0; p < 2; p++)
                for (int j = jlo; j <= jhi; j++)
                    plan.push_back({j, p, h * half, h * half + half, std::max(r0, j * C), std::min(r1, j * C + C),
                                    (int64_t)kb * N, j == jlo, p == 1 && j == jhi});
        }
    return plan;
}

}  // namespace

#ifdef TSG_DIAG
// Column -> wave assignment of one column tile that evens out the waves'
// per-step work (round 6, diagnostic build only; measured no faster --
// configs[1] 59.6 vs 59.4 us, s = 16 428.4 vs 430.0, configs[2] +3%; even
// piling the heaviest columns on the first waves changes nothing:
// profiles/r06s_balance_diag.jsonl -- the per-step barrier costs its sync,
// not the waves' imbalance): every step ends in a workgroup
// barrier, so a step lasts as long as its busiest wave.  The tile's columns
// move between waves in units of `unit` consecutive columns (4 keeps the
// epilogue's float4 stores); a local search swaps units between waves while
// the sum over steps of the busiest wave's entries does not grow.  perm[w *
// nw + c] = the tile-local column the wave's accumulator c holds.
std::vector<int> balance_tile(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                              int N, int n_tile0, int tile_cols, int waves, int nw, int CH, int nch, int unit,
                              bool anti)
{
    const int steps = 2 * nch, units = tile_cols / unit, upw = nw / unit;
    std::vector<int64_t> V((size_t)units * steps, 0);  // entries per (unit, step)
    for (int p = 0; p < 2; p++) {
        const int32_t *cs = p ? csn : csp, *ri = p ? rin : rip;
        for (int cl = 0; cl < tile_cols; cl++) {
            const int n = n_tile0 + cl;
            if (n >= N) continue;
            for (int32_t i = cs[n]; i < cs[n + 1]; i++)
                V[(size_t)(cl / unit) * steps + p * nch + std::min(ri[i] / CH, nch - 1)]++;
        }
    }
    std::vector<int> g(units);  // g[w * upw + j] = unit
    for (int u = 0; u < units; u++) g[u] = u;
    if (anti) {  // the heaviest units on the first waves
        std::vector<int64_t> tot(units, 0);
        for (int u = 0; u < units; u++)
            for (int q = 0; q < steps; q++) tot[u] += V[(size_t)u * steps + q];
        std::stable_sort(g.begin(), g.end(), [&](int a, int b) { return tot[a] > tot[b]; });
    } else if (waves > 1) {
        std::vector<int64_t> S((size_t)waves * steps, 0);
        for (int w = 0; w < waves; w++)
            for (int j = 0; j < upw; j++)
                for (int q = 0; q < steps; q++) S[(size_t)w * steps + q] += V[(size_t)g[w * upw + j] * steps + q];
        uint64_t rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)n_tile0;
        auto rnd = [&](int m) {
            rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
            return (int)(rng % (uint64_t)m);
        };
        const int iters = 40 * units * waves;
        for (int it = 0; it < iters; it++) {
            const int a = rnd(waves), b0 = rnd(waves - 1), b = b0 >= a ? b0 + 1 : b0;
            const int i = rnd(upw), j = rnd(upw);
            const int ua = g[a * upw + i], ub = g[b * upw + j];
            int64_t dcost = 0;
            for (int q = 0; q < steps; q++) {
                int64_t mo = 0;
                for (int w = 0; w < waves; w++)
                    if (w != a && w != b) mo = std::max(mo, S[(size_t)w * steps + q]);
                const int64_t d = V[(size_t)ub * steps + q] - V[(size_t)ua * steps + q];
                const int64_t sa = S[(size_t)a * steps + q], sb = S[(size_t)b * steps + q];
                dcost += std::max(mo, std::max(sa + d, sb - d)) - std::max(mo, std::max(sa, sb));
            }
            if (dcost <= 0) {
                for (int q = 0; q < steps; q++) {
                    const int64_t d = V[(size_t)ub * steps + q] - V[(size_t)ua * steps + q];
                    S[(size_t)a * steps + q] += d;
                    S[(size_t)b * steps + q] -= d;
                }
                g[a * upw + i] = ub;
                g[b * upw + j] = ua;
            }
        }
        for (int w = 0; w < waves; w++) std::sort(g.begin() + w * upw, g.begin() + (w + 1) * upw);
    }
    std::vector<int> perm(tile_cols);
    for (int w = 0; w < waves; w++)
        for (int j = 0; j < upw; j++)
            for (int e = 0; e < unit; e++) perm[w * nw + j * unit + e] = g[w * upw + j] * unit + e;
    return perm;
}
#endif

int jit64_piece_rows()
{
    const char *v = knob_value("TSG_JIT_QBLOCK");
    return !v ? 0 : v[0] == '8' ? 8 : 16;
}

void build_jit_code(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                    int K, int N, int B, JitImage &img, int nw, int waves, bool far, bool r64, bool half)
{
    if (nw <= 0) nw = kJitNW;
    if (!jit_waves_ok(nw, waves)) waves = kJitWaves;
    if (B) r64 = false;  // BlockedTCSC: the 128-row image only
    if (nw > kJitNW && !r64) nw = kJitNW;  // 128 columns per wave: the 64-row image only (callers check)
    if (!r64 || waves != 4) half = false;  // the half ring: 4-wave 64-row workgroups only
    if (r64) far = false;
    // K rows per chunk and per LDS unit (a pair, or a quad in the 64-row image):
    // 48 units of 1 KiB per chunk either way
    // the 64-row image's row layout (default; tsg_internal.h kJit64RowFlag) or
    // its blocked layout (TSG_JIT_QBLOCK; the half ring always)
    const bool rowlay = r64 && !half && jit64_piece_rows() == 0;
    const int CH = r64 ? (half ? kJit64HalfChunk : rowlay ? kJit64RowChunk : kJit64Chunk) : kJitChunk,
              U = r64 ? 4 : 2;
    // one LDS ring buffer: 48 KiB (row layout: 47 KiB used), half ring 24
    const uint32_t kBuf = rowlay ? 48u * 1024u : (uint32_t)(CH / U) * kPairBytes;
    // 64-row image, blocked layout: rows per DMA piece PR (16 or 8) and quads
    // per piece 64 / PR (tsg_internal.h, kJit64R16Flag); 0 = the row layout
    const int PR = r64 && !rowlay ? (jit64_piece_rows() ? jit64_piece_rows() : 16) : 0, PQ = PR ? 64 / PR : 0;
    const JitRegs R(waves, rowlay ? 48 : CH / U);  // (row layout: 47 pieces, the register contract of 48)
    const int streams = waves;  // one stream per wave (no M split)
    const int kPieces = R.pieces;
    const uint32_t kLane128V = R.lane128, kAcc0 = R.acc0;
    const int tile_cols = nw * streams;
    img.K = K;
    img.N = N;
    img.B = B;
    img.nw = nw;
    img.waves = waves;
    img.tile_m = r64 ? kJit64TileM : kJitTileM;
    img.chunk = CH;
    img.piece_rows = PR;
    img.half = half;
    img.Npad = ((N + tile_cols - 1) / tile_cols) * tile_cols;
    img.nch = std::max(1, (K + CH - 1) / CH);
    const int nch = img.nch, ntiles = img.Npad / tile_cols;
    const std::vector<StepSpec> plan = plan_steps(K, N, B, nch, nw, CH);
    const int steps = (int)plan.size();
    // LDS-DMA issue (TSG_JIT_DMA="spread,m0k" overrides, A/B): the pieces that
    // stage step q + kJitRing - 1 go out spread over the first `spread` of step
    // q's read groups instead of all at the step start (every wave of a CU
    // reaches the step start together after the barrier: issued at once, the
    // pieces queue at the CU's vector-memory path and stall every wave);
    // m0k: one M0 write per 4 pieces, the piece offset in the instruction's
    // offset field (the dispatcher subtracts it from the per-piece global
    // offsets; region header word 7, kJitM0kFlag)
    // lag: 1 = a step's pieces are waited for at the end of that step, so the
    // next step's first reads can go out before the barrier (read-ahead
    // across steps); 2 = they are waited for one step later (the DMA gets
    // two steps to land -- for X^T served from far memory) and each step's
    // reads start after its barrier
    //
    // Default spread (profiles/r03_dma_lag_ab.txt, r03c_dma_spread_far_ab.txt):
    // 0 -- every piece at the step start -- for long sparse streams (K >= 8192,
    // density <= 3/16: short steps over X^T from far memory, where a late
    // piece does not land in time: (64000, 16384, 4096) s = 8 15.7 -> 12.6 ms,
    // (16000, 8192, 2048) s = 8 0.92 -> 0.74 ms); else 0.5 (configs[2] 1.229
    // -> 1.197 ms, configs[1] 0.101 -> 0.096 ms, (64000, 16384, 4096) s = 4
    // 26.4 -> 25.2 ms).  Lag 2 gained nowhere (kept as an A/B option).
    const int64_t nnz_all = B ? (int64_t)csp[(int64_t)(K / B) * N] + csn[(int64_t)(K / B) * N]
                              : (int64_t)csp[N] + csn[N];
    const double density = (double)nnz_all / std::max(1.0, (double)K * (double)N);
    // dense W (density > 3/8, s = 2) on the 64-wide image: also 0 -- its long
    // steps leave the late pieces too little time (configs[3] s = 2 2.535 ->
    // 2.452 ms; the 32-wide image of (256, 4096, 16384) s = 2 loses 4% with
    // it, profiles/r03g_s2_ab.txt)
    double dma_spread = (K >= 8192 && density <= 0.1875) || (density > 0.375 && nw == kJitNW) ? 0.0 : 0.5;
    int m0k = 1, lag = 1;
    if (const char *dv = knob_value("TSG_JIT_DMA")) std::sscanf(dv, "%lf,%d,%d", &dma_spread, &m0k, &lag);
    if (lag != 2) lag = 1;
    // Stagger (TSG_JIT_STAGGER=1, 8-wave workgroups; MI355X_MICROARCH.md "Two
    // waves per SIMD" item 9): waves w and w + 4 share a SIMD and run the same
    // step structure in lockstep -- their DMA issue, LDS reads and adds
    // collide.  The first half of the waves then runs half a step AHEAD: its
    // barrier sits in the middle of a step (after half its read groups), the
    // DMA pieces it issues go out after that barrier and are waited for before
    // its next one, and before it a wave reads only its current step's chunk.
    // Barrier k then orders the early waves' mid-step k+1 with the late
    // waves' end of step k: every ring buffer is still written only after all
    // waves finished reading it and read only after all its pieces landed
    // (checked by the CPU emulation, tests/test_jit_codegen.py).
    // TSG_JIT_PRIO=1: s_setprio 1 for the waves of the second half (item 4).
    const char *sv = knob_value("TSG_JIT_STAGGER");
    const bool stagger = sv && sv[0] == '1' && waves == 8 && !B && lag == 1;
    const char *pv = knob_value("TSG_JIT_PRIO");
    const bool prio = pv && pv[0] == '1' && waves == 8;
    // TSG_JIT_MIX="reads,dma" (A/B, 0|1 each): a read group's read-ahead
    // (ds_read) and its share of the DMA pieces go out spread evenly among
    // the group's adds instead of in a burst before them (not with the
    // stagger).  Slot safety is unchanged: the read-ahead of group [i0, i0 +
    // G) refills the previous group's slots only (RA + G <= S).
    int mix_reads = 0, mix_dma = 0;
    if (const char *mv = knob_value("TSG_JIT_MIX")) std::sscanf(mv, "%d,%d", &mix_reads, &mix_dma);
    if (stagger) mix_reads = mix_dma = 0;
    // X slots: all of v[8 : 104) for BaseTCSC; BlockedTCSC keeps y of half the
    // columns (nw registers) at the top of that range
    const int S = B ? (kJitXRegs - nw) / kJitSlotRegs : kJitSlots;
    const uint32_t kTmp0 = kXSlot0 + (uint32_t)(kJitSlotRegs * S);  // y of column c0 + c: v[tmp0 + 2c : +1]
    img.wcode.assign((size_t)ntiles * streams, 0u);
    std::vector<uint32_t> &code = img.code;
    code.clear();
    const int64_t slots = (B ? (int64_t)(K / B) : 1) * N;
    const int64_t nnz = (int64_t)csp[slots] + (int64_t)csn[slots];
    code.reserve((size_t)nnz * 2 + (size_t)ntiles * streams * ((size_t)steps * 150 + 64) + kTailPad + 64);
    // header: magic, then the geometry (tests/test_jit_codegen.py derives the
    // register contract from it), the block size, the X slots in use, the
    // ring and the X^T layout
    code.insert(code.end(), {kJitMagic0, kJitMagic1,
                             (uint32_t)waves | (uint32_t)nw << 8 | (uint32_t)CH << 16,
                             (uint32_t)kJitSlots | (uint32_t)img.tile_m << 16,
                             (uint32_t)streams | (uint32_t)kJitMSplit << 8, (uint32_t)B, (uint32_t)S,
                             (uint32_t)kJitRing | (r64 ? kJit64Format : kJitFormat) << 8 |
                                 (uint32_t)(m0k ? kJitM0kFlag : 0u) | (far ? kJitFarFlag : 0u) |
                                 (PR == 16 ? kJit64R16Flag : 0u) | (half ? kJit64HalfFlag : 0u) |
                                 (rowlay ? kJit64RowFlag : 0u)});
    const char *na = knob_value("TSG_JIT_NOALIGN");
    Emit E{code, !(na && na[0] == '1')};
    // TSG_JIT_CP="dma,touch": cache-policy bits of the LDS-DMA pieces and the
    // code touches (hex; 0x20000 = nt, 0x2000000 = sc1, 0x10000 = sc0; A/B)
    if (const char *cv = knob_value("TSG_JIT_CP")) {
        unsigned a = 0, t = 0;
        std::sscanf(cv, "%x,%x", &a, &t);
        E.dma_cp = a & 0x2030000u;
        E.touch_cp = t & 0x2030000u;
    }
    // far-X^T image (tsg_capi.cpp far_xt): X^T staged non-temporally so its
    // stream does not evict the code from the Infinity Cache, and no code
    // touches
    if (far) E.dma_cp |= 0x20000u;
    // TSG_JIT_DIAG (diagnostic build only, -DTSG_DIAG; results WRONG, timing
    // studies): comma list of nobar (no s_barrier), nodma (no LDS-DMA),
    // notouch (no code prefetch), nolgkm (no LDS waits), noreads (no X reads),
    // novm (the DMA pieces are never waited for: tells the DMA's latency from
    // its issue cost).  The product library never reads it (tsg_knobs.cpp).
#ifdef TSG_DIAG
    const std::string diag = knob_value("TSG_JIT_DIAG") ? knob_value("TSG_JIT_DIAG") : "";
    auto has = [&](const char *f) { return diag.find(f) != std::string::npos; };
    const bool d_nobar = has("nobar"), d_nodma = has("nodma"), d_notouch = has("notouch"),
               d_nolgkm = has("nolgkm"), d_noreads = has("noreads"), d_novm = has("novm");
#else
    constexpr bool d_nobar = false, d_nodma = false, d_notouch = false, d_nolgkm = false, d_noreads = false,
                   d_novm = false;
#endif
    // code-prefetch window: TSG_JIT_TOUCH="first,count" in 8-KiB units (default
    // 1,1), relative to the touch base s[90:91]: the dispatcher moves it 8 KiB
    // back per call (the window then starts at the step's own position) where
    // that pays (tsg_capi.cpp pick_tnear)
    uint32_t touch_first = 1, touch_count = 1;
    if (const char *tv = knob_value("TSG_JIT_TOUCH")) std::sscanf(tv, "%u,%u", &touch_first, &touch_count);
    if (touch_count > 4) touch_count = 4;
    // the prefetch must stay inside the tail padding past the last stream
    if ((touch_first + touch_count) * 8192u > (uint32_t)kTailPad * 4u) touch_first = (uint32_t)kTailPad * 4u / 8192u - touch_count;
    const uint32_t ntouch = d_notouch || far ? 0u : touch_count;
    // TSG_JIT_TROLL=n (A/B; 0 = off): rolling code touches -- instead of
    // `count` touches of 8 KiB at a fixed distance every step, each step
    // (after its last DMA piece, as before) touches the next untouched 8-KiB
    // windows until the stream is covered (touch_first + n) x 8 KiB ahead of
    // the current position: a step whose code is longer than 8 KiB (128-wide
    // streams: ~12.6 KiB at s = 4) gets all of it prefetched, a short one
    // (16-wide: ~2 KiB) touches every few steps.  The step's closing vmcnt
    // lets exactly the step's touches run on.  Not with the stagger or lag 2.
    uint32_t troll = 0;
    if (const char *tr = knob_value("TSG_JIT_TROLL")) troll = (uint32_t)std::atoi(tr);
    const bool rolling = troll > 0 && ntouch > 0 && !stagger && lag == 1;
    // Per-group code touches (round 6; TSG_JIT_TGROUP=0|1|2, TSG_JIT_TGAP=
    // bytes override): a read group after the step's last DMA piece repeats
    // the step's code touch ahead of its own position once the code has
    // advanced >= tgap bytes past the previous touch; 2 = the step's closing
    // vmcnt lets those touches run on (1: it waits for them).  A step's one
    // 8-KiB touch covers a 16-column stream several steps ahead, but a
    // 128-wide dense stream writes ~12.6 KiB of code per step at s = 4 (~25
    // at s = 2): the default (the 64-row image: 2, 4096 B) touches it about
    // twice per step there and exactly as before for every step of <= 4 KiB
    // after its last piece.  Measured, kernel us, alternating
    // (profiles/r06g_tgap_ab.jsonl, r06f_tgroup_ab.jsonl): configs[2]
    // 1217-1223 -> 1157-1167, s = 2 2309 -> 2177, (1024, 4096, 16384) 309.5
    // -> 294.8; s = 8 / 16, configs[1] unchanged (same code); with
    // full-mantissa X configs[2] 1248 vs 1260 (that run is clock-bound).
    // Every group (gap 0) also slows the short streams: s = 16 +14%,
    // configs[1] +45%.  Not with the stagger, lag 2 or the mixed DMA issue.
    int tgroup = r64 ? 2 : 0;
    if (const char *tg = knob_value("TSG_JIT_TGROUP")) tgroup = std::atoi(tg);
    if (stagger || lag != 1 || mix_dma || ntouch == 0) tgroup = 0;
    uint32_t tgap = 4096;
    if (const char *tg = knob_value("TSG_JIT_TGAP")) tgap = (uint32_t)std::atoi(tg);
    if (rolling && (touch_first + troll) * 8192u > (uint32_t)kTailPad * 4u) troll = (uint32_t)kTailPad * 4u / 8192u - touch_first;

    int n0 = 0;  // first column of the current stream
    int tile0 = 0, slot0 = 0;  // first column of the tile, the wave's first slot in tile_perm
    std::vector<int> tile_perm(tile_cols);  // accumulator slot -> tile-local column
    for (int i = 0; i < tile_cols; i++) tile_perm[i] = i;
#ifdef TSG_DIAG
    // TSG_JIT_DIAG=balance4|balance1|anti4 (results WRONG: the dispatcher
    // still writes accumulator c of wave w to column w * nw + c): the
    // timing of a balanced / unbalanced column -> wave assignment
    const int d_bal = has("balance4") ? 4 : has("balance1") ? 1 : has("anti4") ? -4 : 0;
#else
    constexpr int d_bal = 0;
#endif
    std::vector<int32_t> cur((size_t)nw * 2), end((size_t)nw * 2);
    std::vector<uint8_t> live(nw, 0);  // BlockedTCSC: y of the column holds an entry
    // step q's section: the wave's entries in rows [klo, khi) of its pass, as
    // X reads: one per k-row pair with an entry (ascending), its used rows and
    // per row the columns with an entry there
    auto build_section = [&](int q, Section &sec) {
        const StepSpec &sp = plan[(size_t)q];
        // first K row of the chunk in LDS (row layout: the last chunk starts at K - 188)
        const int p = sp.pass, kc = rowlay ? jit64_row_kbase(K, nch, sp.chunk) : sp.chunk * CH;
        const int32_t *cs = p ? csn : csp, *ri = p ? rin : rip;
        if (sp.reset)
            for (int col = sp.c0; col < sp.c1; col++) {
                const int n = d_bal ? tile0 + tile_perm[slot0 + col] : n0 + col;
                cur[(size_t)col * 2 + p] = n < N ? cs[sp.slot0 + n] : 0;
                end[(size_t)col * 2 + p] = n < N ? cs[sp.slot0 + n + 1] : 0;
            }
        std::vector<std::vector<uint8_t>> by_row(CH);
        for (int col = sp.c0; col < sp.c1; col++) {
            int32_t &i = cur[(size_t)col * 2 + p];
            const int32_t e = end[(size_t)col * 2 + p];
            for (; i < e && ri[i] < sp.khi; i++) by_row[ri[i] - kc].push_back((uint8_t)col);
        }
        sec.reads.clear();
        for (int pr = 0; pr < CH / U; pr++) {
            Section::Read rd;
            rd.pair = pr;
            for (int r = 0; r < U; r++)
                if (!by_row[U * pr + r].empty()) {
                    rd.mask |= 1 << r;
                    rd.cols[r] = std::move(by_row[U * pr + r]);
                }
            if (rd.mask) sec.reads.push_back(std::move(rd));
        }
    };
    int base_chunk = -1;  // chunk whose base s[84:85] holds
    bool base_adj = false;  // that base already carries the last chunk's s87 adjustment
    // stage step q's chunk into LDS buffer q % kJitRing: the chunk base, then
    // pieces 0..kPieces-1 (dma_piece); M0 = s83 (this wave's first piece, set
    // by the dispatcher) + buffer + piece offset (m0k: the first of 4 pieces'
    // offset, the others by the instruction offset)
    auto dma_begin = [&](int q) {
        const int j = plan[(size_t)q].chunk;
        if (j == 0 || base_chunk < 0 || j < base_chunk) {
            E.base_reset();
            for (int i = 0; i < j; i++) E.base_next();
            base_adj = false;
        } else {
            for (int i = base_chunk; i < j; i++) E.base_next();
        }
        base_chunk = j;
        if (rowlay && j == nch - 1 && jit64_row_kbase(K, nch, j) != j * CH && !base_adj) {
            // direct X: the last chunk starts s87 = 4 (188 nch - K) bytes below its
            // slot (the staged copy holds it in its slot: s87 = 0); applied once
            // per arrival on the last chunk (a step that stages it again keeps
            // the adjusted base), and a later chunk never follows it without a
            // base reset
            E.base_last_adj();
            base_adj = true;
        }
        E.nop(4);  // SALU-written SGPR base -> VMEM
    };
    int vm_step = 0;  // VMEM operations (DMA pieces, code touches) issued in the current step
    uint32_t touch_step = 0;  // rolling code touches issued in the current step
    uint32_t extra_touch = 0;  // TSG_JIT_TGROUP touches issued in the current step
    uint32_t last_touch_pos = 0;  // code position of the last (non-rolling) touch sequence
    uint32_t touched_to = 0;  // rolling: region offset up to which the stream's code is touched
    int cur_wave = 0;  // the wave whose stream is being generated
    auto dma_piece = [&](int q, int i) {
        // 64-row image: piece pr holds quads PQ * (pr / (64 / PR)) .. + PQ - 1
        // of the chunk (tsg_internal.h, blocked k-quad layout); pieces whose
        // quads all lie at or past K are never staged (no entry reads them):
        // the dispatcher may then stage straight from row-major X, whose rows
        // end at K (tsg_jit_kernel.hip "direct X", K % (4 PQ) == 0).  They are
        // a suffix of the wave's pieces, so no M0 group loses its first piece.
        if (rowlay ? cur_wave * kPieces + i >= kJit64RowQuads
                   : r64 && (int64_t)plan[(size_t)q].chunk * CH + 4 * PQ * (((int64_t)cur_wave * kPieces + i) / (64 / PR)) >= K)
            return;  // (row layout: the chunk's 47 pieces; piece 47 of the register contract is never staged)
        const uint32_t sub = m0k ? (uint32_t)(i & 3) : 0u;
        if (sub == 0) {
            E.m0_wave((uint32_t)(q % kJitRing) * kBuf + (uint32_t)i * kPairBytes);
            E.nop(0);  // M0 -> LDS-DMA
        }
        E.glds_x4(kDmaOffV + (uint32_t)i, sub * kPairBytes);
        vm_step++;
    };
    auto emit_dma = [&](int q) {  // prologue: every piece at once
        if (d_nodma) return;
        dma_begin(q);
        for (int i = 0; i < kPieces; i++) dma_piece(q, i);
    };

    // X read schedule.  The wave's reads (k-row pairs with an entry), over all
    // steps, form one sequence g = 0, 1, ...; read g lives in X slot g % S.
    // Reads are consumed in groups of G (never across a step): at a group's
    // start the wave waits (counted lgkmcnt; LDS returns in order) for the
    // group's reads, then issues the reads of the following pairs up to RA
    // past the group (at most into the next step, whose chunk is already
    // resident: staged two steps ahead, visible since the last barrier), then
    // adds the group's entries column by column (pairs of columns
    // interleaved).  Every column meets its rows in ascending k.
    // Default G = S/3, RA = 2S/3 (8 and 16 of the 24 slots: measured 0.4% faster
    // than 12,12, profiles/r02_jit_knobs_ab.txt); TSG_JIT_READS="G,RA" overrides.
    int G = std::max(1, S / 3), RA = S - std::max(1, S / 3);
    // 64-row image, narrow streams (<= 32 columns) or sparse W (density <=
    // 1/8): groups of 5, read-ahead 19, and of 3 (read-ahead 21) for streams
    // of <= 16 columns -- shorter groups between the waits where a group
    // feeds few adds (round 6, kernel us, alternating, profiles/
    // r06z3_reads_rule_ab.jsonl, r06z5_reads3_ab.jsonl: configs[1] 61.6 ->
    // 60.0 -> 58.1, (1024, 4096, 1024) 56.0 -> 55.0, M = 192 96.4 -> 92.2,
    // s = 16 431.7 -> 424.5, s = 8 664.0 -> 658.3); the wide dense streams
    // keep 8,16 (configs[2] 6,18 and 7,17 +7%, 5,19 even: there the group
    // count moves the per-group code touches, r06z_reads_ab.jsonl), and so
    // do 32-wide streams of dense W (s = 2: (192, 4096, 16384) 162.7 vs 170.9
    // with 5, r06z7_reads_dense_ab.jsonl)
    if (r64 && !B && (nw <= 16 || (nw <= 32 && density <= 0.375) || density <= 0.125)) {
        G = nw <= 16 ? 3 : 5;
        RA = S - G;
    }
    if (const char *rv = knob_value("TSG_JIT_READS")) std::sscanf(rv, "%d,%d", &G, &RA);
    if (G < 1 || RA < 0 || G + RA > S) {
        G = std::max(1, S / 3);
        RA = S - G;
    }
    // register of row `half` of read g's unit (pair: 0 even k, 1 odd k, two
    // VGPRs each; quad: row r of the four, one VGPR each)
    auto xreg = [&](int64_t g, const Section::Read &rd, int half) {
        const uint32_t slot = kXSlot0 + (uint32_t)(kJitSlotRegs * (g % S));
        if (r64) return slot + (uint32_t)(half - quad_read(rd.mask).row0);
        return slot + (rd.mask == 3 ? 2u * (uint32_t)half : 0u);
    };
    for (int t = 0; t < ntiles; t++) {
        for (int w = 0; w < streams; w++) {
            while (code.size() % 64) E.nop();  // 256-B aligned stream start
            img.wcode[(size_t)t * streams + w] = E.pos_bytes();
            cur_wave = w;
            n0 = t * tile_cols + w * nw;
            tile0 = t * tile_cols;
            slot0 = w * nw;
#ifdef TSG_DIAG
            if (d_bal && w == 0 && !B && nw % 4 == 0)
                tile_perm = balance_tile(csp, csn, rip, rin, N, tile0, tile_cols, waves, nw, CH, nch,
                                         d_bal < 0 ? -d_bal : d_bal, d_bal < 0);
#endif
            std::fill(live.begin(), live.end(), 0);
            base_chunk = -1;
            touched_to = 0;
            const bool early = stagger && w < waves / 2;  // runs half a step ahead of waves w + 4
            if (prio && w >= waves / 2) E.setprio(1);
            E.save_m0();
            // prologue: the first kJitRing - 1 steps staged, landed, visible
            if (steps > 0) {
                for (int q = 0; q < std::min(steps, kJitRing - 1); q++) emit_dma(q);
                E.wait_vm0();
                E.barrier();
            }
            std::vector<Section> secs(steps);
            std::vector<int64_t> first(steps + 1, 0);  // global index of each step's first read
            int built = 0;
            auto ensure = [&](int q) {
                while (built <= q && built < steps) {
                    build_section(built, secs[built]);
                    first[built + 1] = first[built] + (int64_t)secs[built].reads.size();
                    built++;
                }
            };
            int64_t issued = 0, ready = 0;  // reads issued / reads known complete
            int rq = 0;                      // step of read `issued`
            // issue reads up to `upto` (exclusive), not past step `qmax`
            auto issue_reads = [&](int64_t upto, int qmax) {
                qmax = std::min(qmax, steps - 1);
                for (; issued < upto; issued++) {
                    while (rq + 1 <= qmax && issued >= first[rq + 1]) rq++;
                    if (issued >= first[rq + 1]) return;  // past step qmax
                    const Section::Read &rd = secs[rq].reads[(size_t)(issued - first[rq])];
                    if (d_noreads) continue;
                    const uint32_t dst = kXSlot0 + (uint32_t)(kJitSlotRegs * (issued % S));
                    const uint32_t lb = kLdsBaseV + (uint32_t)(rq % kJitRing);
                    // 64-row image, blocked k-quad layout: quad q of the chunk at
                    // (q / PQ) * 64 KiB / PR + (q % PQ) * 16 PR B from the lane's base
                    // row layout: quad q at the lane's row base + 16 q
                    const uint32_t off = rowlay ? (uint32_t)rd.pair * 16u
                                         : r64 ? (uint32_t)(rd.pair / PQ) * (65536u / (uint32_t)PR) +
                                                     (uint32_t)(rd.pair % PQ) * 16u * (uint32_t)PR
                                               : (uint32_t)rd.pair * kPairBytes;
                    if (r64) {
                        const QuadRead qr = quad_read(rd.mask);
                        if (qr.nreg == 4) E.ds_read_b128(dst, lb, off);
                        else if (qr.nreg == 2) E.ds_read_b64(dst, lb, off + qr.off);
                        else E.ds_read_b32(dst, lb, off + qr.off);
                    } else if (rd.mask == 3) {
                        E.ds_read_b128(dst, lb, off);
                    } else {
                        E.ds_read_b64(dst, lb, off + (rd.mask == 2 ? 8u : 0u));
                    }
                }
            };
            auto wait_reads = [&](int64_t upto) {  // reads < upto complete
                if (ready >= upto) return;
                const int64_t n = std::min<int64_t>(std::max<int64_t>(issued - upto, 0), 15);
                if (!d_nolgkm) E.wait_lgkm((uint32_t)n);
                ready = issued - n;
            };
            for (int q = 0; q < steps; q++) {
                ensure(q + 1);
                const StepSpec &sp = plan[(size_t)q];
                const bool neg = sp.pass == 1;
                // one entry: BaseTCSC adds into the column's accumulator; a
                // BlockedTCSC block chains in y (0 + first entry, then in place)
                auto add = [&](int col, uint32_t x) {
                    if (r64) {  // one accumulator VGPR per column
                        E.v_addsub(kAcc0 + (uint32_t)col, x, neg);
                        return;
                    }
                    if (!B) {
                        E.pk_add(kAcc0 + 2u * (uint32_t)col, x, neg);
                        return;
                    }
                    const uint32_t d = kTmp0 + 2u * (uint32_t)(col - sp.c0);
                    if (live[col]) {
                        E.pk_add(d, x, neg);
                    } else {
                        E.pk_first(d, x, neg);
                        live[col] = 1;
                    }
                };
                // code touches go out AFTER the step's last DMA piece: VMEM loads
                // return in order, so the step's closing vmcnt(ntouch) waits for
                // every DMA piece but lets the touches (L2 misses) run into the
                // next step
                // (lv: the lane-offset VGPR -- v[lane128] for the step's own
                // touch, v[lane128 + 1] for the per-group ones: the dispatcher
                // zeroes the latter per call, one line then, tsg_capi.cpp xtouch)
                auto touches = [&](uint32_t lv) {
                    if (rolling) {
                        const uint32_t pos = E.pos_bytes();
                        // the stream's first touch starts touch_first windows ahead; later
                        // ones continue where the last stopped (never behind the position)
                        touched_to = touched_to == 0 ? pos + touch_first * 8192u : std::max(touched_to, pos);
                        while (touched_to < pos + (touch_first + troll) * 8192u) {
                            E.touch_addr(touched_to);
                            E.nop(4);
                            E.code_touch(kSinkV, lv);
                            vm_step++;
                            touch_step++;
                            touched_to += 8192u;
                        }
                        return;
                    }
                    last_touch_pos = E.pos_bytes();
                    for (uint32_t d = 0; d < ntouch; d++) {
                        E.touch_addr(E.pos_bytes() + (touch_first + d) * 8192u);
                        E.nop(4);
                        E.code_touch(kSinkV, lv);
                        vm_step++;
                    }
                };
                vm_step = 0;
                touch_step = 0;
                extra_touch = 0;
                const Section &sec = secs[q];
                const int nrd = (int)sec.reads.size();
                const int ngroups = (nrd + G - 1) / G;
                const int qd = q + kJitRing - 1;  // the step whose chunk this step stages
                const bool dma = qd < steps && !d_nodma;
                // the stagger's early waves: the step's barrier (barrier q - 1)
                // before read group `mid`; the DMA pieces after it
                const int mid = early ? ngroups / 2 : 0;
                const int ngd = ngroups - mid;  // the groups the pieces spread over
                // pieces go out before read groups mid .. mid+span-1 (span 0: all at once)
                const int span = dma ? std::min(ngd, (int)std::ceil(dma_spread * ngd)) : 0;
                int pieces_out = 0;
                auto pieces_upto = [&](int upto) {
                    for (; pieces_out < upto; pieces_out++) dma_piece(qd, pieces_out);
                    if (pieces_out == kPieces && upto == kPieces) touches(kLane128V);
                };
                bool released = !early;  // past this step's barrier (early waves) / after the last one
                auto dma_start = [&] {
                    if (early && q >= 1) {
                        // barrier q - 1: the pieces issued in the previous step
                        // (for step q + 1) landed first; then all waves have
                        // finished step q - 1, whose buffer this step's DMA overwrites
                        if (!d_novm) E.wait_vm(ntouch);
                        if (!d_nobar) E.barrier();
                    }
                    released = true;
                    if (dma) {
                        dma_begin(qd);
                        if (span == 0) pieces_upto(kPieces);
                    } else {
                        touches(kLane128V);
                    }
                };
                if (!early) dma_start();
                for (int i0 = 0, grp = 0; i0 < nrd; i0 += G, grp++) {
                    if (early && grp == mid) dma_start();
                    const int i1 = std::min(nrd, i0 + G);
                    const int64_t g1 = first[q] + i1;
                    issue_reads(g1, q);  // (only if the schedule left the group unread)
                    wait_reads(g1);
                    // (early waves before their barrier: this step's chunk only)
                    const int qra = lag == 2 || !released ? q : q + 1;
                    // this group's share of the DMA pieces
                    const int pieces_to = dma && grp >= mid && grp - mid < span && pieces_out < kPieces
                                              ? std::min(kPieces, ((grp - mid + 1) * kPieces + span - 1) / span)
                                              : pieces_out;
                    // per column its entries of the group (ascending k); columns in pairs, interleaved
                    std::vector<std::vector<uint32_t>> xs(nw);
                    for (int i = i0; i < i1; i++) {
                        const Section::Read &rd = sec.reads[(size_t)i];
                        for (int half = 0; half < U; half++)
                            for (uint8_t col : rd.cols[half]) xs[col].push_back(xreg(first[q] + i, rd, half));
                    }
                    std::vector<std::pair<int, uint32_t>> adds;
                    for (int col = sp.c0; col < sp.c1; col += 2)
                        for (size_t k = 0; k < std::max(xs[col].size(), xs[col + 1].size()); k++) {
                            if (k < xs[col].size()) adds.emplace_back(col, xs[col][k]);
                            if (k < xs[col + 1].size()) adds.emplace_back(col + 1, xs[col + 1][k]);
                        }
                    // the group's read-ahead and DMA pieces: before its adds
                    // (default), or spread evenly among them (TSG_JIT_MIX)
                    int64_t reads_to = issued;
                    {
                        const int qm = std::min(qra, steps - 1);
                        reads_to = std::max(issued, std::min<int64_t>(g1 + RA, first[qm + 1]));
                    }
                    if (!mix_reads) issue_reads(g1 + RA, qra);
                    const bool pieces_were_out = dma && pieces_out == kPieces;
                    if (!mix_dma && pieces_to > pieces_out) pieces_upto(pieces_to);
                    if (tgroup && pieces_were_out && !rolling && extra_touch + ntouch <= 15 - ntouch &&
                        E.pos_bytes() >= last_touch_pos + tgap) {
                        // TSG_JIT_TGROUP: every read group after the step's last piece
                        // touches the code (touch_first .. ) windows ahead of it again
                        const int before = vm_step;
                        touches(kLane128V + 1u);
                        extra_touch += (uint32_t)(vm_step - before);
                    }
                    const int nr = mix_reads ? (int)(reads_to - issued) : 0;
                    const int np = mix_dma ? pieces_to - pieces_out : 0;
                    const int items = nr + np, na = (int)adds.size();
                    int done = 0, ri = 0, pi = 0;
                    auto emit_item = [&] {
                        // alternate reads and pieces, reads first, in proportion
                        const bool rd = pi >= np || (ri < nr && (int64_t)ri * np <= (int64_t)pi * nr);
                        if (rd) {
                            issue_reads(issued + 1, qra);
                            ri++;
                        } else {
                            pieces_upto(pieces_out + 1);
                            pi++;
                        }
                        done++;
                    };
                    for (int a = 0; a < na; a++) {
                        add(adds[(size_t)a].first, adds[(size_t)a].second);
                        // item j goes after add (j + 1) * na / (items + 1), on an
                        // 8-byte boundary (an odd position waits one more add)
                        while (done < items && (int64_t)(a + 1) * (items + 1) >= (int64_t)(done + 1) * na &&
                               (!(E.c.size() & 1) || a + 1 == na))
                            emit_item();
                    }
                    while (done < items) emit_item();
                }
                if (sp.flush)  // comp.h:642: Y += y (a block without entries adds +0: a no-op, Y is never -0)
                    for (int col = sp.c0; col < sp.c1; col++)
                        if (live[col]) {
                            E.pk_acc(kAcc0 + 2u * (uint32_t)col, kTmp0 + 2u * (uint32_t)(col - sp.c0));
                            live[col] = 0;
                        }
                if (!released) dma_start();  // (an early wave's step with fewer than mid + 1 read groups)
                if (dma && pieces_out < kPieces) pieces_upto(kPieces);
                if (early) {
                    // no barrier at the step's end: its pieces are waited for
                    // before the next step's mid barrier
                    issue_reads(first[q + 1] + std::max(G, RA), q + 1);  // next step's first reads
                    continue;
                }
                if (lag == 1) {
                    issue_reads(first[q + 1] + std::max(G, RA), q + 1);  // next step's first reads
                    if (!d_novm)  // this step's pieces (the touches may run on)
                        E.wait_vm(rolling ? touch_step : tgroup == 2 ? ntouch + extra_touch : ntouch);
                } else if (!d_novm) {
                    // the previous step's pieces: only its touches and this
                    // step's operations may still be in flight
                    E.wait_vm(ntouch + (uint32_t)vm_step);
                }
                if (!d_nobar) E.barrier();
            }
            if (early && steps > 0 && !d_nobar) E.barrier();  // barrier steps - 1 (the late waves' last)
            if (prio && w >= waves / 2) E.setprio(0);
            E.wait_vm0();  // no load outstanding past the stream
            E.restore_m0();
            E.ret();
        }
    }
    for (int i = 0; i < kTailPad; i++) E.nop();  // the code prefetch reads past the last stream
}

// ------------------------------------------------------------ code object --
namespace {

// The dispatcher of a stream width: tsg_jit.co (kJitNW columns per wave) or
// tsg_jit_w<nw>.co (same kernel built with TSG_JIT_NW=nw, Makefile); 4-wave
// workgroups: tsg_jit_w<nw>_4w.co (TSG_JIT_WAVES=4); the 64-row image:
// tsg_jit64_w<nw>[_4w].co (TSG_JIT_ROWS64=1), its half ring
// tsg_jit64h_w<nw>.co (4 waves, TSG_JIT_HALF=1), its wave pairs
// tsg_jit64p_w<nw>.co (4-wave streams, TSG_JIT_PAIR=1).
std::string template_name(int nw, int waves, bool r64, bool half, bool pair)
{
    return r64 && half ? "tsg_jit64h_w" + std::to_string(nw) + ".co"
           : r64 && pair ? "tsg_jit64p_w" + std::to_string(nw) + ".co"
           : r64 ? "tsg_jit64_w" + std::to_string(nw) + (waves == kJitWaves ? "" : "_4w") + ".co"
           : nw == kJitNW && waves == kJitWaves ? "tsg_jit.co"
           : "tsg_jit_w" + std::to_string(nw) + (waves == kJitWaves ? "" : "_4w") + ".co";
}

}  // namespace
}  // namespace tsg

// Every dispatcher code object, embedded in this library at build time
// (csrc/gen_co_embed.py, Makefile): {file name, bytes, size}, null-terminated.
struct TsgCoEntry {
    const char *name;
    const unsigned char *data;
    uint64_t size;
};
extern "C" const TsgCoEntry tsg_co_table[];

namespace tsg {
namespace {

// The template bytes: from TSG_JIT_DIR when set (tests: a directory with some
// objects missing exercises the fallbacks), else the copy embedded in the
// library, else the file next to the library (a build without the table
// entry).
std::string read_template(int nw, int waves, bool r64, bool half, bool pair, std::vector<unsigned char> &img)
{
    const std::string name = template_name(nw, waves, r64, half, pair);
    std::string path;
    if (const char *dir = knob_value("TSG_JIT_DIR")) {
        path = std::string(dir) + "/" + name;
    } else {
        for (const TsgCoEntry *e = tsg_co_table; e->name; e++)
            if (name == e->name) {
                img.assign(e->data, e->data + e->size);
                return "";
            }
        Dl_info info;
        path = name;
        if (dladdr(reinterpret_cast<void *>(&build_jit_code), &info) && info.dli_fname) {
            const std::string p(info.dli_fname);
            const size_t s = p.rfind('/');
            path = (s == std::string::npos ? std::string(".") : p.substr(0, s)) + "/" + name;
        }
    }
    std::ifstream f(path, std::ios::binary);
    if (!f) return "cannot open jit template " + path;
    img.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return "";
}

}  // namespace

std::string JitModule::load(const std::vector<uint32_t> &code, int nw, int waves, bool r64, bool half, bool pair)
{
    std::vector<unsigned char> img;
    const std::string rerr = read_template(nw, waves, r64, half, pair, img);
    if (!rerr.empty()) return rerr;
    if (img.size() < sizeof(Elf64_Ehdr)) return "jit template too small";
    Elf64_Ehdr eh;
    std::memcpy(&eh, img.data(), sizeof eh);
    if (std::memcmp(eh.e_ident, ELFMAG, SELFMAG) != 0 || eh.e_ident[EI_CLASS] != ELFCLASS64 ||
        eh.e_phentsize != sizeof(Elf64_Phdr) || eh.e_phoff + (size_t)eh.e_phnum * sizeof(Elf64_Phdr) > img.size())
        return "jit template is not an ELF64 code object";
    // highest loaded address; the program header we turn into the code segment
    uint64_t top = 0;
    int spare = -1;
    for (int i = 0; i < eh.e_phnum; i++) {
        Elf64_Phdr ph;
        std::memcpy(&ph, img.data() + eh.e_phoff + (size_t)i * sizeof ph, sizeof ph);
        if (ph.p_type == PT_LOAD) top = std::max<uint64_t>(top, ph.p_vaddr + ph.p_memsz);
        if (ph.p_type == PT_GNU_STACK) spare = i;
    }
    if (spare < 0) return "jit template has no spare program header";
    const uint64_t page = 0x1000;
    const uint64_t vaddr = (top + page - 1) & ~(page - 1);
    // patch the region-base literal of the dispatcher and of the probe kernel
    // (each `s_add_u32 s92, s92, 0x7a5e1234` after its own s_getpc_b64): each
    // becomes (region vaddr - vaddr of that s_add)
    static const unsigned char pat[8] = {0x5c, 0xff, 0x5c, 0x80, 0x34, 0x12, 0x5e, 0x7a};
    std::vector<size_t> sites;
    for (size_t i = 0; i + 8 <= img.size(); i += 4)
        if (std::memcmp(img.data() + i, pat, 8) == 0) sites.push_back(i);
    if (sites.size() != 2) return "jit template: expected 2 region literals, found " + std::to_string(sites.size());
    for (const size_t at : sites) {
        uint64_t insn_vaddr = UINT64_MAX;
        for (int i = 0; i < eh.e_phnum; i++) {
            Elf64_Phdr ph;
            std::memcpy(&ph, img.data() + eh.e_phoff + (size_t)i * sizeof ph, sizeof ph);
            if (ph.p_type == PT_LOAD && at >= ph.p_offset && at < ph.p_offset + ph.p_filesz)
                insn_vaddr = ph.p_vaddr + (at - ph.p_offset);
        }
        if (insn_vaddr == UINT64_MAX || vaddr - insn_vaddr > 0xffffffffull) return "jit template: bad literal location";
        const uint32_t lit = (uint32_t)(vaddr - insn_vaddr);
        std::memcpy(img.data() + at + 4, &lit, 4);
    }
    // append the code segment
    const size_t off = (img.size() + page - 1) & ~(size_t)(page - 1);
    const size_t bytes = code.size() * sizeof(uint32_t);
    img.resize(off + bytes, 0);
    std::memcpy(img.data() + off, code.data(), bytes);
    Elf64_Phdr ph = {};
    ph.p_type = PT_LOAD;
    ph.p_flags = PF_R | PF_X;
    ph.p_offset = off;
    ph.p_vaddr = ph.p_paddr = vaddr;
    ph.p_filesz = ph.p_memsz = bytes;
    ph.p_align = page;
    std::memcpy(img.data() + eh.e_phoff + (size_t)spare * sizeof ph, &ph, sizeof ph);

    hipModule_t m = nullptr;
    hipError_t e = hipModuleLoadData(&m, img.data());
    if (e != hipSuccess) return std::string("hipModuleLoadData: ") + hipGetErrorString(e);
    hipFunction_t fn = nullptr, pf = nullptr;
    e = hipModuleGetFunction(&fn, m, r64 ? "tsg_jit64_kernel" : "tsg_jit_kernel");
    if (e == hipSuccess) e = hipModuleGetFunction(&pf, m, "tsg_jit_probe");
    if (e != hipSuccess) {
        (void)hipModuleUnload(m);
        return std::string("hipModuleGetFunction: ") + hipGetErrorString(e);
    }
    module = m;
    function = fn;
    probe = pf;
    return "";
}

void JitModule::unload()
{
    if (module) (void)hipModuleUnload((hipModule_t)module);
    module = nullptr;
    function = nullptr;
    probe = nullptr;
}

int launch_jit_probe(const JitModule &jm, uint32_t *status, void *stream)
{
    void *params[] = {(void *)&status};
    const hipError_t e =
        hipModuleLaunchKernel((hipFunction_t)jm.probe, 1, 1, 1, 64, 1, 1, 0, (hipStream_t)stream, params, nullptr);
    return e == hipSuccess ? 0 : -1;
}

int launch_tcsc_jit(const JitModule &jm, const float *XT, int Mp, const uint32_t *wcode, const float *b,
                    const float *alpha, float *Y, int M, int N, int Npad, int nch, int prelu,
                    uint32_t *status, int tile_cols, int waves, int gn, int gm, int tmask, void *stream,
                    int tile_m, int xrow, int lastadj, int xtouch, int tnear)
{
    int mtiles = Mp / tile_m, ntiles = Npad / tile_cols;
    void *params[] = {(void *)&XT, (void *)&Mp, (void *)&wcode, (void *)&b, (void *)&alpha, (void *)&Y,
                      (void *)&M, (void *)&N, (void *)&nch, (void *)&mtiles, (void *)&ntiles, (void *)&prelu,
                      (void *)&status, (void *)&gn, (void *)&gm, (void *)&tmask, (void *)&xrow, (void *)&lastadj,
                      (void *)&xtouch, (void *)&tnear};
    hipError_t e = hipModuleLaunchKernel((hipFunction_t)jm.function, (unsigned)(mtiles * ntiles), 1, 1,
                                         (unsigned)waves * 64u, 1, 1, 0, (hipStream_t)stream, params, nullptr);
    return e == hipSuccess ? 0 : -1;
}

}  // namespace tsg

// ---------------------------------------------------------------- C-ABI --
extern thread_local std::string g_tsg_host_err;

extern "C" int tsg_jit_codegen_wv(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                                  int K, int N, int B, int width, int waves, uint32_t *code, int64_t code_cap,
                                  int64_t *code_len, uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len)
{
    if (!tsg::jit_waves_ok(width, waves)) {
        g_tsg_host_err = "tsg_jit_codegen: unsupported waves per workgroup " + std::to_string(waves) +
                         " for width " + std::to_string(width) + " (8; 4 for widths 32, 16, 8)";
        return TSG_ERR_ARG;
    }
    if (!tsg::jit_width_ok(width) || (B && width != tsg::kJitNW)) {
        g_tsg_host_err = "tsg_jit_codegen: unsupported stream width " + std::to_string(width) +
                         (B ? " for BlockedTCSC (64 only)" : " (64, 32, 16 or 8)");
        return TSG_ERR_ARG;
    }
    const std::string e = tsg::validate_tcsc(csp, csn, rip, rin, K, N, B);
    if (!e.empty()) {
        g_tsg_host_err = std::string(B ? "tsg_jit_codegen: malformed BlockedTCSC: " : "tsg_jit_codegen: malformed TCSC: ") + e;
        return TSG_ERR_ARG;
    }
    const std::string ke = tsg::knob_check();
    if (!ke.empty()) {
        g_tsg_host_err = "tsg_jit_codegen: " + ke;
        return TSG_ERR_ARG;
    }
    if (B && (tsg::kJitXRegs - tsg::kJitNW) / tsg::kJitSlotRegs < 2) {
        g_tsg_host_err = "tsg_jit_codegen: this kernel geometry has no registers for BlockedTCSC";
        return TSG_ERR_ARG;
    }
    tsg::JitImage img;
    tsg::build_jit_code(csp, csn, rip, rin, K, N, B, img, width, waves);
    if (code_len) *code_len = (int64_t)img.code.size();
    if (wcode_len) *wcode_len = (int64_t)img.wcode.size();
    if ((code && code_cap < (int64_t)img.code.size()) || (wcode && wcode_cap < (int64_t)img.wcode.size())) {
        g_tsg_host_err = "tsg_jit_codegen: buffer too small";
        return TSG_ERR_ARG;
    }
    if (code) std::memcpy(code, img.code.data(), img.code.size() * 4);
    if (wcode) std::memcpy(wcode, img.wcode.data(), img.wcode.size() * 4);
    return TSG_OK;
}

namespace {
int codegen64(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin, int K, int N,
              int width, int waves, bool half, uint32_t *code, int64_t code_cap, int64_t *code_len,
              uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len);
}

extern "C" int tsg_jit_codegen64(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                                 int K, int N, int width, int waves, uint32_t *code, int64_t code_cap,
                                 int64_t *code_len, uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len)
{
    return codegen64(csp, csn, rip, rin, K, N, width, waves, false, code, code_cap, code_len, wcode, wcode_cap,
                     wcode_len);
}

extern "C" int tsg_jit_codegen64h(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                                  int K, int N, int width, uint32_t *code, int64_t code_cap, int64_t *code_len,
                                  uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len)
{
    if (width >= tsg::kJitNW) {
        g_tsg_host_err = "tsg_jit_codegen64h: the half ring runs widths 32, 16, 8 (4 waves)";
        return TSG_ERR_ARG;
    }
    return codegen64(csp, csn, rip, rin, K, N, width, 4, true, code, code_cap, code_len, wcode, wcode_cap,
                     wcode_len);
}

namespace {
int codegen64(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin, int K, int N,
              int width, int waves, bool half, uint32_t *code, int64_t code_cap, int64_t *code_len,
              uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len)
{
    if (!tsg::jit64_width_ok(width) || !tsg::jit_waves_ok(width, waves)) {
        g_tsg_host_err = "tsg_jit_codegen64: unsupported shape " + std::to_string(width) + " x " +
                         std::to_string(waves) + " (widths 128, 64, 32, 16, 8; 4 waves for 32, 16, 8)";
        return TSG_ERR_ARG;
    }
    const std::string e = tsg::validate_tcsc(csp, csn, rip, rin, K, N, 0);
    if (!e.empty()) {
        g_tsg_host_err = "tsg_jit_codegen64: malformed TCSC: " + e;
        return TSG_ERR_ARG;
    }
    const std::string ke = tsg::knob_check();
    if (!ke.empty()) {
        g_tsg_host_err = "tsg_jit_codegen64: " + ke;
        return TSG_ERR_ARG;
    }
    tsg::JitImage img;
    tsg::build_jit_code(csp, csn, rip, rin, K, N, 0, img, width, waves, false, true, half);
    if (code_len) *code_len = (int64_t)img.code.size();
    if (wcode_len) *wcode_len = (int64_t)img.wcode.size();
    if ((code && code_cap < (int64_t)img.code.size()) || (wcode && wcode_cap < (int64_t)img.wcode.size())) {
        g_tsg_host_err = "tsg_jit_codegen64: buffer too small";
        return TSG_ERR_ARG;
    }
    if (code) std::memcpy(code, img.code.data(), img.code.size() * 4);
    if (wcode) std::memcpy(wcode, img.wcode.data(), img.wcode.size() * 4);
    return TSG_OK;
}

}  // namespace

extern "C" int tsg_jit_codegen_far(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                                   int K, int N, uint32_t *code, int64_t code_cap, int64_t *code_len, uint32_t *wcode,
                                   int64_t wcode_cap, int64_t *wcode_len)
{
    const std::string e = tsg::validate_tcsc(csp, csn, rip, rin, K, N, 0);
    if (!e.empty()) {
        g_tsg_host_err = "tsg_jit_codegen_far: malformed TCSC: " + e;
        return TSG_ERR_ARG;
    }
    const std::string ke = tsg::knob_check();
    if (!ke.empty()) {
        g_tsg_host_err = "tsg_jit_codegen_far: " + ke;
        return TSG_ERR_ARG;
    }
    tsg::JitImage img;
    tsg::build_jit_code(csp, csn, rip, rin, K, N, 0, img, tsg::kJitNW, tsg::kJitWaves, true);
    if (code_len) *code_len = (int64_t)img.code.size();
    if (wcode_len) *wcode_len = (int64_t)img.wcode.size();
    if ((code && code_cap < (int64_t)img.code.size()) || (wcode && wcode_cap < (int64_t)img.wcode.size())) {
        g_tsg_host_err = "tsg_jit_codegen_far: buffer too small";
        return TSG_ERR_ARG;
    }
    if (code) std::memcpy(code, img.code.data(), img.code.size() * 4);
    if (wcode) std::memcpy(wcode, img.wcode.data(), img.wcode.size() * 4);
    return TSG_OK;
}

extern "C" int tsg_jit_tile_map(int L, int mtiles, int ntiles, int gn, int gm, int *nt, int *mt)
{
    if (!nt || !mt || mtiles <= 0 || ntiles <= 0 || gn <= 0 || gm <= 0 || L < 0 ||
        (int64_t)L >= (int64_t)mtiles * ntiles) {
        g_tsg_host_err = "tsg_jit_tile_map: bad arguments";
        return TSG_ERR_ARG;
    }
    tsg_jit_tile(L, mtiles, ntiles, gn, gm, *nt, *mt);
    return TSG_OK;
}

extern "C" int tsg_jit_codegen_w(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                                 int K, int N, int B, int width, uint32_t *code, int64_t code_cap,
                                 int64_t *code_len, uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len)
{
    return tsg_jit_codegen_wv(csp, csn, rip, rin, K, N, B, width, tsg::kJitWaves, code, code_cap, code_len, wcode,
                              wcode_cap, wcode_len);
}

extern "C" int tsg_jit_codegen_blocked(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                                       const int32_t *rin, int K, int N, int B, uint32_t *code,
                                       int64_t code_cap, int64_t *code_len, uint32_t *wcode, int64_t wcode_cap,
                                       int64_t *wcode_len)
{
    return tsg_jit_codegen_w(csp, csn, rip, rin, K, N, B, tsg::kJitNW, code, code_cap, code_len, wcode, wcode_cap,
                             wcode_len);
}

extern "C" int tsg_jit_codegen(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                               const int32_t *rin, int K, int N, uint32_t *code, int64_t code_cap,
                               int64_t *code_len, uint32_t *wcode, int64_t wcode_cap, int64_t *wcode_len)
{
    return tsg_jit_codegen_blocked(csp, csn, rip, rin, K, N, 0, code, code_cap, code_len, wcode, wcode_cap,
                                   wcode_len);
}
