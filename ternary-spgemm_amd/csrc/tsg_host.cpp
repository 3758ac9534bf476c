// tsg_host.cpp -- host-side pieces of the product library that need no GPU:
// the device-image planner, TCSC validation / column slicing for sharding,
// and the synthetic-input generators used by bench.py and the driver.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ternary_spgemm_test.h"
#include "tsg_internal.h"

namespace tsg {

void build_rx_image(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                    const int32_t *rin, int K, int N, RxImage &img)
{
    img.K = K;
    img.N = N;
    img.Npad = ((N + kRxTileCols - 1) / kRxTileCols) * kRxTileCols;
    img.nch = std::max(1, (K + kRxChunk - 1) / kRxChunk);
    const int nch = img.nch, ntiles = img.Npad / kRxTileCols;
    img.wstart.assign((size_t)ntiles * kRxWaves, 0u);
    img.ent.clear();
    const int64_t nnz = (int64_t)csp[N] + (int64_t)csn[N];
    img.ent.reserve((size_t)(nnz / 48) * kRxBlockWords + (size_t)ntiles * kRxWaves * 2 * nch * kRxBlockWords);
    std::vector<int32_t> cur((size_t)kRxNW * 2), end((size_t)kRxNW * 2);
    for (int t = 0; t < ntiles; t++) {
        for (int w = 0; w < kRxWaves; w++) {
            const int n0 = t * kRxTileCols + w * kRxNW;
            img.wstart[(size_t)t * kRxWaves + w] = (uint32_t)img.ent.size();
            for (int c = 0; c < kRxNW; c++)
                for (int p = 0; p < 2; p++) {
                    const int n = n0 + c;
                    const int32_t *cs = p ? csn : csp;
                    cur[(size_t)c * 2 + p] = n < N ? cs[n] : 0;
                    end[(size_t)c * 2 + p] = n < N ? cs[n + 1] : 0;
                }
            for (int q = 0; q < 2 * nch; q++) {
                const int p = q / nch, j = q % nch;
                const int32_t *ri = p ? rin : rip;
                const int klo = j * kRxChunk, khi = klo + kRxChunk;
                size_t last = SIZE_MAX;
                for (;;) {
                    int k0 = INT32_MAX;
                    for (int c = 0; c < kRxNW; c++) {
                        const int32_t i = cur[(size_t)c * 2 + p];
                        if (i < end[(size_t)c * 2 + p] && ri[i] < khi) k0 = std::min(k0, (int)ri[i]);
                    }
                    if (k0 == INT32_MAX) break;
                    // block rows [k0, kend): at most kRxBlockRows, inside the chunk,
                    // at most kRxCap entries per column
                    int kend = std::min(k0 + kRxBlockRows, khi);
                    for (int c = 0; c < kRxNW; c++) {
                        const int32_t i = cur[(size_t)c * 2 + p] + kRxCap;
                        if (i < end[(size_t)c * 2 + p] && ri[i] < kend) kend = ri[i];
                    }
                    last = img.ent.size();
                    img.ent.resize(last + kRxBlockWords, 0u);
                    img.ent[last] = (uint32_t)(k0 - klo) * 1024u;
                    for (int c = 0; c < kRxNW; c++) {
                        int32_t &i = cur[(size_t)c * 2 + p];
                        uint64_t bytes = 0;
                        int f = 0;
                        for (; i < end[(size_t)c * 2 + p] && ri[i] < kend; i++, f++)
                            bytes |= (uint64_t)(4u * (uint32_t)(ri[i] - k0 + 1)) << (8 * f);
                        img.ent[last + 2 + 2 * c] = (uint32_t)bytes;
                        img.ent[last + 3 + 2 * c] = (uint32_t)(bytes >> 32);
                    }
                }
                if (last == SIZE_MAX) {  // no entries in this step: one empty block
                    last = img.ent.size();
                    img.ent.resize(last + kRxBlockWords, 0u);
                }
                img.ent[last] |= 1u << 31;
            }
        }
    }
    img.ent.resize(img.ent.size() + kRxBlockWords, 0u);  // the walk reads one header ahead
}

// Sliced-ELL entry stream of the small-M kernel (tsg_ell.hip header) for an
// M tile of MT rows: per 16-column slice and step every column's entries in
// ascending k as the uint16 float index (k - chunk base) * MT into the LDS
// chunk, padded with C * MT (the zero row) to the slice's longest list rounded
// up to 8; blocks of 256 B = [16 columns][8 entries].  One chunk (K <= C): ONE
// step per slice, the +1 blocks then the -1 blocks; else a step per (pass,
// chunk) in BaseTCSC's order (comp.h:37-63).  tab per (slice, step) =
// {offset in blocks, n8 | n8pos << 16}: the first n8pos blocks add, the rest
// subtract.  Block 0 is all padding (the walk reads it past a list's end).
void build_ell_image(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin, int K, int N,
                     int Cmax, int MT, EllImage &img, int copies, bool sched)
{
    const bool two = copies == 2 && MT == 8;
    sched = sched && MT == 8 && !two;
    if (two) {
        // both copies (and their zero rows) inside the LDS: xb + (C + 1) * MT
        // floats <= kLdsBytes / 4, chunks balanced over K
        const int cmax2 = std::min(Cmax, ((int)(kLdsBytes / 4) - 96) / (2 * MT) - 1) / 4 * 4;
        const int nch2 = std::max(1, (K + cmax2 - 1) / cmax2);
        img.C = std::max(4, ((K + nch2 - 1) / nch2 + 3) / 4 * 4);
    } else if (sched) {
        // the chunk and its 8 zero rows inside the LDS
        img.C = std::min(std::min(Cmax, (int)(kLdsBytes / 4) / MT - kEllSchedZeroRows) / 4 * 4,
                         std::max(4, (K + 3) / 4 * 4));
    } else {
        img.C = std::min(Cmax, std::max(4, (K + 3) / 4 * 4));
    }
    img.zr = sched ? kEllSchedZeroRows : 1;
    img.nch = std::max(1, (K + img.C - 1) / img.C);
    img.steps = img.nch == 1 ? 1 : 2 * img.nch;
    img.nslices = (N + 15) / 16;
    img.xb = two ? ell_copy_offset(img.C, MT) : 0;
    const int C = img.C, nch = img.nch, steps = img.steps, xb = img.xb;
    const uint16_t pad = (uint16_t)(C * MT);
    img.tab.assign((size_t)img.nslices * steps * 2, 0u);
    std::vector<uint16_t> e16((size_t)128, pad);  // block 0: the padding block
    e16.reserve((size_t)((int64_t)csp[N] + csn[N]) * 5 / 4 + (size_t)img.nslices * steps * 256 + 128);
    for (int sl = 0; sl < img.nslices; sl++) {
        int32_t cur[2][16], end[2][16];
        for (int c = 0; c < 16; c++) {
            const int n = sl * 16 + c;
            for (int p = 0; p < 2; p++) {
                const int32_t *cs = p ? csn : csp;
                cur[p][c] = n < N ? cs[n] : 0;
                end[p][c] = n < N ? cs[n + 1] : 0;
            }
        }
        for (int step = 0; step < steps; step++) {
            const size_t at = e16.size();
            uint32_t n8 = 0, n8pos = 0;
            // the (pass, chunk) lists of this step: both passes of chunk 0 when steps == 1
            for (int p = 0; p < 2; p++) {
                if (steps > 1 && p != step / nch) continue;
                const int j = steps > 1 ? step % nch : 0;
                const int32_t *ri = p ? rin : rip;
                const int khi = (j + 1) * C;
                int cnt[16], L = 0;
                for (int c = 0; c < 16; c++) {
                    int q = cur[p][c];
                    while (q < end[p][c] && ri[q] < khi) q++;
                    cnt[c] = q - cur[p][c];
                    L = std::max(L, cnt[c]);
                }
                std::vector<uint16_t> seq[16];  // sched: each column's entries per position
                if (sched) {
                    // per ds_read_b64 lane group (columns 0-7, 8-15) and position:
                    // the columns with most entries left first, each advancing if
                    // its next row's 8-bank window (float index % 64 / 8) is still
                    // free; the rest read the zero row of a free window (one row
                    // for all of them: a broadcast)
                    L = 0;
                    for (int g0 = 0; g0 < 16; g0 += 8) {
                        int at[8] = {0};
                        for (;;) {
                            int order[8], no = 0;
                            for (int c = 0; c < 8; c++)
                                if (at[c] < cnt[g0 + c]) order[no++] = c;
                            if (no == 0) break;
                            std::stable_sort(order, order + no, [&](int a, int b) {
                                return cnt[g0 + a] - at[a] > cnt[g0 + b] - at[b];
                            });
                            unsigned used = 0, moved = 0;
                            for (int o = 0; o < no; o++) {
                                const int c = order[o];
                                const int k = ri[cur[p][g0 + c] + at[c]];
                                const uint16_t a = (uint16_t)((k - j * C) * MT);
                                const int w = a % 64 / 8;
                                if ((used >> w) & 1u) continue;
                                used |= 1u << w;
                                moved |= 1u << c;
                                seq[g0 + c].push_back(a);
                                at[c]++;
                            }
                            int wz = 0;
                            while (wz < 8 && ((used >> wz) & 1u)) wz++;
                            const uint16_t z = (uint16_t)((C + (wz - C % 8 + 8) % 8) * MT);  // zero row in window wz
                            for (int c = 0; c < 8; c++)
                                if (!((moved >> c) & 1u)) seq[g0 + c].push_back(z);
                        }
                        L = std::max(L, (int)seq[g0].size());
                    }
                }
                const int b8 = (L + 7) / 8;
                const size_t base = e16.size();
                e16.resize(base + (size_t)b8 * 128, pad);
                for (int c = 0; c < 16; c++) {
                    if (sched) {
                        for (size_t i = 0; i < seq[c].size(); i++)
                            e16[base + (i / 8) * 128 + (size_t)c * 8 + i % 8] = seq[c][i];
                    } else {
                        for (int i = 0; i < cnt[c]; i++) {
                            const int k = ri[cur[p][c] + i];
                            e16[base + (size_t)(i / 8) * 128 + (size_t)c * 8 + (size_t)(i % 8)] =
                                (uint16_t)((k - j * C) * MT);
                        }
                    }
                    cur[p][c] += cnt[c];
                }
                if (two) {
                    // per entry position (block, entry) and ds_read_b64 lane
                    // group (columns 0-7, 8-15): each entry reads copy A or B,
                    // whichever window (8 banks: float index % 64 / 8) holds
                    // fewer distinct rows of the group so far (greedy; a row
                    // already there broadcasts)
                    for (int i8 = 0; i8 < b8; i8++)
                        for (int h = 0; h < 8; h++)
                            for (int g0 = 0; g0 < 16; g0 += 8) {
                                int nwin[8] = {0};
                                uint32_t seen[8][8];
                                for (int c = g0; c < g0 + 8; c++) {
                                    uint16_t &u = e16[base + (size_t)i8 * 128 + (size_t)c * 8 + (size_t)h];
                                    const uint32_t cand[2] = {u, (uint32_t)(xb + u)};
                                    int best = 0, best_load = 1 << 30;
                                    for (int o = 0; o < 2; o++) {
                                        const int w = (int)(cand[o] % 64 / 8);
                                        bool dup = false;
                                        for (int t = 0; t < nwin[w]; t++) dup |= seen[w][t] == cand[o];
                                        const int load = dup ? nwin[w] : nwin[w] + 1;
                                        if (load < best_load) {
                                            best_load = load;
                                            best = o;
                                        }
                                    }
                                    const int w = (int)(cand[best] % 64 / 8);
                                    bool dup = false;
                                    for (int t = 0; t < nwin[w]; t++) dup |= seen[w][t] == cand[best];
                                    if (!dup) seen[w][nwin[w]++] = cand[best];
                                    u = (uint16_t)cand[best];
                                }
                            }
                }
                n8 += (uint32_t)b8;
                if (p == 0) n8pos = (uint32_t)b8;
            }
            img.tab[((size_t)sl * steps + step) * 2] = (uint32_t)(at / 128);
            img.tab[((size_t)sl * steps + step) * 2 + 1] = n8 | n8pos << 16;
        }
    }
    img.ent.assign((e16.size() + 1) / 2 + 4, 0u);
    std::memcpy(img.ent.data(), e16.data(), e16.size() * sizeof(uint16_t));
}

std::string validate_tcsc(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                          const int32_t *rin, int K, int N, int B)
{
    if (K < 0 || N < 0) return "negative K or N";
    if (B < 0) return "negative block size";
    if (!csp || !csn) return "null col_start array";
    // plain TCSC: one slot per column, rows in [0, K); BlockedTCSC<B>
    // (BlockedTCSC.h:15-41): slot kb*N + n holds column n's rows of block kb,
    // [kb*B, kb*B + B), for the K/B whole blocks
    const int64_t nb = B ? K / B : 1, slots = nb * N;
    if (csp[0] != 0 || csn[0] != 0) return "col_start[0] must be 0";
    for (int64_t s = 0; s < slots; s++) {
        if (csp[s + 1] < csp[s]) return "col_start_pos not monotone at slot " + std::to_string(s);
        if (csn[s + 1] < csn[s]) return "col_start_neg not monotone at slot " + std::to_string(s);
    }
    if ((csp[slots] > 0 && !rip) || (csn[slots] > 0 && !rin)) return "null row_index array";
    for (int64_t s = 0; s < slots; s++) {
        const int n = (int)(s % (N ? N : 1));
        const int64_t klo = B ? (s / N) * B : 0, khi = B ? klo + B : K;
        const std::string where = B ? "block " + std::to_string(s / N) + " column " + std::to_string(n)
                                    : "column " + std::to_string(n);
        for (int p = 0; p < 2; p++) {
            const int32_t *cs = p ? csn : csp;
            const int32_t *ri = p ? rin : rip;
            for (int32_t i = cs[s]; i < cs[s + 1]; i++) {
                if (ri[i] < klo || ri[i] >= khi)
                    return (B ? "row index out of its block in " : "row index out of [0,K) in ") + where;
                if (i > cs[s] && ri[i] <= ri[i - 1]) return "row indices not strictly ascending in " + where;
            }
        }
        // a k may not be both +1 and -1 in one column (the format encodes a
        // single ternary value per (k, n))
        int32_t a = csp[s], b = csn[s];
        while (a < csp[s + 1] && b < csn[s + 1]) {
            if (rip[a] == rin[b]) return "row index in both +1 and -1 runs of " + where;
            if (rip[a] < rin[b]) a++; else b++;
        }
    }
    return std::string();
}

// splitmix64 + unbiased bounded draw: the same stream as the test oracle's
// oracle_gen_ternary, so a seed names one W everywhere.
static inline uint64_t splitmix64(uint64_t &s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint64_t below(uint64_t &s, uint64_t n)
{
    if (n <= 1) return 0;
    const uint64_t thresh = (0 - n) % n;
    uint64_t x;
    do x = splitmix64(s); while (x < thresh);
    return x % n;
}

}  // namespace tsg

// ---------------------------------------------------------------- C-ABI --

thread_local std::string g_tsg_host_err;

extern "C" int tsg_blocked_tcsc_validate(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                                         const int32_t *rin, int K, int N, int B)
{
    if (B <= 0) {
        g_tsg_host_err = "block size must be positive";
        return TSG_ERR_ARG;
    }
    const std::string e = tsg::validate_tcsc(csp, csn, rip, rin, K, N, B);
    if (!e.empty()) {
        g_tsg_host_err = e;
        return TSG_ERR_ARG;
    }
    return TSG_OK;
}

extern "C" int tsg_tcsc_validate(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                                 const int32_t *rin, int K, int N)
{
    std::string e = tsg::validate_tcsc(csp, csn, rip, rin, K, N);
    if (!e.empty()) {
        g_tsg_host_err = e;
        return TSG_ERR_ARG;
    }
    return TSG_OK;
}

extern "C" int tsg_tcsc_slice(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                              const int32_t *rin, int N, int n0, int n1, int32_t *ocsp,
                              int32_t *ocsn, int32_t *orip, int32_t *orin, int64_t *nnz_pos,
                              int64_t *nnz_neg)
{
    if (!csp || !csn || n0 < 0 || n1 < n0 || n1 > N) {
        g_tsg_host_err = "tsg_tcsc_slice: bad arguments";
        return TSG_ERR_ARG;
    }
    const int32_t p0 = csp[n0], p1 = csp[n1], q0 = csn[n0], q1 = csn[n1];
    if (nnz_pos) *nnz_pos = p1 - p0;
    if (nnz_neg) *nnz_neg = q1 - q0;
    if (ocsp)
        for (int i = 0; i <= n1 - n0; i++) ocsp[i] = csp[n0 + i] - p0;
    if (ocsn)
        for (int i = 0; i <= n1 - n0; i++) ocsn[i] = csn[n0 + i] - q0;
    if (orip && p1 > p0) std::memcpy(orip, rip + p0, sizeof(int32_t) * (size_t)(p1 - p0));
    if (orin && q1 > q0) std::memcpy(orin, rin + q0, sizeof(int32_t) * (size_t)(q1 - q0));
    return TSG_OK;
}

// generateSparseMatrix distribution (cpp_impl/sparseUtils.h:52-87), emitted
// as TCSC of the columns [n0, n1).  Row k is drawn exactly as the oracle's
// dense generator draws it; only entries of the slice are kept.
extern "C" int tsg_gen_tcsc(int K, int N, int s, uint64_t seed, int n0, int n1, int32_t *csp,
                            int32_t *csn, int32_t *rip, int32_t *rin, int64_t *nnz_pos,
                            int64_t *nnz_neg)
{
    if (K < 0 || N < 0 || s <= 0 || n0 < 0 || n1 < n0 || n1 > N) {
        g_tsg_host_err = "tsg_gen_tcsc: bad arguments";
        return TSG_ERR_ARG;
    }
    const int W = n1 - n0;
    const int per_row = N / s, half = per_row / 2, vari = per_row / 20 + 1;
    std::vector<int8_t> occ((size_t)N, 0);
    std::vector<int32_t> touched;
    touched.reserve((size_t)per_row + 8);
    // row-major shard: (k, col, sign) in row order; per column counts
    std::vector<int64_t> cntp((size_t)W + 1, 0), cntn((size_t)W + 1, 0);
    std::vector<int32_t> rowcol;   // packed (col - n0) for kept entries, row order
    std::vector<int8_t> rowsgn;
    std::vector<int32_t> rowk;
    const bool fill = csp && csn;
    uint64_t st = seed;
    for (int k = 0; k < K; k++) {
        const int v = (int)tsg::below(st, (uint64_t)vari + 1);
        int npos = half + v, nneg = half - v;
        if (npos > N) npos = N;
        if (nneg < 0) nneg = 0;
        if (nneg > N - npos) nneg = N - npos;
        touched.clear();
        for (int c = 0; c < npos;) {
            const int col = (int)tsg::below(st, (uint64_t)N);
            if (occ[col] == 0) { occ[col] = 1; touched.push_back(col); c++; }
        }
        for (int c = 0; c < nneg;) {
            const int col = (int)tsg::below(st, (uint64_t)N);
            if (occ[col] == 0) { occ[col] = -1; touched.push_back(col); c++; }
        }
        for (int32_t col : touched) {
            if (col >= n0 && col < n1) {
                if (occ[col] > 0) cntp[col - n0 + 1]++; else cntn[col - n0 + 1]++;
                if (fill) {
                    rowk.push_back(k);
                    rowcol.push_back(col - n0);
                    rowsgn.push_back(occ[col]);
                }
            }
            occ[col] = 0;
        }
    }
    for (int i = 0; i < W; i++) {
        cntp[i + 1] += cntp[i];
        cntn[i + 1] += cntn[i];
    }
    if (nnz_pos) *nnz_pos = cntp[W];
    if (nnz_neg) *nnz_neg = cntn[W];
    if (cntp[W] > INT32_MAX || cntn[W] > INT32_MAX) {
        g_tsg_host_err = "tsg_gen_tcsc: slice nnz exceeds int32 (shard the columns)";
        return TSG_ERR_RANGE;
    }
    if (!fill) return TSG_OK;
    for (int i = 0; i <= W; i++) {
        csp[i] = (int32_t)cntp[i];
        csn[i] = (int32_t)cntn[i];
    }
    // counting sort by column; rows arrive in ascending k so each column's
    // list is ascending, as TCSC.h:23-36 produces it
    std::vector<int64_t> curp(cntp.begin(), cntp.end() - 1), curn(cntn.begin(), cntn.end() - 1);
    for (size_t e = 0; e < rowk.size(); e++) {
        const int c = rowcol[e];
        if (rowsgn[e] > 0) rip[curp[c]++] = rowk[e];
        else rin[curn[c]++] = rowk[e];
    }
    return TSG_OK;
}

extern "C" int tsg_gen_x(int64_t len, int range, uint64_t seed, float *X)
{
    if (len < 0 || range < 0 || (len > 0 && !X)) {
        g_tsg_host_err = "tsg_gen_x: bad arguments";
        return TSG_ERR_ARG;
    }
    uint64_t st = seed;
    for (int64_t i = 0; i < len; i++)
        X[i] = (float)((int64_t)tsg::below(st, 2ull * (uint64_t)range + 1) - range);
    return TSG_OK;
}

// ------------------------------------------- CSC + base-3 packed values --
// readme.md:111: "normal CSC with compressed values vector (1s and -1s, 8
// bits for 5 values)".  digit = v + 1, 5 digits per byte, CSC order.

extern "C" int tsg_tcsc_to_csc_packed(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                                      const int32_t *rin, int N, int32_t *col_ptr,
                                      int32_t *row_idx, uint8_t *packed, int64_t *nnz)
{
    if (!csp || !csn || N < 0) {
        g_tsg_host_err = "tsg_tcsc_to_csc_packed: bad arguments";
        return TSG_ERR_ARG;
    }
    const int64_t total = (int64_t)csp[N] + (int64_t)csn[N];
    if (nnz) *nnz = total;
    if (total > INT32_MAX) {
        g_tsg_host_err = "tsg_tcsc_to_csc_packed: nnz exceeds int32";
        return TSG_ERR_RANGE;
    }
    if (!col_ptr || !row_idx || !packed) return TSG_OK;
    static const int pw[5] = {1, 3, 9, 27, 81};
    std::memset(packed, 0, (size_t)((total + 4) / 5));
    int64_t e = 0;
    for (int n = 0; n < N; n++) {  // merge the two ascending runs of column n
        col_ptr[n] = (int32_t)e;
        int32_t a = csp[n], b = csn[n];
        while (a < csp[n + 1] || b < csn[n + 1]) {
            const bool pos = b >= csn[n + 1] || (a < csp[n + 1] && rip[a] < rin[b]);
            row_idx[e] = pos ? rip[a++] : rin[b++];
            packed[e / 5] = (uint8_t)(packed[e / 5] + (pos ? 2 : 0) * pw[e % 5]);
            e++;
        }
    }
    col_ptr[N] = (int32_t)e;
    return TSG_OK;
}

extern "C" int tsg_csc_packed_to_tcsc(const int32_t *col_ptr, const int32_t *row_idx,
                                      const uint8_t *packed, int N, int32_t *csp, int32_t *csn,
                                      int32_t *rip, int32_t *rin, int64_t *nnz_pos,
                                      int64_t *nnz_neg)
{
    if (!col_ptr || N < 0 || col_ptr[0] != 0 || (col_ptr[N] > 0 && (!row_idx || !packed))) {
        g_tsg_host_err = "tsg_csc_packed_to_tcsc: bad arguments";
        return TSG_ERR_ARG;
    }
    int64_t p = 0, q = 0;
    for (int n = 0; n < N; n++) {
        if (col_ptr[n + 1] < col_ptr[n]) {
            g_tsg_host_err = "tsg_csc_packed_to_tcsc: col_ptr not monotone";
            return TSG_ERR_ARG;
        }
        if (csp) csp[n] = (int32_t)p;
        if (csn) csn[n] = (int32_t)q;
        for (int32_t i = col_ptr[n]; i < col_ptr[n + 1]; i++) {
            int d = packed[i / 5];
            for (int j = 0; j < i % 5; j++) d /= 3;
            d %= 3;
            if (d == 1) {
                g_tsg_host_err = "tsg_csc_packed_to_tcsc: stored entry with value 0 at " + std::to_string(i);
                return TSG_ERR_ARG;
            }
            if (d == 2) { if (rip) rip[p] = row_idx[i]; p++; }
            else { if (rin) rin[q] = row_idx[i]; q++; }
        }
    }
    if (csp) csp[N] = (int32_t)p;
    if (csn) csn[N] = (int32_t)q;
    if (nnz_pos) *nnz_pos = p;
    if (nnz_neg) *nnz_neg = q;
    return TSG_OK;
}

// Host-only view of the small-M kernel's sliced-ELL image (tests decode it and
// replay the kernel's walk on the CPU).  NULL buffers query the lengths.
extern "C" int tsg_ell_build(const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin, int K,
                             int N, int Cmax, int MT, int copies, uint32_t *ent, int64_t ent_cap, int64_t *ent_len,
                             uint32_t *tab, int64_t tab_cap, int64_t *tab_len, int32_t *C, int32_t *nch, int32_t *xb)
{
    // copies: 1 or 2 X^T copies; 3 = one copy with the bank-window schedule
    const bool sched = copies == 3;
    if (sched) copies = 1;
    const std::string e = tsg::validate_tcsc(csp, csn, rip, rin, K, N);
    if (!e.empty() || Cmax < 4 || Cmax % 4 || MT < 1 || (int64_t)Cmax * MT >= 65536) {
        g_tsg_host_err = e.empty() ? "tsg_ell_build: Cmax must be a multiple of 4 with Cmax * MT < 65536"
                                   : "tsg_ell_build: " + e;
        return TSG_ERR_ARG;
    }
    if (copies != 1 && copies != 2) {
        g_tsg_host_err = "tsg_ell_build: copies must be 1, 2 or 3 (the schedule)";
        return TSG_ERR_ARG;
    }
    tsg::EllImage img;
    tsg::build_ell_image(csp, csn, rip, rin, K, N, Cmax, MT, img, copies, sched);
    if (xb) *xb = sched ? -img.zr : img.xb;  // (the schedule: minus its zero rows)
    if (ent_len) *ent_len = (int64_t)img.ent.size();
    if (tab_len) *tab_len = (int64_t)img.tab.size();
    if (C) *C = img.C;
    if (nch) *nch = img.nch;
    if ((ent && ent_cap < (int64_t)img.ent.size()) || (tab && tab_cap < (int64_t)img.tab.size())) {
        g_tsg_host_err = "tsg_ell_build: buffer too small";
        return TSG_ERR_ARG;
    }
    if (ent) std::memcpy(ent, img.ent.data(), img.ent.size() * 4);
    if (tab) std::memcpy(tab, img.tab.data(), img.tab.size() * 4);
    return TSG_OK;
}
