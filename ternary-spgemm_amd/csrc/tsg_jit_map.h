// tsg_jit_map.h -- workgroup -> (column tile, M tile) map of the weight-compiled
// kernel, shared by the dispatcher (tsg_jit_kernel.hip) and the host (the
// per-call choice of gn/gm in tsg_capi.cpp, and the bijection test through
// tsg_jit_tile_map).
//
// XCD-aware: workgroup ids are dealt to the 8 XCDs round-robin (id L runs on
// XCD L % 8), so each XCD first gets a contiguous run of logical ids wg; then
// consecutive wg walk groups of gn column tiles x gm M tiles, so the ~32
// workgroups an XCD runs at once share gn code streams and gm X^T slabs
// through its L2.  Measured placement (scripts/hwid_micro.hip):
// an XCD's slot s goes to shader engine s % 4 (rotated), CU s / 4 of it, so
// nt = slot % gn puts every CU of an SE on the same column tile and the CU
// pairs that share an instruction cache fetch one code stream.
#pragma once

#ifdef __HIPCC__
#define TSG_HD __host__ __device__
#else
#define TSG_HD
#endif

TSG_HD inline void tsg_jit_tile(int L, int mtiles, int ntiles, int gn, int gm, int &nt, int &mt)
{
    const int T = mtiles * ntiles;
    const int xcd = L & 7, slot = L >> 3, q8 = T >> 3, r8 = T & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
    const int cb = wg / (gn * mtiles);                                      // column-tile block
    const int wc = ntiles - gn * cb < gn ? ntiles - gn * cb : gn;           // its column tiles
    const int loc = wg - cb * gn * mtiles, g = loc / (wc * gm), i = loc - g * wc * gm;
    nt = gn * cb + i % wc;
    mt = gm * g + i / wc;
}
