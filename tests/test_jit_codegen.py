"""The weight-compiled kernel's machine code, checked on the CPU before any GPU
runs it.  tsg_jit_codegen's region is decoded instruction by instruction (only
the gfx950 encodings the generator may emit are accepted) and a whole
workgroup is emulated against the register contract of
ternary-spgemm_amd/csrc/tsg_jit_kernel.hip and the k-pair X^T layout of
tsg_internal.h: its 8 waves run barrier phase by barrier phase, LDS-DMA
copies (one 1-KiB k-row pair per piece) land at the issuing wave's
`s_waitcnt vmcnt(n)` (VMEM loads return in order: all but the newest n),
ds_read_b128 loads both rows of a pair (ds_read_b64 one of them),
and every LDS read is checked to see data that landed in an EARLIER phase (no
read-after-DMA race) while no DMA may overwrite rows read since it was issued
(no write-after-read race).  Code-prefetch loads must stay inside the region.
The emulated Y must equal the BaseTCSC oracle (comp.h:25-69) bit for bit, for
integer and for order-sensitive non-integer X.  tests/test_gpu_parity.py then
shows the GPU runs that code."""
import os
import struct

import numpy as np
import pytest

MAGIC = (0x7453474A, 0x314A4954)


class Geom:
    """Geometry from the region header (words 2-7) and the register contract
    of tsg_jit_kernel.hip derived from it."""

    def __init__(self, code):
        w2, w3, w4 = int(code[2]), int(code[3]), int(code[4])
        self.waves, self.nw, self.chunk = w2 & 0xFF, (w2 >> 8) & 0xFF, w2 >> 16
        self.slots, self.tile_m = w3 & 0xFFFF, w3 >> 16
        self.streams, self.msplit = w4 & 0xFF, (w4 >> 8) & 0xFF
        self.tile_cols = self.streams * self.nw
        self.ring = int(code[7]) & 0xFF
        fmt = (int(code[7]) >> 8) & 0xFF
        # format 2: k-pair X^T, 128-row tiles, v_pk_add_f32 (2 rows per lane);
        # format 3: the 64-row image -- k-quad X^T, 64-row tiles, VOP2 adds
        assert fmt in (2, 3), "region must use the k-pair (2) or k-quad (3) X^T layout"
        self.r64 = fmt == 3
        # 64-row image: rows per DMA piece (bit 18: 16 rows x 4 quads, else 8 x 8)
        self.pr_rows = (16 if (int(code[7]) >> 18) & 1 else 8) if self.r64 else 0
        assert self.streams == self.waves and self.msplit == 1 and self.tile_m == (64 if self.r64 else 128)
        # DMA pieces take their in-group offset from the instruction offset (one
        # M0 per 4 pieces; the dispatcher subtracts it from the global offsets)
        self.m0k = (int(code[7]) >> 16) & 1
        # 16 m0k, 17 far, 18 R16, 19 the half ring (64-row image, 4 waves, 96-row chunks),
        # 20 the row layout (64-row image: rows of 47 quads, 188-row chunks)
        assert int(code[7]) >> 21 == 0 and (self.r64 or (int(code[7]) >> 18) & 7 == 0)
        self.half = (int(code[7]) >> 19) & 1
        self.rowlay = (int(code[7]) >> 20) & 1
        assert not self.half or (self.waves == 4 and self.chunk == 96)
        assert not self.rowlay or (self.chunk == 188 and not self.half and not (int(code[7]) >> 18) & 1)
        self.unit = 4 if self.r64 else 2              # k rows per LDS unit (quad / pair)
        self.pairs = self.chunk // self.unit          # units per chunk (row layout: 47 quads per row)
        self.pair_bytes = self.tile_m * 4 * self.unit  # one unit row of the tile in LDS: 1 KiB
        assert self.pair_bytes == 1024
        # ring buffer: 48 KiB (row layout: 47 pieces used of the 48 the register contract has)
        self.buf_bytes = 48 * 1024 if self.rowlay else self.pairs * self.pair_bytes
        self.pieces = self.buf_bytes // 1024 // self.waves  # DMA pieces (pair rows) per wave
        self.lds_v = 8 + 4 * self.slots               # X slots: 4 VGPRs each
        self.sink_v = self.lds_v + self.ring
        self.dma_v = self.sink_v + 1
        self.l128_v = self.dma_v + self.pieces
        self.acc0 = (self.l128_v + 2) & ~1
        # BlockedTCSC<B> (B > 0): X slots v[8 : 8 + 4 xslots), block sums y above them
        self.B = int(code[5])
        self.xslots = int(code[6]) or self.slots
        self.tmp0 = 8 + 4 * self.xslots


XT_BASE = 1 << 40  # fake device address of X^T


class Wave:
    def __init__(self, w, pc):
        self.w, self.pc = w, pc
        # registers the dispatcher does not set hold garbage: NaN poisons any
        # use before a def; the accumulators start at +0 (tsg_jit_kernel.hip)
        self.v = np.full((256, 64), np.nan, np.float32)
        self.m0 = 0x5A5A
        self.saved_m0 = None
        self.base = None
        self.touch = None
        self.pending = []  # VMEM loads not yet returned, oldest first: the DMA copies of one
        #                    global_load_lds [(lds_byte, data, issue_phase)...] or [] (code touch)
        self.reads = []    # (first VGPR, count) of LDS reads not yet waited for, oldest first
        self.done = False


def _classify_pk(w0, w1, G):
    """v_pk_add_f32 forms the generator may emit (tsg_jit.cpp Emit):
    add   v[d] = v[d] +/- X slot      (d: accumulator; BlockedTCSC: block sum y)
    first v[d] = +/-X slot + 0        (BlockedTCSC: a block's first entry, 0 + x / 0 - x)
    flush v[d] = v[d] + y             (BlockedTCSC: Y += y at a block's end)"""
    d = w0 & 0xFF
    neg0, neg1 = bool(w0 & 0x100), bool(w0 & 0x200)  # neg_hi of src0 / src1
    assert (w1 >> 29) & 1 == neg0 and (w1 >> 30) & 1 == neg1, "neg_lo and neg_hi disagree"
    assert (w1 >> 18) & 0x1FF == 0 and (w1 >> 27) & 3 == 3 and (w0 >> 11) & 0x1F == 8  # op_sel_hi, clamp/opsel
    s0, s1 = w1 & 0x1FF, (w1 >> 9) & 0x1FF
    x_lo, x_hi = 8, 8 + 4 * G.xslots
    acc = G.acc0 <= d < G.acc0 + 2 * G.nw
    tmp = G.B and G.tmp0 <= d < G.tmp0 + G.nw
    assert d % 2 == 0
    if s1 == 128:  # inline constant 0
        assert tmp and not neg1 and x_lo <= s0 - 256 < x_hi and s0 % 2 == 0
        return "first", (d, s0 - 256, neg0)
    assert s0 == 256 + d and not neg0, "v_pk_add_f32 must accumulate in place"
    if x_lo <= s1 - 256 < x_hi:
        assert (tmp if G.B else acc) and s1 % 2 == 0
        return "add", (d, s1 - 256, neg1)
    assert G.B and acc and not neg1 and G.tmp0 <= s1 - 256 < G.tmp0 + G.nw
    return "flush", (d, s1 - 256)


def _decode(code, pc, G):
    w0 = int(code[pc])
    w1 = int(code[pc + 1]) if pc + 1 < len(code) else None
    if G.r64 and (w0 >> 31) == 0:  # VOP2: v_add_f32 (op 1) / v_sub_f32 (op 2) acc, acc, x
        op, d, x, s0 = (w0 >> 25) & 0x3F, (w0 >> 17) & 0xFF, (w0 >> 9) & 0xFF, w0 & 0x1FF
        assert op in (1, 2) and s0 == 256 + d, f"unexpected VOP2 word {w0:#010x}"
        assert G.acc0 <= d < G.acc0 + G.nw and 8 <= x < 8 + 4 * G.xslots
        return "vadd", (d, x, op == 2), 1
    if (w0 & 0xFFFFFFF0) == 0xBF800000:
        return "nop", (), 1
    if w0 in (0xBF8F0000, 0xBF8F0001):  # s_setprio 0 / 1 (TSG_JIT_PRIO: issue arbitration only)
        return "nop", (), 1
    if (w0 & 0xFFFFF0FF) == 0xBF8CC07F:
        return "wait_lgkm", ((w0 >> 8) & 0xF,), 1
    if (w0 & 0xFFFFFFF0) == 0xBF8C0F70:  # s_waitcnt vmcnt(n), n <= 15
        return "wait_vm", (w0 & 0xF,), 1
    simple = {0xBF8A0000: "barrier", 0xBED6007C: "save_m0", 0x80D45754: "last_adj", 0x82D58055: "last_adjc",
              0xBEFC0056: "restore_m0", 0xBED40150: "base_reset", 0xBE801D5E: "ret", 0x82558055: "base_addc",
              0x8259805B: "touch_addc", 0x80545254: "base_add"}
    if w0 in simple:
        return simple[w0], (), 1
    if w0 == 0x807CFF53:  # s_add_u32 m0, s83, lit
        return "m0", (w1,), 2
    if w0 == 0x8058FF5A:  # s_add_u32 s88, s90, lit: the touch base s[90:91] (region base or 8 KiB below)
        # never less than 8 KiB ahead relative to the base: with the dispatcher's
        # near bias (-8 KiB) the touch still starts inside the region
        assert w1 >= 8192, "code touch closer than 8 KiB to the touch base"
        return "touch_addr", (w1,), 2
    CP = 0x2030000  # cache-policy bits (sc0, nt, sc1): any combination
    if (w0 & ~CP) == 0xDC508000:
        # the step's own touch: v[lane128]; the per-group ones (round 6): v[lane128 + 1]
        assert w1 in ((G.sink_v << 24) | (88 << 16) | G.l128_v, (G.sink_v << 24) | (88 << 16) | (G.l128_v + 1))
        return "touch", (), 2
    if (w0 & ~CP & 0xFFFFF000) == 0xDDF48000:  # global_load_lds_dwordx4 v, s[84:85] offset:(w0 & 0xFFF)
        assert (w1 >> 16) == 84
        return "glds", (w1 & 0xFF, w0 & 0xFFF), 2
    if (w0 & 0xFFFFFC00) == 0xD3B24000:  # v_pk_add_f32
        kind, f = _classify_pk(w0, w1, G)
        return kind, f, 2
    if G.r64 and (w0 & 0xFFFF0000) == 0xD86C0000:  # ds_read_b32
        assert (w1 >> 8) & 0xFFFF == 0
        return "read", (w1 >> 24, w1 & 0xFF, w0 & 0xFFFF, 1), 2
    if (w0 & 0xFFFF0000) == 0xD8EC0000:  # ds_read_b64
        assert (w1 >> 8) & 0xFFFF == 0
        return "read", (w1 >> 24, w1 & 0xFF, w0 & 0xFFFF, 2), 2
    if (w0 & 0xFFFF0000) == 0xD9FE0000:  # ds_read_b128
        assert (w1 >> 8) & 0xFFFF == 0
        return "read", (w1 >> 24, w1 & 0xFF, w0 & 0xFFFF, 4), 2
    raise AssertionError(f"unexpected instruction word {w0:#010x} at word {pc}")


def _overlaps(reads, r0, n):
    return any(a < r0 + n and r0 < a + m for a, m in reads)


def emulate_tile(code, wcode, t, XP, m0, Mp, nch):
    """One workgroup (column tile t, M tile at m0) over the k-pair X^T XP
    [pairs][Mp/2][4] (64-row image: quads [Kp/4][Mp][4]; row layout: per chunk
    [Mp][47][4], XP[j] = the quads from the chunk's first K row,
    jit64_row_kbase): returns acc[tile rows, tile cols]."""
    G = Geom(code)
    WAVES, NW, PAIRS, PAIR_BYTES, BUF_BYTES, PIECES = (G.waves, G.nw, G.pairs, G.pair_bytes, G.buf_bytes,
                                                       G.pieces)
    region_bytes = len(code) * 4
    stride = G.chunk * Mp * 4
    NBUF = G.ring
    lds = np.zeros(NBUF * BUF_BYTES // 4, np.float32)
    landed = np.full(NBUF * BUF_BYTES // PAIR_BYTES, -1)   # phase a 1-KiB piece's data landed
    last_read = np.full(NBUF * BUF_BYTES // PAIR_BYTES, -1)
    S = G.streams
    waves = [Wave(w, int(wcode[t * S + w]) // 4) for w in range(WAVES)]
    RPL = 1 if G.r64 else 2  # M rows per lane
    for wv in waves:
        wv.v[G.acc0:G.acc0 + RPL * NW] = 0.0
        assert int(wcode[t * S + wv.w]) % 256 == 0
    phase = 0
    while not all(wv.done for wv in waves):
        at_barrier = 0
        for wv in waves:
            if wv.done:
                continue
            while True:
                kind, f, n = _decode(code, wv.pc, G)
                wv.pc += n
                if kind == "barrier":
                    at_barrier += 1
                    break
                if kind == "ret":
                    assert not wv.pending and wv.m0 == 0x5A5A
                    wv.done = True
                    break
                if kind == "save_m0":
                    wv.saved_m0 = wv.m0
                elif kind == "restore_m0":
                    wv.m0 = wv.saved_m0
                elif kind == "m0":
                    wv.m0 = wv.w * PIECES * 1024 + f[0]  # s83 = the wave's first DMA piece
                elif kind == "base_reset":
                    wv.base = XT_BASE
                elif kind == "base_add":
                    wv.base += stride
                elif kind == "last_adj":  # s87: 0 for a staged copy (the one emulated here)
                    assert G.rowlay
                elif kind == "last_adjc":
                    assert G.rowlay
                elif kind == "touch_addr":
                    wv.touch = f[0]
                elif kind == "touch":
                    assert wv.touch is not None and wv.touch + 63 * 128 + 4 <= region_bytes, "prefetch past region"
                    wv.pending.append([])
                elif kind == "glds":
                    i, off = f[0] - G.dma_v, f[1]
                    assert 0 <= i < PIECES
                    # the dispatcher's off[i] minus the instruction offset it
                    # expects (m0k: (i & 3) KiB): the global side reads pair row pr
                    assert off == ((i & 3) * PAIR_BYTES if G.m0k else 0), "DMA offset disagrees with the dispatcher"
                    pr = wv.w * PIECES + i  # the pair row this lane set copies (dispatcher off[i])
                    j, rem = divmod(wv.base - XT_BASE, stride)
                    assert rem == 0 and 0 <= j < nch
                    dst = wv.m0 + off  # the offset applies to the LDS address too
                    assert dst % BUF_BYTES == pr * PAIR_BYTES, "DMA lands on the wrong pair row"
                    if G.rowlay:  # lane slot 64 pr + l = (row, quad) of the 64 x 47-quad chunk
                        assert pr < PAIRS, "row layout: piece past the chunk's 47"
                        slots = pr * 64 + np.arange(64)
                        data = XP[j][m0 + slots // PAIRS, slots % PAIRS].reshape(-1).copy()
                    elif G.r64:  # blocked k-quad piece pr = Q qg + rg: lane slot l = row R rg + l % R, quad Q qg + l / R
                        R = G.pr_rows
                        Q = 64 // R
                        qg, rg = divmod(pr, Q)
                        lanes = np.arange(64)
                        q = j * PAIRS + Q * qg + lanes // R
                        data = XP[q, m0 + R * rg + lanes % R].reshape(-1).copy()
                    else:
                        data = XP[j * PAIRS + pr, m0 // RPL:m0 // RPL + 64].reshape(-1).copy()
                    wv.pending.append([(dst, data, phase)])
                elif kind == "wait_vm":  # loads return in order: all but the newest f[0] land
                    n_land = max(len(wv.pending) - f[0], 0)
                    for op in wv.pending[:n_land]:
                        for dst, data, iss in op:
                            row = dst // PAIR_BYTES
                            assert last_read[row] < iss, "DMA overwrites a pair row read since its issue (WAR race)"
                            lds[dst // 4:dst // 4 + 256] = data
                            landed[row] = phase
                    wv.pending = wv.pending[n_land:]
                elif kind == "wait_lgkm":
                    while len(wv.reads) > f[0]:  # LDS returns in order
                        wv.reads.pop(0)
                elif kind == "read":
                    vd, a, off, nreg = f
                    assert not _overlaps(wv.reads, vd, nreg), "X slot reloaded before its previous read was waited for"
                    wv.reads.append((vd, nreg))
                    assert G.lds_v <= a < G.lds_v + NBUF
                    assert 8 <= vd and vd + nreg <= 8 + 4 * G.xslots and (vd - 8) % 4 == 0
                    allowed = {4: (0,), 2: (0, 8), 1: (0, 4, 8, 12)}[nreg]
                    buf = a - G.lds_v
                    if G.rowlay:
                        # row layout: lane l's base (dispatcher) = buffer + l * 752; quad q at + 16 q
                        sub = off % 16
                        assert sub in allowed and off // 16 < PAIRS
                        lanes = np.arange(64)
                        addr = buf * BUF_BYTES + lanes * 16 * PAIRS + off
                        pieces = np.unique(addr // PAIR_BYTES)
                        assert all(0 <= landed[p] < phase for p in pieces), "LDS read of data not yet landed before a barrier"
                        for p in pieces:
                            last_read[p] = max(last_read[p], phase)
                        wv.v[vd:vd + nreg] = np.stack([lds[addr // 4 + t] for t in range(nreg)])
                    elif G.r64:
                        # blocked k-quad layout: lane l's base (dispatcher) = buffer +
                        # (l / R) KiB + (l % R) * 16; quad q at (q / Q) * 64 KiB / R + (q % Q) * 16 R
                        R = G.pr_rows
                        Q = 64 // R
                        sub = off % (16 * R)
                        assert sub in allowed and off // (65536 // R) < PAIRS // Q
                        lanes = np.arange(64)
                        addr = buf * BUF_BYTES + (lanes // R) * 1024 + (lanes % R) * 16 + off
                        pieces = np.unique(addr // PAIR_BYTES)
                        assert len(pieces) == Q and all(0 <= landed[p] < phase for p in pieces), \
                            "LDS read of data not yet landed before a barrier"
                        for p in pieces:
                            last_read[p] = max(last_read[p], phase)
                        wv.v[vd:vd + nreg] = np.stack([lds[addr // 4 + t] for t in range(nreg)])
                    else:
                        assert off // PAIR_BYTES < PAIRS and off % PAIR_BYTES in allowed and nreg != 1
                        j0 = (off % PAIR_BYTES) // 4  # first of the unit's 4 dwords per lane the read loads
                        row = buf * PAIRS + off // PAIR_BYTES
                        assert 0 <= landed[row] < phase, "LDS read of data not yet landed before a barrier"
                        last_read[row] = max(last_read[row], phase)
                        vals = lds[row * 256:row * 256 + 256].reshape(64, 4)  # lane l: 16 B at lane*16
                        wv.v[vd:vd + nreg] = vals[:, j0:j0 + nreg].T
                elif kind == "vadd":
                    d, x, neg = f
                    assert not _overlaps(wv.reads, x, 1), "add reads an X register whose LDS read may not have returned"
                    wv.v[d] = wv.v[d] - wv.v[x] if neg else wv.v[d] + wv.v[x]
                elif kind == "add":
                    d, x, neg = f
                    assert not _overlaps(wv.reads, x, 2), "add reads an X slot whose LDS read may not have returned"
                    wv.v[d:d + 2] = wv.v[d:d + 2] - wv.v[x:x + 2] if neg else wv.v[d:d + 2] + wv.v[x:x + 2]
                elif kind == "first":
                    d, x, neg = f
                    assert not _overlaps(wv.reads, x, 2), "add reads an X slot whose LDS read may not have returned"
                    xv = -wv.v[x:x + 2] if neg else wv.v[x:x + 2]
                    wv.v[d:d + 2] = xv + np.float32(0.0)
                elif kind == "flush":
                    d, t = f
                    wv.v[d:d + 2] = wv.v[d:d + 2] + wv.v[t:t + 2]
                    wv.v[t:t + 2] = np.nan  # a block sum is consumed once
        assert at_barrier in (0, WAVES), "waves disagree on the barrier count"
        phase += 1
    acc = np.zeros((G.tile_m, G.tile_cols), np.float32)
    for wv in waves:
        for c in range(NW):
            for r in range(RPL):
                acc[r:G.tile_m:RPL, wv.w * NW + c] = wv.v[G.acc0 + RPL * c + r]
    return acc


def to_pairs(XT):
    """X^T [Kp][Mp] (Kp, Mp even) -> the k-pair layout [Kp/2][Mp/2][4]
    (tsg_internal.h; tsg_transpose_pairs_kernel)."""
    Kp, Mp = XT.shape
    q = XT.reshape(Kp // 2, 2, Mp // 2, 2)           # [p][k&1][mp][m&1]
    return np.ascontiguousarray(q.transpose(0, 2, 1, 3).reshape(Kp // 2, Mp // 2, 4))


def to_quads(XT):
    """X^T [Kp][Mp] (Kp % 4 == 0) -> quads [Kp/4][Mp][4]: entry [q][m] is the
    16 B X[m][4q .. 4q+3] (the unit the 64-row image's blocked layout moves;
    emulate_tile gathers its DMA pieces from it)."""
    Kp, Mp = XT.shape
    return np.ascontiguousarray(XT.reshape(Kp // 4, 4, Mp).transpose(0, 2, 1))


def emulate(code, wcode, X, K, N):
    assert tuple(int(x) for x in code[:2]) == MAGIC
    G = Geom(code)
    CHUNK, TILE_COLS, TM = G.chunk, G.tile_cols, G.tile_m
    M = X.shape[0]
    nch = max(1, -(-K // CHUNK))
    Mp = -(-max(M, 1) // TM) * TM
    XT = np.zeros((nch * CHUNK, Mp), np.float32)
    XT[:K, :M] = X.T
    if G.rowlay:  # per chunk: the quads from its first K row (the last chunk: K - 188 when K >= 188, K % 4 == 0)
        XT0 = np.zeros((nch * CHUNK + CHUNK, Mp), np.float32)
        XT0[:K, :M] = X.T
        XP = []
        for j in range(nch):
            kb = K - CHUNK if (j == nch - 1 and K >= CHUNK and K % 4 == 0) else j * CHUNK
            XP.append(to_quads(XT0[kb:kb + CHUNK]).transpose(1, 0, 2).copy())  # [Mp][47][4]
    else:
        XP = to_quads(XT) if G.r64 else to_pairs(XT)
    ntiles = len(wcode) // G.streams
    Y = np.zeros((Mp, ntiles * TILE_COLS), np.float32)
    for t in range(ntiles):
        for m0 in range(0, Mp, TM):
            Y[m0:m0 + TM, t * TILE_COLS:(t + 1) * TILE_COLS] = emulate_tile(code, wcode, t, XP, m0, Mp, nch)
    return Y[:M, :N]


def _check(tsg, O, M, K, N, s, seed, frac, W=None, width=64, waves=8, rows64=False, half=False):
    W = O.gen_ternary(K, N, s, seed) if W is None else W
    t = O.tcsc_encode(W)
    if rows64:
        code, wcode = tsg.jit_codegen64(*t.arrays, K, N, width=width, waves=waves, half=half)
        assert Geom(code).half == half
        assert Geom(code).r64 and Geom(code).tile_m == 64
    else:
        code, wcode = tsg.jit_codegen(*t.arrays, K, N, width=width, waves=waves)
    assert Geom(code).nw == width and Geom(code).waves == waves
    X = O.init_x_frac(M, K, seed + 1) if frac else O.init_x_int(M, K, seed + 1)
    b = np.linspace(-2, 3, N).astype(np.float32)
    Y = emulate(code, wcode, X, K, N) + b
    ref = O.base_tcsc(X, t, b)
    assert np.array_equal(Y.view(np.uint32), ref.view(np.uint32)), (M, K, N, s, frac)
    # one v_pk_add_f32 (64-row image: one v_add_f32 / v_sub_f32) per nonzero, nothing else that adds
    if rows64:  # decode the region linearly from the first stream (literals are skipped by the decoder)
        G = Geom(code)
        pc, n_add, n_sub = int(min(wcode)) // 4, 0, 0
        while pc < len(code):
            kind, f, n = _decode(code, pc, G)
            if kind == "vadd":
                n_add += 1
                n_sub += f[2]
            pc += n
        assert n_sub == len(t.arrays[3]), "one v_sub_f32 per -1 entry (comp.h:57)"
    else:
        n_add = sum(1 for i in range(len(code) - 1) if (int(code[i]) & 0xFFFFFD00) == 0xD3B24000
                    and (int(code[i + 1]) >> 27) & 3 == 3)
    assert n_add == len(t.arrays[2]) + len(t.arrays[3])


@pytest.mark.parametrize("M,K,N,s", [(1, 1, 1, 1), (5, 70, 33, 2), (130, 200, 520, 4), (17, 300, 64, 8),
                                     (3, 97, 9, 16)])
def test_jit_code_emulates_base_tcsc(tsg, oracle_mod, M, K, N, s):
    for frac in (False, True):
        _check(tsg, oracle_mod, M, K, N, s, 11 + K + N, frac)


@pytest.mark.parametrize("width", [32, 16, 8])
@pytest.mark.parametrize("M,K,N,s", [(5, 70, 33, 2), (130, 200, 150, 4), (3, 97, 9, 16)])
def test_jit_code_narrow_streams(tsg, oracle_mod, M, K, N, s, width):
    """Narrow streams (small-M widths, tsg_capi.cpp pick_jit_width): same
    register contract, fewer accumulators, more column tiles; same order."""
    for frac in (False, True):
        _check(tsg, oracle_mod, M, K, N, s, 5 + K + N + width, frac, width=width)


@pytest.mark.parametrize("width", [32, 16, 8])
@pytest.mark.parametrize("M,K,N,s", [(5, 70, 33, 2), (130, 300, 150, 4), (3, 97, 9, 16)])
def test_jit_code_four_wave_workgroups(tsg, oracle_mod, M, K, N, s, width):
    """4-wave workgroups (mid-M shapes, lib/tsg_jit_w<nw>_4w.co): each wave
    stages 12 of the chunk's 48 pair rows, the register contract shifts
    (lane*128 v120, accumulators from v122), twice the column tiles; same order."""
    for frac in (False, True):
        _check(tsg, oracle_mod, M, K, N, s, 7 + K + N + width, frac, width=width, waves=4)


@pytest.mark.parametrize("M,K,N,s", [(5, 70, 33, 2), (130, 300, 520, 4), (3, 97, 9, 16)])
def test_jit_code_far_image(tsg, oracle_mod, M, K, N, s):
    """The far-X^T image (tcsc_hip_set_far): the default 64-wide code with the
    code touches removed and every X^T DMA piece non-temporal (nt bit), header
    word 7 bit 17 -- nothing else differs, so the same order."""
    O = oracle_mod
    W = O.gen_ternary(K, N, s, 3 + K)
    t = O.tcsc_encode(W)
    code, wcode = tsg.jit_codegen_far(*t.arrays, K, N)
    base, _ = tsg.jit_codegen(*t.arrays, K, N)
    assert int(code[7]) & (1 << 17) and not int(base[7]) & (1 << 17)
    words = [int(w) for w in code]
    n_dma = sum(1 for w in words if (w & ~0x2030000 & 0xFFFFF000) == 0xDDF48000)
    assert n_dma > 0 and n_dma == sum(1 for w in words if (w & 0xFFFFF000) == 0xDDF48000 | 0x20000)
    assert not any((w & ~0x2030000) == 0xDC508000 for w in words)  # no code touch
    for frac in (False, True):
        X = O.init_x_frac(M, K, 9) if frac else O.init_x_int(M, K, 9)
        b = np.linspace(-2, 3, N).astype(np.float32)
        Y = emulate(code, wcode, X, K, N) + b
        ref = O.base_tcsc(X, t, b)
        assert np.array_equal(Y.view(np.uint32), ref.view(np.uint32)), (M, K, N, s, frac)


@pytest.mark.parametrize("M,K,N,s", [(1, 1, 1, 1), (5, 70, 33, 2), (64, 200, 130, 4), (17, 300, 64, 8),
                                     (3, 97, 9, 16), (100, 390, 40, 4)])
@pytest.mark.parametrize("width,waves", [(128, 8), (64, 8), (16, 4), (8, 8)])
def test_jit_code_64row_image(tsg, oracle_mod, M, K, N, s, width, waves):
    """The 64-row image (one M row per lane, VOP2 v_add_f32 / v_sub_f32, k-quad
    X^T, 192-row chunks; tsg_internal.h): emulated workgroup by workgroup,
    every M tile of 64 rows, equal to the BaseTCSC oracle bit for bit on
    integer and order-sensitive X, one add per nonzero."""
    for frac in (False, True):
        _check(tsg, oracle_mod, M, K, N, s, 5 + K + N + width, frac, width=width, waves=waves, rows64=True)


@pytest.mark.parametrize("layout", ["rows", "16", "8"])
@pytest.mark.parametrize("M,K,N,s", [(64, 188, 70, 4), (70, 376, 40, 2), (5, 189, 30, 4), (33, 1000, 24, 8),
                                     (64, 192, 64, 4), (9, 4096, 16, 8)])
def test_jit_code_64row_layouts(tsg, oracle_mod, monkeypatch, layout, M, K, N, s):
    """The 64-row image's LDS layouts: the row layout (default, round 5: rows
    of 47 quads, 188-row chunks, the last chunk starting at K - 188 when K >=
    188 and K % 4 == 0) and the blocked layouts (TSG_JIT_QBLOCK=16 / 8, 192-row
    chunks) -- K on and around the chunk boundaries, every element bit-exact."""
    if layout != "rows":
        monkeypatch.setenv("TSG_JIT_QBLOCK", layout)
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(K, N, s, K + N))
    code, _ = tsg.jit_codegen64(*t.arrays, K, N, width=16, waves=4)
    G = Geom(code)
    assert G.rowlay == (layout == "rows") and G.chunk == (188 if layout == "rows" else 192)
    assert G.pr_rows == (0 if layout == "rows" else 16 if layout == "16" else 8) or layout == "rows"
    # the last-chunk adjustment (s87) is emitted exactly when the last chunk starts at K - 188
    nch = -(-K // G.chunk)
    shifted = layout == "rows" and K >= 188 and K % 4 == 0 and K % 188 != 0
    assert (any(int(w) == 0x80D45754 for w in code)) == shifted
    for frac in (False, True):
        _check(tsg, O, M, K, N, s, 3 + K, frac, width=16, waves=4, rows64=True)


@pytest.mark.parametrize("width,waves", [(32, 4), (16, 8), (8, 4)])
def test_jit_code_64row_other_shapes(tsg, oracle_mod, width, waves):
    _check(tsg, oracle_mod, 70, 500, 300, 4, 99, True, width=width, waves=waves, rows64=True)


@pytest.mark.parametrize("M,K,N,s", [(1, 1, 1, 1), (5, 70, 33, 2), (64, 200, 130, 4), (17, 300, 64, 8),
                                     (3, 97, 9, 16), (100, 390, 40, 4), (70, 96, 50, 4), (70, 97, 50, 4)])
@pytest.mark.parametrize("width", [32, 16, 8])
def test_jit_code_64row_half_ring(tsg, oracle_mod, M, K, N, s, width):
    """The half ring (96-row chunks of 24 pieces, 4 waves with the 8-wave
    register contract; tsg_internal.h kJit64HalfChunk): emulated, bit for bit
    against the oracle, K on and across chunk boundaries."""
    for frac in (False, True):
        _check(tsg, oracle_mod, M, K, N, s, 7 + K + N + width, frac, width=width, waves=4, rows64=True, half=True)
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(K, N, s, 1))
    with pytest.raises(tsg.TSGError):
        tsg.jit_codegen64(*t.arrays, K, N, width=64, waves=4, half=True)


def test_jit_code_64row_dense_and_empty_columns(tsg, oracle_mod):
    """Every quad read form (b32 at each row, b64 low / high, b128): dense,
    empty, single-row and two-row columns in one W."""
    O = oracle_mod
    K, N = 400, 72  # width 8: stream c // 8 holds columns c..c+7, so each pattern has its own stream
    W = np.zeros((K, N), np.int32)
    W[:, 0] = 1                         # stream 0: dense +1 and -1 columns (b128)
    W[:, 1] = -1
    W[::4, 8] = 1                       # stream 1: row 0 of every quad (b32 at +0)
    W[1::4, 16] = -1                    # b32 at +4
    W[2::4, 24] = 1                     # b32 at +8
    W[3::4, 32] = -1                    # b32 at +12
    W[0::4, 40] = 1                     # rows 0, 1 in one pass (b64 at +0)
    W[1::4, 41] = 1
    W[2::4, 48] = -1                    # rows 2, 3 (b64 at +8)
    W[3::4, 49] = -1
    W[1::4, 56] = 1                     # rows 1, 2 (b128)
    W[2::4, 57] = 1
    W[0::4, 58] = -1                    # and rows 0, 3 of the -1 pass (b128)
    W[3::4, 59] = -1
    W[K - 1, 64] = 1                    # stream 8: one entry at the last row, one at the first
    W[0, 65] = -1
    code, _ = tsg.jit_codegen64(*O.tcsc_encode(W).arrays, K, N, width=8, waves=8)
    ops = {int(w) & 0xFFFF0000 for w in code}
    for op in (0xD86C0000, 0xD8EC0000, 0xD9FE0000):  # ds_read_b32 / b64 / b128 all emitted
        assert op in ops
    for frac in (False, True):
        _check(tsg, O, 64, K, N, 1, 3, frac, W=W, width=8, waves=8, rows64=True)
        _check(tsg, O, 37, K, N, 1, 4, frac, W=W, width=8, waves=8, rows64=True)


def test_jit_width_rejected(tsg, oracle_mod):
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(64, 20, 4, 1))
    with pytest.raises(tsg.TSGError, match="width"):
        tsg.jit_codegen(*t.arrays, 64, 20, width=24)
    with pytest.raises(tsg.TSGError, match="width"):  # 128 columns per wave: the 64-row image only
        tsg.jit_codegen(*t.arrays, 64, 20, width=128)
    with pytest.raises(tsg.TSGError, match="shape"):  # ... with 8 waves
        tsg.jit_codegen64(*t.arrays, 64, 20, width=128, waves=4)
    blk = O.blocked_tcsc_encode(O.gen_ternary(64, 20, 4, 1), 16)
    with pytest.raises(tsg.TSGError, match="BlockedTCSC"):
        tsg.jit_codegen(*blk, 64, 20, B=16, width=16)
    with pytest.raises(tsg.TSGError, match="waves"):
        tsg.jit_codegen(*t.arrays, 64, 20, width=64, waves=4)  # 64-wide streams: 8 waves only
    with pytest.raises(tsg.TSGError, match="waves"):
        tsg.jit_codegen(*t.arrays, 64, 20, width=16, waves=2)


def test_jit_code_dense_and_empty_columns(tsg, oracle_mod):
    """All-+1 / all--1 / alternating / empty columns: every row of a chunk used,
    more rows than one X block holds, and streams with no entries at all."""
    O = oracle_mod
    K, N, M = 250, 40, 9
    W = np.zeros((K, N), np.int32)
    W[:, 0] = 1
    W[:, 1] = -1
    W[::2, 2] = 1
    W[1::2, 2] = -1
    W[:, 5:] = O.gen_ternary(K, N - 5, 2, 3)
    _check(tsg, O, M, K, N, 0, 4, True, W=W)


def _count_entry_adds(code, G):
    """v_pk_add_f32 that apply one nonzero (add / first); flushes excluded."""
    n, i = 0, 0
    while i < len(code) - 1:  # instruction by instruction (8-byte forms aligned or not)
        w0 = int(code[i])
        if (w0 & 0xFFFFFC00) == 0xD3B24000 and (int(code[i + 1]) >> 27) & 3 == 3:
            n += _classify_pk(w0, int(code[i + 1]), G)[0] in ("add", "first")
            i += 2
        elif w0 in (0x807CFF53, 0x8058FF5A) or (w0 >> 26) in (0x36, 0x37) or (w0 >> 24) == 0xDD or (w0 >> 24) == 0xDC:
            i += 2  # literal SALU, DS, global / LDS-DMA: 8 bytes
        else:
            i += 1
    return n


def _check_blocked(tsg, O, M, K, N, s, B, seed, frac, W=None):
    W = O.gen_ternary(K, N, s, seed) if W is None else W
    blk = O.blocked_tcsc_encode(W, B)
    code, wcode = tsg.jit_codegen(*blk, K, N, B=B)
    G = Geom(code)
    assert G.B == B
    X = O.init_x_frac(M, K, seed + 1) if frac else O.init_x_int(M, K, seed + 1)
    b = np.linspace(-2, 3, N).astype(np.float32)
    Y = emulate(code, wcode, X, K, N) + b
    ref = O.base_blocked_tcsc(X, blk, b, K, N, B)
    assert np.array_equal(Y.view(np.uint32), ref.view(np.uint32)), (M, K, N, s, B, frac)
    assert _count_entry_adds(code, G) == len(blk[2]) + len(blk[3])


@pytest.mark.parametrize("M,K,N,s,B", [(5, 70, 33, 2, 16), (130, 200, 520, 4, 64), (17, 300, 64, 8, 100),
                                       (3, 1100, 9, 4, 512), (9, 96, 70, 2, 1), (4, 10, 5, 2, 32)])
def test_jit_code_emulates_base_blocked_tcsc(tsg, oracle_mod, M, K, N, s, B):
    """BaseBlockedTCSC (comp.h:607-658): y per block = 0 + pos - neg, Y += y
    block by block, + b; blocks straddling chunks, K not a multiple of B (the
    tail rows are not in the format), B = 1, K < B (no blocks: Y = b)."""
    for frac in (False, True):
        _check_blocked(tsg, oracle_mod, M, K, N, s, B, 7 + K + B, frac)


def test_jit_code_blocked_kat(tsg, oracle_mod):
    """The 4x4, B = 2 example of plots/data_example_image/blocked.py:12-30."""
    import json
    kat = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_blocked_4x4_B2.json")))
    W = np.array(kat["W"], np.int32)
    _check_blocked(tsg, oracle_mod, 4, 4, 4, 0, 2, 1, True, W=W)


def test_jit_code_base_unchanged_by_block_support(tsg, oracle_mod):
    """B = 0 through the blocked entry point is the BaseTCSC code, word for word."""
    O = oracle_mod
    W = O.gen_ternary(200, 130, 4, 5)
    t = O.tcsc_encode(W)
    c0, w0 = tsg.jit_codegen(*t.arrays, 200, 130)
    c1, w1 = tsg.jit_codegen(*t.arrays, 200, 130, B=0)
    assert np.array_equal(c0, c1) and np.array_equal(w0, w1)
    assert int(c0[5]) == 0


def test_blocked_validation_rejects_malformed(tsg, oracle_mod):
    O = oracle_mod
    W = O.gen_ternary(64, 6, 2, 9)
    csp, csn, rip, rin = O.blocked_tcsc_encode(W, 16)
    tsg.validate_blocked(csp, csn, rip, rin, 64, 6, 16)
    bad = rip.copy()
    j = int(csp[6])  # first +1 row of block 1 (slot N) moved into block 0
    if j < int(csp[7]):
        bad[j] = 3
        with pytest.raises(tsg.TSGError, match="out of its block"):
            tsg.validate_blocked(csp, csn, bad, rin, 64, 6, 16)
    with pytest.raises(tsg.TSGError):
        tsg.validate_blocked(csp, csn, rip, rin, 64, 6, 0)


# ---------------------------------------------------------------------------
# Float mode of the shipped dispatchers (no GPU): the generated adds run under
# the dispatcher's kernel descriptor, which must keep FP32 denormals and IEEE
# mode for the special-value contract of DESIGN.md section 3
# (tests/test_gpu_special.py checks the results on the GPU).

_REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rsrc1_of(co_path, symbol="tsg_jit_kernel.kd"):
    data = open(co_path, "rb").read()
    # ELF64: section headers -> .symtab / .strtab -> the .kd symbol's file offset
    (e_shoff,) = struct.unpack_from("<Q", data, 0x28)
    e_shentsize, e_shnum = struct.unpack_from("<HH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, e_shoff + i * e_shentsize) for i in range(e_shnum)]
    for sh in secs:
        if sh[1] == 2:  # SHT_SYMTAB
            strtab = secs[sh[6]]
            for j in range(sh[5] // 24):
                st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
                    "<IBBHQQ", data, sh[4] + j * 24)
                end = data.index(b"\0", strtab[4] + st_name)
                if data[strtab[4] + st_name:end].decode() == symbol:
                    tgt = secs[st_shndx]
                    off = tgt[4] + (st_value - tgt[3])
                    (rsrc1,) = struct.unpack_from("<I", data, off + 0x30)
                    return rsrc1
    raise AssertionError(f"{symbol} not found in {co_path}")


@pytest.mark.parametrize("co", ["tsg_jit.co", "tsg_jit_w32.co", "tsg_jit_w16.co", "tsg_jit_w8.co",
                                "tsg_jit64_w128.co", "tsg_jit64_w64.co", "tsg_jit64_w16_4w.co"])
def test_kernel_descriptor_float_mode(co):
    sym = "tsg_jit64_kernel.kd" if co.startswith("tsg_jit64") else "tsg_jit_kernel.kd"
    rsrc1 = _rsrc1_of(os.path.join(_REPO_ROOT, "ternary-spgemm_amd", "lib", co), sym)
    assert (rsrc1 >> 16) & 3 == 3, "FP32 denormals must be preserved (FLOAT_DENORM_MODE_32)"
    assert (rsrc1 >> 23) & 1 == 1, "IEEE mode must be on"



@pytest.mark.parametrize("gn,gm", [(2, 16), (4, 8), (1, 1), (3, 5), (8, 4)])
def test_tile_map_is_a_bijection(tsg, gn, gm):
    """Every workgroup of an mtiles x ntiles grid gets a distinct tile, every
    tile gets one (tsg_jit_map.h, the dispatcher's map), for the group sizes
    the library picks (2 x 16, 4 x 8) and odd ones, over grids that are and
    are not multiples of the 8 XCDs and of the groups."""
    for mtiles, ntiles in [(1, 1), (1, 7), (4, 64), (8, 32), (32, 32), (125, 4), (500, 8), (3, 3), (33, 9),
                           (2, 129), (17, 1)]:
        seen = set()
        for L in range(mtiles * ntiles):
            nt, mt = tsg.jit_tile_map(L, mtiles, ntiles, gn, gm)
            assert 0 <= nt < ntiles and 0 <= mt < mtiles
            seen.add((nt, mt))
        assert len(seen) == mtiles * ntiles, (mtiles, ntiles, gn, gm)


@pytest.mark.parametrize("knobs", [{"TSG_JIT_STAGGER": "1"}, {"TSG_JIT_PRIO": "1"},
                                   {"TSG_JIT_STAGGER": "1", "TSG_JIT_PRIO": "1"}])
@pytest.mark.parametrize("M,K,N,s,width,rows64", [(130, 400, 520, 4, 64, False), (70, 500, 1100, 4, 128, True),
                                                  (64, 1000, 300, 16, 16, True), (5, 97, 40, 2, 8, True),
                                                  (200, 188, 600, 8, 32, True), (1, 1, 1, 1, 64, True)])
def test_jit_code_stagger_and_priority(tsg, oracle_mod, monkeypatch, knobs, M, K, N, s, width, rows64):
    """The stagger (TSG_JIT_STAGGER=1: waves 0-3 run half a step ahead of
    waves 4-7, their barrier mid-step, their DMA pieces after it) and the
    static priority (TSG_JIT_PRIO=1: s_setprio 1 for waves 4-7): the emulated
    workgroup checks every LDS read against landed pieces (no read-after-DMA
    race) and every DMA against reads since its issue (no write-after-read
    race), with the barrier counts equal across waves -- and the result equals
    the oracle bit for bit."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    for frac in (False, True):
        _check(tsg, oracle_mod, M, K, N, s, 11 + K, frac, width=width, waves=8, rows64=rows64)


@pytest.mark.parametrize("mix", ["1,0", "0,1", "1,1", "troll=1", "troll=3", "1,1+troll=2", "tgroup=1", "tgroup=2",
                                 "1,0+tgroup=2", "tgroup=2+tgap=4096", "tgroup=1+tgap=1024"])
@pytest.mark.parametrize("M,K,N,s,width,waves,rows64", [(130, 400, 520, 4, 64, 8, False), (70, 500, 1100, 4, 128, 8, True),
                                                        (64, 1000, 300, 16, 16, 8, True), (5, 97, 40, 2, 8, 4, True),
                                                        (200, 188, 600, 8, 32, 8, True), (64, 900, 700, 4, 16, 4, True),
                                                        (1, 1, 1, 1, 64, 8, True)])
def test_jit_code_mixed_issue(tsg, oracle_mod, monkeypatch, mix, M, K, N, s, width, waves, rows64):
    """TSG_JIT_MIX (round 6, A/B): a read group's read-ahead and its share of
    the DMA pieces spread among the group's adds instead of a burst before
    them; TSG_JIT_TROLL: rolling code touches (each step touches the next
    untouched 8-KiB windows, the step's closing vmcnt lets exactly those run
    on).  The emulated workgroup checks every X slot reload against its wait,
    every LDS read against landed pieces and every DMA against reads since its
    issue -- and the result equals the oracle bit for bit."""
    for part in mix.split("+"):
        if part.startswith("troll="):
            monkeypatch.setenv("TSG_JIT_TROLL", part[6:])  # rolling code touches (round 6, A/B)
        elif part.startswith("tgroup="):
            monkeypatch.setenv("TSG_JIT_TGROUP", part[7:])  # per-group code touches (round 6, A/B)
        elif part.startswith("tgap="):
            monkeypatch.setenv("TSG_JIT_TGAP", part[5:])
        else:
            monkeypatch.setenv("TSG_JIT_MIX", part)
    for frac in (False, True):
        _check(tsg, oracle_mod, M, K, N, s, 13 + K, frac, width=width, waves=waves, rows64=rows64)


def test_jit_code_mixed_issue_blocked(tsg, oracle_mod, monkeypatch):
    """TSG_JIT_MIX with BlockedTCSC (per-block sums in the generated code)."""
    monkeypatch.setenv("TSG_JIT_MIX", "1,1")
    for frac in (False, True):
        _check_blocked(tsg, oracle_mod, 130, 512, 300, 4, 128, 7, frac)
