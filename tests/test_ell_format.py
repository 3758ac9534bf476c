"""The small-M kernel's sliced-ELL image (tsg_ell.hip), checked on the CPU
before any GPU runs it: tsg_ell_build's image is decoded and the kernel's walk
replayed in numpy -- per 16-column slice and step (one step with the +1 then
the -1 blocks when K fits one chunk, else one per (pass, K chunk)) each
column's uint16 entries (float indices of X^T rows of an M tile) in order,
y = y + x in the blocks below n8pos and y = y - x after, padding entries on
the zero row -- and Y must equal the BaseTCSC oracle (comp.h:25-69) bit for
bit, for integer and for order-sensitive non-integer X."""
import numpy as np
import pytest


def replay(ent, tab, C, nch, X, K, N, MT, xb=0, zr=1):
    M = X.shape[0]
    steps = 1 if nch == 1 else 2 * nch
    nslices = (N + 15) // 16
    tab = tab.reshape(nslices, steps, 2)
    y = np.zeros((M, nslices * 16), np.float32)
    for st in range(steps):
        j = 0 if steps == 1 else st % nch
        xs = np.zeros((C + zr, M), np.float32)  # X^T chunk + the zero row(s)
        rows = min(C, K - j * C)
        if rows > 0:
            xs[:rows] = X[:, j * C:j * C + rows].T
        for sl in range(nslices):
            off, w = (int(v) for v in tab[sl, st])
            n8, n8pos = w & 0xFFFF, w >> 16
            assert off >= 1 and n8pos <= n8
            if steps > 1:
                assert n8pos == (n8 if st < nch else 0)
            blk = ent[off * 128:(off + n8) * 128].reshape(n8, 16, 8)  # [i8][column][8 entries]
            for c in range(16):
                col = sl * 16 + c
                for i in range(n8):
                    for u in blk[i, c, :]:
                        u = int(u)
                        if xb and u >= xb:  # the second X^T copy (same rows)
                            u -= xb
                        assert u % MT == 0 and u // MT < C + zr
                        x = xs[u // MT]
                        y[:, col] = y[:, col] + x if i < n8pos else y[:, col] - x
    return y[:, :N]


@pytest.mark.parametrize("M,K,N,s,Cmax,MT", [(3, 70, 33, 2, 2048, 4), (5, 300, 40, 4, 256, 32),
                                             (2, 1100, 17, 8, 512, 16), (4, 9, 5, 1, 4, 4), (1, 1, 1, 1, 16380, 1),
                                             (1, 5000, 20, 4, 2044, 1), (2, 700, 40, 4, 1020, 32)])
def test_ell_replay_equals_base_tcsc(tsg, oracle_mod, M, K, N, s, Cmax, MT):
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(K, N, s, M + K + N))
    ent, tab, C, nch = tsg.ell_build(*t.arrays, K, N, Cmax, MT)
    assert C <= Cmax and C % 4 == 0 and nch == max(1, -(-K // C))
    b = np.linspace(-1, 2, N).astype(np.float32)
    for X in (O.init_x_int(M, K, 3), O.init_x_frac(M, K, 4)):
        Y = replay(ent, tab, C, nch, X, K, N, MT) + b
        assert np.array_equal(Y.view(np.uint32), O.base_tcsc(X, t, b).view(np.uint32))
    # block 0 is all padding (read past a list's end); every nonzero appears
    # once; everything else is the zero row, blocks of 8
    assert np.all(ent[:128] == C * MT)
    used = ent[128:int((tab[:, 0] + (tab[:, 1] & 0xFFFF)).max(initial=1)) * 128]  # (the array has tail padding)
    real = used[used != C * MT]
    assert len(real) == len(t.arrays[2]) + len(t.arrays[3])


def test_ell_rejects_bad_chunk(tsg, oracle_mod):
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(64, 20, 4, 1))
    with pytest.raises(tsg.TSGError):
        tsg.ell_build(*t.arrays, 64, 20, 6, 4)
    with pytest.raises(tsg.TSGError):
        tsg.ell_build(*t.arrays, 64, 20, 4096, 16)  # indices past 16 bits


def _window_loads(ent, tab, xb):
    """max over 8-bank windows of the distinct rows a ds_read_b64 lane group
    (8 columns x 4 lanes of 2 rows) reads, per entry position: the LDS cycles
    of that group (MI355X_MICROARCH.md LDS: bank = float index % 64)"""
    loads = []
    for off, w in tab:
        n8 = int(w) & 0xFFFF
        blk = ent[int(off) * 128:(int(off) + n8) * 128].reshape(n8, 16, 8).astype(np.int64)
        for i in range(n8):
            for h in range(8):
                for g0 in (0, 8):
                    addrs = set(int(a) for a in blk[i, g0:g0 + 8, h])
                    win = {}
                    for a in addrs:
                        win[a % 64 // 8] = win.get(a % 64 // 8, 0) + 1
                    loads.append(max(win.values()))
    return np.array(loads)


@pytest.mark.parametrize("M,K,N,s", [(8, 1024, 64, 4), (5, 3000, 48, 4), (3, 700, 33, 2)])
def test_ell_two_copies(tsg, oracle_mod, M, K, N, s):
    """Round 5: the 8-row tile's image with two X^T copies (TSG_ELL_COPIES=2):
    same results bit for bit, both copies and the zero rows inside the LDS,
    and the copy choice lowers the lane groups' bank-window loads."""
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(K, N, s, M + K + N))
    ent, tab, C, nch, xb = tsg.ell_build(*t.arrays, K, N, 5116, 8, copies=2, with_xb=True)
    assert xb % 64 == 32 and xb >= (C + 1) * 8 and xb + (C + 1) * 8 <= 40960 and C % 4 == 0
    b = np.linspace(-1, 2, N).astype(np.float32)
    for X in (O.init_x_int(M, K, 3), O.init_x_frac(M, K, 4)):
        Y = replay(ent, tab, C, nch, X, K, N, 8, xb) + b
        assert np.array_equal(Y.view(np.uint32), O.base_tcsc(X, t, b).view(np.uint32))
    e1, t1, C1, nch1 = tsg.ell_build(*t.arrays, K, N, C, 8)  # one copy, same chunks
    assert (C1, nch1) == (C, nch)
    two, one = _window_loads(ent, tab, xb), _window_loads(e1, t1, 0)
    assert len(two) == len(one) and two.sum() < one.sum() and two.max() <= one.max()
    assert ent.max() < xb + (C + 1) * 8
    with pytest.raises(tsg.TSGError):
        tsg.ell_build(*t.arrays, K, N, 5116, 8, copies=4)


@pytest.mark.parametrize("M,K,N,s", [(8, 1024, 64, 4), (5, 3000, 48, 4), (3, 700, 33, 2), (2, 5200, 40, 8)])
def test_ell_bank_window_schedule(tsg, oracle_mod, M, K, N, s):
    """Round 5: the 8-row tile's image with the bank-window schedule
    (TSG_ELL_SCHED=1): bit for bit the BaseTCSC chains (pads read one of the
    8 zero rows), every lane group's gather conflict-free (one distinct row
    per 8-bank window), every nonzero exactly once, and the chunk plus its
    zero rows inside the LDS."""
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(K, N, s, M + K + N))
    ent, tab, C, nch, xb = tsg.ell_build(*t.arrays, K, N, 5116, 8, copies=3, with_xb=True)
    zr = -xb
    assert zr == 8 and (C + zr) * 8 * 4 <= 160 * 1024 and C % 4 == 0
    b = np.linspace(-1, 2, N).astype(np.float32)
    for X in (O.init_x_int(M, K, 3), O.init_x_frac(M, K, 4)):
        Y = replay(ent, tab, C, nch, X, K, N, 8, 0, zr) + b
        assert np.array_equal(Y.view(np.uint32), O.base_tcsc(X, t, b).view(np.uint32))
    assert _window_loads(ent, tab, 0).max() == 1
    used = ent[128:int((tab[:, 0] + (tab[:, 1] & 0xFFFF)).max(initial=1)) * 128]
    assert np.count_nonzero(used < C * 8) == len(t.arrays[2]) + len(t.arrays[3])
