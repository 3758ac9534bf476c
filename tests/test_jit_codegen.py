"""The weight-compiled kernel's machine code, checked on the CPU before any GPU
runs it: tsg_jit_codegen's region is decoded instruction by instruction (only
the handful of gfx950 encodings the generator may emit are accepted) and
emulated against the register contract of ternary-spgemm_amd/csrc/tsg_jit_kernel.hip;
the emulated Y must equal the BaseTCSC oracle (comp.h:25-69) bit for bit, for
integer and for order-sensitive non-integer X.  This is the test that says the
generated code computes BaseTCSC in BaseTCSC's order; tests/test_gpu_parity.py
then says the GPU runs that code."""
import numpy as np
import pytest

TILE_M, WAVES, NW, TILE_COLS, CHUNK = 256, 8, 32, 256, 64
MAGIC = (0x7453474A, 0x314A4954)


def _decode(w0, w1=None):
    """-> (kind, fields, n_words) for one instruction at w0[, w1]."""
    if w0 == 0xBF800000:
        return "nop", (), 1
    if w0 == 0xBF8CC07F:
        return "wait", (), 1
    if w0 == 0xBEDC1C00 and w1 == 0xBE801D5E:
        return "ret", (), 2
    if (w0 & 0xFFFFFD00) == 0xD3B24000:  # v_pk_add_f32
        d = w0 & 0xFF
        neg = bool(w0 & 0x200)
        src0 = (w1 & 0x1FF) - 256
        src1 = ((w1 >> 9) & 0x1FF) - 256
        assert (w1 >> 18) & 0x1FF == 0, "src2 field must be empty"
        assert (w1 >> 27) & 3 == 3, "op_sel_hi must be [1,1]"
        assert (w1 >> 29) == (2 if neg else 0), "neg_lo must match neg_hi"
        assert src0 == d, "v_pk_add_f32 must accumulate in place"
        return "add", (d, src1, neg), 2
    if (w0 & 0xFFFF0000) == 0xD9FE0000:  # ds_read_b128
        off = w0 & 0xFFFF
        a, vd = w1 & 0xFF, w1 >> 24
        assert (w1 >> 8) & 0xFFFF == 0
        return "read", (vd, a, off), 2
    raise AssertionError(f"unexpected instruction word {w0:#010x}")


def emulate(code, wcode, XT, M, K, N, nch):
    """Runs every (tile, wave) stream on the data a workgroup would see."""
    assert tuple(code[:2]) == MAGIC
    Mp = XT.shape[1]
    ntiles = len(wcode) // WAVES
    acc_out = np.zeros((Mp, ntiles * TILE_COLS), np.float32)
    for t in range(ntiles):
        for w in range(WAVES):
            for mt in range(Mp // TILE_M):
                m0 = mt * TILE_M
                v = np.zeros((256, 64), np.float32)  # VGPR file, one column per lane
                pc = int(wcode[t * WAVES + w]) // 4
                assert int(wcode[t * WAVES + w]) % 256 == 0
                for q in range(2 * nch):
                    j = q % nch
                    chunk = XT[j * CHUNK:(j + 1) * CHUNK, m0:m0 + TILE_M]  # [row][m]
                    while True:
                        kind, f, nw = _decode(int(code[pc]), int(code[pc + 1]) if pc + 1 < len(code) else None)
                        pc += nw
                        if kind == "ret":
                            break
                        if kind == "read":
                            vd, a, off = f
                            assert a == (105 if q & 1 else 104), "read from the wrong LDS buffer"
                            assert off % 1024 == 0 and off // 1024 < CHUNK
                            assert 8 <= vd and vd + 3 <= 103 and (vd - 8) % 4 == 0
                            row = chunk[off // 1024]  # 256 M values; lane l gets 4l..4l+3
                            v[vd:vd + 4] = row.reshape(64, 4).T
                        elif kind == "add":
                            d, x, neg = f
                            assert 112 <= d <= 238 and 8 <= x <= 102
                            if neg:
                                v[d:d + 2] = v[d:d + 2] - v[x:x + 2]
                            else:
                                v[d:d + 2] = v[d:d + 2] + v[x:x + 2]
                    # the dispatcher resumes 4 bytes past the s_setpc
                    pc = pc  # (pc already points past the 2-word return pair)
                n0 = t * TILE_COLS + w * NW
                for c in range(NW):
                    for i in range(4):
                        acc_out[m0 + i:m0 + TILE_M:4, n0 + c] = v[112 + 4 * c + i]
    return acc_out[:M, :N]


def _check(tsg, O, M, K, N, s, seed, frac):
    W = O.gen_ternary(K, N, s, seed)
    t = O.tcsc_encode(W)
    code, wcode = tsg.jit_codegen(*t.arrays, K, N)
    nch = max(1, -(-K // CHUNK))
    Mp = -(-max(M, 1) // TILE_M) * TILE_M
    X = O.init_x_frac(M, K, seed + 1) if frac else O.init_x_int(M, K, seed + 1)
    XT = np.zeros((nch * CHUNK, Mp), np.float32)
    XT[:K, :M] = X.T
    b = np.linspace(-2, 3, N).astype(np.float32)
    Y = emulate(code, wcode, XT, M, K, N, nch) + b
    ref = O.base_tcsc(X, t, b)
    assert np.array_equal(Y.view(np.uint32), ref.view(np.uint32)), (M, K, N, s, frac)
    # one v_pk_add_f32 pair per nonzero, nothing else that adds
    n_add = sum(1 for i in range(len(code) - 1) if (int(code[i]) & 0xFFFFFD00) == 0xD3B24000)
    assert n_add == 2 * (len(t.arrays[2]) + len(t.arrays[3]))


@pytest.mark.parametrize("M,K,N,s", [(1, 1, 1, 1), (5, 70, 33, 2), (256, 130, 300, 4), (300, 64, 257, 8),
                                     (17, 200, 40, 16), (3, 0, 9, 4)])
def test_jit_code_emulates_base_tcsc(tsg, oracle_mod, M, K, N, s):
    for frac in (False, True):
        if K == 0:
            continue
        _check(tsg, oracle_mod, M, K, N, s, 11 + K + N, frac)


def test_jit_code_dense_and_empty_columns(tsg, oracle_mod):
    """All-+1 / all--1 / empty columns: 64 entries per chunk in one column, more
    rows than one X block holds, and streams with no entries at all."""
    O = oracle_mod
    K, N, M = 150, 40, 9
    W = np.zeros((K, N), np.int32)
    W[:, 0] = 1
    W[:, 1] = -1
    W[::2, 2] = 1
    W[1::2, 2] = -1
    W[:, 5:] = O.gen_ternary(K, N - 5, 2, 3)
    t = O.tcsc_encode(W)
    code, wcode = tsg.jit_codegen(*t.arrays, K, N)
    nch = -(-K // CHUNK)
    X = O.init_x_frac(M, K, 4)
    XT = np.zeros((nch * CHUNK, TILE_M), np.float32)
    XT[:K, :M] = X.T
    b = np.zeros(N, np.float32)
    Y = emulate(code, wcode, XT, M, K, N, nch) + b
    ref = O.base_tcsc(X, t, b)
    assert np.array_equal(Y.view(np.uint32), ref.view(np.uint32))
