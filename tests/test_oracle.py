"""Pins the CPU oracle (oracle/) against the reference's own outputs.

CPU only.  The golden vectors were produced by tests/golden/make_golden.py from
the reference's code compiled unmodified (TCSC.h ctor, generateSparseMatrix,
GEMM / GEMM_PreLU of sparseUtils.h) plus the hand-worked 4x4 KATs of
plots/data_example_image/{base_structure,blocked}.py.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _sha(*arrays) -> str:
    return hashlib.sha256(np.concatenate([np.ascontiguousarray(a) for a in arrays]).tobytes()).hexdigest()


def _load_small():
    return np.load(os.path.join(GOLDEN, "ref_small.npz"))


def _case_ids(z):
    return sorted({k.split("_")[0] for k in z.files})


def _dense_from_bits(z, p, K, N):
    pos = np.unpackbits(z[p + "Wpos_bits"])[: K * N].reshape(K, N).astype(np.int32)
    neg = np.unpackbits(z[p + "Wneg_bits"])[: K * N].reshape(K, N).astype(np.int32)
    assert not (pos & neg).any()
    return pos - neg


def test_kat_tcsc_4x4(oracle_mod):
    """TCSC.h:13-41 on plots/data_example_image/base_structure.py:19-30."""
    O = oracle_mod
    kat = json.load(open(os.path.join(GOLDEN, "kat_tcsc_4x4.json")))
    t = O.tcsc_encode(np.array(kat["W"], np.int32))
    assert t.col_start_pos.tolist() == kat["col_start_pos"]
    assert t.row_index_pos.tolist() == kat["row_index_pos"]
    assert t.col_start_neg.tolist() == kat["col_start_neg"]
    assert t.row_index_neg.tolist() == kat["row_index_neg"]
    assert np.array_equal(t.dense(), np.array(kat["W"]))
    X = np.array(kat["X"], np.float32)
    b = np.array(kat["b"], np.float32)
    Y = O.base_tcsc(X, t, b)
    assert np.array_equal(Y, np.array(kat["Y_base_tcsc_oracle"], np.float32))
    # the dense reference GEMM sums in a different order; non-integer X, so
    # compare within the reference's own tolerance (sparseUtils.h:147)
    assert np.max(np.abs(Y - np.array(kat["Y_ref_gemm"], np.float32))) < 1e-5


def test_kat_blocked_4x4(oracle_mod):
    """BlockedTCSC<2> (BlockedTCSC.h:15-41) on plots/data_example_image/blocked.py:19-30."""
    O = oracle_mod
    kat = json.load(open(os.path.join(GOLDEN, "kat_blocked_4x4_B2.json")))
    csp, csn, rip, rin = O.blocked_tcsc_encode(np.array(kat["W"], np.int32), kat["B"])
    assert csp.tolist() == kat["col_start_pos"] and rip.tolist() == kat["row_index_pos"]
    assert csn.tolist() == kat["col_start_neg"] and rin.tolist() == kat["row_index_neg"]
    X = np.array(kat["X"], np.float32)
    b = np.array(kat["b"], np.float32)
    Yb = O.base_blocked_tcsc(X, (csp, csn, rip, rin), b, 4, 4, kat["B"])
    assert np.max(np.abs(Yb - np.array(kat["Y_ref_gemm"], np.float32))) < 1e-5


def test_golden_small_cases(oracle_mod):
    """Oracle == reference TCSC ctor (arrays/hash) and == reference GEMM / GEMM_PreLU
    (integer X: every partial sum exact), bit for bit."""
    O = oracle_mod
    z = _load_small()
    for p in [c + "_" for c in _case_ids(z)]:
        M, K, N, s, seed = (int(v) for v in z[p + "shape"])
        W = _dense_from_bits(z, p, K, N)
        t = O.tcsc_encode(W)
        assert _sha(*t.arrays) == bytes(z[p + "sha256_tcsc"]).decode()
        if p + "csp" in z.files:
            for a, key in zip(t.arrays, ("csp", "csn", "rip", "rin")):
                assert np.array_equal(a, z[p + key]), (p, key)
        assert t.size_bytes() == int(z[p + "ds_bytes"][0])  # getDataStructureSize, TCSC.h:43-49
        X, b, alpha = z[p + "X"], z[p + "b"], z[p + "alpha"]
        assert np.array_equal(O.base_tcsc(X, t, b), z[p + "Y_ref_gemm"]), p
        assert np.array_equal(O.base_tcsc(X, t, b, threads=4), z[p + "Y_ref_gemm"]), p
        assert np.array_equal(O.double_unrolled_tcsc(X, t, b), z[p + "Y_ref_gemm"]), p
        assert np.array_equal(O.base_tcsc_prelu(X, t, b, alpha), z[p + "Y_ref_gemm_prelu"]), p
        Xf = z[p + "Xfrac"]
        assert np.array_equal(O.base_tcsc(Xf, t, b), z[p + "Yfrac_oracle"]), p
        assert np.array_equal(O.base_tcsc_prelu(Xf, t, b, alpha), z[p + "Yfrac_prelu_oracle"]), p


def test_reference_generator_distribution():
    """The reference generator's row law (sparseUtils.h:52-87) -- which the
    in-repo generator restates -- holds on the committed reference outputs."""
    z = _load_small()
    for p in [c + "_" for c in _case_ids(z)]:
        M, K, N, s, seed = (int(v) for v in z[p + "shape"])
        W = _dense_from_bits(z, p, K, N)
        per_row, half = N // s, (N // s) // 2
        pos, neg = (W == 1).sum(1), (W == -1).sum(1)
        v = pos - half
        assert (v >= 0).all() and (v <= per_row // 20 + 1).all()
        assert np.array_equal(neg, np.maximum(half - v, 0))


def test_oracle_generator_law(oracle_mod):
    O = oracle_mod
    for K, N, s in [(64, 4096, 4), (50, 300, 16), (10, 1000, 2)]:
        W = O.gen_ternary(K, N, s, 9)
        per_row, half = N // s, (N // s) // 2
        v = (W == 1).sum(1) - half
        assert (v >= 0).all() and (v <= per_row // 20 + 1).all()
        assert np.array_equal((W == -1).sum(1), half - v)
        assert set(np.unique(W)) <= {-1, 0, 1}


def test_order_matters_for_fractional_x(oracle_mod):
    """The non-integer X vectors really pin order: DoubleUnrolled (other order)
    differs from BaseTCSC on them, while both agree on integer X."""
    O = oracle_mod
    W = O.gen_ternary(512, 256, 4, 3)
    t = O.tcsc_encode(W)
    b = np.full(256, 2.0, np.float32)
    Xi, Xf = O.init_x_int(16, 512, 1), O.init_x_frac(16, 512, 2)
    assert np.array_equal(O.base_tcsc(Xi, t, b), O.double_unrolled_tcsc(Xi, t, b))
    assert (O.base_tcsc(Xf, t, b) != O.double_unrolled_tcsc(Xf, t, b)).mean() > 0.5


def test_roundtrip_and_edges(oracle_mod):
    """DataStructureInterface round trip (DataStructureInterface.hpp:10-13) +
    empty / all-zero / dense-column edge cases."""
    O = oracle_mod
    rng = np.random.default_rng(0)
    for K, N in [(1, 1), (5, 3), (128, 1), (1, 257), (300, 40)]:
        W = rng.integers(-1, 2, size=(K, N)).astype(np.int32)
        t = O.tcsc_encode(W)
        assert np.array_equal(t.dense(), W)
    t = O.tcsc_encode(np.zeros((7, 9), np.int32))
    assert t.col_start_pos.tolist() == [0] * 10 and len(t.row_index_pos) == 0
    Y = O.base_tcsc(np.ones((3, 7), np.float32), t, np.arange(9, dtype=np.float32))
    assert np.array_equal(Y, np.tile(np.arange(9, dtype=np.float32), (3, 1)))


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "libref.so")),
                    reason="oracle/_ref not built (needs /root/reference at build time)")
def test_against_reference_build_directly(oracle_mod):
    """Where oracle/_ref/libref.so exists, check the restatement against the
    reference code itself on fresh seeds (encoder + dense GEMM)."""
    O = oracle_mod
    for K, N, s, seed in [(96, 200, 4, 101), (257, 64, 2, 102)]:
        W = O.ref_generate_sparse(K, N, s, seed)
        csp, csn, rip, rin, ds = O.ref_tcsc_encode(W)
        t = O.tcsc_encode(W)
        for a, r in zip(t.arrays, (csp, csn, rip, rin)):
            assert np.array_equal(a, r)
        X = O.init_x_int(9, K, seed)
        b = np.full(N, 2.0, np.float32)
        assert np.array_equal(O.base_tcsc(X, t, b), O.ref_gemm(X, W, b))
    # BlockedTCSC<B> ctor, incl. K not a multiple of B (the tail rows are dropped)
    for K, N, B in [(1100, 70, 512), (200, 33, 64), (10, 5, 4), (6, 4, 2)]:
        W = O.ref_generate_sparse(K, N, 2, K + B)
        for a, r in zip(O.blocked_tcsc_encode(W, B), O.ref_blocked_tcsc_encode(W, B)):
            assert np.array_equal(a, r), (K, N, B)
