"""Generates the golden fixtures under tests/golden/ (run in the container that
has the reference mounted; the fixtures are committed, the reference is not).

Sources of truth:
  * the reference's own code, compiled unmodified from /root/reference into
    oracle/_ref/libref.so (oracle/Makefile `ref` target):
      generateSparseMatrix (cpp_impl/sparseUtils.h:25-90),
      class TCSC ctor (cpp_impl/data_structures/TCSC.h:13-41),
      BlockedTCSC<B> ctor (cpp_impl/data_structures/BlockedTCSC.h:15-41),
      GEMM / GEMM_PreLU (cpp_impl/sparseUtils.h:92-137)  -- the reference's
      correctness oracle (main.cpp:200-227);
  * the hand-worked 4x4 examples in plots/data_example_image/base_structure.py:12-30
    and blocked.py:12-30 (transcribed below as data);
  * for non-integer X (accumulation ORDER) the CPU restatement in oracle/ only,
    because comp.h (BaseTCSC) cannot be compiled here (it includes <arm_neon.h>).

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "ternary-spgemm_amd")]

import oracle as O  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def kat_files():
    # plots/data_example_image/base_structure.py:12-30 (data transcribed)
    X = [[0.1, -2.2, 0.5, 1.9], [0.4, 4.7, -3.0, -0.6], [2.5, 3.5, 5.2, -4.5], [-2.3, 7.4, 1.2, 1.8]]
    Wb = [[0, -1, 1, 0], [0, 1, 0, 1], [0, 0, -1, 0], [-1, -1, 0, 1]]
    kat = {
        "source": "plots/data_example_image/base_structure.py:12-30",
        "X": X, "W": Wb,
        "col_start_pos": [0, 0, 1, 2, 4], "row_index_pos": [1, 0, 1, 3],
        "col_start_neg": [0, 1, 3, 4, 4], "row_index_neg": [3, 0, 3, 2],
    }
    Xa = np.array(X, np.float32)
    b = np.full(4, 2.0, np.float32)
    kat["b"] = b.tolist()
    kat["Y_ref_gemm"] = O.ref_gemm(Xa, np.array(Wb), b).tolist()
    t = O.tcsc_encode(np.array(Wb, np.int32))
    kat["Y_base_tcsc_oracle"] = O.base_tcsc(Xa, t, b).tolist()
    with open(os.path.join(HERE, "kat_tcsc_4x4.json"), "w") as f:
        json.dump(kat, f, indent=1)

    # plots/data_example_image/blocked.py:12-30, BlockedTCSC<2>
    Wk = [[1, -1, 0, 0], [-1, 1, 0, 1], [1, 0, -1, 0], [-1, -1, 0, 1]]
    blk = {
        "source": "plots/data_example_image/blocked.py:12-30",
        "X": X, "W": Wk, "B": 2,
        "col_start_pos": [0, 1, 2, 2, 3, 4, 4, 4, 5], "row_index_pos": [0, 1, 1, 2, 3],
        "col_start_neg": [0, 1, 2, 2, 2, 3, 4, 5, 5], "row_index_neg": [1, 0, 3, 3, 2],
    }
    tk = O.tcsc_encode(np.array(Wk, np.int32))
    blk["Y_ref_gemm"] = O.ref_gemm(Xa, np.array(Wk), b).tolist()
    blk["Y_base_tcsc_oracle"] = O.base_tcsc(Xa, tk, b).tolist()
    blk["b"] = b.tolist()
    with open(os.path.join(HERE, "kat_blocked_4x4_B2.json"), "w") as f:
        json.dump(blk, f, indent=1)


# (M, K, N, s, seed): small shapes (odd sizes on purpose) + config 1 of BASELINE.json
SMALL_CASES = [
    (1, 64, 96, 2, 11),
    (7, 130, 37, 4, 12),
    (64, 256, 512, 8, 13),
    (33, 512, 300, 16, 14),
    (3, 200, 1, 1, 15),
    (32, 1024, 4096, 4, 42),
]


def small_cases():
    out = {}
    for i, (M, K, N, s, seed) in enumerate(SMALL_CASES):
        W = O.ref_generate_sparse(K, N, s, seed)           # the reference's generator
        csp, csn, rip, rin, ds_bytes = O.ref_tcsc_encode(W)  # the reference's TCSC
        X = O.init_x_int(M, K, 1000 + seed)                # integer X (initX range)
        Xf = O.init_x_frac(M, K, 2000 + seed)              # non-integer X
        b = np.full(N, 2.0, np.float32)                    # main.cpp:194
        alpha = np.full(N, 0.1, np.float32)                # main.cpp:195
        Y = O.ref_gemm(X, W, b)
        Yp = O.ref_gemm_prelu(X, W, b, alpha)
        Yf = O.base_tcsc(Xf, O.TCSC(csp, csn, rip, rin, K, N), b)  # restatement only
        Ypf = O.base_tcsc_prelu(Xf, O.TCSC(csp, csn, rip, rin, K, N), b, alpha)
        p = f"c{i}_"
        if len(rip) + len(rin) <= 20000:  # small: keep the reference's arrays verbatim
            out.update({p + "csp": csp, p + "csn": csn, p + "rip": rip, p + "rin": rin})
        out.update({
            p + "shape": np.array([M, K, N, s, seed], np.int64),
            p + "Wpos_bits": np.packbits((W == 1).ravel()),
            p + "Wneg_bits": np.packbits((W == -1).ravel()),
            p + "sha256_tcsc": np.frombuffer(sha(np.concatenate([csp, csn, rip, rin])).encode(), np.uint8),
            p + "ds_bytes": np.array([ds_bytes], np.int64),
            p + "X": X, p + "b": b, p + "alpha": alpha,
            p + "Y_ref_gemm": Y, p + "Y_ref_gemm_prelu": Yp,
            p + "Xfrac": Xf, p + "Yfrac_oracle": Yf, p + "Yfrac_prelu_oracle": Ypf,
        })
        print("case", i, (M, K, N, s, seed), "nnz", len(rip) + len(rin))
    np.savez_compressed(os.path.join(HERE, "ref_small.npz"), **out)


def hashed_configs():
    """Config 2 in full and config 3 on sampled rows: Y from the reference's
    dense GEMM (exact for integer X), inputs from the in-repo generators
    (tsg_gen_tcsc == oracle_gen_ternary stream; tsg_gen_x == oracle_init_x_int)."""
    res = {"note": "Y from reference GEMM (sparseUtils.h:92-108) compiled from /root/reference; "
                   "W = oracle.gen_ternary(K,N,s,seed_w); X = oracle.init_x_int(M,K,seed_x); b=2"}
    # config 2: M=512 K=4096 N=4096 s=4 (BASELINE.json configs[1])
    M, K, N, s, sw, sx = 512, 4096, 4096, 4, 42, 12345
    W = O.gen_ternary(K, N, s, sw)
    X = O.init_x_int(M, K, sx)
    b = np.full(N, 2.0, np.float32)
    Y = O.ref_gemm(X, W, b)
    t = O.tcsc_encode(W)
    Yo = O.base_tcsc(X, t, b)
    assert np.array_equal(Y, Yo), "restatement disagrees with the reference GEMM at config 2"
    res["config2"] = {"M": M, "K": K, "N": N, "s": s, "seed_w": sw, "seed_x": sx,
                      "nnz_pos": int(len(t.row_index_pos)), "nnz_neg": int(len(t.row_index_neg)),
                      "sha256_tcsc": sha(np.concatenate(t.arrays)), "sha256_Y": sha(Y),
                      "Y_0_0": float(Y[0, 0]), "Y_last": float(Y[-1, -1])}
    print("config2 done")
    # config 3: M=4096 K=4096 N=16384 s=4, sampled rows
    M, K, N, s, sw, sx = 4096, 4096, 16384, 4, 42, 12345
    W = O.gen_ternary(K, N, s, sw)
    X = O.init_x_int(M, K, sx)
    b = np.full(N, 2.0, np.float32)
    rows = np.array(sorted(set([0, 1, 2, 63, 64, 127, 128, 129, 1000, 2047, 2048, 4094, 4095] +
                               list(np.random.default_rng(7).integers(0, M, 19)))), np.int64)
    Ys = O.ref_gemm(np.ascontiguousarray(X[rows]), W, b)
    t = O.tcsc_encode(W)
    Yo = O.base_tcsc(np.ascontiguousarray(X[rows]), t, b)
    assert np.array_equal(Ys, Yo), "restatement disagrees with the reference GEMM at config 3"
    res["config3_rows"] = {"M": M, "K": K, "N": N, "s": s, "seed_w": sw, "seed_x": sx,
                           "rows": rows.tolist(),
                           "nnz_pos": int(len(t.row_index_pos)), "nnz_neg": int(len(t.row_index_neg)),
                           "sha256_tcsc": sha(np.concatenate(t.arrays)),
                           "sha256_Y_rows": sha(Ys)}
    print("config3 rows done")
    res.update(sweep_configs())
    with open(os.path.join(HERE, "ref_hashes.json"), "w") as f:
        json.dump(res, f, indent=1)


SWEEP_ROWS = [0, 1, 127, 128, 2047, 2048, 4094, 4095]


def sweep_configs():
    """BASELINE.json configs[3]: M=4096 K=4096 N=16384 at s in {2, 8, 16} (s=4 is
    config3_rows above), sampled rows.  Y from the reference's dense GEMM
    (sparseUtils.h:92-108), cross-checked against the restatement; the TCSC
    hash pins the generator, the CSC+packed hash pins tsg_tcsc_to_csc_packed."""
    out = {}
    M, K, N, sw, sx = 4096, 4096, 16384, 42, 12345
    rows = np.array(SWEEP_ROWS, np.int64)
    X = O.init_x_int(M, K, sx)
    b = np.full(N, 2.0, np.float32)
    for s in (2, 8, 16):
        W = O.gen_ternary(K, N, s, sw)
        Ys = O.ref_gemm(np.ascontiguousarray(X[rows]), W, b)
        t = O.tcsc_encode(W)
        Yo = O.base_tcsc(np.ascontiguousarray(X[rows]), t, b)
        assert np.array_equal(Ys, Yo), f"restatement disagrees with the reference GEMM at s={s}"
        cp, ri, pk = O.csc_packed_encode(W)
        out[f"config4_s{s}_rows"] = {"M": M, "K": K, "N": N, "s": s, "seed_w": sw, "seed_x": sx,
                                     "rows": rows.tolist(),
                                     "nnz_pos": int(len(t.row_index_pos)), "nnz_neg": int(len(t.row_index_neg)),
                                     "sha256_tcsc": sha(np.concatenate(t.arrays)),
                                     "sha256_csc_packed": sha(np.concatenate([cp.view(np.uint8), ri.view(np.uint8),
                                                                              pk])),
                                     "sha256_Y_rows": sha(Ys)}
        print(f"config4 s={s} rows done")
    return out


if __name__ == "__main__":
    O.build(ref=True)
    assert O.ref_available(), "oracle/_ref/libref.so missing: needs /root/reference"
    if "--sweep-only" not in sys.argv:
        kat_files()
        small_cases()
    if "--sweep-only" in sys.argv:  # add the configs[3] rows to the committed ref_hashes.json
        path = os.path.join(HERE, "ref_hashes.json")
        res = json.load(open(path))
        res.update(sweep_configs())
        with open(path, "w") as f:
            json.dump(res, f, indent=1)
    elif "--no-hash" not in sys.argv:
        hashed_configs()
