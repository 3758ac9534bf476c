"""Host-side logic of the product library (no GPU needed): the C-ABI .so loads
and exports every function include/ternary_spgemm.h declares, the TCSC
validation / slicing / generators agree with the oracle, and GPU entry points
fail loudly (no CPU fallback) when there is no device."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, gpu_available


def _declared_functions(headers=("ternary_spgemm.h", "ternary_spgemm_test.h")):
    names = []
    for hdr in headers:
        text = open(os.path.join(REPO, "include", hdr)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(t\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_header_symbols_exported(tsg):
    declared = _declared_functions()
    assert len(declared) >= 18
    assert sorted(tsg.EXPORTED_SYMBOLS) == declared
    L = ctypes.CDLL(tsg.LIB_PATH)
    for name in declared:
        assert hasattr(L, name), name


def test_library_is_gfx950_code(tsg):
    """The .so carries a gfx950 code object (hipcc --offload-arch=gfx950)."""
    blob = open(tsg.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_generator_matches_oracle(tsg, oracle_mod):
    O = oracle_mod
    for K, N, s, seed in [(64, 256, 4, 1), (100, 37, 2, 5), (33, 7, 16, 3), (512, 1024, 8, 77)]:
        t = O.tcsc_encode(O.gen_ternary(K, N, s, seed))
        g = tsg.gen_tcsc(K, N, s, seed)
        for a, b in zip(t.arrays, g):
            assert np.array_equal(a, b)
        n0, n1 = N // 3, N // 2 + 1
        sl = tsg.gen_tcsc(K, N, s, seed, n0, n1)
        ref = tsg.tcsc_slice(*t.arrays, N, n0, n1)
        for a, b in zip(sl, ref):
            assert np.array_equal(a, b)
        # slice == encoding of the dense column block
        tb = O.tcsc_encode(t.dense()[:, n0:n1])
        for a, b in zip(tb.arrays, ref):
            assert np.array_equal(a, b)
    X = tsg.gen_x(5, 7, 11)
    assert np.array_equal(X, O.init_x_int(5, 7, 11))


def test_slices_tile_the_matrix(tsg, oracle_mod):
    O = oracle_mod
    K, N = 200, 333
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 2))
    cuts = [0, 1, 100, 101, 333]
    parts = [tsg.tcsc_slice(*t.arrays, N, a, b) for a, b in zip(cuts, cuts[1:])]
    Wd = np.concatenate([O.TCSC(*p, K, b - a).dense() for p, (a, b) in zip(parts, zip(cuts, cuts[1:]))], 1)
    assert np.array_equal(Wd, t.dense())


@pytest.mark.parametrize("bad", ["oob", "unsorted", "both", "start", "monotone"])
def test_validate_rejects(tsg, bad):
    csp, csn = np.array([0, 2, 3]), np.array([0, 1, 1])
    rip, rin = np.array([0, 3, 1]), np.array([2])
    tsg.validate(csp, csn, rip, rin, 4, 2)
    if bad == "oob":
        rip = np.array([0, 4, 1])
    elif bad == "unsorted":
        rip = np.array([3, 0, 1])
    elif bad == "both":
        rin = np.array([3])
    elif bad == "start":
        csn = np.array([1, 1, 1])
    elif bad == "monotone":
        csp = np.array([0, 3, 2])
    with pytest.raises(tsg.TSGError) as e:
        tsg.validate(csp, csn, rip, rin, 4, 2)
    assert e.value.code == 1


def test_registry_mirrors_main_cpp(tsg):
    tsg.clear_registry()
    f = lambda X, B, Y, M, N, K: None  # noqa: E731
    tsg.add_function(f, "HipBaseTCSC")
    tsg.add_prelu_function(f, "HipBaseTCSC_PreLU")
    assert tsg.funcNames == ["HipBaseTCSC"] and tsg.userFuncs == [f]
    assert tsg.funcNames_prelu == ["HipBaseTCSC_PreLU"]
    tsg.clear_registry()


def test_metrics_formulas(tsg):
    # readme.md:84-85 / SURVEY 8(d): cfg1 flops 33,685,504; cfg3 bytes 402,849,800
    assert tsg.flops(32, 4096, 1024 * 4096 // 4) == 33_685_504
    assert tsg.algorithmic_bytes(4096, 16384, 4096, 4096 * 16384 // 4) == 402_849_800


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU error path")
def test_no_gpu_fails_loudly(tsg, oracle_mod):
    t = oracle_mod.tcsc_encode(np.eye(4, dtype=np.int32))
    with pytest.raises(tsg.TSGError) as e:
        tsg.TCSCDevice(*t.arrays, 4, 4)
    assert e.value.code == 4  # TSG_ERR_NODEV: never a silent CPU fallback


def test_csc_packed_conversions(tsg, oracle_mod):
    """CSC + base-3 packed values (readme.md:111) <-> TCSC, vs the oracle encoder."""
    O = oracle_mod
    for K, N, s in [(300, 77, 4), (64, 5, 1), (10, 10, 16), (129, 300, 2)]:
        W = O.gen_ternary(K, N, s, 3)
        t = O.tcsc_encode(W)
        ref = O.csc_packed_encode(W)
        got = tsg.tcsc_to_csc_packed(*t.arrays, N)
        for a, b in zip(got, ref):
            assert np.array_equal(a, b)
        back = tsg.csc_packed_to_tcsc(*ref, N)
        for a, b in zip(back, t.arrays):
            assert np.array_equal(a, b)
        X = O.init_x_frac(3, K, 1)
        b = np.ones(N, np.float32)
        assert np.array_equal(O.base_csc_packed(X, *ref, b, K, N).view(np.uint32),
                              O.base_tcsc(X, t, b).view(np.uint32))
    # a stored entry with value 0 (digit 1) is rejected
    with pytest.raises(tsg.TSGError):
        tsg.csc_packed_to_tcsc(np.array([0, 1]), np.array([0]), np.array([1], np.uint8), 1)


@pytest.mark.parametrize("K,N,s,B", [(64, 6, 2, 16), (1100, 70, 4, 512), (300, 33, 8, 100), (10, 5, 2, 32),
                                     (96, 9, 1, 1)])
def test_tcsc_to_blocked_matches_blocked_ctor(tsg, oracle_mod, K, N, s, B):
    """Host TCSC -> BlockedTCSC<B> conversion == the BlockedTCSC ctor
    (BlockedTCSC.h:15-41, restated in the oracle) array for array."""
    O = oracle_mod
    W = O.gen_ternary(K, N, s, K + B)
    got = tsg.tcsc_to_blocked(*O.tcsc_encode(W).arrays, K, N, B)
    want = O.blocked_tcsc_encode(W, B)
    for g, w in zip(got, want):
        assert np.array_equal(np.asarray(g, np.int32), np.asarray(w, np.int32))
    tsg.validate_blocked(*got, K, N, B)


def test_drop_in_header_is_the_product_surface():
    """include/ternary_spgemm.h carries the drop-in surface only; the tuning
    and test hooks live in ternary_spgemm_test.h (both exported by the .so)."""
    product = set(_declared_functions(("ternary_spgemm.h",)))
    hooks = set(_declared_functions(("ternary_spgemm_test.h",)))
    assert not product & hooks
    for f in ("tcsc_hip_create", "tcsc_hip_gemm", "tcsc_hip_gemm_dev", "tcsc_hip_gemm_prelu", "tcsc_hip_destroy",
              "tcsc_hip_reserve", "tcsc_hip_last_error"):
        assert f in product
    for f in ("tcsc_hip_set_jit_width", "tcsc_hip_set_small_m", "tcsc_hip_set_far", "tsg_jit_codegen_wv",
              "tsg_call_plan", "tsg_call_xtouch", "tsg_jit_tile_map", "tsg_ell_build", "tsg_knob_check"):
        assert f in hooks


def _small_tcsc(oracle_mod):
    t = oracle_mod.tcsc_encode(oracle_mod.gen_ternary(64, 32, 4, 3))
    return t.arrays, 64, 32


@pytest.mark.parametrize("var,val,msg", [
    ("TSG_JIT_DIAG", "nodma", "WRONG results"),          # wrong-result diagnostics: diagnostic build only
    ("TSG_JIT_DIAG", "nobar,noreads", "WRONG results"),
    ("TSG_JIT_DMA", "0.5;1", "TSG_JIT_DMA=0.5;1: expected"),
    ("TSG_JIT_DMA", "2,1", "expected"),                  # spread outside [0, 1]
    ("TSG_JIT_TOUCH", "1,9", "expected"),
    ("TSG_JIT_TOUCH", "0,1", "expected"),  # first >= 1: the per-call near bias would reach before the region
    ("TSG_JIT_READS", "20,20", "expected"),
    ("TSG_JIT_CP", "0x40,0", "expected"),
    ("TSG_JIT_GN", "two", "expected"),
    ("TSG_JIT_NOALIGN", "yes", "expected"),
    ("TSG_KERNEL", "fast", "expected"),
    ("TSG_ELL_VARIANT", "7", "expected"),
    ("TSG_JIT_HALF", "2", "expected"),
    ("TSG_JIT_PAIR", "2", "expected"),
    ("TSG_JIT_XDIRECT", "on", "expected"),
    ("TSG_JIT_QBLOCK", "4", "expected"),
    ("TSG_ELL_COPIES", "3", "expected"),
    ("TSG_ELL_WPG", "12", "expected"),
    ("TSG_ELL_SCHED", "yes", "expected"),
])
def test_registration_refuses_bad_knobs(tsg, oracle_mod, monkeypatch, var, val, msg):
    """A set knob outside its accepted values -- and, in the product library,
    TSG_JIT_DIAG at all -- fails registration with TSG_ERR_ARG before any
    device is touched (so this runs on the CPU), and the host codegen refuses
    it too; nothing is parsed leniently."""
    arrays, K, N = _small_tcsc(oracle_mod)
    monkeypatch.setenv(var, val)
    assert msg in tsg.knob_check()
    with pytest.raises(tsg.TSGError, match="TSG_ERR_ARG") as e:
        tsg.TCSCDevice(*arrays, K, N)
    assert var in str(e.value)
    with pytest.raises(tsg.TSGError, match=var):
        tsg.jit_codegen(*arrays, K, N)


@pytest.mark.parametrize("var,val", [
    ("TSG_JIT_DMA", "0.25,1"), ("TSG_JIT_DMA", "0,0,2"), ("TSG_JIT_TOUCH", "1,2"), ("TSG_JIT_READS", "6,12"),
    ("TSG_JIT_CP", "20000,0"), ("TSG_JIT_NOALIGN", "1"), ("TSG_KERNEL", "rx"), ("TSG_ELL_LG", "8"),
    ("TSG_JIT_HALF", "1"), ("TSG_JIT_XDIRECT", "1"), ("TSG_JIT_QBLOCK", "8"), ("TSG_ELL_COPIES", "2"),
    ("TSG_ELL_WPG", "16"), ("TSG_ELL_SCHED", "1"),
])
def test_accepted_knobs_pass(tsg, monkeypatch, var, val):
    monkeypatch.setenv(var, val)
    assert tsg.knob_check() == ""


def test_diag_build_accepts_diag_variants(monkeypatch):
    """The diagnostic build (make diag) is the only one that takes TSG_JIT_DIAG."""
    path = os.path.join(REPO, "ternary-spgemm_amd", "lib", "libternary_spgemm_diag.so")
    if not os.path.exists(path):
        pytest.skip("diagnostic build not present (make -C ternary-spgemm_amd diag)")
    L = ctypes.CDLL(path)
    L.tsg_knob_check.restype = ctypes.c_char_p
    monkeypatch.setenv("TSG_JIT_DIAG", "nodma,novm")
    assert L.tsg_knob_check() == b""
    monkeypatch.setenv("TSG_JIT_DIAG", "nodma,typo")
    assert b"expected" in L.tsg_knob_check()


def test_code_objects_embedded(tsg):
    """The library is one deployable artifact (VERDICT r04 "next" 5): every
    dispatcher code object the call plan can pick is embedded in
    libternary_spgemm.so (csrc/gen_co_embed.py), byte for byte the built
    lib/*.co, so nothing has to sit next to the .so."""
    lib = tsg.lib()

    class Entry(ctypes.Structure):
        _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("size", ctypes.c_uint64)]

    table = (Entry * 64).in_dll(lib, "tsg_co_table")
    got = {}
    for e in table:
        if not e.name:
            break
        got[e.name.decode()] = ctypes.string_at(e.data, e.size)
    libdir = os.path.join(REPO, "ternary-spgemm_amd", "lib")
    on_disk = sorted(f for f in os.listdir(libdir) if f.endswith(".co"))
    expected = (["tsg_jit.co"] + [f"tsg_jit_w{w}.co" for w in (32, 16, 8)]
                + [f"tsg_jit_w{w}_4w.co" for w in (32, 16, 8)]
                + [f"tsg_jit64_w{w}.co" for w in (128, 64, 32, 16, 8)]
                + [f"tsg_jit64_w{w}_4w.co" for w in (32, 16, 8)] + [f"tsg_jit64h_w{w}.co" for w in (32, 16, 8)]
                + [f"tsg_jit64p_w{w}.co" for w in (32, 16, 8)])
    assert sorted(got) == sorted(expected) == on_disk
    for name, blob in got.items():
        with open(os.path.join(libdir, name), "rb") as f:
            assert f.read() == blob, name
        assert blob[:4] == b"\x7fELF"
