"""Special fp32 values through the HIP path: subnormals, +-0, +-inf and NaN in X
and in b, for TCSC, the fused PReLU epilogue and BlockedTCSC, against the CPU
oracle (built with the reference's flags: SSE scalar adds, no FTZ/DAZ, no
contraction).

Contract ("special values"):
  * every output that is not NaN is bit-identical to the oracle -- subnormal
    inputs and subnormal partial sums included: the dispatcher's kernel
    descriptor keeps FP32 denormals (FLOAT_DENORM_MODE_32 = 3, IEEE mode on),
    checked on the shipped code objects by
    tests/test_jit_codegen.py::test_kernel_descriptor_float_mode;
  * an output is NaN exactly where the oracle's is NaN (same IEEE operations
    in the same order raise NaN at the same place), but the NaN payload/sign
    is not compared: x86 `addss` returns the first operand's NaN and makes
    inf - inf the negative default NaN 0xFFC00000, gfx950 returns the
    positive default NaN 0x7FC00000.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(gpu, ref):
    gpu = np.ascontiguousarray(gpu, np.float32)
    ref = np.ascontiguousarray(ref, np.float32)
    assert gpu.shape == ref.shape
    gn, rn = np.isnan(gpu), np.isnan(ref)
    assert np.array_equal(gn, rn), f"NaN positions differ: {int((gn != rn).sum())} outputs"
    ok = ~rn
    bad = gpu.view(np.uint32)[ok] != ref.view(np.uint32)[ok]
    assert not bad.any(), f"{int(bad.sum())} non-NaN outputs differ bitwise"


def _special_x(M, K, seed, kind):
    rng = np.random.default_rng(seed)
    X = (rng.standard_normal((M, K)) * 3).astype(np.float32)
    if kind == "subnormal":
        # subnormal inputs (and sums that stay subnormal): mantissa-only bit patterns
        X = (rng.integers(-(1 << 22), 1 << 22, size=(M, K)).astype(np.int64))
        X = np.where(X < 0, (1 << 31) | (-X), X).astype(np.uint32).view(np.float32)
        X[:, ::7] = np.float32(1e-38)  # tiny normals next to them
    elif kind == "zeros":
        X[:, ::3] = -0.0
        X[:, 1::3] = 0.0
    elif kind == "inf":
        X[rng.random((M, K)) < 0.002] = np.inf
        X[rng.random((M, K)) < 0.002] = -np.inf
    elif kind == "nan":
        X[rng.random((M, K)) < 0.001] = np.nan
        sn = np.array([0x7F800001, 0xFFA00000], np.uint32).view(np.float32)  # signalling NaNs
        X[0, :2] = sn
    elif kind == "mixed":
        X[rng.random((M, K)) < 0.001] = np.nan
        X[rng.random((M, K)) < 0.002] = np.inf
        X[rng.random((M, K)) < 0.002] = -np.inf
        X[:, 5::11] = -0.0
        X[:, 3::13] = np.float32(3e-40)
    return X


KINDS = ["subnormal", "zeros", "inf", "nan", "mixed"]


def _special_b(N, seed):
    rng = np.random.default_rng(seed)
    b = rng.standard_normal(N).astype(np.float32)
    b[0::9] = -0.0
    b[1::9] = np.float32(1e-44)   # subnormal
    b[2::9] = np.inf
    b[3::9] = -np.inf
    b[4::9] = np.nan
    return b


@pytest.mark.parametrize("kind", KINDS)
def test_special_values_tcsc_and_prelu(tsg, oracle_mod, kind):
    O = oracle_mod
    M, K, N = 140, 500, 300
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 31))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    X = _special_x(M, K, 7, kind)
    alpha = np.linspace(-0.5, 0.5, N).astype(np.float32)
    alpha[::17] = np.float32(1e-40)
    for b in (np.full(N, 2.0, np.float32), _special_b(N, 3)):
        _same(h.gemm(X, b), O.base_tcsc(X, t, b))
        _same(h.gemm_prelu(X, b, alpha), O.base_tcsc_prelu(X, t, b, alpha))
    h.close()


@pytest.mark.parametrize("kind", ["subnormal", "mixed"])
def test_special_values_blocked(tsg, oracle_mod, kind):
    O = oracle_mod
    M, K, N, B = 130, 600, 200, 128
    W = O.gen_ternary(K, N, 4, 32)
    blk = O.blocked_tcsc_encode(W, B)
    h = tsg.TCSCDevice.from_blocked(*blk, K, N, B)
    X = _special_x(M, K, 8, kind)
    b = _special_b(N, 4)
    _same(h.gemm(X, b), O.base_blocked_tcsc(X, blk, b, K, N, B))
    h.close()


def test_subnormal_sums_are_not_flushed(tsg, oracle_mod):
    """Every input and every partial sum subnormal: a flush-to-zero mode
    anywhere (kernel descriptor, MODE register) would turn Y into zeros."""
    O = oracle_mod
    M, K, N = 128, 256, 128
    t = O.tcsc_encode(O.gen_ternary(K, N, 8, 33))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    X = (np.arange(M * K, dtype=np.uint32) % 1000 + 1).reshape(M, K).view(np.float32)  # 1..1000 ulp
    b = np.zeros(N, np.float32)
    Y = h.gemm(X, b)
    ref = O.base_tcsc(X, t, b)
    assert np.array_equal(Y.view(np.uint32), ref.view(np.uint32))
    assert (np.abs(ref) < np.float32(1.1754944e-38)).all() and (ref != 0).mean() > 0.5
    h.close()
