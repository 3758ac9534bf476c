"""The small-M kernels (tsg_tcsc_ell_kernel and, for M = 1, its
producer/consumer split tsg_tcsc_ell_pc_kernel; tsg_ell.hip) on the GPU,
through the C-ABI: forced onto every call (tcsc_hip_set_small_m(h, 2); 3 =
without the producer/consumer split) over the edge
shapes of test_gpu_parity.py, every variant (M tiles of 1, 4, 8, 16 and 32
rows, several tiles, one stream or K chunks), PReLU, special values; the
automatic choice; configs[2]'s K and N at M = 1 ... 96 against the oracle;
configs[0] itself; graph capture after reserve.  Bit for bit against the BaseTCSC oracle (comp.h:25-69)."""
import numpy as np
import pytest

from test_gpu_parity import EDGE, _bits_eq

pytestmark = pytest.mark.gpu

SMALL = ("tsg_tcsc_ell_kernel", "tsg_tcsc_ell_pc_kernel")


def _small_kernel(M, K, N, mode):
    """The kernel tcsc_hip_set_small_m(mode) sends a call with M rows to:
    1-row producer/consumer tiles for M = 1, and for M <= 4 while M * N <=
    32768, when K fits the 1-row tile's LDS chunk (tsg_capi.cpp
    pick_ell_variant)."""
    # (the 1-row tile's chunk holds K <= 40956; with the producer/consumer ring
    # beside it in 160 KiB of LDS, K <= 34812: tsg_ell.hip pc_lds)
    pc = mode == 2 and K <= 34812 and (M == 1 or (M <= 4 and M * N <= 32768))
    return "tsg_tcsc_ell_pc_kernel" if pc else "tsg_tcsc_ell_kernel"


@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("M,K,N,s", EDGE)
def test_edges_forced_small_m(tsg, oracle_mod, M, K, N, s, mode):
    O = oracle_mod
    W = O.gen_ternary(K, N, s, M * 7 + K)
    t = O.tcsc_encode(W)
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.set_small_m(mode)
    assert h.call_kernel(M) == _small_kernel(M, K, N, mode)
    b = (np.arange(N, dtype=np.float32) - N / 2) * 0.37
    alpha = np.linspace(-0.5, 0.5, N).astype(np.float32)
    for X in (O.init_x_int(M, K, 5), O.init_x_frac(M, K, 6)):
        assert _bits_eq(h.gemm(X, b), O.base_tcsc(X, t, b)), (M, K, N, s)
        assert _bits_eq(h.gemm_prelu(X, b, alpha), O.base_tcsc_prelu(X, t, b, alpha))
    h.close()


@pytest.mark.parametrize("M,K", [(1, 2300), (2, 2300), (3, 2300), (4, 2300), (5, 2300), (16, 2300), (17, 2300),
                                 (31, 2300), (32, 2300), (33, 2300), (64, 2300), (100, 2300),
                                 (1, 20000), (1, 34812), (1, 34816), (1, 50000), (3, 9000), (16, 6000), (40, 6000)])
@pytest.mark.parametrize("mode", [2, 3])
def test_every_variant_and_tiling(tsg, oracle_mod, M, K, mode):
    """M and K pick the M tile (1 / 4 / 8 / 16 / 32 rows) and the lanes per
    column; M past a tile runs several tiles.  K = 2300 fits one LDS chunk for
    every tile up to 16 rows (one +1/-1 stream per column); K = 6000 and 9000
    split into K chunks for their tiles (a step per pass and chunk, restaged);
    M = 1 holds K = 20000 and 34812 in one chunk beside the producer/consumer
    ring, 34816 without it, 50000 in two chunks."""
    O = oracle_mod
    N = 530
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 40 + M))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.set_small_m(mode)
    assert h.call_kernel(M) == _small_kernel(M, K, N, mode)
    b = np.linspace(-3, 3, N).astype(np.float32)
    X = O.init_x_frac(M, K, M)
    assert _bits_eq(h.gemm(X, b), O.base_tcsc(X, t, b)), M
    h.close()


def test_special_values_small_m(tsg, oracle_mod):
    from test_gpu_special import _same, _special_b, _special_x
    O = oracle_mod
    K, N = 700, 300
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 31))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.set_small_m(2)
    alpha = np.linspace(-0.5, 0.5, N).astype(np.float32)
    for M, kind in ((3, "mixed"), (9, "subnormal"), (20, "nan"), (7, "zeros"), (1, "subnormal"), (4, "nan")):
        for mode in (2, 3):
            h.set_small_m(mode)
            X = _special_x(M, K, 7, kind)
            b = _special_b(N, 3)
            _same(h.gemm(X, b), O.base_tcsc(X, t, b))
            _same(h.gemm_prelu(X, b, alpha), O.base_tcsc_prelu(X, t, b, alpha))
    h.close()


def test_auto_choice_and_structural_edges(tsg, oracle_mod):
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(1024, 4096, 4, 77))
    h = tsg.TCSCDevice(*t.arrays, 1024, 4096)
    assert h.call_kernel(1) == "tsg_tcsc_ell_pc_kernel" and h.call_kernel(4096) == "tsg_jit64_kernel"
    assert h.call_kernel(4) == "tsg_tcsc_ell_pc_kernel" and h.call_kernel(5) == "tsg_tcsc_ell_kernel"
    h.set_small_m(1)
    assert h.call_kernel(1) == "tsg_jit64_kernel"  # small M off: the 64-row weight-compiled image
    h.close()
    # empty / dense / all-zero W and K = 0 on the small-M kernel
    rng = np.random.default_rng(3)
    for W in (np.zeros((300, 70), np.int32), rng.integers(-1, 2, size=(260, 150)).astype(np.int32),
              np.ones((129, 5), np.int32), -np.ones((129, 5), np.int32)):
        K, N = W.shape
        W[:, 0] = 0
        t = O.tcsc_encode(W)
        h = tsg.TCSCDevice(*t.arrays, K, N)
        h.set_small_m(2)
        X = O.init_x_frac(13, K, 9)
        b = rng.standard_normal(N).astype(np.float32)
        assert _bits_eq(h.gemm(X, b), O.base_tcsc(X, t, b))
        h.close()
    h = tsg.TCSCDevice(np.zeros(4, np.int32), np.zeros(4, np.int32), [], [], 0, 3)
    h.set_small_m(2)
    Y = h.gemm(np.zeros((5, 0), np.float32), np.array([1.5, -2.0, 0.0], np.float32))
    assert _bits_eq(Y, np.tile(np.array([1.5, -2.0, 0.0], np.float32), (5, 1)))
    # BlockedTCSC never takes it
    blk = O.blocked_tcsc_encode(O.gen_ternary(64, 8, 2, 1), 16)
    hb = tsg.TCSCDevice.from_blocked(*blk, 64, 8, 16)
    assert hb.call_kernel(1) == "tsg_jit_kernel"
    with pytest.raises(tsg.TSGError):
        hb.set_small_m(2)


@pytest.mark.parametrize("M", [1, 2, 3, 16, 32, 64, 96])
def test_config3_shape_small_m(tsg, oracle_mod, M):
    """configs[2]'s K = 4096, N = 16384 at GEMV-like M (the reference sweep's
    M list, plots/run_benchmark.py:8), automatic choice (the small-M kernel up
    to M = 32 at this K, then the 64-row weight-compiled image), against the
    oracle."""
    import torch
    O = oracle_mod
    K, N = 4096, 16384
    arrs = tsg.gen_tcsc(K, N, 4, 42)
    h = tsg.TCSCDevice(*arrs, K, N)
    assert h.call_kernel(M) == ("tsg_tcsc_ell_pc_kernel" if M <= 2 else "tsg_tcsc_ell_kernel" if M <= 32
                                else "tsg_jit64_kernel")
    Xn = O.init_x_frac(M, K, 5)
    b = np.full(N, 2.0, np.float32)
    Y = h.gemm_torch(torch.from_numpy(Xn).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
    rows = np.unique(np.r_[0, M // 2, M - 1])
    ref = O.base_tcsc(np.ascontiguousarray(Xn[rows]), O.TCSC(*arrs, K, N), b)
    assert _bits_eq(Y[rows], ref)
    h.close()


@pytest.mark.parametrize("M,K,N", [(16, 2048, 8192), (32, 2048, 8192), (16, 2048, 16384), (24, 2048, 16384),
                                   (32, 2048, 16384), (24, 4096, 16384)])
def test_walk_workgroup_shapes_full_y(tsg, oracle_mod, M, K, N):
    """Round 5's waves-per-workgroup rule (tsg_ell.hip launch_lg): these
    shapes run the walk with 4, 8 and 16 waves per workgroup, in one round or
    more; every element against the oracle with order-sensitive X."""
    import torch
    O = oracle_mod
    arrs = tsg.gen_tcsc(K, N, 4, 7)
    h = tsg.TCSCDevice(*arrs, K, N)
    assert h.call_kernel(M) == "tsg_tcsc_ell_kernel"
    Xn = O.init_x_frac(M, K, 11)
    b = np.linspace(-2, 2, N).astype(np.float32)
    Y = h.gemm_torch(torch.from_numpy(Xn).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
    assert _bits_eq(Y, O.base_tcsc(Xn, O.TCSC(*arrs, K, N), b, threads=16))
    h.close()


def test_config0_runs_small_m(tsg, oracle_mod):
    """configs[0] (M = 32, K = 1024, N = 4096, s = 4; BASELINE.json) takes the
    small-M kernel automatically (8-row tiles; 12 us vs 26 us on the jit
    kernel, profiles/r02u_ell_lg.txt) and matches the oracle bit for bit."""
    O = oracle_mod
    M, K, N = 32, 1024, 4096
    arrs = tsg.gen_tcsc(K, N, 4, 42)
    h = tsg.TCSCDevice(*arrs, K, N)
    assert h.call_kernel(M) == "tsg_tcsc_ell_kernel"
    b = np.full(N, 2.0, np.float32)
    for X in (O.init_x_int(M, K, 3), O.init_x_frac(M, K, 4)):
        assert _bits_eq(h.gemm(X, b), O.base_tcsc(X, O.TCSC(*arrs, K, N), b))
    h.close()


@pytest.mark.parametrize("M,K,N,small", [(512, 2048, 512, True), (1000, 2048, 512, True), (256, 4096, 1024, True),
                                         (128, 9000, 1024, False), (1024, 1024, 1024, False), (96, 4096, 16384, False),
                                         (64, 16384, 4096, False)])
def test_starved_jit_shapes_take_small_m(tsg, oracle_mod, M, K, N, small):
    """The reference's cases where the jit kernel would have <= 64 workgroups
    (plots/run_benchmark.py:8-33) take the small-M kernel automatically up to
    M = 1024 while an 8-row chunk holds K (K <= 5116; with K chunked the
    64-row image: (64, 16384, 4096) 156 vs 266 us, profiles/r04g_bound_ab.jsonl);
    bit for bit on sampled rows either way."""
    import torch
    O = oracle_mod
    arrs = tsg.gen_tcsc(K, N, 4, 7)
    h = tsg.TCSCDevice(*arrs, K, N)
    assert (h.call_kernel(M) in SMALL) == small, h.call_kernel(M)
    Xn = O.init_x_frac(M, K, 3)
    b = np.linspace(-1, 1, N).astype(np.float32)
    Y = h.gemm_torch(torch.from_numpy(Xn).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
    rows = np.unique(np.r_[0, 1, M // 2, M - 1])
    assert _bits_eq(Y[rows], O.base_tcsc(np.ascontiguousarray(Xn[rows]), O.TCSC(*arrs, K, N), b))
    h.close()


def test_capture_small_m_after_reserve(tsg, oracle_mod):
    import torch
    O = oracle_mod
    K, N, M = 1024, 2048, 8
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 23))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.reserve(64)
    assert h.call_kernel(M) == "tsg_tcsc_ell_kernel"
    b = torch.full((N,), 2.0, device="cuda")
    Xs = torch.zeros((M, K), device="cuda")
    Ys = torch.empty((M, N), device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        h.gemm_torch(Xs, b, Ys)
    Xn = O.init_x_frac(M, K, 1)
    Xs.copy_(torch.from_numpy(Xn).cuda())
    g.replay()
    torch.cuda.synchronize()
    assert _bits_eq(Ys.cpu().numpy(), O.base_tcsc(Xn, t, np.full(N, 2.0, np.float32)))
    h.close()
