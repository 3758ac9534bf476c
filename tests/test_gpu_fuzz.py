"""Seeded random shapes through every path (round 5): M, K, N and the
sparsity drawn over the regimes the automatic plan distinguishes (walk,
producer/consumer walk, 64-row image with direct or staged X, 128-row image),
K not a multiple of 4 included, each call compared on EVERY element with the
BaseTCSC oracle (comp.h:25-69) on order-sensitive X, automatic and with each
image pinned."""
import numpy as np
import pytest

from test_gpu_parity import _bits_eq

pytestmark = pytest.mark.gpu


def _cases(n=60, seed=2026):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        M = int(rng.choice([1, 2, 3, 5, 8, 13, 17, 31, 33, 47, 64, 65, 100, 129, 200, 257, 513]))
        K = int(rng.integers(1, 6000))
        if rng.random() < 0.5:
            K = K // 4 * 4 + 4  # half the cases on K % 4 == 0 (the row layout's direct X)
        N = int(rng.integers(1, 2500))
        s = int(rng.choice([1, 2, 3, 4, 8, 16, 32]))
        out.append((M, K, N, s))
    return out


@pytest.mark.parametrize("M,K,N,s", _cases())
def test_random_shapes_every_path(tsg, oracle_mod, M, K, N, s):
    import torch
    O = oracle_mod
    W = O.gen_ternary(K, N, s, M * 31 + K * 7 + N)
    t = O.tcsc_encode(W)
    h = tsg.TCSCDevice(*t.arrays, K, N)
    X = O.init_x_frac(M, K, K + N)
    b = (np.arange(N, dtype=np.float32) % 17 - 8) * np.float32(0.41)
    ref = O.base_tcsc(X, t, b, threads=16)
    Xd, bd = torch.from_numpy(X).cuda(), torch.from_numpy(b).cuda()
    for pin in (None, 64, 128):
        h.set_small_m(0 if pin is None else 1)
        h.set_tile_rows(0 if pin is None else pin)
        Y = h.gemm_torch(Xd, bd).cpu().numpy()
        assert _bits_eq(Y, ref), (pin, h.call_kernel(M))
    h.close()
