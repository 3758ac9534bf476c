"""BASELINE.json configs[3] at full size: M=4096 K=4096 N=16384, s in {2, 8, 16}
(s = 4 is test_gpu_parity.py::test_config3_full_size), registered both as TCSC
and as CSC + packed values (readme.md:111).

Pins, per s:
  * the TCSC and CSC+packed arrays (sha256 of the generator / converter output,
    tests/golden/ref_hashes.json, made by tests/golden/make_golden.py);
  * integer X: sampled rows of Y equal the reference's dense GEMM
    (cpp_impl/sparseUtils.h:92-108, compiled from the reference) by hash;
  * the CSC+packed registration gives the same Y as TCSC on every element;
  * non-integer X: sampled rows bit for bit against the BaseTCSC restatement
    (comp.h:37-63 order).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _sha(*arrays) -> str:
    return hashlib.sha256(np.concatenate([np.ascontiguousarray(a).ravel() for a in arrays]).tobytes()).hexdigest()


@pytest.mark.parametrize("s", [2, 8, 16])
def test_config4_sweep_full_size(tsg, oracle_mod, s):
    import torch
    O = oracle_mod
    g = json.load(open(os.path.join(GOLDEN, "ref_hashes.json")))[f"config4_s{s}_rows"]
    M, K, N = g["M"], g["K"], g["N"]
    arrs = tsg.gen_tcsc(K, N, s, g["seed_w"])
    assert _sha(*arrs) == g["sha256_tcsc"]
    cp, ri, pk = tsg.tcsc_to_csc_packed(*arrs, N)
    assert hashlib.sha256(np.concatenate([cp.view(np.uint8), ri.view(np.uint8), pk]).tobytes()).hexdigest() \
        == g["sha256_csc_packed"]
    rows = np.array(g["rows"])
    dev = torch.device("cuda:0")
    rows_t = torch.from_numpy(rows).to(dev)
    b = np.full(N, 2.0, np.float32)
    bt = torch.from_numpy(b).to(dev)
    X = torch.from_numpy(tsg.gen_x(M, K, g["seed_x"])).to(dev)
    Xf_np = O.init_x_frac(M, K, 100 + s)
    Xf = torch.from_numpy(Xf_np).to(dev)

    h = tsg.TCSCDevice(*arrs, K, N)
    assert h.kernel_name() == "tsg_jit_kernel"
    Y = h.gemm_torch(X, bt)
    Yf = h.gemm_torch(Xf, bt)
    torch.cuda.synchronize()
    assert _sha(Y[rows_t].cpu().numpy()) == g["sha256_Y_rows"]
    sub = rows[::2]
    t = O.TCSC(*arrs, K, N)
    ref = O.base_tcsc(np.ascontiguousarray(Xf_np[sub]), t, b)
    assert np.array_equal(Yf[torch.from_numpy(sub).to(dev)].cpu().numpy().view(np.uint32), ref.view(np.uint32))
    h.close()

    hp = tsg.TCSCDevice.from_csc_packed(cp, ri, pk, K, N)
    Yp = hp.gemm_torch(X, bt)
    Ypf = hp.gemm_torch(Xf, bt)
    torch.cuda.synchronize()
    assert torch.equal(Yp.view(torch.int32), Y.view(torch.int32))
    assert torch.equal(Ypf.view(torch.int32), Yf.view(torch.int32))
    hp.close()
