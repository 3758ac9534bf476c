"""ctypes front-end for the CPU oracle (liboracle.so) and the reference shim
(_ref/libref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  Each wrapper
names the reference file:line its C function restates (see tcsc_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i64 = C.c_int64


def build(ref: bool = True) -> None:
    """Compile liboracle.so (and _ref/libref.so when the reference is mounted)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if ref and os.path.isdir(os.environ.get("REF", "/root/reference")):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build(ref=False)
        L = C.CDLL(path)
        L.oracle_gen_ternary.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, _i32p]
        L.oracle_init_x_int.argtypes = [_i64, C.c_int, C.c_uint64, _f32p]
        L.oracle_init_x_frac.argtypes = [_i64, C.c_uint64, _f32p]
        L.oracle_tcsc_count.argtypes = [_i32p, C.c_int, C.c_int, C.POINTER(_i64), C.POINTER(_i64)]
        L.oracle_tcsc_encode.argtypes = [_i32p, C.c_int, C.c_int, _i32p, _i32p, _i32p, _i32p]
        L.oracle_tcsc_decode.argtypes = [_i32p, _i32p, _i32p, _i32p, C.c_int, C.c_int, _i32p]
        L.oracle_tcsc_size_bytes.argtypes = [C.c_int, _i64, _i64]
        L.oracle_tcsc_size_bytes.restype = _i64
        L.oracle_blocked_tcsc_encode.argtypes = [_i32p, C.c_int, C.c_int, C.c_int,
                                                 _i32p, _i32p, _i32p, _i32p]
        kargs = [_f32p, _i32p, _i32p, _i32p, _i32p, _f32p, _f32p, C.c_int, C.c_int, C.c_int]
        L.oracle_base_tcsc.argtypes = kargs
        L.oracle_base_tcsc_omp.argtypes = kargs + [C.c_int]
        L.oracle_double_unrolled_tcsc_k4m4.argtypes = kargs
        L.oracle_base_tcsc_prelu.argtypes = kargs[:6] + [_f32p] + kargs[6:]
        L.oracle_base_blocked_tcsc.argtypes = kargs + [C.c_int]
        L.oracle_gemm_dense.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int, C.c_int]
        _u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
        L.oracle_csc_packed_encode.argtypes = [_i32p, C.c_int, C.c_int, _i32p, _i32p, _u8p]
        L.oracle_csc_packed_encode.restype = None
        L.oracle_base_csc_packed.argtypes = [_f32p, _i32p, _i32p, _u8p, _f32p, _f32p,
                                             C.c_int, C.c_int, C.c_int]
        L.oracle_base_csc_packed.restype = None
        L.oracle_perf_calibrated.argtypes = [C.c_int, C.c_int, C.c_double, _f32p, _i32p, _i32p, _i32p, _i32p,
                                             _f32p, _f32p, C.c_int, C.c_int, C.c_int, C.POINTER(_i64),
                                             C.POINTER(C.c_double)]
        L.oracle_perf_calibrated.restype = C.c_double
        for f in ("oracle_gen_ternary", "oracle_init_x_int", "oracle_init_x_frac",
                  "oracle_tcsc_count", "oracle_tcsc_encode", "oracle_tcsc_decode",
                  "oracle_blocked_tcsc_encode", "oracle_base_tcsc", "oracle_base_tcsc_omp",
                  "oracle_double_unrolled_tcsc_k4m4", "oracle_base_tcsc_prelu",
                  "oracle_base_blocked_tcsc", "oracle_gemm_dense"):
            getattr(L, f).restype = None
        _LIB = L
    return _LIB


def ref_available() -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", "libref.so"))


def ref() -> C.CDLL:
    """The reference's own headers compiled unmodified (oracle/_ref/libref.so)."""
    global _REF
    if _REF is None:
        L = C.CDLL(os.path.join(HERE, "_ref", "libref.so"))
        L.ref_generate_sparse.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, _i32p]
        L.ref_generate_sparse.restype = None
        p64 = C.POINTER(_i64)
        L.ref_tcsc_encode.argtypes = [_i32p, C.c_int, C.c_int, p64, p64,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, p64]
        L.ref_tcsc_encode.restype = None
        L.ref_blocked_tcsc_encode.argtypes = [_i32p, C.c_int, C.c_int, C.c_int, p64, p64,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ref_blocked_tcsc_encode.restype = C.c_int
        L.ref_gemm.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int, C.c_int]
        L.ref_gemm.restype = None
        L.ref_gemm_prelu.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int, C.c_int]
        L.ref_gemm_prelu.restype = None
        L.ref_compare_results.argtypes = [_f32p, _f32p, C.c_int, C.c_int]
        L.ref_compare_results.restype = C.c_int
        _REF = L
    return _REF


# ---------------------------------------------------------------- inputs --

def gen_ternary(K: int, N: int, s: int, seed: int) -> np.ndarray:
    """generateSparseMatrix distribution (sparseUtils.h:52-87), portable PRNG."""
    W = np.empty((K, N), dtype=np.int32)
    lib().oracle_gen_ternary(K, N, s, seed, W)
    return W


def init_x_int(M: int, K: int, seed: int, rng: int = 512) -> np.ndarray:
    """initX (sparseUtils.h:6-23): integer-valued fp32 in [-rng, rng]."""
    X = np.empty((M, K), dtype=np.float32)
    lib().oracle_init_x_int(M * K, rng, seed, X)
    return X


def init_x_frac(M: int, K: int, seed: int) -> np.ndarray:
    """Non-integer X: pins accumulation order (every partial sum rounds)."""
    X = np.empty((M, K), dtype=np.float32)
    lib().oracle_init_x_frac(M * K, seed, X)
    return X


# ---------------------------------------------------------------- formats --

class TCSC:
    """Host TCSC arrays with the layout of class TCSC (TCSC.h:5-50)."""

    def __init__(self, csp, csn, rip, rin, K: int, N: int):
        self.col_start_pos = np.ascontiguousarray(csp, dtype=np.int32)
        self.col_start_neg = np.ascontiguousarray(csn, dtype=np.int32)
        self.row_index_pos = np.ascontiguousarray(rip, dtype=np.int32)
        self.row_index_neg = np.ascontiguousarray(rin, dtype=np.int32)
        self.K, self.N = K, N

    @property
    def arrays(self):
        return (self.col_start_pos, self.col_start_neg, self.row_index_pos, self.row_index_neg)

    def size_bytes(self) -> int:
        return int(lib().oracle_tcsc_size_bytes(self.N, len(self.row_index_pos),
                                                len(self.row_index_neg)))

    def dense(self) -> np.ndarray:
        W = np.empty((self.K, self.N), dtype=np.int32)
        lib().oracle_tcsc_decode(*self.arrays, self.K, self.N, W)
        return W


def tcsc_encode(W: np.ndarray) -> TCSC:
    """class TCSC ctor (TCSC.h:13-41)."""
    W = np.ascontiguousarray(W, dtype=np.int32)
    K, N = W.shape
    p, q = _i64(), _i64()
    lib().oracle_tcsc_count(W, K, N, C.byref(p), C.byref(q))
    csp = np.empty(N + 1, np.int32)
    csn = np.empty(N + 1, np.int32)
    rip_b = np.empty(max(p.value, 1), np.int32)
    rin_b = np.empty(max(q.value, 1), np.int32)
    lib().oracle_tcsc_encode(W, K, N, csp, csn, rip_b, rin_b)
    rip = rip_b[: p.value].copy()
    rin = rin_b[: q.value].copy()
    return TCSC(csp, csn, rip, rin, K, N)


def blocked_tcsc_encode(W: np.ndarray, B: int):
    """BlockedTCSC<B> ctor (BlockedTCSC.h:15-41): K/B whole blocks; rows past
    (K/B)*B are not encoded (BlockedTCSC.h:17)."""
    W = np.ascontiguousarray(W, dtype=np.int32)
    K, N = W.shape
    p, q = _i64(), _i64()
    lib().oracle_tcsc_count(W, K, N, C.byref(p), C.byref(q))
    nslot = (K // B) * N + 1
    csp = np.empty(nslot, np.int32)
    csn = np.empty(nslot, np.int32)
    rip = np.empty(max(p.value, 1), np.int32)
    rin = np.empty(max(q.value, 1), np.int32)
    lib().oracle_blocked_tcsc_encode(W, K, N, B, csp, csn, rip, rin)
    return csp, csn, rip[: csp[-1]].copy(), rin[: csn[-1]].copy()


def csc_packed_encode(W: np.ndarray):
    """CSC + base-3 packed values, 5 per byte (readme.md:111)."""
    W = np.ascontiguousarray(W, dtype=np.int32)
    K, N = W.shape
    nnz = int(np.count_nonzero((W == 1) | (W == -1)))
    col_ptr = np.empty(N + 1, np.int32)
    row_idx = np.empty(max(nnz, 1), np.int32)
    packed = np.zeros(max((nnz + 4) // 5, 1), np.uint8)
    lib().oracle_csc_packed_encode(W, K, N, col_ptr, row_idx, packed)
    return col_ptr, row_idx[:nnz].copy(), packed[: (nnz + 4) // 5].copy()


def base_csc_packed(X, col_ptr, row_idx, packed, b, K: int, N: int) -> np.ndarray:
    X = np.ascontiguousarray(X, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    M = X.shape[0]
    Y = np.empty((M, N), np.float32)
    ri = row_idx if len(row_idx) else np.zeros(1, np.int32)
    pk = packed if len(packed) else np.zeros(1, np.uint8)
    lib().oracle_base_csc_packed(X, np.ascontiguousarray(col_ptr, np.int32), ri, pk, b, Y, M, N, K)
    return Y


# ---------------------------------------------------------------- kernels --

def _prep(X, t: TCSC, b):
    X = np.ascontiguousarray(X, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    M, K = X.shape
    assert K == t.K and b.shape == (t.N,)
    return X, b, M


def base_tcsc(X, t: TCSC, b, threads: int = 0) -> np.ndarray:
    """BaseTCSC<float> (comp.h:25-69); threads>0 -> OpenMP over rows."""
    X, b, M = _prep(X, t, b)
    Y = np.empty((M, t.N), dtype=np.float32)
    if threads:
        lib().oracle_base_tcsc_omp(X, *t.arrays, b, Y, M, t.N, t.K, threads)
    else:
        lib().oracle_base_tcsc(X, *t.arrays, b, Y, M, t.N, t.K)
    return Y


def double_unrolled_tcsc(X, t: TCSC, b) -> np.ndarray:
    """DoubleUnrolledTCSC<float,4,4> (comp.h:1227-1438)."""
    X, b, M = _prep(X, t, b)
    Y = np.empty((M, t.N), dtype=np.float32)
    lib().oracle_double_unrolled_tcsc_k4m4(X, *t.arrays, b, Y, M, t.N, t.K)
    return Y


PERF_KERNELS = {"BaseTCSC": 0, "BaseTCSC_omp": 1, "DoubleUnrolledTCSC_K4_M4": 2}


def perf_calibrated(kernel: str, X, t: TCSC, b, threads: int = 0, cycles_required: float = 1e8):
    """The reference's timing method (perf.cpp:37-71, CALIBRATE on): doubles
    the run count until a batch takes >= 1e8 TSC cycles, then times that many
    runs.  Returns (seconds per call, runs, TSC cycles per call, Y)."""
    X, b, M = _prep(X, t, b)
    Y = np.empty((M, t.N), dtype=np.float32)
    runs, cyc = _i64(), C.c_double()
    rip = t.row_index_pos if len(t.row_index_pos) else np.zeros(1, np.int32)
    rin = t.row_index_neg if len(t.row_index_neg) else np.zeros(1, np.int32)
    sec = lib().oracle_perf_calibrated(PERF_KERNELS[kernel], threads, cycles_required, X, t.col_start_pos,
                                       t.col_start_neg, rip, rin, b, Y, M, t.N, t.K, C.byref(runs), C.byref(cyc))
    return sec, runs.value, cyc.value, Y


def base_tcsc_prelu(X, t: TCSC, b, alpha) -> np.ndarray:
    """BaseTCSC_PreLU<float> (comp_prelu.h:12-70)."""
    X, b, M = _prep(X, t, b)
    alpha = np.ascontiguousarray(alpha, dtype=np.float32)
    Y = np.empty((M, t.N), dtype=np.float32)
    lib().oracle_base_tcsc_prelu(X, *t.arrays, b, alpha, Y, M, t.N, t.K)
    return Y


def base_blocked_tcsc(X, blocked, b, K: int, N: int, B: int) -> np.ndarray:
    """BaseBlockedTCSC<float,B> (comp.h:607-658)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    M = X.shape[0]
    Y = np.empty((M, N), dtype=np.float32)
    csp, csn, rip, rin = (np.ascontiguousarray(a, dtype=np.int32) for a in blocked)
    rip = rip if len(rip) else np.zeros(1, np.int32)
    rin = rin if len(rin) else np.zeros(1, np.int32)
    lib().oracle_base_blocked_tcsc(X, csp, csn, rip, rin, b, Y, M, N, K, B)
    return Y


def gemm_dense(X, W, b) -> np.ndarray:
    """GEMM<float> (sparseUtils.h:92-108)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    Wf = np.ascontiguousarray(W, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    M, K = X.shape
    N = Wf.shape[1]
    Y = np.empty((M, N), dtype=np.float32)
    lib().oracle_gemm_dense(X, Wf, b, Y, M, N, K)
    return Y


# --------------------------------------------------------- reference shim --

def ref_generate_sparse(K: int, N: int, s: int, seed: int) -> np.ndarray:
    W = np.empty((K, N), dtype=np.int32)
    ref().ref_generate_sparse(K, N, s, seed, W)
    return W


def ref_tcsc_encode(W: np.ndarray):
    W = np.ascontiguousarray(W, dtype=np.int32)
    K, N = W.shape
    p, q, ds = _i64(), _i64(), _i64()
    ref().ref_tcsc_encode(W, K, N, C.byref(p), C.byref(q), None, None, None, None, C.byref(ds))
    csp = np.empty(N + 1, np.int32)
    csn = np.empty(N + 1, np.int32)
    rip = np.empty(max(p.value, 1), np.int32)
    rin = np.empty(max(q.value, 1), np.int32)
    ref().ref_tcsc_encode(W, K, N, C.byref(p), C.byref(q), csp.ctypes.data, csn.ctypes.data,
                          rip.ctypes.data, rin.ctypes.data, C.byref(ds))
    return csp, csn, rip[: p.value].copy(), rin[: q.value].copy(), ds.value


def ref_blocked_tcsc_encode(W: np.ndarray, B: int):
    W = np.ascontiguousarray(W, dtype=np.int32)
    K, N = W.shape
    p, q = _i64(), _i64()
    assert ref().ref_blocked_tcsc_encode(W, K, N, B, C.byref(p), C.byref(q),
                                         None, None, None, None) == 0
    nslot = (K // B) * N + 1
    csp = np.empty(nslot, np.int32)
    csn = np.empty(nslot, np.int32)
    rip = np.empty(max(p.value, 1), np.int32)
    rin = np.empty(max(q.value, 1), np.int32)
    ref().ref_blocked_tcsc_encode(W, K, N, B, C.byref(p), C.byref(q), csp.ctypes.data,
                                  csn.ctypes.data, rip.ctypes.data, rin.ctypes.data)
    return csp, csn, rip[: p.value].copy(), rin[: q.value].copy()


def ref_gemm(X, W, b) -> np.ndarray:
    X = np.ascontiguousarray(X, dtype=np.float32)
    Wf = np.ascontiguousarray(W, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    M, K = X.shape
    N = Wf.shape[1]
    Y = np.empty((M, N), dtype=np.float32)
    ref().ref_gemm(X, Wf, b, Y, M, N, K)
    return Y


def ref_gemm_prelu(X, W, b, alpha) -> np.ndarray:
    X = np.ascontiguousarray(X, dtype=np.float32)
    Wf = np.ascontiguousarray(W, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    alpha = np.ascontiguousarray(alpha, dtype=np.float32)
    M, K = X.shape
    N = Wf.shape[1]
    Y = np.empty((M, N), dtype=np.float32)
    ref().ref_gemm_prelu(X, Wf, b, alpha, Y, M, N, K)
    return Y
