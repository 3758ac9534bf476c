"""Python host mirror of the reference's plugin surface, over the C-ABI.

The reference registers kernels as
    using comp_func = std::function<void(float*X, float*B, float*Y, int M, int N, int K)>
    add_function(comp_func f, std::string name)          (cpp_impl/common.h:12-15,
                                                           cpp_impl/main.cpp:21-26)
with a TCSC built once before registration (main.cpp:63,76-81).  This module
keeps that shape for Python callers (tests, bench.py, the multi-GPU launcher):

    h  = TCSCDevice(csp, csn, rip, rin, K, N)           # upload once
    add_function(h.comp_func(), "HipBaseTCSC")          # registry, as main.cpp
    h(X, B, Y, M, N, K)                                  # host pointers, sync

plus device-pointer entry points for torch tensors.  Everything routes to
libternary_spgemm.so (HIP, gfx950); there is no CPU fallback: if the library
or a gfx950 device is missing, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Callable, List, Optional, Tuple

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TSG_LIB") or os.path.join(PKG_DIR, "lib", "libternary_spgemm.so")

TSG_OK = 0
_ERRNAMES = {1: "TSG_ERR_ARG", 2: "TSG_ERR_HIP", 3: "TSG_ERR_NOMEM", 4: "TSG_ERR_NODEV",
             5: "TSG_ERR_RANGE"}

# Every symbol include/ternary_spgemm.h (the drop-in surface) and
# include/ternary_spgemm_test.h (tuning and test hooks) declare; tests check
# the .so exports them.
EXPORTED_SYMBOLS = (
    "tcsc_hip_create", "tcsc_hip_create_dense", "tcsc_hip_destroy", "tcsc_hip_gemm",
    "tcsc_hip_gemm_dev", "tcsc_hip_gemm_prelu", "tcsc_hip_gemm_prelu_dev", "tcsc_hip_reserve",
    "tcsc_hip_info", "tcsc_hip_to_dense", "tcsc_hip_set_timing", "tcsc_hip_kernel_time",
    "tcsc_hip_last_error", "tcsc_hip_device_count", "tsg_tcsc_slice", "tsg_tcsc_validate",
    "tsg_gen_tcsc", "tsg_gen_x", "tcsc_hip_create_csc_packed", "tsg_tcsc_to_csc_packed",
    "tsg_csc_packed_to_tcsc", "tsg_jit_codegen", "tcsc_hip_kernel_name", "tcsc_hip_encode_dense_dev",
    "tcsc_hip_create_blocked", "tsg_jit_codegen_blocked", "tsg_blocked_tcsc_validate",
    "tcsc_hip_jit_width", "tcsc_hip_set_jit_width", "tcsc_hip_jit_waves", "tsg_jit_codegen_w", "tsg_jit_codegen_wv",
    "tcsc_hip_set_small_m", "tcsc_hip_call_kernel", "tsg_ell_build", "tsg_jit_tile_map",
    "tcsc_hip_set_host_chunks", "tcsc_hip_host_chunk_rows", "tcsc_hip_call_image_bytes",
    "tcsc_hip_host_register", "tcsc_hip_host_unregister", "tcsc_hip_set_far", "tcsc_hip_call_far",
    "tsg_jit_codegen_far", "tsg_call_plan", "tsg_call_xtouch", "tsg_knob_check", "tcsc_hip_set_tile_rows", "tcsc_hip_call_tile_rows",
    "tsg_jit_codegen64", "tsg_jit_codegen64h", "tcsc_hip_call_launches",
)


class TSGError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class tsg_info(C.Structure):
    _fields_ = [("K", C.c_int32), ("N", C.c_int32), ("device", C.c_int32),
                ("abi_version", C.c_int32), ("nnz_pos", C.c_int64), ("nnz_neg", C.c_int64),
                ("tcsc_bytes", C.c_int64), ("image_bytes", C.c_int64), ("work_bytes", C.c_int64),
                ("chunk_rows", C.c_int32), ("tile_rows", C.c_int32), ("tile_cols", C.c_int32),
                ("reserved", C.c_int32)]


_LIB: Optional[C.CDLL] = None


def build(jobs: int = 8) -> str:
    """Compile the HIP library in-tree for gfx950 (hipcc cross-compiles; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", PKG_DIR, f"-j{jobs}"], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    """Load libternary_spgemm.so.  torch (when installed) is imported first so
    that the library binds to the same libamdhip64 runtime as torch."""
    global _LIB
    if _LIB is not None:
        return _LIB
    try:  # share one HIP runtime with torch (same soname libamdhip64.so.7)
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} missing: run __graft_entry__.build() or `make -C {PKG_DIR}`")
    L = C.CDLL(LIB_PATH)
    i32p, f32p, vp = C.POINTER(C.c_int32), C.POINTER(C.c_float), C.c_void_p
    H = C.c_void_p
    L.tcsc_hip_create.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.POINTER(H)]
    L.tcsc_hip_create_dense.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.POINTER(H)]
    L.tcsc_hip_create_blocked.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(H)]
    L.tcsc_hip_destroy.argtypes = [H]
    L.tcsc_hip_destroy.restype = None
    L.tcsc_hip_gemm.argtypes = [H, vp, vp, vp, C.c_int, C.c_int, C.c_int]
    L.tcsc_hip_gemm_dev.argtypes = [H, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp]
    L.tcsc_hip_gemm_prelu.argtypes = [H, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int]
    L.tcsc_hip_gemm_prelu_dev.argtypes = [H, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp]
    L.tcsc_hip_reserve.argtypes = [H, C.c_int]
    L.tcsc_hip_info.argtypes = [H, C.POINTER(tsg_info)]
    L.tcsc_hip_to_dense.argtypes = [H, vp, C.c_int, C.c_int]
    L.tcsc_hip_set_timing.argtypes = [H, C.c_int]
    L.tcsc_hip_kernel_time.argtypes = [H, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_int]
    L.tcsc_hip_encode_dense_dev.argtypes = [vp, C.c_int, C.c_int, vp, vp, vp, C.c_int64, vp, C.c_int64,
                                            C.POINTER(C.c_int64), C.POINTER(C.c_int64), vp]
    L.tcsc_hip_kernel_name.argtypes = [H]
    L.tcsc_hip_kernel_name.restype = C.c_char_p
    L.tcsc_hip_last_error.argtypes = []
    L.tcsc_hip_last_error.restype = C.c_char_p
    L.tcsc_hip_device_count.argtypes = [C.POINTER(C.c_int)]
    L.tsg_tcsc_slice.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp,
                                 C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.tsg_tcsc_validate.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int]
    L.tsg_blocked_tcsc_validate.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int]
    L.tsg_gen_tcsc.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int,
                               vp, vp, vp, vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.tsg_gen_x.argtypes = [C.c_int64, C.c_int, C.c_uint64, vp]
    L.tcsc_hip_create_csc_packed.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, C.POINTER(H)]
    L.tsg_tcsc_to_csc_packed.argtypes = [vp, vp, vp, vp, C.c_int, vp, vp, vp, C.POINTER(C.c_int64)]
    L.tsg_csc_packed_to_tcsc.argtypes = [vp, vp, vp, C.c_int, vp, vp, vp, vp,
                                         C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.tsg_jit_codegen.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, vp, C.c_int64,
                                  C.POINTER(C.c_int64), vp, C.c_int64, C.POINTER(C.c_int64)]
    L.tsg_jit_codegen_blocked.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_int64,
                                          C.POINTER(C.c_int64), vp, C.c_int64, C.POINTER(C.c_int64)]
    L.tsg_jit_codegen_w.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int64,
                                    C.POINTER(C.c_int64), vp, C.c_int64, C.POINTER(C.c_int64)]
    L.tsg_jit_codegen_wv.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int64,
                                     C.POINTER(C.c_int64), vp, C.c_int64, C.POINTER(C.c_int64)]
    L.tcsc_hip_set_small_m.argtypes = [H, C.c_int]
    L.tcsc_hip_set_far.argtypes = [H, C.c_int]
    L.tcsc_hip_set_tile_rows.argtypes = [H, C.c_int]
    L.tcsc_hip_call_tile_rows.argtypes = [H, C.c_int]
    L.tcsc_hip_call_launches.argtypes = [H, C.c_void_p, C.c_int]
    L.tsg_jit_codegen64.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int64,
                                    C.POINTER(C.c_int64), vp, C.c_int64, C.POINTER(C.c_int64)]
    L.tsg_jit_codegen64h.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_int64,
                                     C.POINTER(C.c_int64), vp, C.c_int64, C.POINTER(C.c_int64)]
    L.tsg_call_plan.argtypes = [C.c_int, C.c_int, C.c_int64, C.c_int] + [C.POINTER(C.c_int)] * 7
    L.tsg_call_xtouch.argtypes = [C.c_int, C.c_int, C.c_int64, C.c_int]
    L.tcsc_hip_call_far.argtypes = [H, C.c_int]
    L.tsg_jit_codegen_far.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, vp, C.c_int64,
                                      C.POINTER(C.c_int64), vp, C.c_int64, C.POINTER(C.c_int64)]
    L.tcsc_hip_set_host_chunks.argtypes = [H, C.c_int]
    L.tcsc_hip_host_chunk_rows.argtypes = [H, C.c_int]
    L.tcsc_hip_call_image_bytes.argtypes = [H, C.c_int]
    L.tcsc_hip_host_register.argtypes = [vp, C.c_size_t]
    L.tcsc_hip_host_unregister.argtypes = [vp]
    L.tcsc_hip_call_kernel.argtypes = [H, C.c_int]
    L.tcsc_hip_call_kernel.restype = C.c_char_p
    L.tsg_knob_check.argtypes = []
    L.tsg_knob_check.restype = C.c_char_p
    L.tsg_ell_build.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int64,
                                C.POINTER(C.c_int64), vp, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    L.tsg_jit_tile_map.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.tcsc_hip_jit_width.argtypes = [H, C.c_int]
    L.tcsc_hip_jit_waves.argtypes = [H, C.c_int]
    L.tcsc_hip_set_jit_width.argtypes = [H, C.c_int]
    for f in EXPORTED_SYMBOLS:
        if f not in ("tcsc_hip_destroy", "tcsc_hip_last_error", "tcsc_hip_kernel_name", "tcsc_hip_call_kernel",
                     "tcsc_hip_call_image_bytes", "tsg_knob_check"):
            getattr(L, f).restype = C.c_int
    L.tcsc_hip_call_image_bytes.restype = C.c_int64
    _LIB = L
    return L


def knob_check() -> str:
    """"" when every set TSG_* environment knob has an accepted value, else
    the error registration reports (include/ternary_spgemm_test.h)."""
    return lib().tsg_knob_check().decode()


def _check(rc: int, where: str) -> None:
    if rc != TSG_OK:
        raise TSGError(rc, where, lib().tcsc_hip_last_error().decode(errors="replace"))


def _ptr(a: Optional[np.ndarray]):
    return None if a is None or a.size == 0 else a.ctypes.data


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


# ------------------------------------------------------------ host helpers --

def validate(csp, csn, rip, rin, K: int, N: int) -> None:
    """Raise TSGError(TSG_ERR_ARG) unless the arrays form a valid TCSC."""
    csp, csn, rip, rin = map(_i32, (csp, csn, rip, rin))
    _check(lib().tsg_tcsc_validate(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N),
           "tsg_tcsc_validate")


def tcsc_slice(csp, csn, rip, rin, N: int, n0: int, n1: int):
    """Columns [n0, n1) of a TCSC, rebased (the per-rank shard)."""
    csp, csn, rip, rin = map(_i32, (csp, csn, rip, rin))
    p, q = C.c_int64(), C.c_int64()
    L = lib()
    _check(L.tsg_tcsc_slice(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), N, n0, n1,
                            None, None, None, None, C.byref(p), C.byref(q)), "tsg_tcsc_slice")
    o = [np.empty(n1 - n0 + 1, np.int32), np.empty(n1 - n0 + 1, np.int32),
         np.empty(p.value, np.int32), np.empty(q.value, np.int32)]
    _check(L.tsg_tcsc_slice(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), N, n0, n1,
                            o[0].ctypes.data, o[1].ctypes.data, _ptr(o[2]), _ptr(o[3]),
                            C.byref(p), C.byref(q)), "tsg_tcsc_slice")
    return tuple(o)


def gen_tcsc(K: int, N: int, s: int, seed: int, n0: int = 0, n1: Optional[int] = None):
    """Synthetic TCSC (generateSparseMatrix distribution, sparseUtils.h:52-87) of
    columns [n0, n1), rebased; deterministic in seed."""
    n1 = N if n1 is None else n1
    p, q = C.c_int64(), C.c_int64()
    L = lib()
    _check(L.tsg_gen_tcsc(K, N, s, seed, n0, n1, None, None, None, None, C.byref(p), C.byref(q)),
           "tsg_gen_tcsc")
    o = [np.empty(n1 - n0 + 1, np.int32), np.empty(n1 - n0 + 1, np.int32),
         np.empty(max(p.value, 1), np.int32), np.empty(max(q.value, 1), np.int32)]
    _check(L.tsg_gen_tcsc(K, N, s, seed, n0, n1, o[0].ctypes.data, o[1].ctypes.data,
                          o[2].ctypes.data, o[3].ctypes.data, C.byref(p), C.byref(q)),
           "tsg_gen_tcsc")
    return o[0], o[1], o[2][: p.value], o[3][: q.value]


def tcsc_to_csc_packed(csp, csn, rip, rin, N: int):
    """TCSC -> CSC + base-3 packed values (readme.md:111)."""
    csp, csn, rip, rin = map(_i32, (csp, csn, rip, rin))
    nnz = C.c_int64()
    L = lib()
    _check(L.tsg_tcsc_to_csc_packed(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), N, None, None,
                                    None, C.byref(nnz)), "tsg_tcsc_to_csc_packed")
    col_ptr = np.empty(N + 1, np.int32)
    row_idx = np.empty(max(nnz.value, 1), np.int32)
    packed = np.empty(max((nnz.value + 4) // 5, 1), np.uint8)
    _check(L.tsg_tcsc_to_csc_packed(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), N,
                                    col_ptr.ctypes.data, row_idx.ctypes.data, packed.ctypes.data,
                                    C.byref(nnz)), "tsg_tcsc_to_csc_packed")
    return col_ptr, row_idx[: nnz.value], packed[: (nnz.value + 4) // 5]


def csc_packed_to_tcsc(col_ptr, row_idx, packed, N: int):
    col_ptr, row_idx = _i32(col_ptr), _i32(row_idx)
    packed = np.ascontiguousarray(packed, dtype=np.uint8)
    p, q = C.c_int64(), C.c_int64()
    L = lib()
    _check(L.tsg_csc_packed_to_tcsc(_ptr(col_ptr), _ptr(row_idx), _ptr(packed), N, None, None,
                                    None, None, C.byref(p), C.byref(q)), "tsg_csc_packed_to_tcsc")
    o = [np.empty(N + 1, np.int32), np.empty(N + 1, np.int32),
         np.empty(max(p.value, 1), np.int32), np.empty(max(q.value, 1), np.int32)]
    _check(L.tsg_csc_packed_to_tcsc(_ptr(col_ptr), _ptr(row_idx), _ptr(packed), N,
                                    *(a.ctypes.data for a in o), C.byref(p), C.byref(q)),
           "tsg_csc_packed_to_tcsc")
    return o[0], o[1], o[2][: p.value], o[3][: q.value]


def jit_codegen(csp, csn, rip, rin, K: int, N: int, B: int = 0, width: int = 64, waves: int = 8):
    """Host-side machine code of the weight-compiled kernel (TSG_KERNEL=jit):
    (region words uint32[], per-(tile, wave) stream byte offsets uint32[]).
    B > 0: the arrays are BlockedTCSC<B> (tcsc_hip_create_blocked); width:
    columns per stream (64, 32, 16, 8); waves per workgroup (8; 4 for the
    narrow widths)."""
    csp, csn, rip, rin = _i32(csp), _i32(csn), _i32(rip), _i32(rin)
    nc, nw = C.c_int64(), C.c_int64()
    L = lib()
    _check(L.tsg_jit_codegen_wv(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, B, width, waves, None, 0,
                                C.byref(nc), None, 0, C.byref(nw)), "tsg_jit_codegen")
    code = np.empty(nc.value, np.uint32)
    wcode = np.empty(nw.value, np.uint32)
    _check(L.tsg_jit_codegen_wv(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, B, width, waves, _ptr(code),
                                nc.value, C.byref(nc), _ptr(wcode), nw.value, C.byref(nw)),
           "tsg_jit_codegen")
    return code, wcode


def jit_codegen64(csp, csn, rip, rin, K: int, N: int, width: int = 16, waves: int = 4, half: bool = False):
    """Host-side machine code of the 64-row image (one M row per lane, VOP2
    adds, k-quad X^T; include/ternary_spgemm_test.h tsg_jit_codegen64); half:
    its half ring (4 waves, 96-row chunks; tsg_jit_codegen64h)."""
    csp, csn, rip, rin = _i32(csp), _i32(csn), _i32(rip), _i32(rin)
    nc, nw = C.c_int64(), C.c_int64()
    L = lib()

    def gen(code, cap_c, wcode, cap_w):
        if half:
            if waves != 4:
                raise TSGError(-1, "tsg_jit_codegen64h", "the half ring runs 4-wave workgroups")
            return L.tsg_jit_codegen64h(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, width, code, cap_c,
                                        C.byref(nc), wcode, cap_w, C.byref(nw))
        return L.tsg_jit_codegen64(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, width, waves, code, cap_c,
                                   C.byref(nc), wcode, cap_w, C.byref(nw))
    _check(gen(None, 0, None, 0), "tsg_jit_codegen64")
    code = np.empty(nc.value, np.uint32)
    wcode = np.empty(nw.value, np.uint32)
    _check(gen(_ptr(code), nc.value, _ptr(wcode), nw.value), "tsg_jit_codegen64")
    return code, wcode


def jit_codegen_far(csp, csn, rip, rin, K: int, N: int):
    """The far-X^T image of the 64-wide plain-TCSC code (no code touches,
    non-temporal X^T staging; include/ternary_spgemm.h tcsc_hip_set_far)."""
    csp, csn, rip, rin = _i32(csp), _i32(csn), _i32(rip), _i32(rin)
    nc, nw = C.c_int64(), C.c_int64()
    L = lib()
    _check(L.tsg_jit_codegen_far(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, None, 0, C.byref(nc), None, 0,
                                 C.byref(nw)), "tsg_jit_codegen_far")
    code = np.empty(nc.value, np.uint32)
    wcode = np.empty(nw.value, np.uint32)
    _check(L.tsg_jit_codegen_far(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, _ptr(code), nc.value,
                                 C.byref(nc), _ptr(wcode), nw.value, C.byref(nw)), "tsg_jit_codegen_far")
    return code, wcode


def call_plan(K: int, N: int, nnz: int, M: int) -> dict:
    """The automatic per-call plan of a plain-TCSC handle (host only):
    kernel, jit stream width x waves, far-X^T image, tile-map groups and
    code-touch mask (include/ternary_spgemm.h tsg_call_plan)."""
    v = [C.c_int() for _ in range(7)]
    _check(lib().tsg_call_plan(K, N, nnz, M, *[C.byref(x) for x in v]), "tsg_call_plan")
    kernel, width, waves, far, gn, gm, tmask = (x.value for x in v)
    return {"kernel": ("tsg_jit_kernel", "tsg_tcsc_ell_kernel", "tsg_tcsc_ell_pc_kernel", "tsg_jit64_kernel")[kernel],
            "width": width, "waves": waves, "far": bool(far), "map": (gn, gm), "tmask": tmask}


def call_xtouch(K: int, N: int, nnz: int, M: int) -> bool:
    """Whether an M-row call spreads the generated code's per-group code
    touches over the lines (tsg_call_xtouch, host only)."""
    r = lib().tsg_call_xtouch(K, N, nnz, M)
    _check(min(r, 0), "tsg_call_xtouch")
    return bool(r)


def jit_tile_map(L: int, mtiles: int, ntiles: int, gn: int, gm: int):
    """(column tile, M tile) of workgroup L in the weight-compiled kernel's
    grid (tsg_jit_map.h), groups of gn column tiles x gm M tiles per XCD."""
    nt, mt = C.c_int(), C.c_int()
    _check(lib().tsg_jit_tile_map(L, mtiles, ntiles, gn, gm, C.byref(nt), C.byref(mt)), "tsg_jit_tile_map")
    return nt.value, mt.value


def ell_build(csp, csn, rip, rin, K: int, N: int, Cmax: int, MT: int, copies: int = 1, with_xb: bool = False):
    """Host view of the small-M kernel's sliced-ELL image for an M tile of MT
    rows (tsg_ell.hip): (entries uint16[] = LDS float indices, tab
    uint32[slices*steps, 2], C, nch), and the second X^T copy's float offset
    xb when with_xb (copies=2: MT = 8 only, tsg_internal.h ell_copy_offset)."""
    csp, csn, rip, rin = _i32(csp), _i32(csn), _i32(rip), _i32(rin)
    ne, nt, c, nch, xb = C.c_int64(), C.c_int64(), C.c_int32(), C.c_int32(), C.c_int32()
    L = lib()
    _check(L.tsg_ell_build(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, Cmax, MT, copies, None, 0, C.byref(ne),
                           None, 0, C.byref(nt), C.byref(c), C.byref(nch), C.byref(xb)), "tsg_ell_build")
    ent = np.empty(ne.value, np.uint32)
    tab = np.empty(nt.value, np.uint32)
    _check(L.tsg_ell_build(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, Cmax, MT, copies, _ptr(ent), ne.value,
                           C.byref(ne), _ptr(tab), nt.value, C.byref(nt), C.byref(c), C.byref(nch), C.byref(xb)),
           "tsg_ell_build")
    out = (ent.view(np.uint16), tab.reshape(-1, 2), c.value, nch.value)
    return out + (xb.value,) if with_xb else out


def tcsc_to_blocked(csp, csn, rip, rin, K: int, N: int, B: int):
    """TCSC -> BlockedTCSC<B> arrays (the layout BlockedTCSC.h:15-41 builds from
    the dense W): slot kb*N + n = column n's rows of block kb, K/B whole blocks,
    rows past (K/B)*B dropped.  Vectorised host conversion (numpy)."""
    nb = K // B
    out = []
    for cs, ri in ((_i32(csp), _i32(rip)), (_i32(csn), _i32(rin))):
        col = np.repeat(np.arange(N, dtype=np.int64), np.diff(cs[: N + 1]))
        blk = ri[: cs[N]].astype(np.int64) // B
        keep = blk < nb
        slot = blk[keep] * N + col[keep]
        order = np.argsort(slot, kind="stable")  # within a slot: ascending k as in the column
        starts = np.zeros(nb * N + 1, np.int32)
        np.cumsum(np.bincount(slot, minlength=nb * N), out=starts[1:])
        out.append((starts, ri[: cs[N]][keep][order].astype(np.int32)))
    return out[0][0], out[1][0], out[0][1], out[1][1]


def validate_blocked(csp, csn, rip, rin, K: int, N: int, B: int) -> None:
    """Raises TSGError unless the arrays are a well-formed BlockedTCSC<B>."""
    csp, csn, rip, rin = _i32(csp), _i32(csn), _i32(rip), _i32(rin)
    _check(lib().tsg_blocked_tcsc_validate(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), K, N, B),
           "tsg_blocked_tcsc_validate")


def encode_dense_torch(W):
    """GPU-side TCSC encoder (TCSC.h:13-41 on the device): W is a [K, N] int32
    CUDA tensor; returns (csp, csn, rip, rin) as int32 CUDA tensors on W's device,
    on the current stream (tcsc_hip_encode_dense_dev)."""
    import torch
    assert W.is_cuda and W.dtype == torch.int32 and W.dim() == 2 and W.is_contiguous()
    K, N = W.shape
    dev = W.device
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    p, q = C.c_int64(), C.c_int64()
    s = torch.cuda.current_stream(dev).cuda_stream
    L = lib()
    _check(L.tcsc_hip_encode_dense_dev(W.data_ptr(), K, N, csp.data_ptr(), csn.data_ptr(), None, 0, None, 0,
                                       C.byref(p), C.byref(q), s), "tcsc_hip_encode_dense_dev")
    rip = torch.empty(max(p.value, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(q.value, 1), dtype=torch.int32, device=dev)
    _check(L.tcsc_hip_encode_dense_dev(W.data_ptr(), K, N, csp.data_ptr(), csn.data_ptr(), rip.data_ptr(),
                                       rip.numel(), rin.data_ptr(), rin.numel(), C.byref(p), C.byref(q), s),
           "tcsc_hip_encode_dense_dev")
    return csp, csn, rip[: p.value], rin[: q.value]


def gen_x(M: int, K: int, seed: int, rng: int = 512) -> np.ndarray:
    """Integer-valued fp32 X in [-rng, rng] (initX, sparseUtils.h:6-23)."""
    X = np.empty((M, K), np.float32)
    _check(lib().tsg_gen_x(M * K, rng, seed, _ptr(X)), "tsg_gen_x")
    return X


class registered_host:
    """Context manager: page-locks numpy arrays for repeated host-pointer
    calls (tcsc_hip_host_register), unlocks them on exit."""

    def __init__(self, *arrays):
        self.arrays = [a for a in arrays if a is not None and a.size]

    def __enter__(self):
        done = []
        try:
            for a in self.arrays:
                _check(lib().tcsc_hip_host_register(a.ctypes.data, a.nbytes), "tcsc_hip_host_register")
                done.append(a)
        except Exception:
            for a in done:
                lib().tcsc_hip_host_unregister(a.ctypes.data)
            raise
        return self

    def __exit__(self, exc_type, exc, tb):
        # unlock every array even if one fails; report a failure only when the
        # with-block itself did not raise (never mask its exception)
        errors = []
        for a in self.arrays:
            rc = lib().tcsc_hip_host_unregister(a.ctypes.data)
            if rc != TSG_OK:
                errors.append(TSGError(rc, "tcsc_hip_host_unregister", lib().tcsc_hip_last_error().decode(errors="replace")))
        if errors and exc_type is None:
            raise errors[0]
        return False


def device_count() -> int:
    n = C.c_int()
    _check(lib().tcsc_hip_device_count(C.byref(n)), "tcsc_hip_device_count")
    return n.value


# ------------------------------------------------------------------ handle --

class TCSCDevice:
    """One TCSC weight matrix resident on one GPU (tcsc_hip_create)."""

    def __init__(self, csp, csn, rip, rin, K: int, N: int, device: int = -1):
        csp, csn, rip, rin = map(_i32, (csp, csn, rip, rin))
        self.K, self.N = int(K), int(N)
        h = C.c_void_p()
        _check(lib().tcsc_hip_create(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), self.K,
                                     self.N, device, C.byref(h)), "tcsc_hip_create")
        self._h = h

    @classmethod
    def from_csc_packed(cls, col_ptr, row_idx, packed, K: int, N: int,
                        device: int = -1) -> "TCSCDevice":
        """CSC + base-3 packed values (readme.md:111) -> same device image."""
        col_ptr, row_idx = _i32(col_ptr), _i32(row_idx)
        packed = np.ascontiguousarray(packed, dtype=np.uint8)
        self = cls.__new__(cls)
        self.K, self.N = int(K), int(N)
        h = C.c_void_p()
        _check(lib().tcsc_hip_create_csc_packed(_ptr(col_ptr), _ptr(row_idx), _ptr(packed), K, N,
                                                device, C.byref(h)), "tcsc_hip_create_csc_packed")
        self._h = h
        return self

    @classmethod
    def from_blocked(cls, csp, csn, rip, rin, K: int, N: int, B: int,
                     device: int = -1) -> "TCSCDevice":
        """BlockedTCSC<B> arrays (BlockedTCSC.h:15-41): calls compute
        BaseBlockedTCSC (comp.h:607-658) bit for bit (tcsc_hip_create_blocked)."""
        csp, csn, rip, rin = map(_i32, (csp, csn, rip, rin))
        self = cls.__new__(cls)
        self.K, self.N = int(K), int(N)
        h = C.c_void_p()
        _check(lib().tcsc_hip_create_blocked(_ptr(csp), _ptr(csn), _ptr(rip), _ptr(rin), self.K, self.N,
                                             int(B), device, C.byref(h)), "tcsc_hip_create_blocked")
        self._h = h
        return self

    @classmethod
    def from_dense(cls, W, device: int = -1) -> "TCSCDevice":
        W = _i32(W)
        K, N = W.shape
        self = cls.__new__(cls)
        self.K, self.N = int(K), int(N)
        h = C.c_void_p()
        _check(lib().tcsc_hip_create_dense(_ptr(W), K, N, device, C.byref(h)),
               "tcsc_hip_create_dense")
        self._h = h
        return self

    @classmethod
    def from_dense_torch(cls, W, device: int = -1) -> "TCSCDevice":
        """Registration from a dense [K, N] int32 CUDA tensor: the TCSC is built on
        the GPU (encode_dense_torch, TCSC.h:13-41) and compiled from its arrays."""
        csp, csn, rip, rin = encode_dense_torch(W)
        K, N = W.shape
        return cls(csp.cpu().numpy(), csn.cpu().numpy(), rip.cpu().numpy(), rin.cpu().numpy(), K, N,
                   device=W.device.index if device < 0 else device)

    @property
    def device(self) -> int:
        """HIP device index the handle's image lives on (tcsc_hip_info)."""
        if getattr(self, "_device", None) is None:
            self._device = int(self.info()["device"])
        return self._device

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().tcsc_hip_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- comp_func surface (host pointers, synchronous) ----
    def _check_host(self, M: int, N: int, K: int, **arrays) -> None:
        """Host-pointer call contract (main.cpp:214-216): fp32, C-contiguous,
        X holds M*K floats, Y M*N, B (and alpha) N -- checked before the C-ABI
        sees the pointers, so a short buffer raises instead of being overrun."""
        if (N, K) != (self.N, self.K):
            return  # the C-ABI reports the shape mismatch (TSG_ERR_ARG)
        need = {"X": M * K, "B": N, "Y": M * N, "alpha": N}
        for name, a in arrays.items():
            if not isinstance(a, np.ndarray) or a.dtype != np.float32 or not a.flags.c_contiguous:
                raise TSGError(1, "comp_func", f"{name} must be a C-contiguous float32 numpy array")
            if a.size < need[name]:
                raise TSGError(1, "comp_func", f"{name} has {a.size} floats, the call needs {need[name]}")
        X = arrays.get("X")
        if X is not None and X.ndim == 2 and X.shape[1] != K:
            raise TSGError(1, "comp_func", f"X is {X.shape}, rows must have K={K} floats")

    def __call__(self, X, B, Y, M: int, N: int, K: int) -> None:
        """comp_func(X, B, Y, M, N, K) on numpy arrays (common.h:12)."""
        self._check_host(M, N, K, X=X, B=B, Y=Y)
        _check(lib().tcsc_hip_gemm(self._h, X.ctypes.data, B.ctypes.data, Y.ctypes.data, M, N, K),
               "tcsc_hip_gemm")

    def comp_func(self) -> Callable:
        return lambda X, B, Y, M, N, K: self(X, B, Y, M, N, K)

    def prelu(self, X, B, alpha, Y, M: int, N: int, K: int) -> None:
        """comp_func_prelu(X, B, alpha, Y, M, N, K) (common.h:13)."""
        self._check_host(M, N, K, X=X, B=B, alpha=alpha, Y=Y)
        _check(lib().tcsc_hip_gemm_prelu(self._h, X.ctypes.data, B.ctypes.data, alpha.ctypes.data,
                                         Y.ctypes.data, M, N, K), "tcsc_hip_gemm_prelu")

    def gemm(self, X, b) -> np.ndarray:
        X, b = _f32(X), _f32(b)
        M = X.shape[0]
        Y = np.empty((M, self.N), np.float32)
        self(X, b, Y, M, self.N, self.K)
        return Y

    def gemm_prelu(self, X, b, alpha) -> np.ndarray:
        X, b, alpha = _f32(X), _f32(b), _f32(alpha)
        M = X.shape[0]
        Y = np.empty((M, self.N), np.float32)
        self.prelu(X, b, alpha, Y, M, self.N, self.K)
        return Y

    # ---- device pointers (torch tensors), asynchronous on `stream` ----
    def gemm_dev(self, dX: int, db: int, dY: int, M: int, stream: int = 0,
                 dalpha: Optional[int] = None) -> None:
        if dalpha is None:
            _check(lib().tcsc_hip_gemm_dev(self._h, dX, db, dY, M, self.N, self.K, stream or None),
                   "tcsc_hip_gemm_dev")
        else:
            _check(lib().tcsc_hip_gemm_prelu_dev(self._h, dX, db, dalpha, dY, M, self.N, self.K,
                                                 stream or None), "tcsc_hip_gemm_prelu_dev")

    def gemm_torch(self, X, b, Y=None, alpha=None):
        """X [M,K] fp32 cuda tensor -> Y [M,N], enqueued on torch's current stream.
        Every tensor must be float32, contiguous and on the handle's device;
        shapes X (M, K), b (N,), alpha (N,), Y (M, N) are checked here (the
        C-ABI only sees raw pointers)."""
        import torch
        dev = torch.device("cuda", self.device)
        if not (isinstance(X, torch.Tensor) and X.dim() == 2 and X.shape[1] == self.K):
            raise TSGError(1, "gemm_torch", f"X must be a [M, {self.K}] tensor, got "
                                            f"{tuple(X.shape) if isinstance(X, torch.Tensor) else type(X)}")
        M = X.shape[0]
        if Y is None:
            Y = torch.empty((M, self.N), dtype=torch.float32, device=dev)
        for name, t, shape in (("X", X, (M, self.K)), ("b", b, (self.N,)), ("Y", Y, (M, self.N)),
                               ("alpha", alpha, (self.N,))):
            if t is None:
                continue
            if t.dtype != torch.float32 or t.device != dev or not t.is_contiguous() or tuple(t.shape) != shape:
                raise TSGError(1, "gemm_torch", f"{name} must be a contiguous float32 {list(shape)} tensor on "
                                                f"{dev}, got {t.dtype} {list(t.shape)} on {t.device}"
                                                f"{'' if t.is_contiguous() else ' (non-contiguous)'}")
        stream = torch.cuda.current_stream(dev).cuda_stream
        self.gemm_dev(X.data_ptr(), b.data_ptr(), Y.data_ptr(), M, stream,
                      None if alpha is None else alpha.data_ptr())
        return Y

    def reserve(self, max_M: int) -> None:
        _check(lib().tcsc_hip_reserve(self._h, max_M), "tcsc_hip_reserve")

    def jit_width(self, M: int) -> int:
        """Columns per stream a call with M rows runs (0: not the jit kernel)."""
        return int(lib().tcsc_hip_jit_width(self._h, M))

    def jit_waves(self, M: int) -> int:
        """Waves per workgroup of that call's jit image (8, or 4 at mid M)."""
        return int(lib().tcsc_hip_jit_waves(self._h, M))

    def set_jit_width(self, width: int) -> None:
        """0 = automatic per call (default); 64/32/16/8 pins the stream width."""
        _check(lib().tcsc_hip_set_jit_width(self._h, width), "tcsc_hip_set_jit_width")

    def set_small_m(self, mode: int) -> None:
        """Small-M kernel: 0 = automatic (default), 1 = never, 2 = every call,
        3 = every call without the producer/consumer walk (M <= 4)."""
        _check(lib().tcsc_hip_set_small_m(self._h, mode), "tcsc_hip_set_small_m")

    def set_host_chunks(self, chunks: int) -> None:
        """Host-pointer calls: 0 = automatic M-chunk pipeline (default), n =
        force n chunks (1 = one H2D / compute / D2H, no overlap)."""
        _check(lib().tcsc_hip_set_host_chunks(self._h, chunks), "tcsc_hip_set_host_chunks")

    def host_chunk_rows(self, M: int) -> int:
        """Rows per chunk of a host-pointer call with M rows (M = unchunked)."""
        return int(lib().tcsc_hip_host_chunk_rows(self._h, M))

    def call_image_bytes(self, M: int) -> int:
        """Device image bytes a call with M rows reads (ELL image or generated
        code; 0 if not built yet)."""
        return int(lib().tcsc_hip_call_image_bytes(self._h, M))

    def call_kernel(self, M: int) -> str:
        """Device kernel a call with M rows launches."""
        return lib().tcsc_hip_call_kernel(self._h, M).decode()

    def set_far(self, mode: int) -> None:
        """Far-X^T code image: 0 = automatic (default), 1 = never, 2 = every
        64-wide call."""
        _check(lib().tcsc_hip_set_far(self._h, mode), "tcsc_hip_set_far")

    def set_tile_rows(self, rows: int) -> None:
        """Weight-compiled image: 0 = automatic (default), 64 = the 64-row
        image (one row per lane, VOP2 adds), 128 = the 128-row image."""
        _check(lib().tcsc_hip_set_tile_rows(self._h, rows), "tcsc_hip_set_tile_rows")

    def call_tile_rows(self, M: int) -> int:
        """M tile (64 / 128) of the weight-compiled image a call with M rows
        runs; 0 when it runs a small-M walk."""
        return int(lib().tcsc_hip_call_tile_rows(self._h, M))

    def call_launches(self, X, M: int) -> int:
        """Device kernels a device-pointer call with M rows and this X (a cuda
        tensor or a device pointer) launches: 1 (the kernel reads X itself) or
        2 (an X^T staging kernel first)."""
        ptr = X.data_ptr() if hasattr(X, "data_ptr") else int(X)
        return int(lib().tcsc_hip_call_launches(self._h, C.c_void_p(ptr), M))

    def call_far(self, M: int) -> bool:
        """True if a call with M rows runs the far-X^T image."""
        return bool(lib().tcsc_hip_call_far(self._h, M))

    def info(self) -> dict:
        o = tsg_info()
        _check(lib().tcsc_hip_info(self._h, C.byref(o)), "tcsc_hip_info")
        return {f: getattr(o, f) for f, _ in tsg_info._fields_}

    def kernel_name(self) -> str:
        """Device kernel this handle launches (default: the weight-compiled tsg_jit_kernel)."""
        return lib().tcsc_hip_kernel_name(self._h).decode()

    def to_dense(self) -> np.ndarray:
        """getVectorRepresentation (DataStructureInterface.hpp:13)."""
        W = np.empty((self.K, self.N), np.int32)
        _check(lib().tcsc_hip_to_dense(self._h, _ptr(W), self.K, self.N), "tcsc_hip_to_dense")
        return W

    def set_timing(self, on: bool) -> None:
        _check(lib().tcsc_hip_set_timing(self._h, int(bool(on))), "tcsc_hip_set_timing")

    def kernel_time(self, reset: bool = False) -> Tuple[float, int]:
        ms, n = C.c_double(), C.c_int64()
        _check(lib().tcsc_hip_kernel_time(self._h, C.byref(ms), C.byref(n), int(reset)),
               "tcsc_hip_kernel_time")
        return ms.value, n.value


# ------------------------------------------------------- plugin registry --
# Mirrors main.cpp:12-33: global lists of callables + names; "BaseTCSC" is the
# speedup baseline name there (main.cpp:10).

userFuncs: List[Callable] = []
funcNames: List[str] = []
userFuncs_prelu: List[Callable] = []
funcNames_prelu: List[str] = []


def add_function(f: Callable, name: str) -> None:
    userFuncs.append(f)
    funcNames.append(name)


def add_prelu_function(f: Callable, name: str) -> None:
    userFuncs_prelu.append(f)
    funcNames_prelu.append(name)


def clear_registry() -> None:
    for lst in (userFuncs, funcNames, userFuncs_prelu, funcNames_prelu):
        lst.clear()


# --------------------------------------------------------------- metrics --

def flops(M: int, N: int, nnz: int) -> int:
    """Instrumented add/sub count of BaseTCSC (comp.h:28-31,48-50,63):
    one per nonzero per row plus the bias add = M*(nnz + N) = M*N*(K/s+1)."""
    return M * (nnz + N)


def algorithmic_bytes(M: int, N: int, K: int, nnz: int) -> int:
    """main.cpp:267 + TCSC.h:43-49: X, Y, b once, plus the TCSC arrays."""
    return 4 * (M * K + M * N + N) + 4 * (2 * (N + 1) + nnz)
