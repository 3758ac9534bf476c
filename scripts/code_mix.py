#!/usr/bin/env python3
"""Instruction mix of the weight-compiled code (CPU, no GPU): bytes and counts by
class per shape, to see what besides the adds the instruction caches must
supply.   python scripts/code_mix.py [M,K,N,s,width,waves ...]"""
import collections
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ternary-spgemm_amd")]
import tspgemm as T  # noqa: E402


def classify(code, i):
    w0 = int(code[i])
    if (w0 & 0xFFFFFC00) == 0xD3B24000:
        return "pk_add", 2
    if (w0 & 0xFFFF0000) in (0xD8EC0000, 0xD9FE0000):
        return "ds_read", 2
    if (w0 & 0xFFFFF000) == 0xDDF48000:
        return "dma", 2
    if w0 == 0xDC508000:
        return "touch", 2
    if w0 in (0x807CFF53, 0x8058FF5A):
        return "salu_lit", 2
    if w0 == 0xBF800000:
        return "pad_nop0", 1
    if (w0 & 0xFFFFFFF0) == 0xBF800000:
        return "nop", 1
    if (w0 & 0xFFFF0000) == 0xBF8C0000:
        return "waitcnt", 1
    if w0 == 0xBF8A0000:
        return "barrier", 1
    return "salu", 1


def main():
    shapes = sys.argv[1:] or ["512,4096,4096,4,16,4", "4096,4096,16384,4,64,8", "4096,4096,16384,16,64,8",
                              "4096,4096,16384,8,64,8"]
    for sh in shapes:
        M, K, N, s, w, wv = map(int, sh.split(","))
        arrs = T.gen_tcsc(K, N, s, 42)
        code, wcode = T.jit_codegen(*arrs, K, N, width=w, waves=wv)
        end = len(code) - (32768 + 1024)  # the tail padding (tsg_jit.cpp kTailPad)
        cnt, byt = collections.Counter(), collections.Counter()
        i = int(wcode[0]) // 4
        while i < end:
            k, n = classify(code, i)
            cnt[k] += 1
            byt[k] += 4 * n
            i += n
        tot = sum(byt.values())
        print(f"{sh}: {tot / 1e6:.1f} MB of code, {byt['pk_add'] / tot:.3f} of the bytes are adds; "
              + ", ".join(f"{k} {cnt[k]} ({byt[k] / tot:.3f})" for k in sorted(byt, key=lambda k: -byt[k])))


def classify64(code, i):
    """the 64-row image's instruction classes by encoding family (gfx950)"""
    w0 = int(code[i])
    if not (w0 >> 31):  # VOP2: v_add_f32 (op 1) / v_sub_f32 (op 2) are the adds
        op = (w0 >> 25) & 0x3F
        return ("add" if op in (1, 2) else "vop2"), 1
    top = w0 >> 26
    if top == 0x36:
        return "ds_read", 2
    if top == 0x37:
        return "vmem (dma / touch)", 2
    if (w0 >> 28) in (0xD,) or top in (0x34, 0x35):
        return "vop3", 2
    if (w0 & 0xFF800000) == 0xBF800000:  # SOPP
        op = (w0 >> 16) & 0x7F
        return {0: "nop", 0xC: "waitcnt", 0xA: "barrier", 0xF: "setprio"}.get(op, "sopp"), 1
    if (w0 & 0xFF800000) == 0xBE800000:  # SOP1
        return "salu", 2 if (w0 & 0xFF) == 0xFF else 1
    if (w0 >> 30) == 2:  # SOP2
        return "salu", 2 if ((w0 & 0xFF) == 0xFF or ((w0 >> 8) & 0xFF) == 0xFF) else 1
    return "other", 1


def main64(shapes):
    """python scripts/code_mix.py --r64 [K,N,s,width,waves ...]: the 64-row image"""
    for sh in shapes or ["4096,4096,4,16,8", "4096,16384,4,128,8", "4096,16384,8,128,8", "4096,16384,16,128,8"]:
        K, N, s, w, wv = map(int, sh.split(","))
        arrs = T.gen_tcsc(K, N, s, 42)
        code, wcode = T.jit_codegen64(*arrs, K, N, width=w, waves=wv)
        end = len(code) - (32768 + 1024)  # the tail padding (tsg_jit.cpp kTailPad)
        cnt, byt = collections.Counter(), collections.Counter()
        i = int(wcode[0]) // 4
        while i < end:
            k, n = classify64(code, i)
            cnt[k] += 1
            byt[k] += 4 * n
            i += n
        tot = sum(byt.values())
        print(f"{sh}: {tot / 1e6:.1f} MB of code, {byt['add'] / tot:.3f} of the bytes are adds; "
              + ", ".join(f"{k} {cnt[k]} ({byt[k] / tot:.3f})" for k in sorted(byt, key=lambda k: -byt[k])))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--r64":
    main64(sys.argv[2:])
    sys.exit(0)


if __name__ == "__main__":
    main()
