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
    if w0 in (0x807CFF53, 0x8058FF5C):
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


if __name__ == "__main__":
    main()
