#!/bin/bash
# GPU box: kernel time of jit variants: each arg is "<lib dir>:<TSG_JIT_READS>[:<TSG_JIT_TOUCH>]".
for v in "$@"; do
  IFS=: read -r lib reads touch <<< "$v"
  echo "$v $(TSG_LIB=ternary-spgemm_amd/$lib/libternary_spgemm.so TSG_JIT_READS=$reads TSG_JIT_TOUCH=${touch:-1,2} timeout -k 10 120 python scripts/diag_stamps.py 2>/dev/null | grep 'kernel ms')" || exit 1
done
