#!/bin/bash
# TSG_JIT_DIAG code variants exist only in the diagnostic build (make -C ternary-spgemm_amd diag)
export TSG_LIB=${TSG_LIB:-ternary-spgemm_amd/lib/libternary_spgemm_diag.so}
# GPU box: where the per-step time of the weight-compiled kernel goes at mid M
# (configs[1], M = 256, M = 64 forced to jit) and at configs[2]: kernel time of
# the TSG_JIT_DIAG code variants (tsg_jit.cpp; diagnostic, results WRONG, the
# bit flag of each line is meaningless for them).
# Usage: scripts/jit_diag_mid.sh <out file>
set -o pipefail
OUT=${1:-gpurun_out/jit_diag_mid.txt}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
export TSG_KERNEL=jit
for d in "" nobar nodma notouch nolgkm noreads nobar,nodma "nobar,nodma,nolgkm,notouch"; do
  for sh in "configs[1]" "sweep M=64" "sweep M=256" "configs[2]"; do
    line=$(TSG_JIT_DIAG=$d timeout -k 10 150 python scripts/configs.py --only "$sh" --steps 10 2>/dev/null | tail -1) || { echo "diag=[$d] $sh failed"; exit 1; }
    echo "diag=[$d] $line" >> "$OUT"
  done
  echo "diag=[$d] done"
done
