#!/bin/bash
# TSG_JIT_DIAG code variants exist only in the diagnostic build (make -C ternary-spgemm_amd diag)
export TSG_LIB=${TSG_LIB:-ternary-spgemm_amd/lib/libternary_spgemm_diag.so}
# GPU box: where (64000, 16384, 4096) s=4 waits -- kernel time of the
# TSG_JIT_DIAG code variants (tsg_jit.cpp; results WRONG, timing only).
# Usage: scripts/big_diag.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/big_diag.txt}
export TMPDIR=/tmp TSG_KERNEL=jit
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for d in "" nobar nodma nolgkm notouch noreads nobar,nodma; do
  line=$(TSG_JIT_DIAG=$d timeout -k 10 170 python scripts/configs.py --shape 64000,16384,4096,4 --steps 3 2>/dev/null | tail -1) || { echo "diag=[$d] failed"; exit 1; }
  echo "diag=[$d] $line" >> "$OUT"
  echo "diag=[$d] done"
done
