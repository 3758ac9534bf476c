#!/bin/bash
# TSG_JIT_DIAG code variants exist only in the diagnostic build (make -C ternary-spgemm_amd diag)
export TSG_LIB=${TSG_LIB:-ternary-spgemm_amd/lib/libternary_spgemm_diag.so}
# GPU box: does the sparse end wait on the LDS-DMA's latency?  configs[3] at
# s = 8 and 16: default, the pieces never waited for (TSG_JIT_DIAG=novm,
# results WRONG, timing only), lag 2, no DMA (nodma, WRONG).  Kernel ms
# (configs.py), two repetitions.  Usage: scripts/sparse_lag_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/sparse_lag_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for v in default TSG_JIT_DIAG=novm TSG_JIT_DMA=0.5,1,2 TSG_JIT_DIAG=nodma; do
    envs=""; [ "$v" = default ] || envs="$v"
    env $envs timeout -k 10 150 python scripts/configs.py --shape 4096,4096,16384,8 --shape 4096,4096,16384,16 --steps 10 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT"
    rc=$?; [ $rc -eq 0 ] || { echo "$v failed rc=$rc"; exit $rc; }
    echo "rep $rep [$v]: $(tail -n 2 "$OUT" | grep -o '"kernel_ms": [0-9.]*' | cut -d' ' -f2 | tr '\n' ' ')"
  done
done
