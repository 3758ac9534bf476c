#!/bin/bash
# TSG_JIT_DIAG code variants exist only in the diagnostic build (make -C ternary-spgemm_amd diag)
export TSG_LIB=${TSG_LIB:-ternary-spgemm_amd/lib/libternary_spgemm_diag.so}
# GPU box: is the weight-compiled kernel's step waiting on the LDS-DMA's
# latency or paying for its issue?  Kernel ms (configs.py) of configs[1], M = 64
# and 256 (K = 4096, N = 16384, the weight-compiled kernel forced), configs[2]
# under: the DMA never waited for (TSG_JIT_DIAG=novm, results WRONG), no DMA
# (nodma, WRONG), lag 2 (pieces waited one step later), and other spreads.
# Usage: scripts/lag_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/lag_ab.txt}
export TMPDIR=/tmp TSG_KERNEL=jit
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for v in default TSG_JIT_DIAG=novm TSG_JIT_DIAG=nodma TSG_JIT_DMA=0.5,1,2 TSG_JIT_DMA=0.25,1,1 TSG_JIT_DMA=0,1,1 TSG_JIT_DIAG=novm,nobar; do
  envs=""; [ "$v" = default ] || envs="$v"
  env $envs timeout -k 10 200 python scripts/configs.py --shape 512,4096,4096,4 --shape 64,4096,16384,4 \
      --shape 256,4096,16384,4 --shape 4096,4096,16384,4 --steps 10 2>/dev/null | sed "s/^/[$v] /" >> "$OUT"
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v failed rc=$rc"; exit $rc; }
  echo "variant $v done: $(tail -n 4 "$OUT" | grep -o '"kernel_ms": [0-9.]*' | tr '\n' ' ')"
done
