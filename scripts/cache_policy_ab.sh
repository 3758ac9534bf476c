#!/bin/bash
# GPU box: cache policy of the X^T LDS-DMA pieces and the code touches
# (TSG_JIT_CP="dma,touch" hex bits, 0x20000 nt, 0x2000000 sc1) and no code
# touches (TSG_JIT_TOUCH=1,0), on the large reference shapes and the BASELINE
# configs.  Kernel ms (configs.py).  Usage: scripts/cache_policy_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/cache_policy_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
VARS="default TSG_JIT_TOUCH=1,0 TSG_JIT_CP=20000,0 TSG_JIT_CP=2000000,0 TSG_JIT_CP=0,20000 TSG_JIT_CP=20000,20000"
for v in $VARS; do
  envs=""; [ "$v" = default ] || envs="$v"
  env $envs timeout -k 10 170 python scripts/configs.py --shape 64000,16384,4096,4 --shape 64000,16384,4096,8 --steps 3 2>/dev/null | sed "s/^/[$v] rep=1 /" >> "$OUT" || { echo "variant $v big failed"; exit 1; }
  for rep in 1 2; do
    env $envs timeout -k 10 170 python scripts/configs.py --shape 16000,8192,2048,4 --shape 4096,4096,16384,4 --shape 512,4096,4096,4 --shape 4096,4096,16384,16 --shape 1024,16384,1024,4 --steps 20 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT" || { echo "variant $v failed"; exit 1; }
  done
  echo "variant $v done"
done
