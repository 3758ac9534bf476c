#!/bin/bash
# GPU box: configs[3] at s = 2 (dense W: 268 MB of code, past the Infinity
# Cache) and s = 4 under DMA-issue spreads (TSG_JIT_DMA="spread,m0k,lag"):
# round 2 ran s = 2 in 2.44 ms with every piece at the step start, round 3's
# default spread 0.5 in 2.55.  Kernel ms (configs.py), two repetitions.
# Usage: scripts/s2_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/s2_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for v in default TSG_JIT_DMA=0,1,1 TSG_JIT_DMA=0.25,1,1 TSG_JIT_DMA=0.5,0,1 TSG_JIT_DMA=0,0,1; do
    envs=""; [ "$v" = default ] || envs="$v"
    env $envs timeout -k 10 150 python scripts/configs.py --shape 4096,4096,16384,2 --shape 4096,4096,16384,4 --shape 256,4096,16384,2 --shape 256,4096,16384,4 --steps 10 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT"
    rc=$?; [ $rc -eq 0 ] || { echo "$v failed rc=$rc"; exit $rc; }
    echo "rep $rep [$v]: $(tail -n 4 "$OUT" | grep -o '"kernel_ms": [0-9.]*' | tr '\n' ' ')"
  done
done
