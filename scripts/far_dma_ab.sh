#!/bin/bash
# GPU box: DMA-issue variants of the far-X^T image (TSG_JIT_DMA="spread,m0k,lag")
# on the shapes that run it; each in its own process, two repetitions.
# Kernel ms (configs.py, bit-checked rows).  Usage: scripts/far_dma_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/far_dma_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for v in default TSG_JIT_DMA=0,1,1 TSG_JIT_DMA=0.25,1,1 TSG_JIT_DMA=0.75,1,1 TSG_JIT_DMA=0.5,1,2; do
    envs=""; [ "$v" = default ] || envs="$v"
    for sh in 64000,16384,4096,4 32000,16384,4096,4; do
      env $envs timeout -k 10 150 python scripts/configs.py --shape $sh --steps 3 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT"
      rc=$?; [ $rc -eq 0 ] || { echo "$sh $v failed rc=$rc"; exit $rc; }
      echo "rep $rep $sh [$v]: $(tail -n 1 "$OUT" | grep -o '"kernel_ms": [0-9.]*')"
    done
  done
done
