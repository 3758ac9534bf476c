#!/bin/bash
# GPU box: the "far X^T" code image (no code touches, non-temporal X^T DMA:
# TSG_JIT_TOUCH=1,0 TSG_JIT_CP=20000,0) and each half of it, against the
# default image, on long-K shapes whose X^T is far larger than the 256 MiB
# Infinity Cache; each shape in its own process, two repetitions.  Kernel ms
# (configs.py, bit-checked rows).  Usage: scripts/far_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/far_ab.txt}
export TMPDIR=/tmp TSG_JIT_FAR=0  # the env knobs below, not the automatic far image
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for sh in 64000,16384,4096,8 64000,16384,4096,16 32000,16384,4096,4 16000,16384,4096,4 64000,8192,4096,4; do
    for v in default TSG_JIT_TOUCH=1,0:TSG_JIT_CP=20000,0 TSG_JIT_TOUCH=1,0 TSG_JIT_CP=20000,0; do
      envs=""; [ "$v" = default ] || envs="${v//:/ }"
      env $envs timeout -k 10 150 python scripts/configs.py --shape $sh --steps 3 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT"
      rc=$?; [ $rc -eq 0 ] || { echo "$sh $v failed rc=$rc"; exit $rc; }
      echo "rep $rep $sh [$v]: $(tail -n 1 "$OUT" | grep -o '"kernel_ms": [0-9.]*')"
    done
  done
done
timeout -k 10 150 python scripts/configs.py --shape 512,4096,4096,4 --shape 1024,4096,1024,4 --shape 4096,4096,16384,4 --steps 10 2>/dev/null | sed "s/^/[tmask rule] /" >> "$OUT" && echo "tmask rule: $(tail -n 3 "$OUT" | grep -o '"kernel_ms": [0-9.]*' | tr '\n' ' ')"
