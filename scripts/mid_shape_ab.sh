#!/bin/bash
# GPU box: (width x waves) shapes at mid M with the round-3 touch thinning:
# automatic pick vs pinned widths (TSG_JIT_NW; TSG_JIT_WAVES=4 for 4-wave
# workgroups).  Kernel ms (configs.py, bit-checked rows), two repetitions.
# Usage: scripts/mid_shape_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/mid_shape_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for v in default TSG_JIT_NW=16 TSG_JIT_NW=32:TSG_JIT_WAVES=4 TSG_JIT_NW=8 TSG_JIT_NW=8:TSG_JIT_WAVES=4 TSG_JIT_NW=32; do
    envs=""; [ "$v" = default ] || envs="${v//:/ }"
    env $envs timeout -k 10 150 python scripts/configs.py --shape 512,4096,4096,4 --shape 1024,4096,1024,4 --shape 256,4096,16384,4 --steps 20 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT"
    rc=$?; [ $rc -eq 0 ] || { echo "$v failed rc=$rc"; exit $rc; }
    echo "rep $rep [$v]: $(tail -n 3 "$OUT" | grep -o '"kernel_ms": [0-9.]*' | cut -d' ' -f2 | tr '\n' ' ')"
  done
done
