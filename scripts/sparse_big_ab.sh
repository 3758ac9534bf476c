#!/bin/bash
# GPU box: the reference's largest shape with sparse W (s = 8, 16) under the
# tile maps and the far-X^T image: default (4 x 8 map), 1 x 32, 1 x 32 + far,
# 2 x 16 (+ far); each shape in its own process, two repetitions.  Kernel ms
# (configs.py, bit-checked rows).  Usage: scripts/sparse_big_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/sparse_big_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for sh in 64000,16384,4096,8 64000,16384,4096,16; do
    for v in default TSG_JIT_GN=1:TSG_JIT_GM=32 TSG_JIT_GN=1:TSG_JIT_GM=32:TSG_JIT_FAR=1 TSG_JIT_GN=2:TSG_JIT_GM=16 TSG_JIT_GN=4:TSG_JIT_GM=8:TSG_JIT_FAR=1; do
      envs=""; [ "$v" = default ] || envs="${v//:/ }"
      env $envs timeout -k 10 150 python scripts/configs.py --shape $sh --steps 3 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT"
      rc=$?; [ $rc -eq 0 ] || { echo "$sh $v failed rc=$rc"; exit $rc; }
      echo "rep $rep $sh [$v]: $(tail -n 1 "$OUT" | grep -o '"kernel_ms": [0-9.]*')"
    done
  done
done
