#!/bin/bash
# GPU box: the weight-compiled kernel's tile map (TSG_JIT_GN x TSG_JIT_GM: column
# tiles x M tiles per XCD group) against density: X^T slab re-staging vs code
# streaming.  Kernel time per (shape, map), 2 alternating reps.
# Usage: scripts/map_density_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/map_density_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
SH="--shape 4096,4096,16384,16 --shape 4096,4096,16384,8 --shape 4096,4096,16384,4 --shape 4096,4096,16384,2 --shape 512,4096,4096,4 --shape 1024,4096,16384,4"
for rep in 1 2; do
  for m in default 1,32 2,16 4,8 8,4 16,2 32,1; do
    if [ $m = default ]; then unset TSG_JIT_GN TSG_JIT_GM; else export TSG_JIT_GN=${m%,*} TSG_JIT_GM=${m#*,}; fi
    timeout -k 10 170 python scripts/configs.py $SH --steps 20 2>/dev/null | sed "s/^/map=$m rep=$rep /" >> "$OUT" || { echo "map $m failed"; exit 1; }
    echo "rep $rep map=$m done"
  done
done
unset TSG_JIT_GN TSG_JIT_GM
for m in default 1,32 4,8 8,4 8,1 1,8; do
  if [ $m = default ]; then unset TSG_JIT_GN TSG_JIT_GM; else export TSG_JIT_GN=${m%,*} TSG_JIT_GM=${m#*,}; fi
  timeout -k 10 170 python scripts/configs.py --shape 64000,16384,4096,4 --steps 4 2>/dev/null | sed "s/^/map=$m rep=1 /" >> "$OUT" || { echo "big map $m failed"; exit 1; }
  echo "big map=$m done"
done
