#!/bin/bash
# GPU box: tile-map groups (TSG_JIT_GN x TSG_JIT_GM) on the mid-M shapes with the
# round-3 code-touch thinning; two repetitions.  Kernel ms (configs.py,
# bit-checked rows).  Usage: scripts/mid_map_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/mid_map_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for v in default TSG_JIT_GN=1:TSG_JIT_GM=4 TSG_JIT_GN=2:TSG_JIT_GM=4 TSG_JIT_GN=8:TSG_JIT_GM=4 TSG_JIT_GN=16:TSG_JIT_GM=4 TSG_JIT_GN=2:TSG_JIT_GM=16; do
    envs=""; [ "$v" = default ] || envs="${v//:/ }"
    env $envs timeout -k 10 150 python scripts/configs.py --shape 512,4096,4096,4 --shape 1024,4096,1024,4 --shape 1024,16384,1024,4 --steps 20 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT"
    rc=$?; [ $rc -eq 0 ] || { echo "$v failed rc=$rc"; exit $rc; }
    echo "rep $rep [$v]: $(tail -n 3 "$OUT" | grep -o '"kernel_ms": [0-9.]*' | cut -d' ' -f2 | tr '\n' ' ')"
  done
done
