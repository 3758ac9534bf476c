#!/bin/bash
# GPU box: X read schedule (TSG_JIT_READS="G,RA": group size, read-ahead in
# slots of 24) and code-prefetch window (TSG_JIT_TOUCH="first,count" in 8-KiB
# units) at the sparse end, mid M and configs[2].  Kernel ms (configs.py), 2 reps.
# Usage: scripts/reads_touch_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/reads_touch_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
SH="--shape 4096,4096,16384,16 --shape 4096,4096,16384,8 --shape 512,4096,4096,4 --shape 4096,4096,16384,4"
for rep in 1 2; do
  for v in "default" "TSG_JIT_READS=12,12" "TSG_JIT_READS=6,18" "TSG_JIT_READS=4,20" "TSG_JIT_TOUCH=2,1" "TSG_JIT_TOUCH=1,2" "TSG_JIT_TOUCH=2,2" "TSG_JIT_TOUCH=3,1"; do
    envs=""; [ "$v" = default ] || envs="$v"
    env $envs timeout -k 10 170 python scripts/configs.py $SH --steps 20 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT" || { echo "variant $v failed"; exit 1; }
  done
  echo "rep $rep done"
done
