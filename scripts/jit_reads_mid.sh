#!/bin/bash
# GPU box: configs[1] (M = 512, jit width 8) kernel time by read schedule
# (TSG_JIT_READS="G,RA": group size, read-ahead; S = 24 X slots).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${1:-x}_jit_reads_mid.txt
: > $out
for gr in "8,16" "4,20" "2,22" "12,12" "6,18"; do
  echo "# TSG_JIT_READS=$gr" >> $out
  TSG_JIT_READS=$gr timeout -k 10 120 python scripts/configs.py --only "configs[1]" >> $out 2>&1 || exit 1
  TSG_JIT_READS=$gr timeout -k 10 120 python scripts/configs.py --only "sweep M=256" >> $out 2>&1 || exit 1
done
