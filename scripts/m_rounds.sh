#!/bin/bash
# GPU box: kernel time vs M at configs[2]'s K, N (workgroup rounds = M / 1024 at
# 256 CUs): intercept = per-launch fixed cost, slope = cost of one round.
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/m_rounds_${1:-x}.txt; : > $OUT
for rep in 1 2; do
  for M in 1024 2048 3072 4096 6144 8192; do
    timeout -k 10 120 python bench.py --M $M --steps 20 --warmup 3 --cpu-rows 0 > /tmp/mr.log 2>&1 || { echo "M=$M failed"; tail -3 /tmp/mr.log; exit 1; }
    python3 - $M $rep >> $OUT <<'P'
import json, sys
d = json.loads([l for l in open("/tmp/mr.log") if l.startswith("{")][-1])
print(sys.argv[2], "M", sys.argv[1], "kernel_ms", d["roofline"]["kernel_ms"], "valu", d["roofline"]["binding"]["frac"], "ms_step", d["ms_per_step"])
P
    tail -1 $OUT
  done
done
