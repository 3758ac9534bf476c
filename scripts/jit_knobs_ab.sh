#!/bin/bash
# GPU box: A/B of the weight-compiled kernel's generator knobs (env at
# registration) at config 3, interleaved repeats, kernel ms from the bench line.
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/knobs_${1:-x}.txt; shift || true
: > $OUT
for rep in 1 2; do
  for v in "$@"; do
    env $(echo "$v" | tr '|' ' ') timeout -k 10 120 python bench.py --steps 30 --warmup 3 --cpu-rows 0 > /tmp/ab.log 2>&1 || { echo "$v failed"; tail -3 /tmp/ab.log; exit 1; }
    python3 - "$v" "$rep" >> $OUT <<'P'
import json, sys
d = json.loads([l for l in open("/tmp/ab.log") if l.startswith("{")][-1])
print(sys.argv[2], sys.argv[1], "kernel_ms", d["roofline"]["kernel_ms"], "valu", d["roofline"]["binding"]["frac"], "ms_step", d["ms_per_step"])
P
    tail -1 $OUT
  done
done
