#!/bin/bash
# GPU box, round 4: the 64-row image's 128 x 8 at configs[3]'s s = 8 / 16
# under its tile map (TSG_JIT_GN x TSG_JIT_GM) and DMA spread (TSG_JIT_DMA)
# alternatives -- one process per setting (the knobs are read once).
# Usage: scripts/r04_sparse_knobs_ab.sh <tag>
set -o pipefail
TAG=${1:-r04y}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/sparse_knobs_$TAG.jsonl; : > $O
run() { echo "{\"env\": \"$1\"}" >> $O; env $1 timeout -k 10 200 python scripts/rows64_ab.py --xint --modes jit64 --K 4096 --N 16384 --M 4096 --s $2 --reps 20 >> $O 2>> gpurun_out/sparse_knobs_$TAG.err; }
for s in 8 16; do
  run "AB_DEFAULT=1" $s && run "TSG_JIT_GN=2 TSG_JIT_GM=16" $s && run "TSG_JIT_GN=1 TSG_JIT_GM=32" $s &&
  run "TSG_JIT_GN=8 TSG_JIT_GM=4" $s && run "TSG_JIT_DMA=0,1,1" $s && run "TSG_JIT_DMA=1,1,1" $s || exit 1
done
python3 - $O <<'PY'
import json, sys
env = None
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    if "env" in d:
        env = d["env"]
        continue
    v = d["jit64"]
    print(d["s"], env, v["width"], v["waves"], round(v["kernel_ms"] * 1e3, 1), round(v["step_ms"] * 1e3, 1), v["bit_identical"])
PY
