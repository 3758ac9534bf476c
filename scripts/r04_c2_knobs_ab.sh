#!/bin/bash
# GPU box, round 4: configs[2] on the 64-row image's 128 x 8 with direct X
# (the automatic plan) under tile-map, touch-mask and DMA-spread alternatives
# -- one process per setting (the knobs are read once).  Usage: scripts/r04_c2_knobs_ab.sh <tag>
set -o pipefail
TAG=${1:-r04c2}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/c2_knobs_$TAG.jsonl; : > $O
run() { echo "{\"env\": \"$1\"}" >> $O; env $1 timeout -k 10 200 python scripts/rows64_ab.py --xint --modes jit64 --K 4096 --N 16384 --M 4096 --reps 20 >> $O 2>> gpurun_out/c2_knobs_$TAG.err; }
run "AB_DEFAULT=1" && run "TSG_JIT_GN=4 TSG_JIT_GM=8" && run "TSG_JIT_GN=1 TSG_JIT_GM=32" && run "TSG_JIT_TMASK=3" &&
run "TSG_JIT_DMA=0,1,1" && run "TSG_JIT_DMA=1,1,1" && run "TSG_JIT_DMA=0.25,1,1" && run "AB_DEFAULT=2" || exit 1
python3 - $O <<'PY'
import json, sys
env = None
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    if "env" in d:
        env = d["env"]
        continue
    v = d["jit64"]
    print(env, v["width"], v["waves"], round(v["kernel_ms"] * 1e3, 1), round(v["step_ms"] * 1e3, 1), v["bit_identical"])
PY
