#!/bin/bash
# GPU box, round 4: the 64-row image at 128 columns per wave (8 waves,
# tcsc_hip_set_jit_width(128)) against its 64-wide stream and the 128-row
# image -- the bench workload, the sparse end, mid-to-large M.
# Usage: scripts/r04_w128_ab.sh <tag>
set -o pipefail
TAG=${1:-r04l}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/w128_ab_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/w128_ab_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --widths 128,64 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --s 8 --widths 128,64 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --s 16 --widths 128,64 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 16384 --M 640,1024,2048 --widths 128,64,32 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 4096 --M 512,2048 --widths 128,64,16 --reps 20 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 2048 --widths 128,64 --reps 20 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], " ".join(cells))
PY
