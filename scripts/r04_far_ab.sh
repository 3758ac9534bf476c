#!/bin/bash
# GPU box, round 4: the 128-row far-X^T image against the 64-row image's
# 128 x 8 on the reference's long-K, large-M cases (both data kinds), and the
# sparse clause at mid M.  Usage: scripts/r04_far_ab.sh <tag>
set -o pipefail
TAG=${1:-r04p}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/far_ab_$TAG.jsonl; : > $O
run() { timeout -k 10 400 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/far_ab_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --xint --modes jit128,jit64 --K 16384 --N 4096 --M 64000 --reps 3 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 64000 --reps 3 &&
run --xint --modes jit128,jit64 --K 16384 --N 4096 --M 16000 --reps 5 &&
run --xint --modes jit128,jit64 --K 4096 --N 16384 --M 1024,2048 --s 8 --reps 20 &&
run --xint --modes jit128,jit64 --K 4096 --N 16384 --M 1024,2048 --s 16 --reps 20 &&
run --xint --modes jit128,jit64 --K 4096 --N 4096 --M 2048,4096 --s 16 --reps 20 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["x"], d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], " ".join(cells))
PY
