#!/bin/bash
# GPU box, round 4: each image's automatic shape (the 64-row image now
# including 128 columns per wave) on the shapes the new rule moves to it --
# N = 8192 / 4096 at large M, the long-K reference cases, s = 2.
# Usage: scripts/r04_w128_big.sh <tag>
set -o pipefail
TAG=${1:-r04m}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/w128_big_$TAG.jsonl; : > $O
run() { timeout -k 10 400 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/w128_big_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --modes jit128,jit64 --K 4096 --N 8192 --M 2048,4096 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 4096 --M 4096 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --s 2 --reps 10 &&
run --modes jit128,jit64 --K 1024 --N 1024 --M 4096 --reps 20 &&
run --modes jit128,jit64 --K 8192 --N 2048 --M 16000 --reps 10 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 8192 --reps 10 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 64000 --s 8 --reps 3 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 64000 --s 16 --reps 3 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 64000 --s 2 --reps 3 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], " ".join(cells))
PY
