#!/bin/bash
# GPU box, round 4: the 64-row image (X staged) against the 128-row image at
# M >= 512 over N and K -- the upper boundary of the automatic choice.
# Usage: scripts/r04_big_ab.sh <tag>
set -o pipefail
TAG=${1:-r04h}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/big_ab_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/big_ab_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --modes jit128,jit64 --K 4096 --N 16384 --M 640,768,1024,1536,2048,4096 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 8192 --M 768,1024,2048,4096 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 4096 --M 512,1024,2048,4096 --reps 20 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 1024,2048 --reps 20 &&
run --modes jit128,jit64 --K 1024 --N 1024 --M 1024,4096 &&
run --modes jit128,jit64 --K 2048 --N 2048 --M 1024 &&
run --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --s 8 --reps 20 &&
run --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --s 16 --reps 20 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], " ".join(cells))
PY
