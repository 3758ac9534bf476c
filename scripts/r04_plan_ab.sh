#!/bin/bash
# GPU box, round 4: the calls whose automatic kernel changed with the round-4
# rules and were not yet timed both ways -- (1024, 4096, 1024), the starved
# shapes with K in several chunks, (512, 2048, 512) -- each kernel forced.
# Usage: scripts/r04_plan_ab.sh <tag>
set -o pipefail
TAG=${1:-r04i}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/plan_ab_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/plan_ab_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --modes ell,jit128,jit64 --K 4096 --N 1024 --M 1024 &&
run --modes ell,jit128,jit64 --K 9000 --N 1024 --M 128 &&
run --modes ell,jit128,jit64 --K 16384 --N 1024 --M 64,256 &&
run --modes ell,jit128,jit64 --K 2048 --N 512 --M 512 &&
run --modes ell,jit64 --K 16384 --N 16384 --M 16,24 &&
run --modes ell,jit64 --K 8192 --N 8192 --M 8,16,32 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], " ".join(cells))
PY
