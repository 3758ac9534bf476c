#!/bin/bash
# GPU box, round 4: the 64-row image at mid and large M (the VOP2 add issues
# at the packed rate on gfx950 when two waves share a SIMD) against the
# 128-row image: configs[1], configs[2], configs[3] s = 2/8/16, by stream
# width.  Usage: scripts/r04_big.sh <tag>
set -o pipefail
TAG=${1:-r04c}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/rows64_big_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py --modes jit128,jit64 "$@" >> $O 2>> gpurun_out/rows64_big_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --K 4096 --N 16384 --M 4096 --widths 0,64,32 --reps 20 &&
run --K 4096 --N 4096 --M 512 --widths 0,32,16,8 &&
TSG_JIT_WAVES=4 run --K 4096 --N 4096 --M 512 --widths 32,16,8 &&
run --K 4096 --N 16384 --s 2 --M 4096 --widths 0,64 --reps 20 &&
run --K 4096 --N 16384 --s 8 --M 4096 --widths 0,64 --reps 20 &&
run --K 4096 --N 16384 --s 16 --M 4096 --widths 0,64 --reps 20 &&
run --K 4096 --N 16384 --M 256,1024,2048 --widths 0,64,32 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}us/{v['step_ms']*1e3:.1f}({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d["s"], d.get("waves_env"), " ".join(cells))
PY
