#!/bin/bash
# GPU box, round 4: the 64-row image's stream shapes, 4 waves against 8 per
# workgroup (one vs two waves per SIMD), at configs[1] and the small / mid M
# shapes where the cost model picks 4-wave shapes.  Usage: scripts/r04_waves_ab.sh <tag>
set -o pipefail
TAG=${1:-r04j}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/waves_ab_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/waves_ab_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --modes jit64 --K 4096 --N 4096 --M 512,256 --widths 0,64,32,16,8 &&
TSG_JIT_WAVES=4 run --modes jit64 --K 4096 --N 4096 --M 512,256 --widths 32,16,8 &&
run --modes jit64 --K 4096 --N 16384 --M 64,128 --widths 0,32,16,8 &&
TSG_JIT_WAVES=4 run --modes jit64 --K 4096 --N 16384 --M 64,128 --widths 32,16,8 &&
run --modes jit64 --K 4096 --N 4096 --M 512 --widths 0 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], "waves_env=%s" % d.get("waves_env"), " ".join(cells))
PY
