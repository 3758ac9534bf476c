#!/bin/bash
# GPU box, round 4: the 128-row image against the 64-row image (automatic
# shapes) with bench.py's integer X and with order-sensitive fractional X, on
# one box: the kernels' speed depends on the data (power / clock).
# Usage: scripts/r04_xdata_ab.sh <tag>
set -o pipefail
TAG=${1:-r04o}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/xdata_ab_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/xdata_ab_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
for x in --xint ""; do
  run $x --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --reps 20 &&
  run $x --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --s 8 --reps 20 &&
  run $x --modes jit128,jit64 --K 4096 --N 16384 --M 4096 --s 16 --reps 20 &&
  run $x --modes jit128,jit64 --K 4096 --N 16384 --M 1024,2048 --reps 20 &&
  run $x --modes jit128,jit64 --K 16384 --N 4096 --M 8192 --reps 10 &&
  run $x --modes jit128,jit64 --K 4096 --N 4096 --M 512 --reps 30 || exit 1
done
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["x"], d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], " ".join(cells))
PY
