#!/bin/bash
# GPU box, round 4: the small-M walk against the 64-row image for sparse W
# (s = 8, 16) at M = 32 ... 128 -- where the automatic ELL boundary should sit
# when W is sparse.  Usage: scripts/r04_sparse_small_ab.sh <tag>
set -o pipefail
TAG=${1:-r04r}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/sparse_small_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/sparse_small_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
for s in 8 16; do
  run --xint --modes ell,jit64 --K 2048 --N 8192 --s $s --M 48,64,96,128 &&
  run --xint --modes ell,jit64 --K 4096 --N 16384 --s $s --M 48,64,96,128 &&
  run --xint --modes ell,jit64 --K 4096 --N 4096 --s $s --M 48,64,96,128 &&
  run --xint --modes ell,jit64 --K 1024 --N 4096 --s $s --M 48,64,96,128 || exit 1
done
run --xint --modes ell,jit64 --K 2048 --N 8192 --s 4 --M 48,64 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["x"], d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], " ".join(cells))
PY
