#!/bin/bash
# GPU box, round 4: the automatic kernel choice's boundaries, measured -- the
# small-M walk against the 64-row image at M <= 48 and on the "starved grid"
# shapes (few jit workgroups), the 64-row against the 128-row image at
# M >= 1024 over N, and direct vs staged X at configs[1].  JSON lines through
# scripts/rows64_ab.py (bit-identity across kernels checked per line).
# Usage: scripts/r04_bound_ab.sh <tag>
set -o pipefail
TAG=${1:-r04g}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/bound_ab_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/bound_ab_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --modes ell,jit64 --K 16384 --N 16384 --M 1,8,16,32 &&
run --modes ell,jit64 --K 4096 --N 16384 --M 1,8,16,24,32,48 &&
run --modes ell,jit64 --K 16384 --N 4096 --M 16,32,64,128 &&
run --modes ell,jit128,jit64 --K 2048 --N 512 --M 1000 &&
run --modes ell,jit128,jit64 --K 4096 --N 1024 --M 256 &&
run --modes ell,jit128,jit64 --K 1024 --N 1024 --M 1024 &&
run --modes ell,jit128,jit64 --K 2048 --N 2048 --M 256,1024 &&
run --modes jit128,jit64 --K 4096 --N 16384 --M 1024,1536,2048 &&
run --modes jit128,jit64 --K 4096 --N 8192 --M 768,1024,2048 &&
run --modes jit128,jit64 --K 4096 --N 4096 --M 1024,2048,4096 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 2048 &&
TSG_JIT_XDIRECT=0 run --modes jit64 --K 4096 --N 4096 --M 512,512,256 &&
run --modes jit64 --K 4096 --N 4096 --M 512,512,256 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], "xdirect=%s" % d.get("xdirect_env"), " ".join(cells))
PY
