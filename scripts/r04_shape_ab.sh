#!/bin/bash
# GPU box, round 4: the automatic choice around its boundaries -- the 64-row
# image vs the 128-row image over M at configs[2]'s K, N (M = 192 ... 1024),
# the small-M walk vs both at K = N = 16384 (M = 33 ... 128), configs[1]
# repeated (noise), then rocprofv3 counters of M = 64 on the three kernels.
# Usage: scripts/r04_shape_ab.sh <tag>
set -o pipefail
TAG=${1:-r04f}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/shape_ab_$TAG.jsonl; : > $O
run() { timeout -k 10 300 python scripts/rows64_ab.py "$@" >> $O 2>> gpurun_out/shape_ab_$TAG.err; rc=$?; echo "ab $* rc=$rc"; return $rc; }
run --modes jit128,jit64 --K 4096 --N 16384 --M 192,320,384,512,640,768,1024 &&
run --modes ell,jit128,jit64 --K 16384 --N 16384 --M 33,40,64,128 &&
run --modes jit128,jit64 --K 4096 --N 4096 --M 512,512,256,1024 &&
run --modes jit128,jit64 --K 16384 --N 4096 --M 64,256,1024 &&
TSG_JIT_QBLOCK=8 run --modes jit64 --K 4096 --N 16384 --M 64,128,512 &&
TSG_JIT_QBLOCK=8 TSG_JIT_XDIRECT=0 run --modes jit64 --K 4096 --N 16384 --M 64,128,512 &&
TSG_JIT_XDIRECT=0 run --modes jit64 --K 4096 --N 16384 --M 64,128,512 &&
run --modes jit64 --K 4096 --N 16384 --M 64,128,512 &&
TSG_JIT_QBLOCK=8 run --modes jit64 --K 4096 --N 4096 --M 512 || exit 1
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d["s"], "auto=" + d["auto"], "xdirect=%s" % d.get("xdirect_env"), " ".join(cells))
PY
bash scripts/r04_small_pmc.sh $TAG 64
