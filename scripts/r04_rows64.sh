#!/bin/bash
# GPU box, round 4: the 64-row image -- its GPU parity tests, then the A/B
# against the 128-row image and the small-M walk (scripts/rows64_ab.py) at
# configs[2]'s K, N and at configs[0] / configs[1].  Usage: scripts/r04_rows64.sh <tag>
set -o pipefail
TAG=${1:-r04b}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows64.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_rows64_$TAG.log 2>&1
rc=$?; echo "rows64 tests rc=$rc: $(tail -1 gpurun_out/pytest_rows64_$TAG.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_rows64_$TAG.log; exit $rc; }
timeout -k 10 300 python scripts/rows64_ab.py > gpurun_out/rows64_ab_$TAG.jsonl 2> gpurun_out/rows64_ab_$TAG.err
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rows64_ab_$TAG.err; exit $rc; }
TSG_JIT_WAVES=4 timeout -k 10 300 python scripts/rows64_ab.py --modes jit64 --widths 32,16,8 --M 32,64,128,256,512 >> gpurun_out/rows64_ab_$TAG.jsonl 2>> gpurun_out/rows64_ab_$TAG.err
rc=$?; echo "ab 4w rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rows64_ab_$TAG.err; exit $rc; }
timeout -k 10 300 python scripts/rows64_ab.py --modes jit64 --widths 32,16,8 --M 32,64,128,256,512 >> gpurun_out/rows64_ab_$TAG.jsonl 2>> gpurun_out/rows64_ab_$TAG.err
rc=$?; echo "ab 8w rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rows64_ab_$TAG.err; exit $rc; }
TSG_JIT_XDIRECT=0 timeout -k 10 300 python scripts/rows64_ab.py --modes jit64 --M 32,64,128,512 >> gpurun_out/rows64_ab_$TAG.jsonl 2>> gpurun_out/rows64_ab_$TAG.err
rc=$?; echo "ab staged rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rows64_ab_$TAG.err; exit $rc; }
timeout -k 10 300 python scripts/rows64_ab.py --K 1024 --N 4096 --M 1,8,16,32,64,128 >> gpurun_out/rows64_ab_$TAG.jsonl 2>> gpurun_out/rows64_ab_$TAG.err
rc=$?; echo "ab c0 rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rows64_ab_$TAG.err; exit $rc; }
timeout -k 10 300 python scripts/rows64_ab.py --K 4096 --N 4096 --M 256,512,1024 --modes jit128,jit64 >> gpurun_out/rows64_ab_$TAG.jsonl 2>> gpurun_out/rows64_ab_$TAG.err
rc=$?; echo "ab c1 rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rows64_ab_$TAG.err; exit $rc; }
python3 - gpurun_out/rows64_ab_$TAG.jsonl <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    d["waves_env"] = d.get("waves_env") or d.get("xdirect_env")
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d["M"], d["K"], d["N"], d.get("waves_env"), " ".join(cells))
PY
