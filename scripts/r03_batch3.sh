#!/bin/bash
# GPU box: full-Y tests at BASELINE sizes, read/touch knob A/B, big-shape diag.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_y.py -x -v --timeout 170 --timeout-method thread > gpurun_out/full_y_r03.log 2>&1
rc=$?; echo "full-Y rc=$rc: $(tail -1 gpurun_out/full_y_r03.log)"; [ $rc -eq 0 ] || { grep -E "PASS|FAIL|Error|assert" gpurun_out/full_y_r03.log | tail -20; exit $rc; }
bash scripts/big_diag.sh gpurun_out/big_diag_r03.txt || exit 1
bash scripts/reads_touch_ab.sh gpurun_out/reads_touch_ab_r03.txt || exit 1
