#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats of the small-M sweep (configs[2]'s K,
# N at M = 1, 2, 16, 64, and configs[0]), to set beside its HIP-event times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/small_trace -o run -- \
    python3 scripts/small_m_sweep.py --M 1,2,16,64 > gpurun_out/small_trace_sweep.jsonl 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/small_trace_c0 -o run -- \
    python3 scripts/configs.py --only "configs[0]" > gpurun_out/small_trace_c0.jsonl 2>&1 || exit 1
