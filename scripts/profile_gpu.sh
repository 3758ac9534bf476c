#!/bin/bash
# Runs on the GPU box (via gpurun): kernel-trace stats + PMC passes of bench.py.
# Usage: scripts/profile_gpu.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
ARGS="$@"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 5 --warmup 1 --cpu-rows 0 $ARGS > $OUT/trace_bench.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
i=0
for CTR in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-rows 0 $ARGS > $OUT/pmc${i}_bench.log 2>&1 || echo "pmc pass $i ($CTR) failed rc=$?"
done
echo profile done
