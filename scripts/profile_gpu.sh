#!/bin/bash
# Runs on the GPU box (via gpurun): kernel-trace stats of the exact default
# bench command, then PMC passes of a 1-step bench (same workload).
# Usage: [PMC_SETS="A B;C D"] [NO_TRACE=1] [NO_PMC=1] scripts/profile_gpu.sh <tag> [bench args...]
# Each ';'-separated set is one rocprofv3 --pmc pass (kernel-trace only, never
# combined with sys/runtime traces), within the per-block limits (8 SQ, 4 TCC,
# 2 GRBM; FETCH_SIZE uses 3 TCC, WRITE_SIZE 2: each in its own pass).
set -u
TAG=${1:-r02}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
DEFAULT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT;\
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA;\
FETCH_SIZE;WRITE_SIZE;\
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;\
SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_INPUT_VALID_READYB SQ_IFETCH GRBM_GUI_ACTIVE"
IFS=';' read -ra SETS <<< "${PMC_SETS:-$DEFAULT}"
if [ -z "${NO_TRACE:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
      python3 bench.py "$@" > $OUT/trace_bench.log 2>&1 || { echo "trace failed rc=$?"; tail -5 $OUT/trace_bench.log; exit 1; }
  tail -1 $OUT/trace_bench.log
fi
[ -n "${NO_PMC:-}" ] && { echo profile done; exit 0; }
i=0
for CTR in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-rows 0 "$@" > $OUT/pmc${i}_bench.log 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc ($CTR)"
  if [ $rc -ne 0 ]; then tail -3 $OUT/pmc${i}_bench.log; [ $rc -ge 124 ] && exit $rc; fi
done
echo profile done
