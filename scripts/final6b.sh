#!/bin/bash
# GPU box, round 6's final evidence, part 2: PMC passes of configs[1] (its
# own summary, with the call plan), BASELINE's configs and the configs[3]
# sweep (scripts/configs.py, scripts/sweep.py).
#   bash scripts/final6b.sh <tag>
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/prof_c1_$TAG; mkdir -p $OUT
i=0
for CTR in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- \
      python3 bench.py --M 512 --K 4096 --N 4096 --steps 1 --warmup 0 --cpu-rows 0 > $OUT/pmc${i}_bench.log 2>&1
  rc=$?; echo "configs[1] pmc pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $OUT/pmc${i}_bench.log; [ $rc -ge 124 ] && exit $rc; fi
done
python3 scripts/make_profile_summary.py $OUT gpurun_out/summary_c1_$TAG 512 4096 4096 4 > /dev/null && echo configs1 summary ok
timeout -k 10 400 python scripts/configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err
rc=$?; echo "configs rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/configs_$TAG.err; exit $rc; }
timeout -k 10 400 python scripts/sweep.py > gpurun_out/sweep_$TAG.jsonl 2> gpurun_out/sweep_$TAG.err
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sweep_$TAG.err; exit $rc; }
