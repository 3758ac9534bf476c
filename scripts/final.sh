#!/bin/bash
# GPU box, a round's final evidence: the whole GPU suite, the default bench
# line, rocprofv3 --kernel-trace --stats of the exact default bench command
# plus PMC passes of it (scripts/profile_gpu.sh), and PMC passes of
# configs[1] (HBM bytes per launch).  Summaries under gpurun_out/summary_<tag>*.
#   bash scripts/final.sh <tag> [skip-suite]
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$2" != skip-suite ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "gpu suite rc=$rc: $(tail -1 gpurun_out/pytest_$TAG.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_$TAG.log; exit $rc; }
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.jsonl 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
tail -1 gpurun_out/bench_$TAG.jsonl | cut -c1-400
bash scripts/profile_gpu.sh $TAG || exit $?
python3 scripts/make_profile_summary.py gpurun_out/prof_$TAG gpurun_out/summary_$TAG 4096 4096 16384 4 > /dev/null && echo summary ok
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
