#!/bin/bash
# GPU box: PMC passes of one shape through scripts/configs.py (2 timed steps;
# every dispatch of the process is counted: divide by the launch count), one
# rocprofv3 --pmc pass per counter set, never combined with traces.
# Usage: scripts/big_pmc.sh <tag> <M,K,N,s>
set -u
TAG=${1:-big}; SHAPE=${2:-64000,16384,4096,4}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT;\
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE;\
SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE;\
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE"
IFS=';' read -ra S <<< "$SETS"
i=0
for CTR in "${S[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- \
      python3 scripts/configs.py --shape $SHAPE --steps 2 > $OUT/pmc${i}.log 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc ($CTR)"
  if [ $rc -ne 0 ]; then tail -3 $OUT/pmc${i}.log; [ $rc -ge 124 ] && exit $rc; fi
done
python3 - $OUT <<'P'
import csv, glob, os, sys, collections, json
d = sys.argv[1]
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for f in sorted(glob.glob(os.path.join(d, 'pmc*/run_counter_collection.csv'))):
    for r in csv.DictReader(open(f)):
        if 'tsg_jit_kernel' not in r['Kernel_Name']:
            continue
        tot[r['Counter_Name']] += float(r['Counter_Value'])
        n[r['Counter_Name']].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
per = {k: v / max(len(n[k]), 1) for k, v in tot.items()}
per['launches_per_pass'] = {k: len(v) for k, v in n.items()}
json.dump(per, open(os.path.join(d, 'per_launch.json'), 'w'), indent=1)
print(json.dumps({k: per[k] for k in ('FETCH_SIZE', 'WRITE_SIZE', 'TCC_HIT_sum', 'TCC_MISS_sum', 'SQ_WAIT_INST_ANY', 'SQ_WAVE_CYCLES') if k in per}))
P
