#!/bin/bash
# GPU box: alternating same-lease runs of the default bench command under two
# (or more) environments, e.g. the row layout against the blocked one:
#   bash scripts/bench_ab.sh <tag> <reps> "" "TSG_JIT_QBLOCK=16" [...]
# Each run's JSON line gets the environment under "ab_env"; lines in
# gpurun_out/bench_ab_<tag>.jsonl; a summary (ms_per_step, kernel_ms) at the end.
set -o pipefail
TAG=${1:?tag}; REPS=${2:?reps}; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/bench_ab_$TAG.jsonl; : > $O
for r in $(seq $REPS); do
  for e in "$@"; do
    env $e timeout -k 10 200 python bench.py --cpu-rows 0 ${BENCH_ARGS:-} 2>> gpurun_out/bench_ab_$TAG.err |
      python3 -c "import json,sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1]); d['ab_env'] = sys.argv[1]; print(json.dumps(d))" "$e" >> $O
    rc=$?; [ $rc -eq 0 ] || { echo "bench [$e] rc=$rc"; tail -5 gpurun_out/bench_ab_$TAG.err; exit $rc; }
  done
done
python3 - $O <<'PY'
import json, sys, collections
by = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    by[d["ab_env"]].append((d["ms_per_step"], d["roofline"]["kernel_ms"]))
for e, v in by.items():
    print(f"[{e}] ms_per_step {' '.join(f'{a:.4f}' for a, _ in v)} | kernel_ms {' '.join(f'{b:.4f}' for _, b in v)}")
PY
