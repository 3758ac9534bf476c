#!/bin/bash
# GPU box: per-launch durations of tsg_jit_kernel over a long run (clock ramp
# after idle vs steady state), from a rocprofv3 kernel trace of bench.py.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ramp_${1:-x}; shift || true
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
    python3 bench.py --cpu-rows 0 "$@" > $OUT/bench.log 2>&1 || { echo "failed rc=$?"; tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-400
python3 - $OUT <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
r = [x for x in csv.DictReader(open(f)) if x["Kernel_Name"] == "tsg_jit_kernel"]
d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6 for x in r]
print("launches", len(d))
for i in range(0, len(d), 10):
    print(i, " ".join(f"{v:.3f}" for v in d[i:i + 10]))
P
