#!/bin/bash
# GPU box: one A/B batch of scripts/rows64_ab.py runs from a plan file, one
# process per line (the environment knobs are read once per process).
#   bash scripts/ab.sh <tag> scripts/plans/<name>.plan
# A plan line is `[KNOB=value ...] <rows64_ab.py arguments>`; `#` lines are
# comments.  Results (one JSON object per shape, each with the line's
# environment under "env") go to gpurun_out/ab_<tag>.jsonl; a compact table is
# printed at the end.  Stops at the first failing line.
set -o pipefail
TAG=${1:?tag}
PLAN=${2:?plan file}
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_$TAG.jsonl; : > $O
E=gpurun_out/ab_$TAG.err; : > $E
while IFS= read -r line; do
  [[ -z "${line// }" || "$line" == \#* ]] && continue
  envs=(); args=()
  for w in $line; do
    if [[ ${#args[@]} -eq 0 && "$w" =~ ^[A-Z_][A-Z_0-9]*= ]]; then envs+=("$w"); else args+=("$w"); fi
  done
  env "${envs[@]}" timeout -k 10 300 python scripts/rows64_ab.py "${args[@]}" 2>> $E |
    python3 -c "import json,sys
for ln in sys.stdin:
    d = json.loads(ln); d['env'] = sys.argv[1]; print(json.dumps(d))" "${envs[*]}" >> $O
  rc=$?; echo "ab [${envs[*]}] ${args[*]} rc=$rc"
  [ $rc -eq 0 ] || { tail -20 $E; exit $rc; }
done < "$PLAN"
python3 - $O <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    cells = [f"{k}={v['kernel_ms']*1e3:.1f}/{v['step_ms']*1e3:.1f}us({v['width']}x{v['waves']}){'' if v['bit_identical'] else ' MISMATCH'}"
             for k, v in d.items() if isinstance(v, dict)]
    print(d.get("x", ""), d["M"], d["K"], d["N"], d["s"], "auto=" + str(d.get("auto")), f"[{d['env']}]", " ".join(cells))
PY
