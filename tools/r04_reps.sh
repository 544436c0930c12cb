#!/bin/bash
# round 4: the headline in five more fresh processes on another box (placement spread), then the
# plain default line (cpu_baseline and fp32-master line included) at the round's final code
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04reps"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
: > "$O/headline_rep5.jsonl"
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-fp32-master-line > "$O/rep$i.json" 2> "$O/rep$i.err" || { tail -10 "$O/rep$i.err"; exit 1; }
  tail -1 "$O/rep$i.json" >> "$O/headline_rep5.jsonl"
done
python3 -c "
import json
for l in open('$O/headline_rep5.jsonl'):
    d = json.loads(l); print(round(d['ms_per_step'], 3), round(d['roofline']['frac'], 4), d['placement']['state']['gbs'])"
timeout -k 10 600 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -10 "$O/bench_default.err"; exit 1; }
tail -1 "$O/bench_default.json" | cut -c1-400
echo "[r04reps] done"
