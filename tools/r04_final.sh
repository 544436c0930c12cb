#!/bin/bash
# round 4 closing measurements: the default line in three fresh processes, SmolLM3 training at N=1
# (ZeRO-2 / ZeRO-3) on the final code
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04z"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
: > "$O/headline_rep.jsonl"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-fp32-master-line > "$O/rep$i.json" 2> "$O/rep$i.err" || { tail -10 "$O/rep$i.err"; exit 1; }
  tail -1 "$O/rep$i.json" >> "$O/headline_rep.jsonl"
done
python3 -c "
import json
for l in open('$O/headline_rep.jsonl'):
    d = json.loads(l); print(round(d['ms_per_step'], 3), round(d['roofline']['frac'], 4), d['placement']['state']['gbs'])"
for z in 2 3; do
  timeout -k 10 400 python3 bench.py --train smollm3 --zero $z > "$O/smollm3_z$z.json" 2> "$O/smollm3_z$z.err" || { tail -10 "$O/smollm3_z$z.err"; exit 1; }
  tail -1 "$O/smollm3_z$z.json" | cut -c1-260
done
echo "[r04z] done"
