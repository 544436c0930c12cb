#!/bin/bash
# the simulated ws=8 C5 ZeRO-3 iteration (bench diagnostic) in five fresh processes: median
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03zr"; mkdir -p "$O"; : > "$O/rep.jsonl"
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 "$R/bench.py" --zero 3 --config C5 --simulate-ws 8 --steps 20 --warmup 3 2>/dev/null | grep '^{' >> "$O/rep.jsonl" || exit 1
done
python3 -c "
import json, statistics
ms = [json.loads(l)['ms_per_step'] for l in open('$O/rep.jsonl')]
print('ms', [round(x, 2) for x in ms], 'median', round(statistics.median(ms), 2))"
