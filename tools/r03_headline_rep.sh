#!/bin/bash
# the default bench line repeated in fresh processes on one box: the spread of the headline
# (placement of the state / arena, kept vs first candidate) at the final code
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03rep"; mkdir -p "$O"; : > "$O/rep.jsonl"
for i in 1 2 3 4; do
  timeout -k 10 300 python3 "$R/bench.py" --steps 300 --no-cpu-baseline --no-fp32-master-line 2>/dev/null | grep '^{' >> "$O/rep.jsonl" || exit 1
done
python3 - "$O/rep.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); p = d["placement"]
    print(round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4), "state", p["state"]["gbs"], "arena", p["arena"]["gbs"], "grads", p["grads"]["gbs"])
PY
