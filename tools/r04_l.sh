#!/bin/bash
# round 4: SmolLM3-3B training N=1, 10 steps each, interleaved twice: ZeRO-2 flat + overlap (the
# default), flat without overlap, buckets + overlap, ZeRO-3
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04l"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
: > "$O/train.jsonl"
for rep in 1 2; do
  for v in "z2flat:--zero 2" "z2flat_noov:--zero 2 --no-overlap" "z2buck:--zero 2 --arena buckets" "z3:--zero 3"; do
    tag=${v%%:*}; a=${v#*:}
    timeout -k 10 300 python3 bench.py --train smollm3 $a --steps 10 --warmup 2 > "$O/$tag.json" 2> "$O/$tag.err" || { tail -10 "$O/$tag.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print(json.dumps({'variant':'$tag','rep':$rep,'ms':round(d['ms_per_step'],2),'tok_s':round(d['value'])}))" | tee -a "$O/train.jsonl"
  done
done
