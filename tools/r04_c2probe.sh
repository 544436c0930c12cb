#!/bin/bash
# round 4: does probing buffers below 1 GiB lift C2 (100.7M fp32 params, every buffer < 1 GiB)?
# interleaved fresh processes: default threshold vs 256 MiB
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04c2"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
: > "$O/c2.jsonl"
for i in 1 2 3; do
  for thr in default 268435456; do
    if [ $thr = default ]; then
      timeout -k 10 200 python3 bench.py --config C2 --dtype fp32 --steps 2000 --no-cpu-baseline > "$O/c2_${thr}_${i}.json" 2> "$O/c2_err" || { tail -10 "$O/c2_err"; exit 1; }
    else
      ZERO_AMD_PROBE_MIN_BYTES=$thr timeout -k 10 200 python3 bench.py --config C2 --dtype fp32 --steps 2000 --no-cpu-baseline > "$O/c2_${thr}_${i}.json" 2> "$O/c2_err" || { tail -10 "$O/c2_err"; exit 1; }
    fi
    python3 -c "
import json,sys
d=json.loads(open('$O/c2_${thr}_${i}.json').read().strip().splitlines()[-1])
print(json.dumps({'thr':'$thr','rep':$i,'ms':round(d['ms_per_step'],4),'frac':round(d['roofline']['frac'],4),'placement':d.get('placement')}))" | tee -a "$O/c2.jsonl"
  done
done
