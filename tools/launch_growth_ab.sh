#!/bin/bash
# A/B of the bucket arena's copy launch-group growth (ZERO_AMD_LAUNCH_GROWTH 2 / 4 / 8) on the
# pack / unpack at the simulated ws=8 C4 layout, interleaved runs
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/growth_ab"; mkdir -p "$O"
for rep in 1 2; do
  for g in 2 4 8; do
    ZERO_AMD_LAUNCH_GROWTH=$g timeout -k 10 240 python3 "$R/bench.py" --config C4 --simulate-ws 8 \
      --arena buckets --steps 30 --warmup 3 > "$O/g${g}_r${rep}.json" 2>> "$O/err.log" || exit 1
  done
done
python3 - "$O" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "g*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    ck = d["copy_kernels"]
    print(os.path.basename(f), {k: (round(v["frac"], 4), v["launches_per_step"]) for k, v in ck.items()}, round(d["ms_per_step"], 3))
PY
