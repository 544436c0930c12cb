#!/bin/bash
# A/B of the segment-copy kernel's accesses in flight per lane (ZERO_AMD_COPY_UNROLL 4 vs 8) on
# the bucket arena's pack / unpack at the simulated ws=8 C4 layout, interleaved runs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/copy_ab"; mkdir -p "$O"
for u in 4 8 4 8; do
  ZERO_AMD_COPY_UNROLL=$u timeout -k 10 240 python3 "$R/bench.py" --config C4 --simulate-ws 8 \
    --arena buckets --steps 20 --warmup 3 > "$O/u${u}_$RANDOM.json" 2>> "$O/err.log" || exit 1
done
python3 - "$O" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "u*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    ck = d["copy_kernels"]
    print(os.path.basename(f), {k: round(v["frac"], 4) for k, v in ck.items()}, round(d["ms_per_step"], 3))
PY
