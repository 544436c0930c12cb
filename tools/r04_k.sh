#!/bin/bash
# round 4: where SmolLM3-3B training (N=1) spends GPU time, ZeRO-2 (flat arena, overlap) vs ZeRO-3
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04k"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
for z in 2 3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/z$z" -o run -- python3 bench.py --train smollm3 --zero $z --steps 4 --warmup 2 > "$O/z$z.json" 2> "$O/z$z.err" || { tail -10 "$O/z$z.err"; exit 1; }
  tail -1 "$O/z$z.json" | cut -c1-200
  find "$O/z$z" -type f ! -name "*kernel_stats.csv" -delete  # the traces exceed what comes back
done
find "$O" -name "*kernel_stats.csv" | head
