#!/bin/bash
# round 4: is the HIP runtime thread's CPU per cross-stream wait or per pending time?
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04e"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 180 python3 tools/hip_event_cost.py > "$O/hip_event_cost.log" 2>&1 || { tail -5 "$O/hip_event_cost.log"; exit 1; }
grep '^{' "$O/hip_event_cost.log"
echo "[r04e] done"
