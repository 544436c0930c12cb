#!/bin/bash
# round 4: zs_scale cache policy by size (tests + A/B), then the N = 8 C4 rehearsal
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04g"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py -k scale_kernel -q --timeout 120 --timeout-method thread > "$O/pytest_scale.log" 2>&1 || { tail -30 "$O/pytest_scale.log"; exit 1; }
tail -2 "$O/pytest_scale.log"
timeout -k 10 300 python -u tools/scale_ab.py --out "$O/scale_ab.json" > "$O/scale_ab.log" 2>&1 || { tail -20 "$O/scale_ab.log"; exit 1; }
cat "$O/scale_ab.log"
bash tools/r04_rehearsal8.sh
