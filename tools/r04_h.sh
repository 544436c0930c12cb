#!/bin/bash
# round 4: zs_scale / zs_convert cache policy by size — tests and the A/B over both kernels
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04h"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_kernels.py -k "scale_kernel or convert or copy" -q --timeout 120 --timeout-method thread > "$O/pytest_policy.log" 2>&1 || { tail -30 "$O/pytest_policy.log"; exit 1; }
tail -2 "$O/pytest_policy.log"
timeout -k 10 400 python -u tools/scale_ab.py --out "$O/policy_ab.json" > "$O/policy_ab.log" 2>&1 || { tail -20 "$O/policy_ab.log"; exit 1; }
cat "$O/policy_ab.log"
