#!/bin/bash
# launch growth 8 (default): the bucket-arena GPU tests + the sim ws=8 bucket line
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03g"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layouts.py tests/test_gpu_scale.py "tests/test_gpu_rccl.py::test_rccl_zero12" -x -q --timeout 170 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python3 "$R/bench.py" --config C4 --simulate-ws 8 --arena buckets --steps 30 --warmup 3 > "$O/c4_sim8_buckets.json" 2> "$O/err.log" || exit 1
grep '^{' "$O/c4_sim8_buckets.json" | cut -c1-600
