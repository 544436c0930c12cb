#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03sc"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py -k "scale or ddp" -x -q --timeout 170 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 240 python3 "$R/tools/kernel_table.py" --out "$O/kernels_table.json" > "$O/kernels_table.log" 2>&1 || exit 1
grep scale "$O/kernels_table.log" | cut -c1-200
