#!/bin/bash
# scale-kernel rewrite: its GPU test + DDP tests, then the kernel table (+ rocprof trace)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03k3"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_fp8.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 240 python3 "$R/tools/kernel_table.py" --out "$O/kernels_table.json" > "$O/kernels_table.log" 2>&1 || exit 1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_kernels" -o run -- python3 "$R/tools/kernel_table.py" --iters 10 ) > "$O/kt_kernels.log" 2>&1 || exit 1
echo "[r03k3] done"
