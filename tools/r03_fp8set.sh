#!/bin/bash
# fused fp8 gather forms: fp8 / ZeRO-3 / RCCL-fp8 GPU tests, then the kernel table (+ rocprof)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03f"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_zero3.py "tests/test_gpu_rccl.py::test_rccl_zero3" -x -q --timeout 170 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 240 python3 "$R/tools/kernel_table.py" --out "$O/kernels_table.json" > "$O/kernels_table.log" 2>&1 || { tail -20 "$O/kernels_table.log"; exit 1; }
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_kernels" -o run -- python3 "$R/tools/kernel_table.py" --iters 10 ) > "$O/kt_kernels.log" 2>&1 || exit 1
echo "[r03f] done"
# end to end: C5 ZeRO-3 at N=1 with fp8 gathers (the only N=1 config whose hooks gather: per layer
# one fused quantise + dequantise in forward and backward)
timeout -k 10 300 python3 "$R/bench.py" --zero 3 --config C5 --gather fp8 --steps 20 --warmup 3 --no-cpu-baseline > "$O/c5z3_fp8_n1.json" 2> "$O/c5z3_fp8_n1.err" || exit 1
grep '^{' "$O/c5z3_fp8_n1.json" | cut -c1-300
