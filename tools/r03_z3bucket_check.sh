#!/bin/bash
# ZeRO-3 RS bucket default 512 MB: ZeRO-3 / bench / RCCL ZeRO-3 GPU tests + the sim C5 line x2
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03zb"; mkdir -p "$O"
timeout -k 10 700 python -u -m pytest tests/test_gpu_zero3.py tests/test_gpu_bench.py "tests/test_gpu_rccl.py::test_rccl_zero3" "tests/test_gpu_rccl.py::test_bench_share_gpu_zero3_paramset" "tests/test_gpu_rccl.py::test_bench_share_gpu_zero3_mlp" -x -q --timeout 170 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for i in 1 2; do
  timeout -k 10 300 python3 "$R/bench.py" --zero 3 --config C5 --simulate-ws 8 --steps 20 --warmup 3 2>/dev/null | grep '^{' >> "$O/c5z3_sim8.jsonl" || exit 1
done
cut -c1-220 "$O/c5z3_sim8.jsonl"
