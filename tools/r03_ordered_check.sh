#!/bin/bash
# ordered group calls (ABI v9): ZeRO-3 GPU tests incl. real RCCL, then host time (in-process A/B vs
# round 2, and the sim bench x3)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03o"; mkdir -p "$O"
timeout -k 10 800 python -u -m pytest tests/test_gpu_zero3.py tests/test_gpu_train.py tests/test_gpu_fp8.py tests/test_gpu_checkpoint.py tests/test_gpu_bench.py "tests/test_gpu_rccl.py::test_rccl_zero3" "tests/test_gpu_rccl.py::test_bench_share_gpu_zero3_paramset" "tests/test_gpu_rccl.py::test_bench_share_gpu_zero3_mlp" "tests/test_gpu_rccl.py::test_bench_share_gpu_smollm3" -x -q --timeout 170 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python3 "$R/tools/z3_host_ab.py" > "$O/z3_host_ab.json" 2> "$O/z3_host_ab.err" || exit 1
tail -1 "$O/z3_host_ab.json"
for i in 1 2 3; do
  timeout -k 10 300 python3 "$R/bench.py" --zero 3 --config C5 --simulate-ws 8 --steps 20 --warmup 3 2>/dev/null | grep '^{' >> "$O/c5z3_sim8.jsonl" || exit 1
done
cut -c1-200 "$O/c5z3_sim8.jsonl"
