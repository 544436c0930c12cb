#!/bin/bash
# round 4: gather waves — ZeRO-3 GPU tests, then the host breakdown at wave 1 / 2 / 4 and with
# 1 GiB reduce-scatter buckets, and the in-process A/B against the round-3 runtime
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04c"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_placement.py tests/test_gpu_zero3.py "tests/test_gpu_rccl.py::test_rccl_zero3" \
  "tests/test_gpu_bench.py::test_bench_zero3_parameter_set_two_ranks_gloo_staged" -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; grep -E "^(FAILED|ERROR)" "$O/pytest.log" | head; case $rc in 124|134|137|139) exit 1;; esac
for v in "--wave 1" "--wave 2" "--wave 4" "--wave 2 --bucket-mb 1024"; do
  tag=$(echo "$v" | tr -d ' -')
  timeout -k 10 300 python3 tools/z3_host_threads.py --blocks 3 $v --out "$O/z3_threads_$tag.json" > "$O/z3_threads_$tag.log" 2>&1 || { tail -20 "$O/z3_threads_$tag.log"; exit 1; }
  grep '^{' "$O/z3_threads_$tag.log" | tail -1
done
timeout -k 10 400 python3 tools/z3_host_ab.py --baseline r03 --blocks 4 --out "$O/z3_ab.json" > "$O/z3_ab.log" 2>&1 || { tail -20 "$O/z3_ab.log"; exit 1; }
tail -1 "$O/z3_ab.log"
echo "[r04c] done"
