#!/bin/bash
# round 4: weak hook callbacks + gather waves — the affected GPU tests, then the ZeRO-3 host A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04d"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 900 python -u -m pytest tests/test_gpu_placement.py tests/test_gpu_zero3.py tests/test_gpu_overlap.py \
  tests/test_gpu_train.py tests/test_gpu_fp8.py "tests/test_gpu_rccl.py::test_rccl_zero3" \
  "tests/test_gpu_bench.py::test_bench_zero3_parameter_set_two_ranks_gloo_staged" -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; grep -E "^(FAILED|ERROR)" "$O/pytest.log" | head; case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 400 python3 tools/z3_host_ab.py --baseline r03 --blocks 4 --out "$O/z3_ab.json" > "$O/z3_ab.log" 2>&1 || { tail -20 "$O/z3_ab.log"; exit 1; }
tail -1 "$O/z3_ab.log"
timeout -k 10 300 python3 tools/z3_host_threads.py --blocks 3 --out "$O/z3_threads.json" > "$O/z3_threads.log" 2>&1 || { tail -20 "$O/z3_threads.log"; exit 1; }
grep '^{' "$O/z3_threads.log" | tail -1
# the runtime thread's CPU: HIP runtime knobs for cross-queue dependencies (diagnostic)
for e in "ROC_CPU_WAIT_FOR_SIGNAL=0" "ROC_ACTIVE_WAIT_TIMEOUT=0" "HSA_ENABLE_INTERRUPT=0"; do
  tag=$(echo "$e" | tr '=' '_')
  env $e timeout -k 10 120 python3 tools/hip_event_cost.py > "$O/hip_event_cost_$tag.log" 2>&1 || { tail -5 "$O/hip_event_cost_$tag.log"; exit 1; }
  echo "== $e"; grep '"ordered' "$O/hip_event_cost_$tag.log"
  env $e timeout -k 10 300 python3 tools/z3_host_threads.py --blocks 3 --out "$O/z3_threads_$tag.json" > "$O/z3_threads_$tag.log" 2>&1 || { tail -5 "$O/z3_threads_$tag.log"; exit 1; }
  grep '^{' "$O/z3_threads_$tag.log" | tail -1
done
echo "[r04d] done"
