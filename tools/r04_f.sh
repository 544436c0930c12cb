#!/bin/bash
# round 4: single-stream ZeRO-3 mode — its GPU tests, the host A/B (round 3 / current two-stream /
# current single-stream), and the simulated ws=8 C5 bench line
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04f"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 900 python -u -m pytest tests/test_gpu_zero3.py "tests/test_gpu_rccl.py::test_rccl_zero3" \
  "tests/test_gpu_rccl.py::test_bench_share_gpu_zero3_paramset" "tests/test_gpu_bench.py::test_bench_zero3_parameter_set_two_ranks_gloo_staged" \
  "tests/test_gpu_bench.py::test_bench_zero3_parameter_set_simulated_ws8" -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; grep -E "^(FAILED|ERROR)" "$O/pytest.log" | head; case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 500 python3 tools/z3_host_ab.py --baseline r03 --single --blocks 4 --out "$O/z3_ab.json" > "$O/z3_ab.log" 2>&1 || { tail -20 "$O/z3_ab.log"; exit 1; }
tail -1 "$O/z3_ab.log"
for m in single side; do
  timeout -k 10 300 python3 bench.py --zero 3 --config C5 --simulate-ws 8 --z3-stream $m --steps 30 --warmup 5 --no-cpu-baseline > "$O/c5z3_sim8_$m.json" 2> "$O/c5z3_sim8_$m.err" || { tail -10 "$O/c5z3_sim8_$m.err"; exit 1; }
  tail -1 "$O/c5z3_sim8_$m.json" | cut -c1-300
done
echo "[r04f] done"
