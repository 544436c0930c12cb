#!/bin/bash
# round 4: where the ZeRO-3 host CPU goes (runtime threads), the placement test, and one
# headline bench line on the private-allocation placement
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04b"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 120 python -u -m pytest tests/test_gpu_placement.py -v --timeout 100 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 120 python3 tools/hip_event_cost.py > "$O/hip_event_cost.log" 2>&1 || { tail -20 "$O/hip_event_cost.log"; exit 1; }
grep '^{' "$O/hip_event_cost.log"
timeout -k 10 300 python3 tools/z3_host_threads.py --blocks 3 --out "$O/z3_threads.json" > "$O/z3_threads.log" 2>&1 || { tail -20 "$O/z3_threads.log"; exit 1; }
grep '^{' "$O/z3_threads.log" | tail -2
timeout -k 10 300 python3 tools/z3_host_threads.py --blocks 3 --no-events --out "$O/z3_threads_noev.json" > "$O/z3_threads_noev.log" 2>&1 || { tail -20 "$O/z3_threads_noev.log"; exit 1; }
grep '^{' "$O/z3_threads_noev.log" | tail -2
timeout -k 10 400 python3 bench.py --steps 300 > "$O/bench_n1.json" 2> "$O/bench_n1.err" || { tail -20 "$O/bench_n1.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'], d['placement']['state'], d['cpu_baseline'])"
timeout -k 10 300 python3 tools/dq_ab.py --out "$O/dq_ab.json" > "$O/dq_ab.log" 2>&1 || { tail -20 "$O/dq_ab.log"; exit 1; }
grep "^{" "$O/dq_ab.log"
echo "[r04b] done"
