#!/bin/bash
# ZeRO-3 host time: the simulated ws=8 C5 iteration (bench diagnostic) + cProfile of both hook styles
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03z"; mkdir -p "$O"
export TMPDIR=/tmp
step() { local t="$1"; shift; echo "[r03z] $*" >&2; timeout -k 10 "$t" "$@"; }
step 300 python3 "$R/bench.py" --zero 3 --config C5 --simulate-ws 8 --steps 20 --warmup 3 > "$O/c5z3_sim8.json" 2> "$O/c5z3_sim8.err" || exit 1
step 300 python3 "$R/tools/z3_host_profile.py" --iters 20 --profile 3 --bwd-hooks module > "$O/z3_host_module.json" 2> "$O/z3_host_profile_module.txt" || exit 1
step 300 python3 "$R/tools/z3_host_profile.py" --iters 20 --profile 3 --bwd-hooks tensor > "$O/z3_host_tensor.json" 2> "$O/z3_host_profile_tensor.txt" || exit 1
step 300 python3 "$R/tools/z3_host_ab.py" > "$O/z3_host_ab.json" 2> "$O/z3_host_ab.err" || exit 1
echo "[r03z] done" >&2
