#!/bin/bash
# round-3 final numbers on one box: kernel table (+ rocprof), SmolLM3 ZeRO-2 / ZeRO-3 training
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03final"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 240 python3 "$R/tools/kernel_table.py" --out "$O/kernels_table.json" > "$O/kernels_table.log" 2>&1 || exit 1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_kernels" -o run -- python3 "$R/tools/kernel_table.py" --iters 10 ) > "$O/kt_kernels.log" 2>&1 || exit 1
timeout -k 10 400 python3 "$R/bench.py" --train smollm3 > "$O/sm3_z2.json" 2> "$O/sm3_z2.err" || exit 1
timeout -k 10 400 python3 "$R/bench.py" --train smollm3 --zero 3 > "$O/sm3_z3.json" 2> "$O/sm3_z3.err" || exit 1
grep -h '^{' "$O/sm3_z2.json" "$O/sm3_z3.json" | cut -c1-400
