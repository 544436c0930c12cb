#!/bin/bash
# Round-3 measurement session (run on the GPU box from the repo root):
#   1. kernel roofline table (HIP events) and the same under rocprofv3 --kernel-trace --stats
#   2. ZeRO-3 host time: simulated ws=8 C5 iteration (bench diagnostic line + cProfile)
#   3. bucket-arena pack/unpack at the simulated ws=8 C4 layout (doubling launch groups)
#   4. the default bench line (C4 ZeRO-2, N=1) incl. the fp32-master line
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03n"; mkdir -p "$O"
export TMPDIR=/tmp
step() { local t="$1"; shift; echo "[r03] $*" >&2; timeout -k 10 "$t" "$@"; }
step 240 python3 "$R/tools/kernel_table.py" --out "$O/kernels_table.json" > "$O/kernels_table.log" 2>&1 || exit 1
( cd /tmp && step 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_kernels" -o run -- python3 "$R/tools/kernel_table.py" --iters 10 ) > "$O/kt_kernels.log" 2>&1 || exit 1
step 300 python3 "$R/bench.py" --zero 3 --config C5 --simulate-ws 8 --steps 20 --warmup 3 > "$O/c5z3_sim8.json" 2> "$O/c5z3_sim8.err" || exit 1
step 300 python3 "$R/tools/z3_host_profile.py" --iters 20 --profile 3 --bwd-hooks module > "$O/z3_host_module.json" 2> "$O/z3_host_profile_module.txt" || exit 1
step 300 python3 "$R/tools/z3_host_profile.py" --iters 20 --profile 3 --bwd-hooks tensor > "$O/z3_host_tensor.json" 2> "$O/z3_host_profile_tensor.txt" || exit 1
step 300 python3 "$R/bench.py" --config C4 --simulate-ws 8 --arena buckets --steps 20 --warmup 3 > "$O/c4_sim8_buckets.json" 2> "$O/c4_sim8_buckets.err" || exit 1
step 600 python3 "$R/bench.py" > "$O/bench_default.json" 2> "$O/bench_default.err" || exit 1
echo "[r03] done" >&2
