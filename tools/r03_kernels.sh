#!/bin/bash
# kernel roofline table (HIP events) + the same under rocprofv3 --kernel-trace --stats, and the
# bucket-arena pack/unpack at the simulated ws=8 C4 layout
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03k"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 240 python3 "$R/tools/kernel_table.py" --out "$O/kernels_table.json" > "$O/kernels_table.log" 2>&1 || exit 1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_kernels" -o run -- python3 "$R/tools/kernel_table.py" --iters 10 ) > "$O/kt_kernels.log" 2>&1 || exit 1
timeout -k 10 300 python3 "$R/bench.py" --config C4 --simulate-ws 8 --arena buckets --steps 20 --warmup 3 > "$O/c4_sim8_buckets.json" 2> "$O/c4_sim8_buckets.err" || exit 1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_sim8_buckets" -o run -- python3 "$R/bench.py" --config C4 --simulate-ws 8 --arena buckets --steps 10 --warmup 2 --no-cpu-baseline > "$O/c4_sim8_buckets_under_rocprof.json" ) || exit 1
echo "[r03k] done"
