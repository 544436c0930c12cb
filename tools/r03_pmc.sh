#!/bin/bash
# round-3 PMC passes (separate FETCH_SIZE / WRITE_SIZE runs) of the headline C4 N=1 Adam
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -s KILL 240 bash "$R/tools/prof_bench.sh" r03 fetch --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-master-line > "$R/gpurun_out/pmc_fetch.log" 2>&1 || exit 1
timeout -s KILL 240 bash "$R/tools/prof_bench.sh" r03 write --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-master-line > "$R/gpurun_out/pmc_write.log" 2>&1 || exit 1
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/prof_r03_fetch" "$R/gpurun_out/prof_r03_write" \
  "adam_segments_kernel<unsigned short, false, false, true>" "$R/gpurun_out/r03_c4_n1_adam_pmc.json" 79952564224 \
  '{"workload": "C4", "zero": 2, "param_dtype": "bf16", "layout": "reference", "n_gpus": 1, "master": "split"}' \
  "tools/r03_pmc.sh (prof_bench.sh r03 fetch|write --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-master-line)" || exit 1
python3 -c "import json; d=json.load(open('$R/gpurun_out/r03_c4_n1_adam_pmc.json')); print(d['hbm_bytes_per_launch'], d['traffic_over_algorithmic'])"
