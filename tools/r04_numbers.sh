#!/bin/bash
# Round-4 measurement session (GPU box, repo root): kernel table + rocprof stats + PMC traffic,
# the default bench line, its rocprof kernel stats and PMC passes, and the N=1 config table.
# Every GPU step has its own limit; the first failure stops the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04n"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
step() { local t="$1"; shift; echo "[r04n] $*" >&2; timeout -k 10 "$t" "$@"; }
step 240 python3 tools/kernel_table.py --out "$O/kernels_table.json" > "$O/kernels_table.log" 2>&1 || exit 1
( cd /tmp && step 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_kernels" -o run -- python3 "$R/tools/kernel_table.py" --iters 10 ) > "$O/kt_kernels.log" 2>&1 || exit 1
( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/kpmc_fetch" -o run -- python3 "$R/tools/kernel_table.py" --iters 3 --out "$O/kernels_table_pmc.json" ) > "$O/kpmc_fetch.log" 2>&1 || exit 1
( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/kpmc_write" -o run -- python3 "$R/tools/kernel_table.py" --iters 3 ) > "$O/kpmc_write.log" 2>&1 || exit 1
python3 tools/kernel_pmc.py "$O/kernels_table_pmc.json" "$O/kpmc_fetch" "$O/kpmc_write" "$O/kernels_pmc.json" "$O/kernels_table.json" || exit 1
step 600 python3 bench.py > "$O/bench_n1.json" 2> "$O/bench_n1.err" || exit 1
tail -1 "$O/bench_n1.json" | cut -c1-400
( cd /tmp && step 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_bench" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$O/bench_under_rocprof.json" ) > "$O/kt_bench.log" 2>&1 || exit 1
( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-master-line ) > "$O/pmc_fetch.log" 2>&1 || exit 1
( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-master-line ) > "$O/pmc_write.log" 2>&1 || exit 1
python3 tools/pmc_summary.py "$O/pmc_fetch" "$O/pmc_write" "adam_segments_kernel<unsigned short, false, false, true>" "$O/r04_c4_n1_adam_pmc.json" 79952564224 \
  '{"workload": "C4", "zero": 2, "param_dtype": "bf16", "layout": "reference", "n_gpus": 1, "master": "split"}' \
  "tools/r04_numbers.sh (rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE -- bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-master-line)" > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/r04_c4_n1_adam_pmc.json')); print('traffic/alg', d['traffic_over_algorithmic'])"
out="$O/config_table_n1.jsonl"; : > "$out"
run() {
  echo "=== bench.py $*" >&2
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$O/cfg.log" 2>&1
  local rc=$?
  grep '^{' "$O/cfg.log" | sed "s|^{|{\"args\": \"$*\", |" >> "$out"
  [ $rc -eq 0 ] || { tail -5 "$O/cfg.log"; echo "=== stopping: exit $rc"; exit $rc; }
}
run --config C4 --zero 1 --steps 300 --no-fp32-master-line
run --config C2 --dtype fp32 --zero 2 --steps 300
run --config C3 --dtype fp32 --zero 2 --steps 300
run --config C5 --zero 2 --steps 50 --no-fp32-master-line
run --config C5 --zero 3 --steps 50
run --config C3 --zero 3 --steps 200
run --config C4 --simulate-ws 8 --arena flat --steps 50 --warmup 5
run --config C4 --simulate-ws 8 --arena buckets --steps 50 --warmup 5
run --config C4 --zero 1 --simulate-ws 8 --arena flat --steps 50 --warmup 5
run --config C5 --zero 3 --simulate-ws 8 --steps 100 --warmup 20
run --config C5 --zero 3 --simulate-ws 8 --z3-stream side --steps 100 --warmup 20
python3 -c "
import json
for l in open('$out'):
    d = json.loads(l); print(d['args'][:60], round(d['ms_per_step'], 3), round(d.get('roofline', {}).get('frac', d.get('adam_achieved_gbs', 0) / 8000), 3))"
echo "[r04n] done" >&2
