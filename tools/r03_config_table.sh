#!/bin/bash
# Round-3 N=1 config table (run on the GPU box from the repo root): one JSON line per config into
# gpurun_out/r03_config_table_n1.jsonl.  Each run has its own limit; the first failure stops it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/r03_config_table_n1.jsonl
mkdir -p gpurun_out && : > "$out"
run() {
  echo "=== bench.py $*"
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/cfg3.log 2>&1
  rc=$?
  grep '^{' gpurun_out/cfg3.log | sed "s|^{|{\"args\": \"$*\", |" >> "$out"
  tail -n 2 gpurun_out/cfg3.log
  [ $rc -eq 0 ] || { echo "=== stopping: exit $rc"; exit $rc; }
}
run --config C4 --zero 2 --steps 500                 # headline config (+ its fp32-master line)
run --config C4 --zero 1 --steps 300 --no-fp32-master-line
run --config C2 --dtype fp32 --zero 2 --steps 300
run --config C3 --dtype fp32 --zero 2 --steps 300
run --config C5 --zero 2 --steps 50 --no-fp32-master-line
run --config C5 --zero 3 --steps 50
run --config C3 --zero 3 --steps 200                 # the reference MLP's ZeRO-3 iteration, fp32
run --config C3 --zero 3 --dtype bf16 --steps 200
run --config C4 --simulate-ws 8 --arena flat --steps 50 --warmup 5
run --config C4 --simulate-ws 8 --arena buckets --steps 50 --warmup 5
run --config C4 --zero 1 --simulate-ws 8 --arena flat --steps 50 --warmup 5
run --config C5 --zero 3 --simulate-ws 8 --steps 100 --warmup 50
