#!/bin/bash
# N=1 bench line of every BASELINE.json config the bench covers (run on the GPU box from the repo
# root); one JSON line each into gpurun_out/config_table_n1.jsonl.  Each run has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
out=gpurun_out/config_table_n1.jsonl
mkdir -p gpurun_out && : > "$out"
run() {
  echo "=== bench.py $*"
  timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > gpurun_out/cfg.log 2>&1
  rc=$?
  grep '^{' gpurun_out/cfg.log >> "$out"
  tail -n 2 gpurun_out/cfg.log
  [ $rc -eq 0 ] || { echo "=== stopping: exit $rc"; exit $rc; }
}
run --config C2 --dtype fp32 --zero 2
run --config C2 --dtype fp32 --zero 1
run --config C3 --dtype fp32 --zero 2
run --config C4 --zero 2
run --config C4 --zero 2 --master fp32
run --config C4 --zero 1
run --config C5 --zero 2 --steps 50
run --config C5 --zero 3 --steps 50
run --config C3 --dtype fp32 --zero 3
run --config C4 --simulate-ws 8 --steps 20 --warmup 2
run --config C4 --zero 1 --simulate-ws 8 --steps 20 --warmup 2
run --config C5 --simulate-ws 8 --steps 10 --warmup 2
run --config C5 --zero 3 --simulate-ws 8 --steps 10 --warmup 2
