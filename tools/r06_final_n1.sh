#!/bin/bash
# Round-6 N=1 evidence in one call: the default bench line, its rocprof kernel stats, the two PMC
# passes over the same command shape, then (last: it ends in an injected hang by design) the N=2
# hang rehearsal of the watchdog's partial line.  Each step under its own limit; && chains.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 2
CFG='{"workload": "C4", "zero": 2, "param_dtype": "bf16", "layout": "reference", "n_gpus": 1, "master": "split", "grad_handoff": "default"}'
bash tools/r06.sh bench n1_final && \
bash tools/r06.sh kstats c4_n1 --steps 100 --warmup 5 --no-cpu-baseline && \
bash tools/r06.sh pmc c4_n1_default 79952564224 "$CFG" --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-master-line --no-default-leg && \
{ ZS_BENCH_INJECT_HANG="exchange check (buckets" ZS_BENCH_INJECT_RANK=1 timeout -k 10 240 \
    python3 bench.py --gpus 2 --share-gpu --config C2 --steps 3 --warmup 1 --no-cpu-baseline \
    --no-comm-sweep --watchdog-s 100 > gpurun_out/r06/hang_rehearsal.json 2> gpurun_out/r06/hang_rehearsal.err
  echo "[hang rehearsal] rc=$? (non-zero expected)"; cat gpurun_out/r06/hang_rehearsal.json | cut -c1-400; }
