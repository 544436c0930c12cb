#!/bin/bash
# round 4: the driver's N>1 runs rehearsed on the ONE GPU through real RCCL (--share-gpu), launched
# the way the driver may launch them: plain `python bench.py --gpus N` (bench.py starts the ranks)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04r"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 90 tools/event_poll_probe 200 > "$O/event_poll_probe.jsonl" 2>&1 || { tail -5 "$O/event_poll_probe.jsonl"; exit 1; }
cat "$O/event_poll_probe.jsonl"
run() {
  local tag=$1 t=$2; shift 2
  GPU_MAX_HW_QUEUES=2 timeout -k 10 $t python3 bench.py --share-gpu --no-cpu-baseline --watchdog-s $((t - 20)) "$@" > "$O/$tag.json" 2> "$O/$tag.err"
  local rc=$?
  echo "== $tag rc=$rc"; tail -1 "$O/$tag.json" | cut -c1-250
  case $rc in 0) ;; *) tail -15 "$O/$tag.err"; exit 1;; esac
}
run c5z3_n8_4layers_single 400 --gpus 8 --zero 3 --config C5 --set-layers 4 --steps 3 --warmup 1
run c5z3_n8_4layers_side 400 --gpus 8 --zero 3 --config C5 --set-layers 4 --steps 3 --warmup 1 --z3-stream side
run c4_n2_full 400 --gpus 2 --steps 3 --warmup 1 --no-comm-sweep
run c4_n4_full 500 --gpus 4 --steps 2 --warmup 1 --no-comm-sweep
echo "[r04r] done"
