#!/bin/bash
# round 4: more of the N > 1 lines at full size on the ONE GPU through real RCCL (--share-gpu):
# C5 ZeRO-3 (configs[4], all 32 layers) at N = 4 — at N = 8 the eight ranks' resident synthetic
# full-size grads (16 GB each) and state do not fit one card (HIP OOM, gpurun_out/r04r8b first run)
# — and C4 ZeRO-1 at N = 8
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04r8b"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
run() {
  local tag=$1 t=$2; shift 2
  GPU_MAX_HW_QUEUES=2 timeout -k 10 $t python3 bench.py --share-gpu --no-cpu-baseline --watchdog-s $((t - 20)) "$@" > "$O/$tag.json" 2> "$O/$tag.err"
  local rc=$?
  echo "== $tag rc=$rc"; tail -1 "$O/$tag.json" | cut -c1-250
  case $rc in 0) ;; *) tail -15 "$O/$tag.err"; exit 1;; esac
}
run c5z3_n4_full 560 --gpus 4 --zero 3 --config C5 --steps 2 --warmup 1
run c4z1_n8_full 500 --gpus 8 --zero 1 --steps 2 --warmup 1 --no-comm-sweep
echo "[r04r8b] done"
