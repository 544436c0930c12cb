#!/bin/bash
# round 4: the driver's default N = 8 line (C4 ZeRO-2, arena auto: exchange checks, both arenas
# calibrated, the faster timed) rehearsed on the ONE GPU through real RCCL (--share-gpu: 8 ranks on
# one card, sockets between them), launched as plain `python bench.py --gpus 8`
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04r8"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
GPU_MAX_HW_QUEUES=2 timeout -k 10 840 python3 bench.py --share-gpu --no-cpu-baseline --watchdog-s 800 \
  --gpus 8 --steps 2 --warmup 1 --no-comm-sweep > "$O/c4_n8_full.json" 2> "$O/c4_n8_full.err"
rc=$?
echo "== c4_n8_full rc=$rc"; tail -1 "$O/c4_n8_full.json" | cut -c1-300
[ $rc -eq 0 ] || { tail -20 "$O/c4_n8_full.err"; exit 1; }
echo "[r04r8] done"
