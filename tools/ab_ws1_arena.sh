#!/bin/bash
# N=1 A/B of the ZeRO-2 step: flat arena (params/grads in probed arena) vs caller's buffers.
set -o pipefail
mkdir -p gpurun_out/ab1
for i in 1 2; do
  for a in flat buckets; do
    timeout -k 10 240 python bench.py --arena $a --no-cpu-baseline --steps 50 > gpurun_out/ab1/${a}_$i.json 2> gpurun_out/ab1/${a}_$i.err || exit $?
  done
done
