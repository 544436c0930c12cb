#!/bin/bash
set -o pipefail
o=gpurun_out/sm3d; mkdir -p $o
export ZERO_AMD_DIAG_BW=1
for z in 2 3; do
  timeout -k 10 300 python bench.py --train smollm3 --zero $z --steps 3 --warmup 1 > $o/z$z.json 2> $o/z$z.err || exit $?
done
