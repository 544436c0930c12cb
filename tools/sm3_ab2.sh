#!/bin/bash
# SmolLM3-3B ZeRO-2 training: flat-arena overlap vs bucket-arena overlap vs ZeRO-3, alternating on one box
set -o pipefail
o=gpurun_out/sm3ab2; mkdir -p $o
for i in 1 2; do
  for a in flat buckets; do
    timeout -k 10 300 python tools/sm3_variant.py none --train smollm3 --arena $a > $o/z2_${a}_$i.json 2> $o/z2_${a}_$i.err || exit $?
  done
  timeout -k 10 300 python tools/sm3_variant.py none --train smollm3 --zero 3 > $o/z3_$i.json 2> $o/z3_$i.err || exit $?
done
