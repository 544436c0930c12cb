#!/bin/bash
set -o pipefail
o=gpurun_out/sm3v; mkdir -p $o
A="--train smollm3 --steps 3 --warmup 1"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > $o/z2_$i.json 2> $o/z2_$i.err || exit $?
  for v in ${VARIANTS:-none nohooks}; do
    timeout -k 10 300 python tools/sm3_variant.py $v $A --zero 3 > $o/z3_${v}_$i.json 2> $o/z3_${v}_$i.err || exit $?
  done
done
