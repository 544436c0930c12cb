#!/bin/bash
# the headline bench three times on one box (placement spread), plus the simulated ws=8 flat step
set -o pipefail
o=gpurun_out/rep; mkdir -p $o
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $o/c4_$i.json 2> $o/c4_$i.err || exit $?
done
timeout -k 10 300 python bench.py --simulate-ws 8 --arena flat --no-cpu-baseline --steps 50 > $o/sim8.json 2> $o/sim8.err || exit $?
