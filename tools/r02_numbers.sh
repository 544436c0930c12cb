#!/bin/bash
# round-2 headline numbers on one box: default bench, simulated ws=8 flat, C5 ZeRO-3, SmolLM3 ZeRO-2/3
set -o pipefail
o=gpurun_out/r02n; mkdir -p $o
timeout -k 10 300 python bench.py > $o/c4_n1.json 2> $o/c4_n1.err || exit $?
timeout -k 10 300 python bench.py --simulate-ws 8 --arena flat --no-cpu-baseline --steps 50 > $o/c4_sim8.json 2> $o/c4_sim8.err || exit $?
timeout -k 10 300 python bench.py --zero 3 --config C5 --steps 20 > $o/c5_z3.json 2> $o/c5_z3.err || exit $?
timeout -k 10 300 python bench.py --zero 3 --config C3 --steps 50 > $o/c3_z3.json 2> $o/c3_z3.err || exit $?
timeout -k 10 300 python bench.py --train smollm3 > $o/sm3_z2.json 2> $o/sm3_z2.err || exit $?
timeout -k 10 300 python bench.py --train smollm3 --zero 3 > $o/sm3_z3.json 2> $o/sm3_z3.err || exit $?
