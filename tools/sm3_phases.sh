#!/bin/bash
set -o pipefail
o=gpurun_out/sm3p; mkdir -p $o
A="--train smollm3 --steps 3 --warmup 1"
timeout -k 10 300 python tools/sm3_variant.py none $A > $o/z2.json 2> $o/z2.err || exit $?
timeout -k 10 300 python tools/sm3_variant.py none $A --zero 3 > $o/z3.json 2> $o/z3.err || exit $?
timeout -k 10 300 python tools/sm3_variant.py nohooks $A --zero 3 > $o/z3nh.json 2> $o/z3nh.err || exit $?
