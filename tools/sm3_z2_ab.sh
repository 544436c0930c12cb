# SmolLM3-3B N=1: phase timings (forward / backward / step+zero_grad, GPU and host) of ZeRO-2 with
# and without the backward-overlap hooks, and ZeRO-3
set -o pipefail
o=gpurun_out/sm3ab; mkdir -p $o
A="--train smollm3 --steps 3 --warmup 1"
timeout -k 10 300 python tools/sm3_variant.py none $A > $o/z2.json 2> $o/z2.err || exit $?
timeout -k 10 300 python tools/sm3_variant.py nooverlap $A > $o/z2_noov.json 2> $o/z2_noov.err || exit $?
timeout -k 10 300 python tools/sm3_variant.py none $A --zero 3 > $o/z3.json 2> $o/z3.err || exit $?
