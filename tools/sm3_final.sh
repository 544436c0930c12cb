# SmolLM3-3B training (§8(f) 3) at N=1, seq 8192, at the current state: ZeRO-2, ZeRO-3, ZeRO-3 kept
# gathered through backward (FSDP2 reshard_after_forward=False)
set -o pipefail
o=gpurun_out/sm3f; mkdir -p $o
timeout -k 10 300 python bench.py --train smollm3 > $o/z2.json 2> $o/z2.err || exit $?
timeout -k 10 300 python bench.py --train smollm3 --zero 3 > $o/z3.json 2> $o/z3.err || exit $?
timeout -k 10 300 python bench.py --train smollm3 --zero 3 --no-reshard > $o/z3nr.json 2> $o/z3nr.err || exit $?
