#!/bin/bash
# SmolLM3-3B training, ZeRO-2 vs ZeRO-3 on one box, with allocation variants (why is ZeRO-3 slower?)
set -o pipefail
o=gpurun_out/sm3ab; mkdir -p $o
run() { tag=$1; shift; timeout -k 10 300 env "$@" > $o/$tag.json 2> $o/$tag.err || exit $?; tail -1 $o/$tag.json | cut -c1-200; }
run z2      python bench.py --train smollm3 --steps 4 --warmup 2
run z3      python bench.py --train smollm3 --zero 3 --steps 4 --warmup 2
run z3_np   ZERO_AMD_PROBE_TRIES=1 python bench.py --train smollm3 --zero 3 --steps 4 --warmup 2
run z2_np   ZERO_AMD_PROBE_TRIES=1 python bench.py --train smollm3 --steps 4 --warmup 2
run z3_exp  PYTORCH_HIP_ALLOC_CONF=expandable_segments:True python bench.py --train smollm3 --zero 3 --steps 4 --warmup 2
