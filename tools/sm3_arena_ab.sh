# SmolLM3-3B ZeRO-2 at N=1: flat arena (grads accumulate into arena views) vs bucket arena (fresh
# grads, read where backward left them), alternating, phase timings
set -o pipefail
o=gpurun_out/sm3arena; mkdir -p $o
A="--train smollm3 --steps 3 --warmup 1"
for i in 1 2; do
  timeout -k 10 300 python tools/sm3_variant.py none $A > $o/flat_$i.json 2> $o/flat_$i.err || exit $?
  timeout -k 10 300 python tools/sm3_variant.py none $A --arena buckets > $o/buckets_$i.json 2> $o/buckets_$i.err || exit $?
done
