#!/bin/bash
# Kernel traces of the SmolLM3-3B ZeRO-2 and ZeRO-3 training steps (gaps between kernels = host starvation?)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; o=$R/gpurun_out/sm3tr; mkdir -p $o
export TMPDIR=/tmp
cd /tmp || exit 2
for z in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sm3tr_$z -o run -- python3 $R/bench.py --train smollm3 --zero $z --steps 3 --warmup 1 > $o/z$z.json 2> $o/z$z.err || exit $?
  gzip -c /tmp/sm3tr_$z/run_kernel_trace.csv > $o/z${z}_trace.csv.gz || exit $?
done
