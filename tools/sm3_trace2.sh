#!/bin/bash
# kernel traces: ZeRO-3 SmolLM3 as is vs without module hooks (tools/sm3_variant.py)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; o=$R/gpurun_out/sm3tr2; mkdir -p $o
export TMPDIR=/tmp
cd /tmp || exit 2
for v in none nohooks; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_$v -o run -- python3 $R/tools/sm3_variant.py $v --train smollm3 --zero 3 --steps 3 --warmup 1 > $o/$v.json 2> $o/$v.err || exit $?
  gzip -c /tmp/tr_$v/run_kernel_trace.csv > $o/${v}_trace.csv.gz || exit $?
done
