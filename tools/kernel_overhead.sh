#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; o=$R/gpurun_out/kov; mkdir -p $o
timeout -k 10 180 python3 $R/tools/kernel_overhead_probe.py > $o/plain.jsonl 2> $o/plain.err || exit $?
export TMPDIR=/tmp; cd /tmp || exit 2
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kov -o run -- python3 $R/tools/kernel_overhead_probe.py > $o/prof.jsonl 2> $o/prof.err || exit $?
cp /tmp/kov/run_kernel_stats.csv $o/kernel_stats.csv
