#!/bin/bash
# rocprofv3 kernel trace + roctx marker trace over bench.py (run on the GPU box from the repo root):
# the step's phase ranges (all_reduce_gradients / optimizer_step / broadcast_parameters,
# zero1.py:80-91) beside the kernels each one enqueued.  No PMC counters in this pass.
# usage: tools/prof_marker.sh <tag> [bench args...]
R="${GRAFT_REPO_ROOT:-$(pwd)}"; tag="$1"; shift
export TMPDIR=/tmp
cd /tmp || exit 2
rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/prof_${tag}_marker" -o run -- python3 "$R/bench.py" "$@"
