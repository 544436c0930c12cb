#!/bin/bash
# round-end evidence on one box, as the driver runs it: the full -m gpu suite (incl. the real-RCCL
# shared-GPU tests), then (tools/gpu_round_check.sh <dir> bench) smoke() and the default bench
set -o pipefail
o=gpurun_out/${1:-r02f}; mkdir -p $o
if [ "${2:-tests}" = tests ]; then
  ZS_FAIL_LOG=$o/failures.log timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 170 \
    --timeout-method thread --durations=25 > $o/pytest.log 2>&1; echo "pytest rc=$?"
else
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $o/smoke.log 2>&1 && \
  timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err; echo "smoke+bench rc=$?"
fi
