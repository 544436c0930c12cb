#!/bin/bash
# session-2 final evidence on one box: full -m gpu suite, smoke(), the default bench (as the driver
# runs it), a rocprofv3 kernel trace of the bench
set -o pipefail
o=gpurun_out/final_s2; mkdir -p $o
ZS_FAIL_LOG=$o/failures.log timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 170 \
  --timeout-method thread > $o/pytest.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $o/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err && \
timeout -k 10 300 bash tools/prof_bench.sh final_s2 kt --steps 30 --warmup 2 --no-cpu-baseline > $o/prof_bench.json 2> $o/prof.err; echo "smoke+bench+prof rc=$?"
