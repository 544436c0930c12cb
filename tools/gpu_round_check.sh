#!/bin/bash
# round-end evidence on one box: full -m gpu suite, smoke(), the default bench, rocprof kernel
# trace + PMC passes of the headline (tools/prof_bench.sh)
set -o pipefail
o=gpurun_out/r02f; mkdir -p $o
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $o/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err
