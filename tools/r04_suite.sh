#!/bin/bash
# round 4: the whole -m gpu suite as the driver runs it (+ per-test durations), then smoke()
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04s"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
ZS_FAIL_LOG="$O/failures.txt" timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread --durations=40 > "$O/pytest.log" 2>&1
rc=$?
tail -60 "$O/pytest.log"
case $rc in 124|134|137|139) echo "pytest rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1; tail -3 "$O/smoke.log"
echo "[r04s] done rc=$rc"
