#!/bin/bash
# smoke() + the default bench line + the same bench under rocprofv3 --kernel-trace --stats
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r03b"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > "$O/smoke.log" 2>&1 || exit 1
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit 1
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_bench" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_under_rocprof.json" ) || exit 1
echo "[r03b] done"
