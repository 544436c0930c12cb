#!/bin/bash
# rocprofv3 passes over bench.py (run on the GPU box from the repo root).
#   kt   : kernel trace + stats (per-kernel durations)
#   fetch: PMC FETCH_SIZE pass      write: PMC WRITE_SIZE pass   (separate passes: TCC slots)
# usage: tools/prof_bench.sh <tag> <kt|fetch|write> [bench args...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; tag="$1"; kind="$2"; shift 2
export TMPDIR=/tmp
cd /tmp || exit 2
out="$R/gpurun_out/prof_${tag}_${kind}"
case "$kind" in
  kt)    exec_args=(--kernel-trace --stats) ;;
  fetch) exec_args=(--pmc FETCH_SIZE) ;;
  write) exec_args=(--pmc WRITE_SIZE) ;;
  *) echo "unknown kind $kind"; exit 2 ;;
esac
rocprofv3 "${exec_args[@]}" --output-format csv -d "$out" -o run -- python3 "$R/bench.py" "$@"
