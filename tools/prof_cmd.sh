#!/bin/bash
# rocprofv3 pass over an arbitrary program (run on the GPU box from the repo root).
# usage: tools/prof_cmd.sh <tag> <kt|fetch|write> <program> [args...]
R="${GRAFT_REPO_ROOT:-$(pwd)}"; tag="$1"; kind="$2"; shift 2
export TMPDIR=/tmp
case "$kind" in
  kt)    a=(--kernel-trace --stats) ;;
  fetch) a=(--pmc FETCH_SIZE) ;;
  write) a=(--pmc WRITE_SIZE) ;;
  *) echo "unknown kind $kind"; exit 2 ;;
esac
prog="$1"; shift
case "$prog" in /*) ;; *) prog="$R/$prog" ;; esac
cd /tmp || exit 2
rocprofv3 "${a[@]}" --output-format csv -d "$R/gpurun_out/prof_${tag}_${kind}" -o run -- "$prog" "$@"
