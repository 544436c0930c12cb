#!/bin/bash
# Run GPU steps in order on the gpurun box.  Each step has its own time limit; an ordinary test
# failure (exit 1) lets the next step run, but a crash / abort / timeout (anything else non-zero)
# ends the script so nothing else touches a possibly-faulted GPU.
#   usage: tools/gpu_steps.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc after $(( $(date +%s) - start )) s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name ended with $rc"
    exit $rc
  fi
done
