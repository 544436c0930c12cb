#!/bin/bash
# round 4: arena="auto" — gloo-staged edge cases (ws 4, an owner of nothing), real RCCL at ws 2 / 8,
# and the N = 8 share-gpu bench (library choice reported beside the full-step calibration)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04i"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_multirank_fewer_params_than_ranks" \
  "tests/test_gpu_rccl.py::test_rccl_zero12[2]" "tests/test_gpu_rccl.py::test_rccl_zero12[8]" \
  "tests/test_gpu_rccl.py::test_bench_share_gpu_n8_both_arenas" > "$O/pytest.log" 2>&1
rc=$?; tail -15 "$O/pytest.log"; exit $rc
