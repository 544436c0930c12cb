# real RCCL between ranks sharing the box's one GPU (tests/test_gpu_rccl.py); $2 = pytest -k expr
set -o pipefail
o=gpurun_out/${1:-rccl}; mkdir -p $o
ZS_FAIL_LOG=$o/failures.log timeout -k 10 1000 python -u -m pytest tests/test_gpu_rccl.py -m gpu -v --timeout 170 --timeout-method thread -k "${2:-}" > $o/pytest.log 2>&1; echo "pytest rc=$?"
