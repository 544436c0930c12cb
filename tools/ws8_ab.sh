set -o pipefail
O=gpurun_out/r06; mkdir -p $O
ZS_CASE_LOG=$O/cases_default.txt timeout -k 10 400 python -u -m pytest "tests/test_gpu_rccl.py::test_rccl_ws8" -m gpu -q --timeout 380 --timeout-method thread > $O/ws8_default.log 2>&1 || exit 1
NCCL_MAX_NCHANNELS=2 NCCL_NSOCKS_PERTHREAD=1 NCCL_SOCKET_NTHREADS=1 ZS_CASE_LOG=$O/cases_ch2.txt timeout -k 10 400 python -u -m pytest "tests/test_gpu_rccl.py::test_rccl_ws8" -m gpu -q --timeout 380 --timeout-method thread > $O/ws8_ch2.log 2>&1 || exit 1
tail -n 2 $O/ws8_default.log $O/ws8_ch2.log
