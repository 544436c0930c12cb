# test_rccl_ws8 (eight ranks on one card over RCCL's socket transport) under RCCL environment
# variants: which settings make the suite's longest test shorter.  Logs under gpurun_out/r06/.
set -o pipefail
O=gpurun_out/r06; mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u -m pytest "tests/test_gpu_rccl.py::test_rccl_ws8" -m gpu -q \
    --timeout 280 --timeout-method thread > $O/ws8env_$tag.log 2>&1 || { tail -5 $O/ws8env_$tag.log; exit 1; }
  echo "$tag $(grep -E 'passed|failed' $O/ws8env_$tag.log | tail -1)"
}
run default ZS_X=0
run ll NCCL_PROTO=LL
run simple NCCL_PROTO=Simple
run ch1 NCCL_MIN_NCHANNELS=1 NCCL_MAX_NCHANNELS=1
