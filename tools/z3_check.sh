set -o pipefail
mkdir -p gpurun_out/z3c gpurun_out/sync
timeout -k 10 600 python -u -m pytest tests/test_gpu_zero3.py tests/test_gpu_train.py tests/test_gpu_fp8.py -x -q --timeout 200 --timeout-method thread > gpurun_out/z3c/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --zero 3 --config C5 --steps 5 --warmup 2 > gpurun_out/z3c/c5.json 2> gpurun_out/z3c/c5.err && \
SYNC_DEBUG=1 timeout -k 10 300 python tools/sm3_variant.py none --train smollm3 --zero 3 --steps 2 --warmup 1 > gpurun_out/sync/z3.json 2> gpurun_out/sync/z3.err && \
SYNC_DEBUG=1 timeout -k 10 300 python tools/sm3_variant.py none --train smollm3 --steps 2 --warmup 1 > gpurun_out/sync/z2.json 2> gpurun_out/sync/z2.err
