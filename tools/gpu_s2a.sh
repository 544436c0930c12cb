set -o pipefail
o=gpurun_out/r02s2a; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_overlap.py -m gpu -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1; echo "pytest rc=$?"
rc=$(tail -1 $o/pytest.log >/dev/null; echo 0)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $o/smoke.log 2>&1 && echo smoke ok && \
timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err && echo bench ok && \
NCCL_DEBUG=INFO timeout -k 10 150 python -u tools/rccl_net_probe.py --ws 2 > $o/net2.log 2>&1; echo "net2 rc=$?"
