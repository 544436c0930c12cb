set -o pipefail
mkdir -p gpurun_out/r02f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02f/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r02f/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r02f/bench.json 2> gpurun_out/r02f/bench.err && \
timeout -k 10 300 bash tools/prof_bench.sh r02h kt --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02f/kt.json 2> gpurun_out/r02f/kt.err && \
timeout -k 10 300 bash tools/prof_bench.sh r02h fetch --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02f/fetch.json 2> gpurun_out/r02f/fetch.err && \
timeout -k 10 300 bash tools/prof_bench.sh r02h write --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02f/write.json 2> gpurun_out/r02f/write.err
