# PMC HBM traffic of the C5 ZeRO-3 N=1 step's Adam (configs[4]): separate FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
timeout -s KILL 240 bash tools/prof_bench.sh c5z3 fetch --zero 3 --config C5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5z3_fetch.json 2> gpurun_out/c5z3_fetch.err || exit $?
timeout -s KILL 240 bash tools/prof_bench.sh c5z3 write --zero 3 --config C5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5z3_write.json 2> gpurun_out/c5z3_write.err || exit $?
