set -o pipefail
O=gpurun_out/z3drift; mkdir -p $O
timeout -k 10 300 python3 bench.py --zero 3 --config C5 --simulate-ws 8 --steps 20 --warmup 3 > $O/a_20_3.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --zero 3 --config C5 --simulate-ws 8 --steps 100 --warmup 50 > $O/b_100_50.json 2>/dev/null || exit 1
timeout -k 10 300 python3 tools/z3_host_profile.py --iters 20 --blocks 10 --profile 1 > $O/c_blocks.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --zero 3 --config C5 --simulate-ws 8 --steps 20 --warmup 3 > $O/d_20_3.json 2>/dev/null || exit 1
grep -h '^{' $O/*.json | cut -c1-400
