#!/bin/bash
# round 4, first GPU call: placement (private allocations), fp8 dequantise rewrite, bench
# self-launch; then the kernel table, its rocprof stats and the PMC traffic passes
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r04a"; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 2
timeout -k 10 500 python -u -m pytest tests/test_gpu_placement.py tests/test_gpu_fp8.py tests/test_gpu_kernels.py \
  "tests/test_gpu_rccl.py::test_bench_share_gpu_exchange_check" -v --timeout 240 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?
tail -3 "$O/pytest.log"; grep -E "^(FAILED|ERROR)" "$O/pytest.log" | head -20
# a test failure is read afterwards; a crash / kill / time limit ends the call here
case $rc in 124|134|137|139) echo "pytest rc=$rc: stopping"; exit 1;; esac
timeout -k 10 240 python3 tools/kernel_table.py --out "$O/kernels_table.json" > "$O/kernels_table.log" 2>&1 || { tail -20 "$O/kernels_table.log"; exit 1; }
ZERO_AMD_DQ_WG_PER_CU=8 timeout -k 10 240 python3 tools/kernel_table.py --out "$O/kernels_table_dq8.json" > "$O/kernels_table_dq8.log" 2>&1 || exit 1
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/tools/kernel_table.py" --iters 10 --out "$O/kernels_table_kt.json" ) > "$O/kt.log" 2>&1 || exit 1
( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- python3 "$R/tools/kernel_table.py" --iters 3 --out "$O/kernels_table_pmc.json" ) > "$O/pmc_fetch.log" 2>&1 || exit 1
( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- python3 "$R/tools/kernel_table.py" --iters 3 ) > "$O/pmc_write.log" 2>&1 || exit 1
python3 tools/kernel_pmc.py "$O/kernels_table_pmc.json" "$O/pmc_fetch" "$O/pmc_write" "$O/kernels_pmc.json" || exit 1
grep -h '"frac"' "$O/kernels_table.log" | python3 -c "import sys,json; [print(f\"{json.loads(l)['kernel'][:80]:80s} {json.loads(l)['frac']:.3f}\") for l in sys.stdin]"
echo "--- dq8"; grep -h 'dequant' "$O/kernels_table_dq8.log" | python3 -c "import sys,json; [print(f\"{json.loads(l)['kernel'][:80]:80s} {json.loads(l)['frac']:.3f}\") for l in sys.stdin]"
timeout -k 10 300 python3 tools/z3_host_threads.py --out "$O/z3_threads.json" > "$O/z3_threads.log" 2>&1 || { tail -20 "$O/z3_threads.log"; exit 1; }
tail -1 "$O/z3_threads.log"
timeout -k 10 400 python3 tools/z3_host_ab.py --baseline r03 --blocks 4 --out "$O/z3_ab.json" > "$O/z3_ab.log" 2>&1 || { tail -20 "$O/z3_ab.log"; exit 1; }
tail -1 "$O/z3_ab.log"
echo "[r04a] done"
