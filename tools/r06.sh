#!/bin/bash
# Round-6 GPU session driver: `tools/r06.sh <step> [args]`, each step under its own time limit,
# outputs under gpurun_out/r06/<step>_<stamp>* — every invocation its own log names (UTC time and
# PID), so a killed run's log survives the next call.  Steps are chained by the caller with && (a
# fault, an abort or a time limit ends the call: nothing more runs on the GPU after it).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r06"; mkdir -p "$O"
TS="$(date -u +%H%M%S)_$$"
export TMPDIR=/tmp
cd "$R" || exit 2
step="$1"; shift
fatal() { case $1 in 124|134|137|139) echo "[$step] rc=$1: stop"; exit 1;; esac; }
case "$step" in
  tests)  # a subset of the -m gpu suite: tools/r06.sh tests <pytest node ids / files>
    ZS_FAIL_LOG="$O/failures_tests_$TS.txt" timeout -k 10 900 python -u -m pytest "$@" -m gpu -v \
      --timeout 300 --timeout-method thread --durations=20 > "$O/tests_$TS.log" 2>&1; rc=$?
    tail -40 "$O/tests_$TS.log"; fatal $rc; echo "[tests $TS] rc=$rc";;
  suite)  # the whole -m gpu suite as the driver runs it, then smoke()
    ZS_CASE_LOG="$O/cases_suite_$TS.txt" ZS_FAIL_LOG="$O/failures_suite_$TS.txt" timeout -k 10 1000 python -u -m pytest tests -m gpu -q \
      --timeout 600 --timeout-method thread --durations=60 > "$O/suite_$TS.log" 2>&1; rc=$?
    tail -80 "$O/suite_$TS.log"; fatal $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
      > "$O/smoke_$TS.log" 2>&1; tail -3 "$O/smoke_$TS.log"; echo "[suite $TS] rc=$rc";;
  bench)  # tools/r06.sh bench <tag> <bench.py args>
    tag="$1"; shift
    timeout -k 10 900 python -u bench.py "$@" > "$O/bench_$tag.json" 2> "$O/bench_$tag.err"; rc=$?
    tail -c 3000 "$O/bench_$tag.json"; tail -5 "$O/bench_$tag.err"; fatal $rc; echo "[bench $tag] rc=$rc";;
  kstats)  # rocprofv3 kernel trace + stats of a bench command: tools/r06.sh kstats <tag> <args>
    tag="$1"; shift
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$tag" -o run -- \
      python3 bench.py "$@" > "$O/kstats_$tag.json" 2> "$O/kstats_$tag.err"; rc=$?
    tail -c 1500 "$O/kstats_$tag.json"; fatal $rc
    find "$O/prof_$tag" -name '*kernel_stats.csv' -exec head -12 {} \; ; echo "[kstats $tag] rc=$rc";;
  pmc)  # separate FETCH_SIZE / WRITE_SIZE passes + summary: tools/r06.sh pmc <tag> <alg bytes> <config json> <bench args>
    tag="$1"; alg="$2"; cfg="$3"; shift 3
    for c in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_${tag}_$c" -o run -- \
        python3 "$R/bench.py" "$@" > "$O/pmc_${tag}_$c.json" 2> "$O/pmc_${tag}_$c.err"); rc=$?
      tail -c 300 "$O/pmc_${tag}_$c.json"; fatal $rc
      [ $rc -eq 0 ] || { echo "[pmc $c] rc=$rc"; tail -5 "$O/pmc_${tag}_$c.err"; exit 1; }
    done
    python3 tools/pmc_summary.py "$O/pmc_${tag}_FETCH_SIZE" "$O/pmc_${tag}_WRITE_SIZE" "adam_segments_kernel<unsigned short, false, false, true>" \
      "$O/${tag}_pmc.json" "$alg" "$cfg" "python3 bench.py $*" | tail -8; echo "[pmc $tag] done";;
  ktable)  # the kernel roofline table: timed run, rocprof stats of it, FETCH / WRITE passes, summary
    timeout -k 10 300 python3 tools/kernel_table.py --out "$O/kernels_table.json" > "$O/ktable_$TS.log" 2>&1; rc=$?
    tail -3 "$O/ktable_$TS.log"; fatal $rc; [ $rc -eq 0 ] || exit 1
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_ktable" -o run -- \
      python3 "$R/tools/kernel_table.py" --out "$O/kernels_table_rocprof.json" > "$O/ktable_rocprof_$TS.log" 2>&1); rc=$?
    fatal $rc; [ $rc -eq 0 ] || { tail -5 "$O/ktable_rocprof_$TS.log"; exit 1; }
    for c in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_ktable_$c" -o run -- \
        python3 "$R/tools/kernel_table.py" --iters 2 --out "$O/kernels_table_$c.json" > "$O/pmc_ktable_$c.log" 2>&1); rc=$?
      fatal $rc; [ $rc -eq 0 ] || { echo "[ktable $c] rc=$rc"; tail -5 "$O/pmc_ktable_$c.log"; exit 1; }
    done
    python3 tools/kernel_pmc.py "$O/kernels_table_FETCH_SIZE.json" "$O/pmc_ktable_FETCH_SIZE" \
      "$O/pmc_ktable_WRITE_SIZE" "$O/kernels_pmc.json" "$O/kernels_table.json" | tail -12; echo "[ktable] done";;
  rehearsal8)  # the driver's default N = 8 line (C4 ZeRO-2, arena auto) on the ONE GPU through real
    # RCCL (--share-gpu: 8 ranks on one card, sockets between them), as plain `python bench.py --gpus 8`
    GPU_MAX_HW_QUEUES=2 timeout -k 10 840 python3 bench.py --share-gpu --no-cpu-baseline --watchdog-s 800 \
      --gpus 8 --steps 2 --warmup 1 --no-comm-sweep "$@" > "$O/c4_n8_full_$TS.json" 2> "$O/c4_n8_full_$TS.err"; rc=$?
    tail -1 "$O/c4_n8_full_$TS.json" | cut -c1-600; fatal $rc
    [ $rc -eq 0 ] || { tail -20 "$O/c4_n8_full_$TS.err"; exit 1; }; echo "[rehearsal8] done";;
  *) echo "unknown step $step"; exit 2;;
esac
