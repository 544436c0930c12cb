# A/B of the placement probe's acceptance threshold: default bench runs alternating two
# thresholds on one box (no CPU baseline); prints one JSON line per run
set -o pipefail
o=gpurun_out/probe_ab; mkdir -p $o
for i in 1 2 3; do
  for a in ${AB:-5950 6150}; do
    ZERO_AMD_PROBE_ACCEPT_GBS=$a timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 > $o/b_${a}_$i.json 2> $o/b_${a}_$i.err || exit 1
    python -c "import json,sys; d=json.loads([l for l in open('$o/b_${a}_$i.json') if l.startswith('{')][0]); print(json.dumps({'accept': $a, 'run': $i, 'ms': round(d['ms_per_step'],3), 'frac': round(d['roofline']['frac'],4), 'placement': d['placement']}))" | tee -a $o/summary.jsonl
  done
done
