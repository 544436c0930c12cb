# A/B: does a longer timed region (sustained load) change the C4 step? alternating 300 / 1500 steps
set -o pipefail
o=gpurun_out/steps_ab; mkdir -p $o; : > $o/summary.jsonl
for i in 1 2; do
  for s in 300 1500; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps $s > $o/b_${s}_$i.json 2> $o/b_${s}_$i.err || exit 1
    python -c "import json; d=json.loads([l for l in open('$o/b_${s}_$i.json') if l.startswith('{')][0]); print(json.dumps({'steps': $s, 'run': $i, 'ms': round(d['ms_per_step'],3), 'adam_ms': round(d['roofline']['avg_launch_ms'],3), 'state_gbs': d['placement']['state']['gbs']}))" | tee -a $o/summary.jsonl
  done
done
