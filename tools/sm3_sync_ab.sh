mkdir -p gpurun_out/r06
B="--train smollm3 --zero 3 --simulate-ws 8 --steps 6 --warmup 2"
for v in "base:" "nofence:sync_write_fence=0" "waitk:sync_wait_kernel=1" "both:sync_write_fence=0 sync_wait_kernel=1"; do
  n=${v%%:*}; k=${v#*:}
  timeout -k 10 300 python tools/tune_run.py $k -- $B > gpurun_out/r06/sm3ab_$n.json 2> gpurun_out/r06/sm3ab_$n.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06/prof_sm3_both -o run -- python3 $GRAFT_REPO_ROOT/tools/tune_run.py sync_write_fence=0 sync_wait_kernel=1 -- $B > $GRAFT_REPO_ROOT/gpurun_out/r06/prof_sm3_both.json 2> $GRAFT_REPO_ROOT/gpurun_out/r06/prof_sm3_both.err
