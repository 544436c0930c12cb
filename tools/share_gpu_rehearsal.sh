# bench.py at N ranks on the box's ONE GPU with real RCCL between them (--share-gpu): the driver's
# N>1 configurations rehearsed end to end (exchange checks, calibration, sweep); timings are not
# xGMI's.  $1 = out dir, $2 = N, rest = bench args
set -o pipefail
o=gpurun_out/${1}; n=$2; shift 2; mkdir -p $o
GPU_MAX_HW_QUEUES=2 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
  --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus $n --share-gpu --no-cpu-baseline \
  --watchdog-s 560 "$@" > $o/bench_n$n.json 2> $o/bench_n$n.err; echo "bench n=$n rc=$?"
