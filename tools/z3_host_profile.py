"""Host time of the hooked ZeRO-3 iteration: rank 0 of a simulated ws-rank job on
the configs[4] parameter set (C5 by default: 34 layer modules, 291 tensors), collectives replaced by
no-ops, so the GPU runs only Adam and the step time beyond it is host time.  Prints the iteration
time (HIP-event-free wall clock over --iters iterations after warmup) and a cProfile of a few
iterations (top functions by total time).

Usage: python tools/z3_host_profile.py [--config C5] [--ws 8] [--iters 20] [--profile 5]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--ws", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--profile", type=int, default=5)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--bwd-hooks", default="tensor", choices=["tensor", "module"])
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import bench
    from zero_amd import zero3
    from zero_amd.paramset import ParamSetModel, decoder_layer_groups
    from zero_amd.shapes import CONFIGS, decoder_shapes

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    shapes = CONFIGS[args.config][1]() if args.layers is None else decoder_shapes(args.config, args.layers)
    gen = torch.Generator(device=dev).manual_seed(0)
    params = [torch.nn.Parameter(torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(
        0.0, 0.02, generator=gen)) for s in shapes]
    grads = [torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(0.0, 1e-3, generator=gen)
             for s in shapes]
    model = ParamSetModel(params, decoder_layer_groups(len(shapes)))
    model.set_grad_source(grads)
    ws = args.ws
    real_get = zero3.get
    zero3.get = lambda what, dm=None: {"ws": ws, "rank": 0}.get(what) if what in ("ws", "rank") \
        else real_get(what, dm)
    opt = zero3.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), update=True,
                                 sync=False, comm=bench._NoComm(ws))
    zero3.register_zero3_hooks(model, opt.param_managers, backward_hooks=args.bwd_hooks)
    x = torch.zeros(1, device=dev, requires_grad=True)

    def step():
        opt.zero_grad()
        model(x).sum().backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    opt.timing_events = []
    t0 = time.perf_counter()
    for _ in range(args.iters):
        step()
    host = (time.perf_counter() - t0) / args.iters * 1e3
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.iters * 1e3
    ev, opt.timing_events = opt.timing_events, None
    adam_ms = sum(a.elapsed_time(b) for a, b, _ in ev) / args.iters
    out = {"config": args.config, "simulated_ws": ws, "backward_hooks": args.bwd_hooks,
           "layers": len(model.layers),
           "tensors": len(shapes), "ms_per_iteration": el, "host_enqueue_ms_per_iteration": host,
           "adam_ms_per_iteration": adam_ms, "gathers_per_iteration": 2 * len(model.layers),
           "reduce_buckets": opt._reducer.K}
    print(json.dumps(out), flush=True)
    if args.profile:
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.profile):
            step()
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
        print(s.getvalue(), file=sys.stderr)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
