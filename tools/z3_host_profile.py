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
    ap.add_argument("--blocks", type=int, default=5, help="timing blocks of --iters iterations")
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
    import gc

    blocks = []
    for gc_on in [True] * args.blocks:
        (gc.enable if gc_on else gc.disable)()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.iters):
            step()
        torch.cuda.synchronize()
        blocks.append((gc_on, round((time.perf_counter() - t1) / args.iters * 1e3, 3)))
    gc.enable()
    out_blocks = {"blocks_ms_per_iteration(gc_enabled, ms)": blocks}
    out = {"config": args.config, "simulated_ws": ws, "backward_hooks": args.bwd_hooks, **out_blocks,
           "layers": len(model.layers),
           "tensors": len(shapes), "ms_per_iteration": el, "host_enqueue_ms_per_iteration": host,
           "adam_ms_per_iteration": adam_ms, "gathers_per_iteration": 2 * len(model.layers),
           "reduce_buckets": opt._reducer.K}
    print(json.dumps(out), flush=True)
    # inclusive host time of the runtime's entry points, on whatever thread runs them (backward
    # hooks run on autograd's device thread, which cProfile does not see)
    acc = {}

    def timed(owner, name):
        fn = getattr(owner, name)

        def wrapper(*a, **k):
            t = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                key = f"{owner.__name__}.{name}"
                tot, n = acc.get(key, (0.0, 0))
                acc[key] = (tot + time.perf_counter() - t, n + 1)
        setattr(owner, name, wrapper)
        return fn

    patched = [(o, n, timed(o, n)) for o, n in (
        (zero3._GatherRuntime, "launch"), (zero3._GatherRuntime, "materialize"),
        (zero3.Zero3ParamManager, "release"), (zero3._GradReducer, "on_grad_ready"),
        (zero3._GradReducer, "_launch"), (zero3._GradReducer, "_end_backward"),
        (zero3.ShardedOptimizer, "step"), (zero3.ShardedOptimizer, "zero_grad"))]
    n_t = 10
    phases = {"zero_grad": 0.0, "forward": 0.0, "backward": 0.0, "step": 0.0}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_t):
        ta = time.perf_counter()
        opt.zero_grad()
        tb = time.perf_counter()
        y = model(x).sum()
        tc = time.perf_counter()
        y.backward()
        td = time.perf_counter()
        opt.step()
        te = time.perf_counter()
        for k, d in zip(phases, (tb - ta, tc - tb, td - tc, te - td)):
            phases[k] += d
    wall = (time.perf_counter() - t0) / n_t * 1e3
    torch.cuda.synchronize()
    for o, n, fn in patched:
        setattr(o, n, fn)
    print(json.dumps({"instrumented_ms_per_iteration": wall,
                      "phase_ms_per_iteration": {k: round(v / n_t * 1e3, 3) for k, v in phases.items()},
                      "inclusive_ms_per_iteration": {k: round(v[0] / n_t * 1e3, 3)
                                                     for k, v in sorted(acc.items())},
                      "calls_per_iteration": {k: v[1] / n_t for k, v in sorted(acc.items())}}),
          flush=True)
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
