"""Where the host time of the hooked ZeRO-3 iteration goes, by library function: rank 0 of a
simulated ws-rank job on the configs[4] parameter set (collectives no-ops, as tools/z3_host_ab.py),
with the runtime's entry points wrapped in per-thread CPU-time accumulators (time.thread_time: the
backward hooks run on autograd's device thread).  Inclusive times per iteration; a wrapped call
inside another wrapped call is counted in both.

Usage: python tools/z3_host_parts.py [--config C5] [--ws 8] [--iters 30] [--single] [--out …]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--ws", type=int, default=8)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--single", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--floor", action="store_true",
                    help="also time the synthetic model alone (full parameters, no ZeRO-3 hooks, no "
                         "optimizer): zero_grad + forward + backward, the host floor of the iteration")
    ap.add_argument("--cprofile", type=int, default=0,
                    help="after the timed block, N more iterations under cProfile (main thread "
                         "and autograd's: threading.setprofile is not enough, so the profiler is "
                         "enabled from the hooks' thread too); prints the top functions by own time")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import bench
    from zero_amd import zero3
    from zero_amd.paramset import ParamSetModel, decoder_layer_groups
    from zero_amd.shapes import CONFIGS

    acc = defaultdict(float)
    calls = defaultdict(int)

    def wrap(owner, name, label):
        fn = getattr(owner, name)

        def timed(*a, **k):
            t0 = time.thread_time()
            try:
                return fn(*a, **k)
            finally:
                acc[label] += time.thread_time() - t0
                calls[label] += 1
        setattr(owner, name, timed)

    R, G = zero3._GatherRuntime, zero3._GradReducer
    wrap(R, "materialize", "runtime.materialize (incl. launches)")
    wrap(R, "launch", "runtime.launch")
    wrap(R, "_launch_wave", "runtime._launch_wave")
    wrap(G, "on_grad_ready", "reducer.on_grad_ready (incl. bucket launches)")
    wrap(G, "_launch", "reducer._launch (one bucket)")
    wrap(G, "_end_backward", "reducer._end_backward")
    wrap(zero3, "_release_group", "_release_group")
    wrap(zero3.ShardedOptimizer, "step", "optimizer.step")
    wrap(zero3.ShardedOptimizer, "zero_grad", "optimizer.zero_grad")

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    shapes = CONFIGS[args.config][1]()
    ws = args.ws
    gen = torch.Generator(device=dev).manual_seed(0)
    params = [torch.nn.Parameter(torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(
        0.0, 0.02, generator=gen)) for s in shapes]
    grads = [torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(0.0, 1e-3, generator=gen)
             for s in shapes]
    model = ParamSetModel(params, decoder_layer_groups(len(shapes)))
    model.set_grad_source(grads)
    real_get = zero3.get
    zero3.get = lambda what, dm=None: {"ws": ws, "rank": 0}.get(what) if what in ("ws", "rank") \
        else real_get(what, dm)
    opt = zero3.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), update=True,
                                 sync=False, comm=bench._NoComm(ws), side_stream=not args.single)
    zero3.register_zero3_hooks(model, opt.param_managers)
    x = torch.zeros(1, device=dev, requires_grad=True)
    fwd = [0.0]
    bwd = [0.0]

    def step():
        opt.zero_grad()
        t0 = time.thread_time()
        y = model(x).sum()
        fwd[0] += time.thread_time() - t0
        t0 = time.perf_counter()
        y.backward()
        bwd[0] += time.perf_counter() - t0
        opt.step()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    acc.clear()
    calls.clear()
    fwd[0] = bwd[0] = 0.0
    w0, c0 = time.perf_counter(), time.process_time()
    for _ in range(args.iters):
        step()
    torch.cuda.synchronize()
    n = args.iters
    res = {"config": args.config, "simulated_ws": ws, "side_stream": not args.single,
           "hostext": zero3._hostext is not None, "iters": n,
           "wall_ms": (time.perf_counter() - w0) / n * 1e3,
           "process_cpu_ms": (time.process_time() - c0) / n * 1e3,
           "forward_main_thread_cpu_ms": fwd[0] / n * 1e3,
           "backward_wall_ms": bwd[0] / n * 1e3,
           "parts_thread_cpu_ms": {k: round(v / n * 1e3, 4) for k, v in sorted(acc.items())},
           "calls_per_iteration": {k: v / n for k, v in sorted(calls.items())}}
    if args.cprofile:
        res["cprofile_top"] = profile_iters(step, args.cprofile)
    if args.floor:
        res["model_only"] = model_floor(model, params, x, args.warmup, n)
    print(json.dumps(res, indent=1), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
    dist.destroy_process_group()


def profile_iters(step, n):
    """Own time per function over n iterations, per thread (main: forward, step; autograd: the
    backward hooks), one cProfile each."""
    import cProfile
    import pstats
    import threading

    import torch

    profs = {}

    def enable_here():
        tid = threading.get_ident()
        if tid not in profs:
            profs[tid] = cProfile.Profile()
            profs[tid].enable()

    # autograd's device thread: enable its profiler from the first hook that runs there
    from zero_amd import zero3
    orig = zero3._GatherRuntime.materialize

    def mat(self, *a, **k):
        enable_here()
        return orig(self, *a, **k)
    zero3._GatherRuntime.materialize = mat
    enable_here()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    for p in profs.values():
        p.disable()
    zero3._GatherRuntime.materialize = orig
    main = threading.get_ident()
    out = {}
    for tid, p in profs.items():
        st = pstats.Stats(p)
        rows = []
        for (fn, line, name), (cc, nc, tt, ct, _) in st.stats.items():
            rows.append((tt, ct, nc, f"{Path(fn).name}:{line}:{name}"))
        rows.sort(reverse=True)
        out["main" if tid == main else "autograd"] = [
            {"fn": r[3], "own_ms_per_iter": round(r[0] / n * 1e3, 4),
             "cum_ms_per_iter": round(r[1] / n * 1e3, 4), "calls_per_iter": r[2] / n}
            for r in rows[:30]]
    return out


def model_floor(model, shards, x, warmup, n):
    """The same ParamSetModel over full-size parameters with no hooks and no optimizer."""
    import torch

    from zero_amd.paramset import ParamSetModel

    full = [torch.nn.Parameter(torch.zeros(tuple(g.shape), device=g.device, dtype=g.dtype))
            for g in (src for layer in model.layers for src in layer.grads())]
    del shards
    m2 = ParamSetModel(full, model.groups)
    m2.set_grad_source([src for layer in model.layers for src in layer.grads()])

    def it():
        for p in full:
            p.grad = None
        m2(x).sum().backward()

    for _ in range(warmup):
        it()
    torch.cuda.synchronize()
    w0, c0 = time.perf_counter(), time.process_time()
    for _ in range(n):
        it()
    torch.cuda.synchronize()
    return {"wall_ms": (time.perf_counter() - w0) / n * 1e3,
            "process_cpu_ms": (time.process_time() - c0) / n * 1e3}


if __name__ == "__main__":
    main()
