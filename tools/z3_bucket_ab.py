"""Host-time A/B of the hooked ZeRO-3 iteration over the reduce-scatter bucket size: the current
runtime with each --buckets value (MB), in ONE process, alternating blocks of iterations, each on
its own copy of the configs[4] parameter set as rank 0 of a simulated ws-rank job (collectives
no-ops, so the GPU runs only Adam and the rest is host time).  Wall and process CPU time per
iteration per block — the box's host speed drifts over minutes, so only the interleaved comparison
means anything.

Usage: python tools/z3_bucket_ab.py [--config C5] [--ws 8] [--buckets 128,512] [--blocks 6]
"""
from __future__ import annotations

import argparse
import json
import os
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
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--buckets", default="128,512")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import bench
    from zero_amd import zero3 as z3_new
    from zero_amd.paramset import ParamSetModel, decoder_layer_groups
    from zero_amd.shapes import CONFIGS

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29563")
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    shapes = CONFIGS[args.config][1]()
    ws = args.ws

    def build(mod, seed, bucket_mb):
        gen = torch.Generator(device=dev).manual_seed(seed)
        params = [torch.nn.Parameter(torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(
            0.0, 0.02, generator=gen)) for s in shapes]
        grads = [torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(0.0, 1e-3, generator=gen)
                 for s in shapes]
        model = ParamSetModel(params, decoder_layer_groups(len(shapes)))
        model.set_grad_source(grads)
        real_get = mod.get
        mod.get = lambda what, dm=None: {"ws": ws, "rank": 0}.get(what) if what in ("ws", "rank") \
            else real_get(what, dm)
        opt = mod.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), update=True,
                                   sync=False, comm=bench._NoComm(ws), bucket_mb=bucket_mb)
        mod.register_zero3_hooks(model, opt.param_managers)
        x = torch.zeros(1, device=dev, requires_grad=True)

        def step():
            opt.zero_grad()
            model(x).sum().backward()
            opt.step()
        return step

    variants = {f"bucket_{mb}MB": build(z3_new, 0, float(mb)) for mb in args.buckets.split(",")}
    for st in variants.values():
        for _ in range(args.warmup):
            st()
    torch.cuda.synchronize()
    rows = []
    for b in range(args.blocks):
        names = list(variants)
        for name in (names if b % 2 == 0 else names[::-1]):
            st = variants[name]
            torch.cuda.synchronize()
            w0, c0 = time.perf_counter(), time.process_time()
            for _ in range(args.iters):
                st()
            torch.cuda.synchronize()
            w, c = time.perf_counter() - w0, time.process_time() - c0
            rows.append({"block": b, "variant": name, "wall_ms": round(w / args.iters * 1e3, 3),
                         "cpu_ms": round(c / args.iters * 1e3, 3)})
            print(json.dumps(rows[-1]), flush=True)
    summ = {}
    for name in variants:
        ws_ = sorted(r["wall_ms"] for r in rows if r["variant"] == name)
        cs_ = sorted(r["cpu_ms"] for r in rows if r["variant"] == name)
        summ[name] = {"wall_ms_median": ws_[len(ws_) // 2], "wall_ms_min": ws_[0],
                      "cpu_ms_median": cs_[len(cs_) // 2], "cpu_ms_min": cs_[0]}
    print(json.dumps({"config": args.config, "simulated_ws": ws, "iters_per_block": args.iters,
                      "summary": summ}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
