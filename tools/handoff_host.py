"""Per-step host enqueue time of the C4 ZeRO-2 step through the default gradient hand-off
(``zero_grad()`` -> None, fresh gradient tensors from two alternating sets, ``step()``: Adam reads
them in place after a gradient-pointer patch launch) and through the views hand-off, without any
synchronisation inside the loop: shows how far the host runs ahead of the GPU before a launch has
to wait, i.e. whether bench.py's ``host_enqueue_ms_per_step`` measures host work or the GPU.

Round 6 (is the bound the kernel-argument pool?): the same step with the
patch launches' argument payload taken out or put back —
  default_same_grads  one gradient set every step: the pointers never change, no patch launch;
  views_plus_patch    the views step + two patch launches (1,808-B GradPatch arguments) per step
                      on a one-segment dummy set (negligible GPU work);
  views_plus_small    the views step + two launches with small arguments (zs_scale of 64 floats).
If views_plus_patch blocks like default and views_plus_small like views, the depth follows the
argument bytes (tools/queue_depth_probe.hip measures the pool itself).

Usage: python tools/handoff_host.py [--config C4] [--steps 400] [--out …]
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
    ap.add_argument("--config", default="C4")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    from zero_amd import zero2
    from zero_amd.shapes import CONFIGS

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    shapes = CONFIGS[args.config][1]()
    gen = torch.Generator(device=dev).manual_seed(0)
    params = [torch.nn.Parameter(torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(
        0.0, 0.02, generator=gen)) for s in shapes]
    sets = [[torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(0.0, 1e-3, generator=gen)
             for s in shapes] for _ in range(2)]
    opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), sync=False)
    res = {"config": args.config, "steps": args.steps}

    def run(name, step):
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t = []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            step()
            t.append((time.perf_counter() - t0) * 1e3)
        w0 = time.perf_counter()
        torch.cuda.synchronize()
        drain = (time.perf_counter() - w0) * 1e3
        t = np.array(t)
        slow = np.nonzero(t > 1.0)[0]
        res[name] = {"first_blocked_step": int(slow[0]) if len(slow) else None,
                     "host_ms_before": float(t[:slow[0]].mean()) if len(slow) and slow[0] else float(t.mean()),
                     "host_ms_after": float(t[slow[0]:].mean()) if len(slow) else None,
                     "host_ms_mean": float(t.mean()), "drain_ms_after_loop": drain}
        print(json.dumps({name: res[name]}), flush=True)

    k = [0]

    def default_step():
        opt.zero_grad()
        for p, g in zip(params, sets[k[0] % 2]):
            p.grad = g
        k[0] += 1
        opt.step()

    run("default", default_step)

    def default_same():
        opt.zero_grad()
        for p, g in zip(params, sets[0]):
            p.grad = g
        opt.step()

    run("default_same_grads", default_same)
    opt.zero_grad(set_to_none=False)
    with torch.no_grad():
        for p, g in zip(params, sets[0]):
            p.grad.copy_(g)
    run("views", lambda: opt.step())

    from zero_amd import _lib
    from zero_amd.kernels import AdamSet

    dp = torch.zeros(256, device=dev)
    dm, dv = torch.zeros_like(dp), torch.zeros_like(dp)
    dg = [torch.zeros_like(dp), torch.zeros_like(dp)]
    rows = np.array([[0, dp.data_ptr(), dp.data_ptr(), 0, dm.data_ptr(), dv.data_ptr(), 0, 0, 256]],
                    np.uint64)
    dummy = AdamSet(rows, _lib.ZS_F32)
    ptrs = [np.array([g.data_ptr()], np.uint64) for g in dg]
    st = torch.cuda.current_stream()

    def views_plus_patch():
        opt.step()
        dummy.set_grads(ptrs[0], st)  # (alternating pointers: each call launches one patch)
        dummy.set_grads(ptrs[1], st)

    run("views_plus_patch", views_plus_patch)
    small = torch.ones(64, device=dev)

    def views_plus_small():
        opt.step()
        for _ in range(2):
            _lib.call("zs_scale", small.data_ptr(), 64, _lib.ZS_F32, 1.0, st.cuda_stream)

    run("views_plus_small", views_plus_small)
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
