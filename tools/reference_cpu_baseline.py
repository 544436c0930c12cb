"""Time the REFERENCE's own ShardedOptimizer on CPU / gloo in this container.

Imports xo-toybox/distributed-training-sandbox's zero/zero{1,2,3}.py from /root/reference (only
possible here; the reference never travels to the GPU box), unmodified except that
``torch.cuda.synchronize`` is a no-op (zero1.py:104 calls it unconditionally).  Per world size
ws in {1, 2, 4, 8}: ws gloo processes, ``torch.set_num_threads(8 // ws)`` each, the reference
harness model 6 x nn.Linear(D, D) + ReLU (zero1.py:237-249, D=4096: config C2, 100,687,872 fp32
params), batch 16, identical data on every rank (zero1.py:115-117).  Per variant: 1 warm-up
iteration, then 5 timed iterations of zero_grad -> forward -> MSE -> backward -> barrier -> step;
``perf_counter`` brackets ``opt.step()`` (after the barrier) and the full iteration; the slowest
rank's median is reported, with the reference's own ``communication_time`` counter.

    PYTHONDONTWRITEBYTECODE=1 python tools/reference_cpu_baseline.py [--width 4096] [--out F]

Writes profiles/r02_reference_cpu_gloo.json.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import platform
import statistics
import sys
import time
from pathlib import Path

REF_ZERO = Path("/root/reference/zero")
REPO = Path(__file__).resolve().parents[1]


def _load(variant: int):
    sys.dont_write_bytecode = True
    if str(REF_ZERO) not in sys.path:
        sys.path.insert(0, str(REF_ZERO))
    import torch

    torch.cuda.synchronize = lambda *a, **k: None
    spec = importlib.util.spec_from_file_location(f"ref_zero{variant}", REF_ZERO / f"zero{variant}.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _worker(rank, ws, port, variant, width, iters, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(max(1, 8 // ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    ref = _load(variant)
    torch.manual_seed(0)
    layers = []
    for i in range(6):
        layers += [torch.nn.Linear(width, width)] + ([torch.nn.ReLU()] if i < 5 else [])
    model = torch.nn.Sequential(*layers)
    opt = ref.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3))
    if variant == 3:
        ref.register_zero3_hooks(model, opt.param_managers)
    g = torch.Generator().manual_seed(42)
    x = torch.randn(16, width, generator=g)
    y = torch.randn(16, width, generator=g)
    step_s, iter_s, comm_s = [], [], []
    for it in range(iters + 1):
        t0 = time.perf_counter()
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(x), y)
        loss.backward()
        dist.barrier()
        c0 = opt.communication_time
        t1 = time.perf_counter()
        opt.step()
        t2 = time.perf_counter()
        if it:  # the first iteration is the warm-up (zero1.py:120-125)
            step_s.append(t2 - t1)
            iter_s.append(t2 - t0)
            comm_s.append(opt.communication_time - c0)
    t = torch.tensor([statistics.median(step_s), statistics.median(iter_s), statistics.median(comm_s)],
                     dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put([float(v) for v in t])
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    sys.path.insert(0, str(REPO / "tests"))
    from conftest import free_port

    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--ws", default="1,2,4,8")
    ap.add_argument("--variants", default="1,2,3")
    ap.add_argument("--out", default=str(REPO / "profiles" / "r02_reference_cpu_gloo.json"))
    a = ap.parse_args()
    params = 6 * (a.width * a.width + a.width)
    rows = []
    ctx = mp.get_context("spawn")
    for variant in (int(v) for v in a.variants.split(",")):
        for ws in (int(w) for w in a.ws.split(",")):
            q = ctx.Queue()
            mp.spawn(_worker, args=(ws, free_port(), variant, a.width, a.iters, q), nprocs=ws, join=True)
            step, it, comm = q.get()
            row = {"variant": f"zero{variant}", "ws": ws, "step_s": step, "iteration_s": it,
                   "communication_time_s": comm, "params_per_s": params / step,
                   "threads_per_rank": max(1, 8 // ws)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    out = {"what": "the reference's own zero/zeroN.py ShardedOptimizer on CPU/gloo (unmodified; "
                   "torch.cuda.synchronize stubbed)",
           "model": f"6 x nn.Linear({a.width},{a.width}) + ReLU, {params:,} fp32 params, batch 16",
           "timing": "median of %d iterations after 1 warm-up, slowest rank; step_s = opt.step() "
                     "after a barrier; iteration_s = zero_grad+forward+backward+barrier+step" % a.iters,
           "host": {"cpu": platform.processor() or platform.machine(), "cores": os.cpu_count(),
                    "python": platform.python_version()},
           "rows": rows}
    import torch

    out["host"]["torch"] = torch.__version__
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
