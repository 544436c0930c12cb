"""Golden fixtures for the DDP drop-in, computed by the reference's own
``SimpleDistributedDataParallelism`` (DDP/ddp.py:30-60).

Runs ONLY in the build container.  ``DDP/ddp.py`` cannot be imported as a module: its body reads
``DDP_TRACE_DIR``, builds an accelerate ``PartialState`` and downloads GLUE MRPC and a tokenizer
(ddp.py:22-27, 58-60), then trains.  So this script reads the file as text, takes the ``ast`` of
the ``SimpleDistributedDataParallelism`` class alone and executes that class definition — the
reference's own code, nothing rewritten — in a namespace holding ``torch`` and
``torch.distributed``.  Nothing of the source is stored: the fixtures hold only inputs and the
outputs the reference computed from them.

Per world size ws in {2, 3} (gloo, CPU processes) and dtype in {float32, bfloat16}:
``Sequential(Linear(40,24), ReLU, Linear(24,8), Linear(8,8))`` seeded identically on every rank,
wrapped by the reference class (its ``__init__`` broadcast check runs); for 3 steps every rank
sets seeded local gradients on the first four parameters (the last Linear gets none) and calls
``sync_gradients()``.  Saved: ``r{r}_t{t}_in{i}`` (local gradient), ``r{r}_t{t}_out{i}`` (after
the reference's all_reduce and ``/= ws``), ``has{i}``; bf16 tensors as their uint16 bits.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ddp_golden.py
"""
from __future__ import annotations

import ast
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REF = Path("/root/reference/DDP/ddp.py")
OUT = Path(__file__).resolve().parent
SHAPES = [(24, 40), (24,), (8, 24), (8,), (8, 8), (8,)]
STEPS = 3


def reference_class():
    tree = ast.parse(REF.read_text(), filename=str(REF))
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef)
           and n.name == "SimpleDistributedDataParallelism"]
    assert len(cls) == 1, "class not found in the reference"
    mod = ast.Module(body=cls, type_ignores=[])
    ns = {"torch": torch, "dist": dist}
    exec(compile(mod, str(REF), "exec"), ns)  # the reference's class definition, as written
    return ns["SimpleDistributedDataParallelism"]


def local_grad(step, rank, i, dtype):
    g = torch.Generator().manual_seed(1000 * step + 10 * rank + i)
    return torch.randn(SHAPES[i], generator=g).to(dtype)


def _bits(t):
    return t.view(torch.int16).numpy().view(np.uint16).copy() if t.dtype == torch.bfloat16 \
        else t.numpy().copy()


def worker(rank, ws, port, dtype_name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    dtype = getattr(torch, dtype_name)
    Ref = reference_class()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(40, 24), torch.nn.ReLU(), torch.nn.Linear(24, 8),
                                torch.nn.Linear(8, 8)).to(dtype)
    ddp = Ref(model)
    out = {}
    params = list(model.parameters())
    for t in range(STEPS):
        for i, p in enumerate(params):
            p.grad = local_grad(t, rank, i, dtype) if i < 4 else None
            if i < 4:
                out[f"r{rank}_t{t}_in{i}"] = _bits(p.grad)
        ddp.sync_gradients()
        for i, p in enumerate(params):
            if p.grad is not None:
                out[f"r{rank}_t{t}_out{i}"] = _bits(p.grad)
    for i, p in enumerate(params):
        out[f"has{i}"] = np.array(p.grad is not None)
    q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def run(ws, dtype_name, port):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, ws, port, dtype_name, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(ws):
        res.update(q.get(timeout=120))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res["ws"] = np.array(ws)
    res["dtype"] = np.array(dtype_name)
    np.savez_compressed(OUT / f"ddp_sync_ws{ws}_{dtype_name}.npz", **res)
    print(f"ddp_sync_ws{ws}_{dtype_name}.npz: {len(res)} arrays")


if __name__ == "__main__":
    port = 29870
    for ws in (2, 3):
        for dn in ("float32", "bfloat16"):
            run(ws, dn, port)
            port += 1
    sys.exit(0)
