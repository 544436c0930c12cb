"""Optimizer-state save / restore on the flat state (zero_amd/checkpoint.py).

The reference's ``ShardedOptimizer.optimizer`` is a plain torch Adam (zero1.py:45), so its state
round-trips through ``state_dict()`` / ``load_state_dict()``; memory.py:15-24 walks the same state.
Here: 5 steps, ``state_dict()`` (through ``torch.save`` / ``torch.load(weights_only=True)``), a fresh
optimizer over fresh parameters holding the saved values, ``load_state_dict()``, 5 more steps —
the parameters and the whole optimizer state equal 10 uninterrupted steps bit for bit.  Cases:
ZeRO-1 (the gradient carry), ZeRO-2 with bf16 parameters (split master and fp32 master), the
bucket arena, AdamW + amsgrad, ZeRO-3 update mode (each rank saves its chunks); loading through
the inner optimizer's ``load_state_dict`` (what a reference user calls) as well.  ws 1 and 2 on
the gloo-staged communicator here, ws 2 through real RCCL in tests/test_gpu_rccl.py.
"""
import io

import numpy as np
import pytest
import torch
import torch.distributed as dist

from _zero_run import init_pg, spawn_batch

pytestmark = pytest.mark.gpu

SHAPES = [(48, 8), (48,), (20, 9), (20,), (7,), (64, 3)]

CASES = {
    # name: (variant, param dtype, optimizer class, optimizer kwargs, wrapper kwargs, via_inner)
    "z1_fp32": (1, torch.float32, torch.optim.Adam, {}, {}, False),
    "z2_bf16_split": (2, torch.bfloat16, torch.optim.Adam, {}, {}, False),
    "z2_bf16_fp32master": (2, torch.bfloat16, torch.optim.Adam, {}, {"master": "fp32"}, True),
    "z2_buckets": (2, torch.float32, torch.optim.Adam, {}, {"arena": "buckets"}, False),
    "z2_adamw_amsgrad": (2, torch.float32, torch.optim.AdamW,
                         {"weight_decay": 0.05, "amsgrad": True}, {}, True),
    "z3_bf16": (3, torch.bfloat16, torch.optim.Adam, {}, {"update": True}, False),
    "z3_fp32_inner": (3, torch.float32, torch.optim.Adam, {}, {"update": True}, True),
}


def _grad(t, rank, i, dtype, dev):
    g = torch.Generator().manual_seed(7919 * t + 104 * rank + i)
    return (torch.randn(SHAPES[i], generator=g) * 1e-2).to(dtype).to(dev)


def _bits(t):
    t = t.detach().reshape(-1).cpu()
    return t.view(torch.int16 if t.element_size() == 2 else torch.int32).numpy().copy()


def _ckpt_worker(rank, ws, port, case):
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from zero_amd import zero1, zero2, zero3

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    variant, dt, cls, okw, wkw, via_inner = CASES[case]
    mod = {1: zero1, 2: zero2, 3: zero3}[variant]
    g0 = torch.Generator().manual_seed(3)
    init = [torch.randn(s, generator=g0).to(dt) for s in SHAPES]

    def make():
        params = [torch.nn.Parameter(a.clone().to(dev)) for a in init]
        opt = mod.ShardedOptimizer(cls(params, lr=1e-3, **okw), comm=test_comm(), **wkw)
        return params, opt

    def steps(params, opt, t0, t1):
        for t in range(t0, t1):
            opt.zero_grad()
            for i, p in enumerate(params):
                g = _grad(t, rank, i, dt, dev)
                if variant == 3 and g.shape != p.data.shape:  # a full-size grad on a shard
                    shard = p.data
                    p.data = torch.empty(g.shape, dtype=dt, device=dev)
                    p.grad = g
                    p.data = shard
                elif p.grad is not None and p.grad.shape == g.shape:
                    p.grad.copy_(g)  # (the flat arena's view: ZeRO-1's carry survives)
                else:
                    p.grad = g
            opt.step()
        torch.cuda.synchronize()

    pa, oa = make()
    steps(pa, oa, 0, 10)
    want_p = [_bits(p) for p in pa]
    want_sd = oa.state_dict()
    del pa, oa

    pb, ob = make()
    steps(pb, ob, 0, 5)
    buf = io.BytesIO()
    torch.save({"params": [p.detach().cpu() for p in pb], "opt": ob.state_dict()}, buf)
    del pb, ob
    buf.seek(0)
    ck = torch.load(buf, weights_only=True)  # plain tensors / numbers / strings only
    pc, oc = make()
    with torch.no_grad():  # the model's own checkpoint (ZeRO-3: this rank's chunks)
        for p, saved in zip(pc, ck["params"]):
            p.data.copy_(saved)
    if via_inner:  # what a reference user calls: the inner torch optimizer's loader
        oc.optimizer.load_state_dict(ck["opt"])
    else:
        oc.load_state_dict(ck["opt"])
    steps(pc, oc, 5, 10)
    for i, p in enumerate(pc):
        assert np.array_equal(_bits(p), want_p[i]), (case, ws, rank, "param", i)
    got_sd = oc.state_dict()
    assert sorted(got_sd["state"]) == sorted(want_sd["state"]), case
    for k, entry in want_sd["state"].items():
        assert set(got_sd["state"][k]) == set(entry), (case, k)
        for name, v in entry.items():
            assert np.array_equal(_bits(got_sd["state"][k][name]), _bits(v)), (case, rank, k, name)
    assert got_sd["param_groups"] == want_sd["param_groups"]
    # optimizer.state holds live views again (memory.py walks them)
    for p in oc.optimizer.param_groups[0]["params"]:
        st = oc.optimizer.state[p]
        assert int(st["step"].item()) == 10 and "exp_avg" in st
    # a state dict of another rank / world size is refused, not mis-assigned
    bad = dict(ck["opt"], zero_amd=dict(ck["opt"]["zero_amd"], world_size=ws + 1))
    with pytest.raises(ValueError, match="world_size"):
        oc.load_state_dict(bad)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


@pytest.mark.parametrize("ws", [1, 2])
def test_checkpoint_roundtrip_bit_exact(gpu, ws):
    spawn_batch(ws, [(_ckpt_worker, (c,)) for c in CASES])
