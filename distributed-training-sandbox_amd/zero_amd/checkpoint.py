"""Optimizer-state save / restore for the ShardedOptimizer drop-ins.

The reference's ``ShardedOptimizer.optimizer`` is a plain ``torch.optim.Adam`` over the owned
parameters (zero1.py:45,71-74), so ``opt.optimizer.state_dict()`` / ``load_state_dict()`` round-trip
its state natively (and memory.py:15-24 walks the same ``state``).  Here that state lives in the
engine's flat buffers and ``optimizer.state[p]`` only holds views of them; torch's own loader would
replace the views with fresh tensors the engine never reads (and cast fp32 moments of bf16
parameters to bf16).  So both the wrapper's ``state_dict()`` / ``load_state_dict()`` and the inner
optimizer's ``load_state_dict`` (re-bound on the instance) go through this module: the dict keeps
torch's format — ``{"state": {index: {...}}, "param_groups": [...]}`` with indices over the inner
optimizer's parameters in group order — and the tensors are copied into and out of the flat state.

Per-parameter entries: ``step`` (fp32 CPU scalar, torch's convention), ``exp_avg``, ``exp_avg_sq``
(+ ``max_exp_avg_sq``) and, beyond torch's Adam, what the engine needs to continue bit for bit:
``master_residual`` (int16; bf16 params, split master: master = bf16 param bits << 16 + residual),
``master_param`` (fp32 master), ``zero1_carry`` (ZeRO-1's A_{t-1}).  A
``zero_amd`` header names the variant, world size, rank and ownership; loading a dict written at a
different world size or rank raises instead of silently mis-assigning shards.  A dict without the
header (a plain torch Adam state dict, e.g. the reference's ``opt.optimizer.state_dict()``) loads
by index; missing extras start from the parameter as it is (residual 0 / master = param, carry 0).
"""
from __future__ import annotations

import torch
from torch.optim import Optimizer

FORMAT = 1


def header(variant: int, ws: int, rank: int, owned, update=None) -> dict:
    h = {"format": FORMAT, "variant": int(variant), "world_size": int(ws), "rank": int(rank),
         "local_param_indices": [int(i) for i in owned]}
    if update is not None:
        h["update"] = bool(update)
    return h


def check_header(sd: dict, expect: dict) -> None:
    h = sd.get("zero_amd")
    if h is None:
        return
    if int(h.get("format", 0)) != FORMAT:
        raise ValueError(f"zero_amd state dict format {h.get('format')} (this build reads {FORMAT})")
    for k in ("variant", "world_size", "rank", "local_param_indices", "update"):
        if k in expect and k in h and h[k] != expect[k]:
            raise ValueError(f"zero_amd state dict was written with {k}={h[k]!r}; this optimizer has "
                             f"{k}={expect[k]!r} (each rank loads its own shard's state)")


def inner_params(optimizer: Optimizer):
    """The inner optimizer's parameters in torch's state_dict index order."""
    return [p for g in optimizer.param_groups for p in g["params"]]


def load_param_groups(optimizer: Optimizer, sd: dict) -> None:
    """Hyper-parameters only, through torch's own loader (group / size validation included); the
    per-parameter state is copied by the caller."""
    Optimizer.load_state_dict(optimizer, {"state": {}, "param_groups": sd["param_groups"]})


def step_of(entry: dict) -> int:
    s = entry.get("step", 0)
    return int(s.item()) if torch.is_tensor(s) else int(s)


def clone_entry(entry: dict) -> dict:
    return {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in entry.items()}


def bind_inner_load(owner) -> None:
    """Route ``owner.optimizer.load_state_dict`` through ``owner.load_state_dict``, so loading the
    inner optimizer (what a reference user calls) fills the flat state instead of desyncing it."""
    def load_state_dict(state_dict):
        owner.load_state_dict(state_dict)
    owner.optimizer.load_state_dict = load_state_dict
