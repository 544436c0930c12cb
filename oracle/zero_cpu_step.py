"""TEST INFRASTRUCTURE / CPU BASELINE — the reference's ZeRO step restated on CPU with gloo.

A from-scratch restatement (no reference code) of what ``ShardedOptimizer.step()`` does per
step, used as ``bench.py``'s ``cpu_baseline`` (SURVEY.md §8(d) "CPU baseline timing" (2),
BASELINE.md §3.2): the same per-tensor algorithm on the host cores, so the GPU step can be read
beside the reference's own path on the same box (the reference itself cannot travel there; its
timings in this container are profiles/r02_reference_cpu_gloo.json).

ZeRO-2 (zero2.py:94-133), per parameter tensor, in index order:
  * flatten the grad and concatenate ws copies (zero2.py:99-104);
  * ``reduce_scatter_tensor`` over the default group (zero2.py:107) — the full summed grad;
  * the owner divides by ws and keeps it, everyone else drops it (zero2.py:109-113);
then ``torch.optim.Adam.step`` on the owned parameters (zero2.py:120, CPU single-tensor path) and
one ``broadcast`` per parameter from its owner (zero2.py:122-133).  ZeRO-1 (zero1.py:80-102) is the
same with an in-place ``all_reduce`` + ``/= ws`` on every grad instead.  Checked against the
reference fixtures by tests/test_oracle.py.  Never imported by the product (zero_amd).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .zero_oracle import owner_of, owner_range


class ReferenceStepCPU:
    """The reference step on CPU tensors over the default (gloo) process group."""

    def __init__(self, params, variant: int = 2, lr: float = 1e-3):
        if variant not in (1, 2):
            raise ValueError("variant must be 1 or 2")
        self.params = list(params)
        self.variant = variant
        self.ws = dist.get_world_size()
        self.rank = dist.get_rank()
        s, e = owner_range(len(self.params), self.ws, self.rank)
        self.owned = set(range(s, e))
        self.adam = torch.optim.Adam([self.params[i] for i in sorted(self.owned)], lr=lr,
                                     foreach=False)

    @torch.no_grad()
    def step(self):
        ws, n = self.ws, len(self.params)
        for i, p in enumerate(self.params):
            if p.grad is None:
                continue
            if self.variant == 1:  # zero1.py:81-84
                dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
                p.grad /= ws
                continue
            flat = p.grad.contiguous().view(-1)  # zero2.py:99-107
            out = torch.empty_like(flat)
            dist.reduce_scatter_tensor(out, torch.cat([flat] * ws), op=dist.ReduceOp.SUM)
            if i in self.owned:
                p.grad = (out / ws).view_as(p)
            else:
                p.grad = None
        self.adam.step()  # zero1.py:88 / zero2.py:120
        for i, p in enumerate(self.params):  # zero1.py:91-102 / zero2.py:122-133
            dist.broadcast(p.data, src=owner_of(n, ws, i))

    def zero_grad(self):
        self.adam.zero_grad()
