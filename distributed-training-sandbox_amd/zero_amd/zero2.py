"""ZeRO-2 drop-in: ``ShardedOptimizer`` of reference zero/zero2.py:38-139, MI355X-native.

Reference behaviour: every rank reduces every gradient
(``reduce_scatter_tensor`` over ws copies of the flattened grad is an all-reduce in disguise,
zero2.py:99-107), the owner averages it (zero2.py:111) and steps Adam on its index-owned params
(zero2.py:120), then each param is broadcast from its owner (zero2.py:122-133).  The result is
exactly data-parallel Adam.

Here: grads are packed into buckets laid out owner-major (Layout R), one in-place RCCL
reduce-scatter per bucket delivers each owner the summed grads of exactly the params it owns,
the fused HIP Adam divides by ws and updates them, and one in-place all-gather per bucket
replaces the per-param broadcasts.  Ownership, and therefore optimizer-state placement, is
bit-identical to the reference.
"""
from __future__ import annotations

from ._sharded import ShardedOptimizerBase


class Zero2Hook:
    """zero2.py:23-35 (defined but unused by the reference): keeps local grads, drops others.
    Returning ``None`` from a tensor hook leaves the grad unchanged, so this is a no-op there too."""

    def __init__(self, param, is_local_param: bool = False):
        self.param = param
        self.is_local_param = is_local_param

    def __call__(self, grad):
        if not self.is_local_param:
            return None
        return grad


class ShardedOptimizer(ShardedOptimizerBase):
    _carry = False
    _variant = 2

    def __init__(self, optimizer, **kw):
        super().__init__(optimizer, **kw)
        self.grad_hooks = {}
        self.register_gradient_hooks()

    def register_gradient_hooks(self):
        """zero2.py:75-86.  The reference's hooks return the grad or ``None``; both leave the grad
        unchanged, so they are registered as the same no-op (kept for API parity)."""
        for param in self.params:
            if param.requires_grad:
                self.grad_hooks[param] = param.register_hook(lambda grad: None)
