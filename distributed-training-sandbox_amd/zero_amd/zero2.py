"""ZeRO-2 drop-in: ``ShardedOptimizer`` of reference zero/zero2.py:38-139, MI355X-native.

Reference behaviour: every rank reduces every gradient
(``reduce_scatter_tensor`` over ws copies of the flattened grad is an all-reduce in disguise,
zero2.py:99-107), the owner averages it (zero2.py:111) and steps Adam on its index-owned params
(zero2.py:120), then each param is broadcast from its owner (zero2.py:122-133).  The result is
exactly data-parallel Adam.

Here:
  * default ``arena="flat"``: every parameter is a view of one owner-major *flat parameter
    arena* (rank r's owned parameters, Layout R, are the contiguous stretch [base_r, base_r+L_r)).
    ``zero_grad()`` sets the grads to None (as the reference's), and what happens to the fresh
    gradients backward then produces depends on the world size:
      - ws = 1: nothing is exchanged, so Adam reads them in place where backward left them (the
        fused-Adam tables re-pointed in stream order, ``zs_adamset_set_grads``); no copy, and no
        gradient arena unless the caller asks for grad views (``zero_grad(set_to_none=False)``);
      - ws > 1: they are copied into a flat gradient arena of the same layout from the
        post-accumulate-grad hooks — one copy launch per overlap bucket with ``overlap=True``,
        per batch of ``land_batch_bytes`` (64 MiB) otherwise — and ``p.grad`` becomes the slot's
        view, so backward never holds the arena plus a whole second set of gradients.
    A step at ws > 1 is a few *rounds* (window j of every
    owner's stretch): ONE RCCL group of per-owner ``ncclReduce`` — each owner's window of the
    gradient arena summed into its reduced buffer, the reduce-scatter-v of zero2.py:94-113 —, the
    fused HIP Adam on the own window (``/ws`` folded in) writing the updated parameters straight
    into the arena, and ONE RCCL group of in-place ``ncclBroadcast`` of every owner's window, the
    all-gather-v of zero2.py:122-133.  No pack, no unpack: the parameters are the arena.  After
    the step ``p.grad`` is still the arena view holding this rank's local gradient (the reduce is
    out of place) until ``zero_grad()`` (``set_to_none=False`` zeroes the views instead).
    ``overlap=True`` launches each round's reduces from
    backward hooks as buckets complete.
  * ``arena="buckets"``: parameters and grads stay where the caller put them; grads are packed
    into rank-major buckets, one in-place RCCL reduce-scatter per even bucket (grouped per-owner
    reduce / broadcast for the ragged tail) delivers each owner its summed grads, Adam updates
    them, an in-place all-gather per bucket replaces the per-param broadcasts, then unpack; grads
    are released after the step.
  * ``arena="auto"``: at construction (ws > 1, a collective call) a 256 MiB sample of the gradient
    is exchanged both ways on this job's interconnect — grouped per-owner reduce + broadcast
    against reduce-scatter + all-gather plus the pack / unpack copies — and the arena whose
    estimate per step is lower (buckets only when >= 5 % faster) is built on every rank;
    ``arena_calibration`` holds the times (``_sharded.calibrate_arena``).
Ownership, and therefore optimizer-state placement, is bit-identical to the reference on all.
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
