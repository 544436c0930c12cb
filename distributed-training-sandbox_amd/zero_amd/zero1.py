"""ZeRO-1 drop-in: ``ShardedOptimizer`` of reference zero/zero1.py:43-108, MI355X-native.

Reference behaviour: ``zero_grad()`` only clears *owned* grads because the
inner optimizer's groups were filtered (zero1.py:71-74, 107-108).  Non-owners therefore still hold
last step's averaged grad A_{t-1} when the next backward accumulates into it, and the per-tensor
all-reduce + ``/ws`` (zero1.py:81-84) computes

    A_t = (Σ_r G_t^r + (ws-1) · A_{t-1}) / ws

which is the gradient the owner's Adam consumes.  This implementation reproduces that carry
without keeping full-size averaged grads on non-owners: the owner keeps A_{t-1} for its shard in
an fp32 *carry* buffer and the fused Adam kernel computes (sum + carry_mul·carry)/ws and stores
the new carry (+8 B/elem of HBM traffic); parameters follow the reference trajectory
(tests/test_gpu_parity.py).

Mechanism (the same engine as ZeRO-2, ``zero2.py``):
  * default ``arena="flat"``: every parameter is a view of one owner-major *flat parameter
    arena*, and after ``zero_grad()`` every ``p.grad`` is a view of the matching slot of a flat
    gradient arena, so backward accumulates straight into it.  A step is a few *rounds*, each ONE
    RCCL group of per-owner ``ncclReduce`` (each owner's window of the gradient arena, summed
    into its reduced buffer: the reference's per-tensor all-reduce, zero1.py:81-84, delivered only
    where it is consumed), the fused Adam on the own window (carry folded in), and ONE RCCL group
    of in-place ``ncclBroadcast`` of every owner's updated window (zero1.py:91-102).  No pack, no
    unpack.  The grads stay arena views holding this rank's local gradient after the step;
    ``zero_grad()`` zeroes them.  The carry multiplier is (ws-1) for a parameter whose grad is
    still the arena view at the next step (``opt.zero_grad()`` keeps the non-owned A_{t-1}
    semantics) and 0 when the caller replaced it (``model.zero_grad()``), per parameter.
  * ``arena="buckets"``: parameters and grads stay where the caller put them; grads are packed
    into rank-major buckets, moved by in-place reduce-scatter / all-gather (plus per-owner grouped
    reduce / broadcast for the ragged tail), unpacked; grads are released after the step.
  * ``arena="auto"``: the two exchanges timed on a gradient sample at construction, the faster
    built on every rank (as zero2.py describes).
"""
from __future__ import annotations

from ._sharded import ShardedOptimizerBase


class ShardedOptimizer(ShardedOptimizerBase):
    _carry = True
    _variant = 1
