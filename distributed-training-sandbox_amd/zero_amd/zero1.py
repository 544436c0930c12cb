"""ZeRO-1 drop-in: ``ShardedOptimizer`` of reference zero/zero1.py:43-108, MI355X-native.

Reference behaviour: ``zero_grad()`` only clears *owned* grads because the
inner optimizer's groups were filtered (zero1.py:71-74, 107-108).  Non-owners therefore still hold
last step's averaged grad A_{t-1} when the next backward accumulates into it, and the per-tensor
all-reduce + ``/ws`` (zero1.py:81-84) computes

    A_t = (Σ_r G_t^r + (ws-1) · A_{t-1}) / ws

which is the gradient the owner's Adam consumes.  This implementation reproduces that carry
without keeping full-size grads on non-owners: the owner keeps A_{t-1} for its shard in an fp32
*carry* buffer and the fused Adam kernel computes (RS_sum + (ws-1)·carry)/ws and stores the new
carry (+8 B/elem of HBM traffic).  All grads are released after the step, so ``zero_grad`` has
nothing left to clear; parameters follow the reference trajectory (tests/test_gpu_parity.py).
"""
from __future__ import annotations

from ._sharded import ShardedOptimizerBase


class ShardedOptimizer(ShardedOptimizerBase):
    _carry = True
    _variant = 1
