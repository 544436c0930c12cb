"""DDP drop-in: ``SimpleDistributedDataParallelism`` of reference DDP/ddp.py:30-60, MI355X-native
(SURVEY.md §8(f) rank 2).

Reference behaviour: ``__init__`` broadcasts every parameter from rank 0 and raises ``ValueError``
if any rank's copy differs (ddp.py:33-40); ``sync_gradients()`` all-reduces every ``param.grad``
(SUM) and divides it by the world size, one blocking c10d call per tensor (ddp.py:43-47);
``__call__`` / ``train`` / ``eval`` forward to the module.

Here the gradients live in backward-overlapped buckets (overlap.py): a post-accumulate-grad hook
launches each bucket's in-place RCCL all-reduce on a side HIP stream as soon as backward has
produced all of its grads, followed on the same stream by the gfx950 ``zs_scale`` kernel
(``/= world_size``); ``sync_gradients()`` only flushes the buckets backward did not complete,
makes the compute stream wait, and leaves every ``param.grad`` as a view of its averaged bucket
slot.  Parameters that received no gradient keep ``grad = None`` (the reference skips them).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .comm import zs_dtype
from .kernels import stream_handle
from .overlap import GradBuckets
from .training_utils.utils import get


class SimpleDistributedDataParallelism:
    def __init__(self, model: torch.nn.Module, *, bucket_mb: float = 64.0, overlap: bool = True,
                 comm=None):
        self.model = model
        self.world_size = get("ws")
        self.rank = get("rank")
        self.params = [p for p in model.parameters() if p.requires_grad]
        if not self.params:
            raise ValueError("SimpleDistributedDataParallelism: model has no trainable parameters")
        if self.world_size > 1 and comm is None:
            from .comm import RcclComm
            comm = RcclComm()
        self.comm = comm
        self._check_identical()
        self.buckets = GradBuckets(self.params, [0] * len(self.params), int(bucket_mb * (1 << 20)),
                                   self._all_reduce_mean)
        self._hooks = self.buckets.register_hooks() if overlap else []

    def _check_identical(self):
        """ddp.py:33-40 in one collective: rank 0's flat copy of every parameter, compared locally."""
        with torch.no_grad():
            flat = torch.cat([p.detach().reshape(-1).float() for p in self.model.parameters()])
            ref = flat.clone()
            if self.world_size > 1:
                dist.broadcast(ref, src=0)
            if not torch.equal(flat, ref):
                raise ValueError(
                    "Expected model parameters to be identical during `__init__`, but this is not "
                    "true. Make sure to set the seeds before creating your model")

    def _all_reduce_mean(self, k, region, stream):
        if self.world_size == 1:
            return
        self.comm.all_reduce(region, stream)
        _lib.call("zs_scale", region.data_ptr(), region.numel(), zs_dtype(region.dtype),
                  float(self.world_size), stream_handle(stream))

    def zero_grad(self):
        """Optional: zeroed bucket views as grads (autograd then accumulates in place, no copy)."""
        self.buckets.install_views()

    def sync_gradients(self):
        gb = self.buckets
        base, es = gb.buf.data_ptr(), gb.es
        # a param has a gradient if backward accumulated one (hook) or one was set by hand
        has = np.array([gb.marked[i] or (p.grad is not None and
                                         p.grad.data_ptr() != base + int(gb.slot[i]) * es)
                        for i, p in enumerate(self.params)])
        with torch.no_grad():
            gb.flush()
            cur = torch.cuda.current_stream(gb.device)
            for ev in gb.ev_done:
                cur.wait_event(ev)
            for i, p in enumerate(self.params):
                p.grad = gb.view(i) if has[i] else None
        gb.views_installed = False
        gb.reset()
        if len(gb.retired) > 64:  # tables replaced because grads moved: free at an idle point
            torch.cuda.synchronize(gb.device)
            gb.retired.clear()

    def __call__(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    def train(self):
        self.model.train()

    def eval(self):
        self.model.eval()
