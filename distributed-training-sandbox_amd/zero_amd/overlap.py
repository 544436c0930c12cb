"""Backward-overlapped gradient buckets.

The reference reduces gradients only inside ``step()`` (zero1.py:80-84, zero2.py:94-113) or
``sync_gradients()`` (DDP/ddp.py:43-47), one blocking collective per tensor, after backward has
finished.  ``GradBuckets`` moves that exchange into backward:

* parameters are grouped, in reverse index order (the order a sequential model's backward
  produces them), into buckets of at most ``bucket_bytes``; a bucket never mixes parameters with
  different *keys* (the owning rank for ZeRO, so each bucket is one reduce to one root);
* every bucket is a contiguous region of one flat buffer, and ``install_views()`` (called by
  ``zero_grad``) zeroes the buffer and makes each ``p.grad`` a view of its slot, so autograd
  accumulates straight into the bucket — no pack copy;
* a post-accumulate-grad hook on every parameter counts the bucket's ready grads; when a bucket is
  complete (and every earlier bucket has been launched — the launch order is fixed, so every rank
  issues the same collective sequence) its collective is enqueued on a side HIP stream behind an
  event on the stream that produced the grad, and backward continues;
* ``flush()`` launches whatever backward did not complete (unused parameters, grads set by hand):
  a grad that is not the slot's view is copied in by the gfx950 segment-copy kernel, a missing
  grad is zero-filled.

The collective itself is the caller's (``collective(k, region, stream)``): one RCCL reduce to the
owner for ZeRO-1/2, one RCCL all-reduce for DDP.  Gradient accumulation over several backward
passes per step is not supported in this mode (a second accumulation into a launched bucket
raises).
"""
from __future__ import annotations

import numpy as np
import torch

from ._hooks import WeakCall
from .comm import StreamEvent, comm_stream
from .kernels import CopySet

ALIGN = 64  # elements: every slot 16-byte aligned for the vector kernels


def plan_grad_buckets(numels, keys, bucket_bytes: int, elem_size: int, order=None, align: int = ALIGN):
    """Greedy grouping of parameters along ``order`` (default: reverse index) into buckets of at
    most ``bucket_bytes`` (a larger parameter gets a bucket of its own) that never mix keys.
    Returns (groups, key per bucket, slot offset per param, bucket per param, bucket offsets,
    bucket lengths), offsets in elements of one flat buffer, every slot ``align``-aligned."""
    n = len(numels)
    order = list(range(n))[::-1] if order is None else [int(i) for i in order]
    if sorted(order) != list(range(n)):
        raise ValueError("order must be a permutation of the parameter indices")
    keys = list(keys)
    cap = max(1, int(bucket_bytes) // int(elem_size))
    rnd = lambda x: -(-int(x) // align) * align  # noqa: E731
    groups, cur, cur_elems = [], [], 0
    for i in order:
        if cur and (keys[i] != keys[cur[0]] or cur_elems + rnd(numels[i]) > cap):
            groups.append(cur)
            cur, cur_elems = [], 0
        cur.append(i)
        cur_elems += rnd(numels[i])
    if cur:
        groups.append(cur)
    slot = np.zeros(n, np.int64)
    bucket_of = np.zeros(n, np.int64)
    boff = np.zeros(len(groups), np.int64)
    blen = np.zeros(len(groups), np.int64)
    off = 0
    for k, g in enumerate(groups):
        boff[k] = off
        for i in g:
            slot[i] = off
            bucket_of[i] = k
            off += rnd(numels[i])
        blen[k] = off - boff[k]
    return groups, [keys[g[0]] for g in groups], slot, bucket_of, boff, blen


class GradBuckets:
    def __init__(self, params, keys, bucket_bytes: int, collective, *, order=None,
                 align: int = ALIGN):
        if not params:
            raise ValueError("GradBuckets: no parameters")
        self.params = list(params)
        self.device = params[0].device
        self.dtype = params[0].dtype
        if self.device.type != "cuda":
            raise RuntimeError("zero_amd: backward overlap needs GPU parameters")
        self.es = params[0].element_size()
        self.collective = collective
        n = len(self.params)
        (self.groups, self.key, self.slot, self.bucket_of, self.bucket_off,
         self.bucket_len) = plan_grad_buckets([p.numel() for p in self.params], keys, bucket_bytes,
                                              self.es, order=order, align=align)
        self.K = len(self.groups)
        off = int(self.bucket_off[-1] + self.bucket_len[-1])
        from .engine import probed_zeros  # grads stream through Adam every step: place by probe

        self.buf, self.placement = probed_zeros(max(off, align), self.dtype, self.device)
        self.comm_stream = comm_stream(self.device)
        self.ev_ready = [StreamEvent() for _ in range(self.K)]  # (comm.StreamEvent: stream flags)
        self.ev_done = [StreamEvent() for _ in range(self.K)]
        self._size = np.array([len(g) for g in self.groups], np.int64)
        self._cache = {}
        self.retired = []
        self.views_installed = False
        self.launched_in_backward = 0
        self.reset()

    # ------------------------------------------------------------------------------------------
    def region(self, k: int) -> torch.Tensor:
        o, n = int(self.bucket_off[k]), int(self.bucket_len[k])
        return self.buf[o:o + n]

    def view(self, i: int) -> torch.Tensor:
        p = self.params[i]
        o = int(self.slot[i])
        return self.buf[o:o + p.numel()].view(p.shape)

    def reset(self):
        self.pending = self._size.copy()
        self.marked = np.zeros(len(self.params), bool)
        self.next = 0

    def install_views(self):
        """zero_grad(): zero the buffer and point every p.grad at its slot."""
        self.buf.zero_()
        for i, p in enumerate(self.params):
            p.grad = self.view(i)
        self.views_installed = True

    def release(self):
        for p in self.params:
            p.grad = None
        self.views_installed = False

    def register_hooks(self):
        handles = []
        for i, p in enumerate(self.params):
            if p.requires_grad:
                # weakly: the buckets are owned by the engine (engine.gb); a strong closure would
                # be a cycle through the parameter's C++-held hook dict (_hooks.py)
                handles.append(p.register_post_accumulate_grad_hook(
                    WeakCall(self, "on_grad_ready", i)))
        return handles

    # ------------------------------------------------------------------------------------------
    def on_grad_ready(self, i: int):
        if self.marked[i]:
            raise RuntimeError(
                "zero_amd overlap: gradient of parameter %d accumulated twice before step(); "
                "backward-overlapped buckets support one backward pass per step" % i)
        self.marked[i] = True
        self.pending[self.bucket_of[i]] -= 1
        while self.next < self.K and self.pending[self.next] == 0:
            self._launch(self.next)
            self.launched_in_backward += 1
            self.next += 1

    def flush(self):
        """Launch every bucket backward did not complete, in the fixed order."""
        while self.next < self.K:
            self._launch(self.next)
            self.next += 1

    def _launch(self, k: int):
        stream = torch.cuda.current_stream(self.device)
        src, dst, nb = [], [], []
        base = self.buf.data_ptr()
        for i in self.groups[k]:
            p = self.params[i]
            g = p.grad
            slot = base + int(self.slot[i]) * self.es
            if g is not None and g.data_ptr() == slot:
                continue  # autograd accumulated into the view
            if g is None and self.views_installed:
                continue  # unused parameter: its zeroed view is the gradient
            if g is not None and (g.dtype != self.dtype or g.shape != p.shape or not g.is_contiguous()):
                raise ValueError("zero_amd: grads must be contiguous and match their param's "
                                 "dtype and shape")
            src.append(0 if g is None else g.data_ptr())
            dst.append(slot)
            nb.append(p.numel() * self.es)
        if src:
            sig = np.array(src + dst, np.uint64).tobytes()
            cs = self._cache.get(k)
            if cs is None or cs[0] != sig:
                if cs is not None:  # queued kernels may still read the old table (see engine)
                    self.retired.append(cs[1])
                cs = (sig, CopySet(src, dst, nb))
                self._cache[k] = cs
            cs[1].run(stream)
        self.ev_ready[k].record(stream)
        self.comm_stream.wait_event(self.ev_ready[k])
        self.collective(k, self.region(k), self.comm_stream)
        self.ev_done[k].record(self.comm_stream)
