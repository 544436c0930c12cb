# Round-2 snapshot of zero_amd/zero3.py (commit 1653aab), loaded only by tools/z3_host_ab.py as
# the host-time A/B baseline; not part of the product.
"""ZeRO-3 drop-in: ``Zero3ParamManager``, ``register_zero3_hooks`` and ``ShardedOptimizer`` of
reference zero/zero3.py:25-168, MI355X-native.

Reference behaviour:
  * every parameter's ``.data`` is replaced by its dim-0 chunk ``chunk(ws, 0)[rank]``
    (zero3.py:105-110) — Layout Z;
  * module hooks all-gather the chunks into the full tensor before forward and backward
    (``materialize``, zero3.py:36-41) and re-chunk after (``release``, zero3.py:43-52, which also
    shrinks a full-size grad to the local chunk);
  * ``step()`` chunks any still-full grad, all-reduces every (shard-sized) grad and divides by ws
    (zero3.py:131-147) — and then the ``for … else`` at zero3.py:150-153 sets EVERY ``param.grad``
    to None, so the inner Adam never sees a gradient and parameters never change.

Here every rank's chunks of every parameter live in ONE flat *chunk arena* (slot i holds param
i's padded chunk of S_i = ceil(d0/ws)·row elements, 64-element aligned, zero beyond the rank's
real rows), and ``param.data`` is a view of its slot between gathers.  Two modes:

  * ``update=False`` (default): reference semantics, bit-for-bit in what is observable — the
    reduced shard grads are computed (one grouped RCCL all-reduce per step, exposed as
    ``last_reduced_grads``) and then discarded; parameters stay at their initial values.
  * ``update=True``: the ZeRO-3 the reference intends.  A post-accumulate-grad hook on every
    parameter hands its full-size gradient, as soon as backward has produced it, to a bucketed
    reduce-scatter (one RCCL group per bucket, buckets in backward order, launched strictly in
    order so every rank issues the same sequence) that writes the summed chunk straight into a
    flat *grad chunk arena*; the full gradient is released right after, so gradient memory is one
    bucket in flight plus 1/ws of the model.  ``step()`` is one fused HIP Adam launch over the
    chunk arena (grad /ws folded in) — data-parallel Adam, sliced.  Every rank updates its chunk
    of every parameter, so the inner optimizer's groups are not filtered in this mode and
    ``optimizer.state[p]`` holds chunk-shaped views of the flat fp32 state.

``materialize`` is a zero-copy RCCL all-gather from the chunk slot (already padded to S) straight
into the full tensor (rows of torch.chunk are contiguous: full = [chunk_0 | … | chunk_{ws-1}]),
grouped per module, on a side HIP stream, and the NEXT module's gather is prefetched there while
the current module computes (the order is learned on the first iteration).  Reduce-scatters run
on the same side stream, so one communicator sees one totally ordered sequence of collectives.
"""
from __future__ import annotations

import contextlib
import time

import numpy as np
import torch
from torch.optim import Optimizer

from . import _lib
from ._lib import ZS_BF16, ZS_BF16_SPLIT, ZS_F32
from ._sharded import adam_group_hparams
from .comm import RcclComm, comm_stream, zs_dtype
from .engine import ALIGN_ELEMS, probed_zeros
from .kernels import AdamSet, adam_hparams, stream_handle
from .training_utils.utils import get


def _chunk_geom(d0: int, ws: int, rank: int):
    """torch.chunk(ws, dim=0) rows: chunk size cs = ceil(d0/ws), rank's rows [r0, r1)."""
    cs = -(-d0 // ws) if d0 else 0
    r0, r1 = min(rank * cs, d0), min((rank + 1) * cs, d0)
    return cs, r0, r1


def _round_up(x: int, a: int) -> int:
    return -(-int(x) // a) * a


def _group_ctx(comm):
    grp = getattr(comm, "group", None)
    return grp() if grp is not None else contextlib.nullcontext()


class _GatherRuntime:
    """Side-stream collectives of one ShardedOptimizer: module all-gathers with one-ahead prefetch
    (and, in update mode, the gradient reduce-scatters, on the same stream).

    The first iteration records the order in which module groups are materialised (forward, then
    backward); afterwards each materialise also launches the gather of the next group in that
    order, so the all-gather overlaps the current module's compute.  ``end_iteration`` (called at
    the end of step()) prefetches the first group of the next iteration."""

    def __init__(self, ws, rank, comm, device):
        self.ws, self.rank, self.comm, self.device = ws, rank, comm, device
        self.stream = comm_stream(device)
        self.pending = {}      # key -> (list[(manager, full_tensor)], event, holding tensor)
        self.sequence = []     # learned order of group keys
        self.pos = 0
        self.recording = True
        self.key_managers = {}
        self.n_gathers = 0
        self.n_prefetch_hits = 0
        self.gather_events = None  # optional list of (start, end, bus_bytes) per gather group
        self._tables = {}          # key -> grouped all-gather pointer table (see _table)

    def launch(self, key, managers):
        """Enqueue the all-gather of ``managers`` on the side stream; returns immediately."""
        if key in self.pending or not managers:
            return
        if self.ws == 1 and not any(m.fp8 for m in managers):
            # the shard is the whole parameter: nothing to gather, no stream to synchronise with
            self.pending[key] = ([(m, m._gather_prepare(None)[1]) for m in managers], None, None)
            self.n_gathers += 1
            return
        ev_ready = torch.cuda.Event()
        ev_ready.record(torch.cuda.current_stream(self.device))  # shards may just have been updated
        timed = self.gather_events is not None and self.ws > 1
        plan = self._table(key, managers)
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev_ready)
            if timed:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(self.stream)
            hold = None
            if plan is not None:
                # one allocation for the module's full tensors and ONE library call for its RCCL
                # group of all-gathers (zero-copy from the chunk-arena slots)
                send, count, offs, total, dt, es, spans = plan
                hold = torch.empty(total, dtype=managers[0].shard.dtype, device=self.device)
                recv = np.uint64(hold.data_ptr()) + offs * np.uint64(es)
                self.comm.all_gather_group(send, recv, count, dt, self.stream)
                out = [(m, hold[o:o + n]) for m, (o, n) in zip(managers, spans)]
            else:
                # kernels (fp8 quantisation) before the RCCL group, dequantisation after: an RCCL
                # group only launches its collectives at group end; every buffer a collective of
                # the group touches is referenced from `states` until the group has ended
                states = [m._gather_prepare(self.stream) for m in managers]
                with _group_ctx(self.comm):
                    for m, st in zip(managers, states):
                        m._gather_issue(self.comm, self.stream, st)
                out = [(m, m._gather_finish(self.stream, st)) for m, st in zip(managers, states)]
            ev = torch.cuda.Event()
            ev.record(self.stream)
            if timed:  # ring all-gather bus bytes: (ws-1)/ws of the gathered tensor, per rank
                bus = sum(m.gather_bytes() for m in managers) * (self.ws - 1)
                self.gather_events.append((e0, _timed_after(self.stream), bus))
        self.pending[key] = (out, ev, hold)
        self.n_gathers += 1

    def _table(self, key, managers):
        """The cached pointer table of a module's grouped all-gather (chunk-arena managers with
        a communicator that takes tables), or None for the per-parameter path."""
        if key in self._tables:
            return self._tables[key]
        plan = None
        if (hasattr(self.comm, "all_gather_group") and managers
                and all(m.send_slot is not None and not m.fp8 for m in managers)
                and len({m.shard.dtype for m in managers}) == 1):
            ws = self.ws
            es = managers[0].shard.element_size()
            sizes = [ws * m.S for m in managers]
            offs, o = [], 0
            for n in sizes:
                offs.append(o)
                o += -(-n // ALIGN_ELEMS) * ALIGN_ELEMS  # every full tensor 64-element aligned
            from .comm import zs_dtype

            plan = (np.array([m.send_slot.data_ptr() for m in managers], np.uint64),
                    np.array([m.S for m in managers], np.int64), np.array(offs, np.uint64),
                    max(o, 1), zs_dtype(managers[0].shard.dtype), es,
                    [(off, m.numel) for off, m in zip(offs, managers)])
        self._tables[key] = plan
        return plan

    def _prefetch(self, i):
        if 0 <= i < len(self.sequence):
            key = self.sequence[i]
            self.launch(key, self.key_managers.get(key))

    def materialize(self, key, managers):
        if self.recording:
            self.sequence.append(key)
        else:
            if self.pos < len(self.sequence) and self.sequence[self.pos] == key:
                self.pos += 1
            elif key in self.sequence[self.pos:]:
                self.pos = self.sequence.index(key, self.pos) + 1
            self._prefetch(self.pos)  # the next group, while this one computes
        if key in self.pending:
            self.n_prefetch_hits += 1
        self.launch(key, managers)
        out, ev, hold = self.pending.pop(key)
        if ev is None:  # ws == 1
            for m, full in out:
                m._install_full(full)
            return
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        if hold is not None:  # one allocation behind all of the module's full tensors
            hold.record_stream(cur)
        for m, full in out:
            if hold is None:
                full.record_stream(cur)
            m._install_full(full)

    def end_iteration(self):
        if self.sequence:
            self.recording = False
        self.pending.clear()
        self.pos = 0
        self._prefetch(0)


def _timed_after(stream):
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    return e


class Zero3ParamManager:
    """zero3.py:25-52: tracks one parameter's dim-0 shard and gathers / releases the full tensor.

    Standalone use (the reference's constructor): ``param.data`` must already be this rank's
    chunk; the gathers then run on a private side-stream runtime over a communicator created on
    first use (a collective call, so every rank must materialise the same parameters)."""

    def __init__(self, param, shard_idx, world_size, shard_dim=0, *, runtime=None, shard=None,
                 full_shape=None, keep_full_grad=False, gather_dtype=None, send_slot=None):
        if shard_dim != 0:
            raise NotImplementedError("zero_amd ZeRO-3 shards along dim 0 (as zero3.py:106)")
        self.param = param
        self.shard_idx = shard_idx
        self.world_size = world_size
        self.shard_dim = shard_dim
        self.full_data = None
        self.runtime = runtime
        self.full_shape = tuple(full_shape if full_shape is not None else param.shape)
        self.shard = shard if shard is not None else param.data
        self.keep_full_grad = keep_full_grad
        d0 = self.full_shape[0] if self.full_shape else 1
        self.row = int(np.prod(self.full_shape[1:])) if len(self.full_shape) > 1 else 1
        self.cs, self.r0, self.r1 = _chunk_geom(d0, world_size, shard_idx)
        self.S = self.cs * self.row  # padded chunk elements (equal on every rank)
        self.numel = int(np.prod(self.full_shape)) if self.full_shape else 1
        # S elements starting at the shard, zero beyond its rows (the chunk arena's slot): the
        # all-gather sends it as it is, so uneven chunks need no padding copy
        self.send_slot = send_slot
        if gather_dtype not in (None, "fp8"):
            raise ValueError(f"gather_dtype must be None or 'fp8' (got {gather_dtype!r})")
        # fp8 only for matrices (row-wise scales); vectors (biases, norms) gather as they are
        self.fp8 = gather_dtype == "fp8" and len(self.full_shape) >= 2

    def gather_bytes(self) -> int:
        """Bytes this rank contributes to one all-gather of the parameter."""
        return self.S + 4 * self.cs if self.fp8 else self.S * self.shard.element_size()

    # -- gather ----------------------------------------------------------------------------------
    # Three phases so a module's managers share one RCCL group: prepare (kernels on the side
    # stream), issue (collectives, inside the group), finish (kernels after the group).
    def _gather_prepare(self, stream):
        dev, ws = self.shard.device, self.world_size
        rows = self.r1 - self.r0
        if self.fp8:  # 1 byte per element + one fp32 scale per row
            q = torch.zeros(self.S, dtype=torch.uint8, device=dev)
            sc = torch.ones(self.cs, dtype=torch.float32, device=dev)
            if rows:
                _lib.call("zs_fp8_quantize_rows", self.shard.data_ptr(), zs_dtype(self.shard.dtype),
                          q.data_ptr(), sc.data_ptr(), rows, self.row, stream_handle(stream))
            return (q, sc, torch.empty(ws * self.S, dtype=torch.uint8, device=dev),
                    torch.empty(ws * self.cs, dtype=torch.float32, device=dev))
        if self.send_slot is not None:
            send = self.send_slot
        else:
            send = self.shard.reshape(-1)
            if send.numel() != self.S:  # standalone short / empty chunk: pad to S elements
                pad = torch.zeros(self.S, dtype=send.dtype, device=dev)
                pad[:send.numel()].copy_(send)
                send = pad
        if ws == 1:  # the shard is the whole parameter: nothing to gather
            return (send, send)
        return (send, torch.empty(ws * self.S, dtype=self.shard.dtype, device=dev))

    def _gather_issue(self, comm, stream, st):
        if self.fp8:
            q, sc, full_q, full_sc = st
            comm.all_gather(q, full_q, stream)
            comm.all_gather(sc, full_sc, stream)
        else:
            send, full = st
            if full is not send:
                comm.all_gather(send, full, stream)

    def _gather_finish(self, stream, st):
        if not self.fp8:
            return st[1]
        _, _, full_q, full_sc = st
        full = torch.empty(self.world_size * self.S, dtype=self.shard.dtype, device=self.shard.device)
        _lib.call("zs_fp8_dequantize_rows", full_q.data_ptr(), full_sc.data_ptr(), full.data_ptr(),
                  zs_dtype(full.dtype), self.world_size * self.cs, self.row, stream_handle(stream))
        return full

    def _install_full(self, full):
        self.full_data = full[:self.numel].view(self.full_shape)
        self.param.data = self.full_data

    def _runtime(self):
        if self.runtime is None:
            self.runtime = _GatherRuntime(self.world_size, self.shard_idx, RcclComm(),
                                          self.shard.device)
        return self.runtime

    def materialize(self):
        """zero3.py:36-41 for this one parameter."""
        rt = self._runtime()
        key = ("param", id(self))
        rt.launch(key, [self])
        out, ev, hold = rt.pending.pop(key)
        cur = torch.cuda.current_stream(self.shard.device)
        if ev is not None:
            cur.wait_event(ev)
        if hold is not None:
            hold.record_stream(cur)
        for m, full in out:
            full.record_stream(cur)
            m._install_full(full)

    def release(self):
        """zero3.py:43-52: back to the local shard; shrink a full-size grad to its local rows
        (reference mode) or leave it to the reduce-scatter hook (update mode)."""
        self.param.data = self.shard
        g = self.param.grad
        if g is not None and g.shape != self.shard.shape and not self.keep_full_grad:
            self.param.grad.data = g.data.reshape(self.full_shape)[self.r0:self.r1].clone()
        self.full_data = None


def register_zero3_hooks(model, param_managers, units=None, reshard_after_forward=True):
    """zero3.py:56-77: forward / backward pre-hooks materialise a module's direct parameters (one
    grouped all-gather, prefetched on the side stream), post-hooks release them.

    ``units`` (an extension; None = the reference's per-module hooks): modules gathered as ONE
    group each — every managed parameter anywhere inside a unit is materialised by the unit's
    pre-hooks and released by its post-hooks, as FSDP2's ``fully_shard`` of each transformer block
    does (fsdp/train_fsdp.py:90-97).  One RCCL group and four hooks per block instead of per
    Linear / norm.  Modules outside every unit keep per-module gathers of their direct params.

    ``reshard_after_forward`` (FSDP2's flag, fsdp/train_fsdp.py:84-94): True (the reference's
    hooks, FSDP2 "ZeRO-3") releases after forward and gathers again for backward; False (FSDP2
    "ZeRO-2") keeps the gathered parameters from forward through backward — one gather per group
    per step instead of two, full parameters resident between forward and backward."""
    if all(m.world_size == 1 and not m.fp8 for m in param_managers.values()):
        # one rank: every shard is its whole parameter, so materialize / release are identities —
        # hooks would only cost host time (a forward whose host enqueue falls behind the GPU)
        return []
    runtimes = {m.runtime for m in param_managers.values() if m.runtime is not None}
    mod_managers = {}
    covered = set()
    unit_ids = set()
    for u in units or ():
        ms, seen = [], set()
        for p in u.parameters():
            if p in param_managers and id(p) not in seen:
                seen.add(id(p))
                ms.append(param_managers[p])
        mod_managers[id(u)] = ms
        unit_ids.add(id(u))
        covered |= seen
    for mod in model.modules():
        if id(mod) in unit_ids:
            continue
        ms = [param_managers[p] for _, p in mod.named_parameters(recurse=False)
              if p in param_managers and id(p) not in covered]
        mod_managers[id(mod)] = ms
    for rt in runtimes:
        rt.key_managers = {}
        rt._tables = {}  # a key's managers may differ from an earlier registration
        for mod in model.modules():
            ms = mod_managers[id(mod)]
            if ms:
                rt.key_managers[("fwd", id(mod))] = ms
                rt.key_managers[("bwd", id(mod))] = ms

    def make_pre(phase):
        def pre_hook(module, *args):
            ms = mod_managers.get(id(module)) or []
            if not ms:
                return None
            if phase == "bwd" and not reshard_after_forward and all(
                    m.full_data is not None for m in ms):
                return None  # still gathered from forward
            rt = ms[0].runtime
            if rt is None:
                for m in ms:
                    m.materialize()
            else:
                rt.materialize((phase, id(module)), ms)
            return None
        return pre_hook

    def make_post(phase):
        def post_hook(module, *args):
            if phase == "fwd" and not reshard_after_forward:
                return None  # kept for backward
            for m in mod_managers.get(id(module)) or []:
                m.release()
            return None
        return post_hook

    handles = []
    for m in model.modules():
        # the reference hooks every module (zero3.py:73-77); a module without managed parameters
        # has nothing to gather or release, so it is left unhooked (a full backward hook would
        # only wrap its inputs and outputs in autograd nodes for nothing)
        if not mod_managers[id(m)]:
            continue
        handles.append(m.register_forward_pre_hook(make_pre("fwd")))
        handles.append(m.register_forward_hook(make_post("fwd")))
        handles.append(m.register_full_backward_pre_hook(make_pre("bwd")))
        handles.append(m.register_full_backward_hook(make_post("bwd")))
    return handles


class _ChunkArena:
    """This rank's dim-0 chunks of every parameter in one flat buffer (Layout Z, zero3.py:107-108).

    slot i: S_i = ceil(d0/ws)·row elements (the padded chunk every rank gathers), 64-element
    aligned; the rank's real rows fill the first ln_i elements and the rest stays zero."""

    def __init__(self, params, ws: int, rank: int, align: int = ALIGN_ELEMS):
        self.ws, self.rank = ws, rank
        self.full_shapes, self.rows, self.S, self.ln, self.slot, self.shard_shapes = [], [], [], [], [], []
        self.numel = []
        off = 0
        for p in params:
            fs = tuple(p.shape)
            d0 = fs[0] if fs else 1
            row = int(np.prod(fs[1:])) if len(fs) > 1 else 1
            cs, r0, r1 = _chunk_geom(d0, ws, rank)
            self.full_shapes.append(fs)
            self.rows.append((r0, r1, row))
            self.S.append(cs * row)
            self.ln.append((r1 - r0) * row)
            self.shard_shapes.append((r1 - r0,) + fs[1:])
            self.numel.append(int(np.prod(fs)) if fs else 1)
            self.slot.append(off)
            off += _round_up(cs * row, align)
        self.total = max(off, align)
        self.S = np.asarray(self.S, np.int64)
        self.ln = np.asarray(self.ln, np.int64)
        self.slot = np.asarray(self.slot, np.int64)
        p0 = params[0]
        self.dtype, self.device = p0.dtype, p0.device
        self.P = torch.zeros(self.total, dtype=self.dtype, device=self.device)
        for i, p in enumerate(params):
            r0, r1, row = self.rows[i]
            n, s = int(self.ln[i]), int(self.slot[i])
            if n:
                self.P[s:s + n].copy_(p.detach().reshape(-1)[r0 * row:r0 * row + n])

    def shard(self, i: int) -> torch.Tensor:
        s, n = int(self.slot[i]), int(self.ln[i])
        return self.P[s:s + n].view(self.shard_shapes[i])

    def send_slot(self, i: int) -> torch.Tensor:
        s = int(self.slot[i])
        return self.P[s:s + int(self.S[i])]


class _GradReducer:
    """update mode: full-size gradients → summed chunks in the grad chunk arena, from backward.

    Parameters are grouped in reverse index order (the order backward produces a sequential
    model's grads) into buckets of at most ``bucket_bytes`` of full gradient.  A
    post-accumulate-grad hook marks a parameter ready; a complete bucket whose predecessors have
    all been launched is reduce-scattered at once — one RCCL group on the side stream, behind an
    event on the stream that produced the grads — and its full gradients are released (their
    memory returns to torch's allocator once the side stream has passed the collective).  The end
    of backward (an autograd callback) launches whatever is left in the same fixed order, so every
    rank issues the same collective sequence, and makes the compute stream wait for the last one."""

    def __init__(self, opt, bucket_bytes: int):
        self.opt = opt
        arena = opt._arena
        n = len(opt.params)
        es = opt.params[0].element_size()
        groups, cur, cur_b = [], [], 0
        for i in reversed(range(n)):
            b = arena.numel[i] * es
            if cur and cur_b + b > bucket_bytes:
                groups.append(cur)
                cur, cur_b = [], 0
            cur.append(i)
            cur_b += b
        if cur:
            groups.append(cur)
        self.groups = groups
        self.K = len(groups)
        self.bucket_of = np.zeros(n, np.int64)
        for k, g in enumerate(groups):
            self.bucket_of[g] = k
        self._size = np.array([len(g) for g in groups], np.int64)
        self.ev_done = [torch.cuda.Event() for _ in range(self.K)]
        self.timing = None  # optional list of (start, end, bus_bytes) per launched bucket
        self._rs_tables = {}
        self.reset()

    def reset(self):
        n = len(self.opt.params)
        # buckets the last backward launched before it ended (the rest: flushed at its end)
        self.last_launched_in_backward = getattr(self, "launched_in_backward", 0)
        self.pending = self._size.copy()
        self.marked = np.zeros(n, bool)
        self.had_grad = np.zeros(n, bool)
        self.local_grads = [None] * n  # ws == 1: the grad itself is the chunk's gradient
        self.next = 0
        self.callback_queued = False
        self.launched_in_backward = 0

    def register_hooks(self):
        return [p.register_post_accumulate_grad_hook(lambda _p, i=i: self.on_grad_ready(i))
                for i, p in enumerate(self.opt.params) if p.requires_grad]

    def on_grad_ready(self, i: int):
        if self.marked[i]:
            raise RuntimeError(
                "zero_amd ZeRO-3: gradient of parameter %d accumulated twice before step(); "
                "update mode reduce-scatters each gradient once per step" % i)
        self.marked[i] = True
        self.pending[self.bucket_of[i]] -= 1
        if not self.callback_queued:
            self.callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._end_backward)
        while self.next < self.K and self.pending[self.next] == 0:
            self._launch(self.next)
            self.launched_in_backward += 1
            self.next += 1

    def _end_backward(self):
        self.flush()
        self.install_shard_grads()

    def flush(self):
        """Launch every bucket not launched yet, in the fixed order."""
        while self.next < self.K:
            self._launch(self.next)
            self.next += 1

    def install_shard_grads(self):
        """After backward every parameter shows its (summed, not yet averaged) gradient chunk, the
        shard-size grad the reference's release() leaves (zero3.py:49-51)."""
        opt = self.opt
        if opt.world_size == 1:
            return
        cur = torch.cuda.current_stream(opt._arena.device)
        if self.K:
            cur.wait_event(self.ev_done[self.K - 1])
        for i, p in enumerate(opt.params):
            if (self.had_grad[i] and p.data.shape == opt._arena.shard_shapes[i]
                    and opt._G.dtype == p.dtype):  # (a bf16 exchange's chunks stay internal)
                s, n = int(opt._arena.slot[i]), int(opt._arena.ln[i])
                p.grad = opt._G[s:s + n].view(opt._arena.shard_shapes[i])

    def _rs_table(self, k: int):
        """Bucket k's reduce-scatter destinations (grad chunk-arena slots) and counts, cached."""
        t = self._rs_tables.get(k)
        if t is None:
            from .comm import zs_dtype

            opt, idx = self.opt, np.asarray(self.groups[k], np.int64)
            G = opt._G
            t = (np.uint64(G.data_ptr()) + (opt._arena.slot[idx] * G.element_size()).astype(np.uint64),
                 np.ascontiguousarray(opt._arena.S[idx], np.int64), zs_dtype(G.dtype))
            self._rs_tables[k] = t
        return t

    def _launch(self, k: int):
        opt = self.opt
        ar, ws = opt._arena, opt.world_size
        if ws == 1:  # nothing to exchange: Adam reads the local grad in place
            for i in self.groups[k]:
                g = opt.params[i].grad
                if g is not None:
                    if g.numel() != ar.numel[i] or not g.is_contiguous() or g.dtype != ar.dtype:
                        raise ValueError("zero_amd ZeRO-3: grads must be contiguous, full-size and "
                                         "of the parameter dtype")
                    self.had_grad[i] = True
                    self.local_grads[i] = g
            return
        dev = ar.device
        cur = torch.cuda.current_stream(dev)
        wdt = opt._G.dtype  # on the wire: the param dtype, or bf16 for grad_comm="bf16"
        sends = []  # (param index, send buffer): alive until the RCCL group has been enqueued
        for i in self.groups[k]:
            p = opt.params[i]
            g = p.grad
            S, N = int(ar.S[i]), int(ar.numel[i])
            if g is None:
                send = torch.zeros(ws * S, dtype=wdt, device=dev)  # every rank takes part
            else:
                if g.numel() != N or g.dtype != ar.dtype:
                    raise ValueError("zero_amd ZeRO-3 update mode needs the full-size gradient "
                                     "(param %d: got %s)" % (i, tuple(g.shape)))
                self.had_grad[i] = True
                flat = g.reshape(-1) if g.is_contiguous() else g.contiguous().reshape(-1)
                if wdt != ar.dtype:  # bf16 exchange: gfx950 RNE conversion into the send buffer
                    from .kernels import convert

                    send = torch.empty(ws * S, dtype=wdt, device=dev) if N == ws * S else \
                        torch.zeros(ws * S, dtype=wdt, device=dev)
                    convert(flat, send[:N], cur)
                elif N == ws * S:
                    send = flat  # zero-copy: rows of torch.chunk are contiguous
                else:  # uneven chunks: every rank sends ws*S elements
                    send = torch.zeros(ws * S, dtype=wdt, device=dev)
                    send[:N].copy_(flat)
            sends.append((i, send))
        ready = torch.cuda.Event()
        ready.record(cur)
        cs = opt.runtime.stream
        cs.wait_event(ready)
        if self.timing is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(cs)
        if hasattr(opt.comm, "reduce_scatter_group"):  # the bucket's RCCL group: ONE call
            recv, count, dt = self._rs_table(k)
            sp = np.fromiter((t.data_ptr() for _, t in sends), np.uint64, len(sends))
            opt.comm.reduce_scatter_group(sp, recv, count, dt, cs)
        else:
            with _group_ctx(opt.comm):
                for i, send in sends:
                    s = int(ar.slot[i])
                    opt.comm.reduce_scatter(send, opt._G[s:s + int(ar.S[i])], cs)
        # the group has been enqueued: a buffer freed from here on is only reused after it
        for i, send in sends:
            send.record_stream(cs)
            opt.params[i].grad = None
        self.ev_done[k].record(cs)
        if self.timing is not None:
            bus = sum(int(ar.S[i]) * ws for i, _ in sends) * opt._G.element_size() * (ws - 1) / ws
            self.timing.append((e0, _timed_after(cs), bus))
        del sends


class ShardedOptimizer:
    """zero3.py:81-168 with ``update`` selecting reference (no-op) or real ZeRO-3 updates."""

    def __init__(self, optimizer: Optimizer, *, update: bool = False, comm=None, sync: bool = True,
                 gather_dtype=None, bucket_mb: float = 128.0, grad_comm: str | None = None):
        if not isinstance(optimizer, torch.optim.Adam):
            raise TypeError("zero_amd ShardedOptimizer wraps torch.optim.Adam / AdamW")
        self.optimizer = optimizer
        self.original_param_groups = optimizer.param_groups
        self.params = [p for group in self.original_param_groups for p in group["params"]]
        self._group_of = [gi for gi, g in enumerate(self.original_param_groups) for _ in g["params"]]
        self._groups = list(self.original_param_groups)
        world_size = get("ws")
        rank = get("rank")
        params_per_rank = len(self.params) // world_size
        remainder = len(self.params) % world_size
        start_idx = rank * params_per_rank + min(rank, remainder)
        end_idx = start_idx + params_per_rank + (1 if rank < remainder else 0)
        self.local_param_indices = list(range(start_idx, end_idx))
        self.local_params = set(self.params[i] for i in self.local_param_indices)
        self.world_size, self.rank = world_size, rank
        self.update = bool(update)
        self._sync = sync
        # grad_comm="bf16" (update mode, fp32 params): full grads are converted to bf16 before the
        # reduce-scatter, so the exchange moves 2 B per element; opt-in
        if grad_comm not in (None, "bf16"):
            raise ValueError(f"grad_comm must be None or 'bf16' (got {grad_comm!r})")
        if grad_comm and not update:
            raise ValueError("grad_comm='bf16' applies to update mode (reference mode keeps the "
                             "reference's fp32 all-reduce)")
        self._grad_comm = grad_comm if self.params[0].dtype == torch.float32 else None

        dev = self.params[0].device
        if dev.type != "cuda":
            raise RuntimeError("zero_amd: parameters must live on a GPU; there is no CPU path")
        dtype = self.params[0].dtype
        for p in self.params:
            if p.device != dev or p.dtype != dtype:
                raise TypeError("zero_amd: all parameters must share one device and dtype")
        if comm is None:
            comm = RcclComm()
        self.comm = comm
        self.runtime = _GatherRuntime(world_size, rank, comm, dev)
        # zero3.py:104-110: every param becomes its dim-0 chunk — here a view of the chunk arena
        # (the full tensor is released); one manager per param
        self._arena = _ChunkArena(self.params, world_size, rank)
        self.param_managers = {}
        for i, param in enumerate(self.params):
            shard = self._arena.shard(i)
            param.data = shard
            self.param_managers[param] = Zero3ParamManager(
                param, rank, world_size, 0, runtime=self.runtime, shard=shard,
                full_shape=self._arena.full_shapes[i], keep_full_grad=self.update,
                gather_dtype=gather_dtype, send_slot=self._arena.send_slot(i))
        if not self.update:
            for group in self.optimizer.param_groups:  # zero3.py:114-115
                group["params"] = [p for p in group["params"] if p in self.local_params]
        self.grad_hooks = {}
        self.communication_time = 0.0
        self.step_time = 0.0
        self.last_reduced_grads = None
        self.timing_events = None  # optional list of (start, end, bytes) around each Adam launch
        self._comm_spans = []      # (start event, end event) pairs not yet added to comm time
        self._reducer = None
        self._G = None
        self._hook_handles = []
        if self.update:
            self._build_update_state()
            self._reducer = _GradReducer(self, int(bucket_mb * (1 << 20)))
            self._hook_handles = self._reducer.register_hooks()

    # ------------------------------------------------------------------------------------------
    def _build_update_state(self):
        ar = self._arena
        L = ar.total
        split = ar.dtype == torch.bfloat16
        # exp_avg, exp_avg_sq (+ for bf16 params the split master's int16 residual: the fp32
        # master is the bf16 chunk + residual, include/zero_amd.h ZS_BF16_SPLIT; starts at 0)
        nlo = (L + 1) // 2 if split else 0
        state, self.placement = probed_zeros(2 * L + nlo, torch.float32, ar.device)
        self._state = state
        self._m, self._v = state[:L], state[L:2 * L]
        self._lo = state[2 * L:].view(torch.int16)[:L] if split else None
        self._vmax = None
        self._split = split
        gdt = torch.bfloat16 if self._grad_comm else ar.dtype
        self._G = torch.zeros(L, dtype=gdt, device=ar.device) if self.world_size > 1 else None
        self._steps = np.zeros(len(self.params), np.int64)
        self._adam_cache = {}
        self._retired = []
        for i, p in enumerate(self.params):
            s, n = int(ar.slot[i]), int(ar.ln[i])
            st = self.optimizer.state[p]
            st["exp_avg"] = self._m[s:s + n].view(ar.shard_shapes[i])
            st["exp_avg_sq"] = self._v[s:s + n].view(ar.shard_shapes[i])

    def grad_arena(self):
        """The flat gradient chunk arena (update mode, ws > 1): slot i holds param i's summed chunk."""
        return self._G

    # ------------------------------------------------------------------------------------------
    def _reduce_reference(self):
        """zero3.py:131-153: chunk full grads, all-reduce shard grads, /ws, then discard all."""
        cur = torch.cuda.current_stream()
        shards = []
        for param in self.params:
            g = param.grad
            if g is None:
                continue
            man = self.param_managers[param]
            if g.shape != param.data.shape:  # zero3.py:141-143
                g = g.reshape(man.full_shape)[man.r0:man.r1].contiguous()
            n = g.numel()
            if n != man.S:  # uneven torch.chunk: every rank all-reduces S elements (the
                pad = torch.zeros(man.S, dtype=g.dtype, device=g.device)  # reference deadlocks)
                pad[:n].copy_(g.reshape(-1))
                shards.append((pad, n, g.shape))
            else:
                shards.append((g.contiguous(), n, g.shape))
        ready = torch.cuda.Event()
        ready.record(cur)
        cs = self.runtime.stream
        cs.wait_event(ready)
        with _group_ctx(self.comm):
            for buf, _, _ in shards:
                self.comm.all_reduce(buf, cs)
        # after the group: the division runs behind the collectives on the side stream
        with torch.cuda.stream(cs):
            self.last_reduced_grads = [buf.reshape(-1)[:n].view(shp).div_(self.world_size)
                                       for buf, n, shp in shards]
        for buf, _, _ in shards:
            buf.record_stream(cs)
        done = _timed_after(cs)
        cur.wait_event(done)
        for param in self.params:  # zero3.py:150-153 for-else: every grad is dropped
            param.grad = None
        return done

    def _adam_rows(self, idx):
        """zs_adam_seg rows (g, master, master_out, p_out, m, v, vmax, carry, n) of the chunks of
        the params in ``idx``."""
        ar, red = self._arena, self._reducer
        es = ar.P.element_size()
        so = ar.slot[idx].astype(np.uint64)
        rows = np.zeros((len(idx), 9), np.uint64)
        if self.world_size > 1:
            rows[:, 0] = np.uint64(self._G.data_ptr()) + so * np.uint64(self._G.element_size())
        else:
            rows[:, 0] = [red.local_grads[i].data_ptr() for i in idx]
        pp = np.uint64(ar.P.data_ptr()) + so * np.uint64(es)
        if self._split:  # master = bf16 chunk (in and out) + int16 residual
            rows[:, 1], rows[:, 3] = pp, pp
            rows[:, 2] = np.uint64(self._lo.data_ptr()) + so * np.uint64(2)
        else:
            rows[:, 1], rows[:, 2] = pp, pp
        rows[:, 4] = np.uint64(self._m.data_ptr()) + so * np.uint64(4)
        rows[:, 5] = np.uint64(self._v.data_ptr()) + so * np.uint64(4)
        if self._vmax is not None:
            rows[:, 6] = np.uint64(self._vmax.data_ptr()) + so * np.uint64(4)
        rows[:, 8] = ar.ln[idx].astype(np.uint64)
        return rows

    def _step_update(self):
        red, ar = self._reducer, self._arena
        cur = torch.cuda.current_stream(ar.device)
        red.flush()  # grads assigned outside backward (or backward without hooks firing)
        done = None
        if self.world_size > 1 and red.K:
            done = red.ev_done[red.K - 1]
            cur.wait_event(done)
        idx = np.nonzero(red.had_grad & (ar.ln > 0))[0]
        self._steps[idx] += 1
        hps = {gi: adam_group_hparams(self._groups[gi], self.optimizer) for gi in set(self._group_of)}
        if any(h["amsgrad"] for h in hps.values()) and self._vmax is None:
            self._vmax = torch.zeros(ar.total, dtype=torch.float32, device=ar.device)
            for i, p in enumerate(self.params):
                s, n = int(ar.slot[i]), int(ar.ln[i])
                self.optimizer.state[p]["max_exp_avg_sq"] = self._vmax[s:s + n].view(ar.shard_shapes[i])
        if len(idx):
            rows = self._adam_rows(idx)
            keys = np.stack([np.asarray(self._group_of)[idx], self._steps[idx]], axis=1)
            for key in np.unique(keys, axis=0):
                sel = np.nonzero((keys == key).all(axis=1))[0]
                sub = np.ascontiguousarray(rows[sel])
                ck = (int(key[0]), len(sel), int(sel[0]))
                hit = self._adam_cache.get(ck)
                if hit is None or hit[0] != sub.tobytes():
                    if hit is not None:  # keep until the device is idle (hipFree would sync it)
                        self._retired.append(hit[1])
                    gz = ZS_BF16 if (self._split or (self._grad_comm and self.world_size > 1)) \
                        else ZS_F32
                    hit = (sub.tobytes(), AdamSet(sub, ZS_BF16, ZS_BF16_SPLIT) if self._split
                           else AdamSet(sub, gz))
                    self._adam_cache[ck] = hit
                h = hps[int(key[0])]
                hp = adam_hparams(h["lr"], h["beta1"], h["beta2"], h["eps"], h["weight_decay"],
                                  int(key[1]), decoupled=h["decoupled"], amsgrad=h["amsgrad"],
                                  maximize=h["maximize"], grad_div=float(self.world_size))
                if self.timing_events is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(cur)
                    hit[1].run(hp, cur)
                    self.timing_events.append((e0, _timed_after(cur), hit[1].bytes))
                else:
                    hit[1].run(hp, cur)
        step_t = {}
        for i in idx:
            s = int(self._steps[i])
            t = step_t.get(s)
            if t is None:
                t = step_t[s] = torch.tensor(float(s))
            self.optimizer.state[self.params[i]]["step"] = t
        for p in self.params:  # zero3.py:150-153: no grad survives the step
            p.grad = None
        red.reset()
        return done

    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        step_start = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream(self.params[0].device))
        with torch.no_grad():
            done = self._step_update() if self.update else self._reduce_reference()
        if done is not None and self.world_size > 1:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(self.runtime.stream)  # after the last gradient collective
            self._comm_spans.append((e0, e1))
        retired = len(self._retired) if self.update else 0
        if self._sync or retired > 64:
            torch.cuda.synchronize()
            if self.update:
                self._retired.clear()
            self._collect_comm_time()
        self.runtime.end_iteration()
        self.step_time += time.perf_counter() - step_start
        return loss

    def _collect_comm_time(self):
        """zero3.py:125,158: communication_time = from step() entry until the gradient reduction is
        done.  Measured on the device: step-entry event on the compute stream → event after the
        last gradient collective on the side stream (0 when backward already finished them)."""
        for e0, e1 in self._comm_spans:
            self.communication_time += max(0.0, e0.elapsed_time(e1) / 1e3)
        self._comm_spans.clear()

    def zero_grad(self, set_to_none: bool = True):
        self.optimizer.zero_grad(set_to_none=set_to_none)
