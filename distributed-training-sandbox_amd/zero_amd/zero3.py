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
import ctypes
import os
import time
import weakref
from collections import OrderedDict, deque

import numpy as np
import torch
from torch.optim import Optimizer
from torch.utils.weak import WeakIdKeyDictionary

from . import _lib
from ._lib import ZS_BF16, ZS_BF16_SPLIT, ZS_F32
from . import checkpoint as ckpt
from ._hooks import WeakArgCall, WeakCall, on_param_device
from ._sharded import adam_group_hparams
from .comm import STREAM_SYNC, RcclComm, Sync, comm_stream, sync_kind, zs_dtype
from .engine import ALIGN_ELEMS, probed_zeros
from .kernels import AdamSet, adam_hparams, stream_handle
from .training_utils.utils import get

try:  # the hooks' per-module install / release in C++ (csrc/zs_host_ext.cpp, built with the library)
    from . import _hostext
except ImportError:  # (an image whose torch ABI differs: the same steps per parameter in Python)
    _hostext = None
if os.environ.get("ZERO_AMD_HOSTEXT", "1") == "0":  # A/B switch (tools/z3_host_ab.py)
    _hostext = None
# the backward's per-parameter gradient counting (reduce-scatter buckets, module releases) in C++
# hooks when the extension has them; False: one Python post-accumulate hook per parameter and
# counter (read when hooks are registered; tools/z3_host_ab.py --no-counting)
HOSTEXT_COUNTING = True
# Side-stream gathers: at most this many bytes of gathered allocations the GPU has not released
# yet (0: 1/8 of the device's memory).  Each module's allocation is made on the side stream and its
# consumer's use recorded on it, so the caching allocator reuses a block only once the consumer
# stream has passed its release; a host that runs ahead of the GPU (a GPU-bound iteration) kept
# allocating new blocks, ~68 per C5 iteration, until hipMalloc failed and the allocator
# synchronised the device and freed its cache — single host iterations of 1.4-5 s
# (profiles/r06_z3_thr_stall.json, stacks in torch.empty of _side_empty).  The runtime records a
# release marker on the consumer stream every GATHER_MARKER_EVERY releases, and before a new
# allocation waits on the host for the oldest marker while the limit would be exceeded (FSDP's
# all-gather rate limit).  In bytes, not allocations: a limit of a few modules starved a GPU whose
# iteration ends in a long step (the next forward's releases queue behind it) — the host should
# stay about an iteration ahead, as far as memory allows (profiles/r06_z3_thr_limit_*.json).
GATHER_INFLIGHT_BYTES = int(os.environ.get("ZERO_AMD_GATHER_INFLIGHT_BYTES", "0"))
GATHER_MARKER_EVERY = 4


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


# One post-accumulate-grad hook per parameter, dispatching to every ZeRO-3 callback registered for
# it (update mode has two per parameter: the reduce-scatter bucket count and the tensor-style
# backward release count).  Each hook autograd runs is a C++ -> Python transition; one per
# parameter instead of two halves that cost on every backward (291 parameters in C5).
# param -> (autograd hook handle, weak reference to its callback list).  The list itself lives in
# the dispatch closure the parameter's hook holds, so this table keeps nothing of the parameter's
# (or its optimizer's) alive.
_post_acc = WeakIdKeyDictionary()


class _Callbacks(list):
    """A parameter's callbacks (a list subclass, so the table above can hold it weakly)."""


class _PostAccHandle:
    """``remove()`` drops one callback; the autograd hook goes with the parameter's last one."""

    def __init__(self, param, fn):
        self._param, self._fn = weakref.ref(param), fn

    def remove(self):
        p = self._param()
        ent = _post_acc.get(p) if p is not None else None
        fns = ent[1]() if ent is not None else None
        if fns is None or self._fn not in fns:
            return
        fns.remove(self._fn)
        if not fns:
            ent[0].remove()
            del _post_acc[p]


def _add_post_accumulate_hook(param, fn):
    """``fn(param)`` after ``param``'s gradient has been accumulated, in registration order."""
    ent = _post_acc.get(param)
    fns = ent[1]() if ent is not None else None
    if fns is None:
        fns = _Callbacks()

        def dispatch(p, fns=fns):
            for f in tuple(fns) if len(fns) > 1 else fns:
                f(p)

        _post_acc[param] = (param.register_post_accumulate_grad_hook(dispatch), weakref.ref(fns))
    fns.append(fn)
    return _PostAccHandle(param, fn)


class _CounterHandle:
    """``remove()`` detaches a parameter from a C++ gradient counter (the counting hook stays on the
    parameter, passing through to its Python hooks)."""

    __slots__ = ("_param", "_counter")

    def __init__(self, param, counter, index: int, slot: int):
        if param._post_accumulate_grad_hooks is None:
            # torch's Python hooks dict first: a later Python registration then adds to it instead
            # of replacing the hook slot the counter shares (csrc/zs_host_ext.cpp CountingHook)
            param._post_accumulate_grad_hooks = OrderedDict()
        _hostext.attach(param, counter, int(index), int(slot))
        self._param, self._counter = weakref.ref(param), counter

    def remove(self):
        p = self._param()
        if p is not None and self._counter is not None:
            _hostext.detach(p, self._counter)
        self._counter = None


class _Gathered:
    """A module's gathered allocation (``hold``) with its managers: iterating gives the
    (manager, full tensor) pairs the per-parameter paths hold, built only when asked;
    ``_GatherRuntime.materialize`` installs them through the module's ViewPlan in one call."""

    __slots__ = ("ms", "hold", "views", "vplan")

    def __init__(self, ms, hold, views, vplan):
        self.ms, self.hold, self.views, self.vplan = ms, hold, views, vplan

    def __iter__(self):
        if self.vplan is not None:
            return iter(list(zip(self.ms, self.vplan.views(self.hold))))
        return iter([(m, self.hold.as_strided(shape, stride, off))
                     for m, (shape, stride, off) in zip(self.ms, self.views)])


def _release_group(ms):
    """Every manager of ``ms`` back to its shard (zero3.py:43-52): one ViewPlan call when the
    module has one (update mode's chunk-arena managers), else per parameter."""
    rt = ms[0].runtime if ms else None
    ent = rt._vplans.get(id(ms)) if rt is not None else None
    if ent is not None and ent[0] is ms and ent[1] is not None:
        ent[1].release()
        for m in ms:
            m._full = None  # (full_data = None, without the property call)
        if getattr(rt, "_throttled", False):
            rt.note_release(ms)
        return
    for m in ms:
        m.release()
    if getattr(rt, "_throttled", False):
        rt.note_release(ms)


class _GatherRuntime:
    """Side-stream collectives of one ShardedOptimizer: module all-gathers prefetched one wave
    ahead (and, in update mode, the gradient reduce-scatters, on the same stream).

    The first iteration records the order in which module groups are materialised (forward, then
    backward); afterwards the learned sequence is cut into *waves* of ``wave`` consecutive groups,
    and materialising the first group of wave w launches wave w + 1, so the all-gathers overlap the
    current wave's compute.  A wave is ordered as a unit: ONE ready event on the compute stream
    before its first gather, ONE done event after its last, and its consumers wait once per wave —
    a cross-stream wait on a pending HIP event costs ~10 µs of a HIP runtime thread plus ~5 µs of
    the caller (profiles/r04_hip_event_cost.json), and at one wait pair per module those were 6 of
    the 12 ms of host CPU of a simulated ws = 8 C5 iteration.  ``wave = 1`` is the per-module
    ordering.  ``end_iteration`` (called at the end of step()) prefetches the first wave of the next
    iteration.

    ``side_stream=False``: every collective is enqueued on the stream that asks for it (the current
    stream), in order with the compute — no events, no cross-stream waits, the reference's own
    structure (zero3.py:36-41 gathers synchronously in the hook).  For a model with nothing to
    overlap the collectives with (the synthetic parameter-set model of BASELINE.json configs[4])
    the GPU time is the same, and the host saves the stream ordering and the HIP runtime thread
    that polls while a cross-stream dependency is pending (≈ one core for as long as the host runs
    ahead of the GPU: profiles/r04_hip_event_cost.jsonl)."""

    def __init__(self, ws, rank, comm, device, wave: int = 1, side_stream: bool = True,
                 stream_sync: str | None = None):
        self.ws, self.rank, self.comm, self.device = ws, rank, comm, device
        # the cross-stream ordering: stream flags (the GPU resolves the wait; no HIP runtime
        # thread polls while one is pending) or HIP events (comm.Sync)
        self.sync_kind = sync_kind(stream_sync or STREAM_SYNC)
        if int(wave) < 1:
            raise ValueError(f"gather wave must be >= 1 (got {wave})")
        self.wave = int(wave)
        self._waves_launched = set()  # wave indices launched this iteration
        self._waited = {}             # done-event handle -> stream handle that waited on it
        self.stream = comm_stream(device) if side_stream else None
        self._side_h = self.stream.cuda_stream if side_stream else None
        self._side_ids = ((self.stream.stream_id, self.stream.device_index, self.stream.device_type)
                          if side_stream else None)
        # the current stream as a raw handle (torch.cuda.current_stream builds a Stream object per
        # call; the hot path only needs the handle for the library's ordered calls)
        self._dev_idx = device.index if device.index is not None else torch.cuda.current_device()
        # key -> (list[(manager, full_tensor)], done event, holding tensor, stream handle the gather
        # was ordered after, raw handle of the done event its consumers wait on)
        self.pending = {}
        self.sequence = []     # learned order of group keys
        self.pos = 0
        self.recording = True
        self.key_managers = {}
        self.n_gathers = 0
        self.n_prefetch_hits = 0
        self.gather_events = None  # optional list of (start, end, bus_bytes) per gather group
        self._tables = {}          # key -> grouped all-gather pointer table (see _table)
        self._fp8_tables = {}      # key -> fp8 gather tables (see _fp8_plan)
        # (key, producing stream) -> ready sync and key -> done sync, re-recorded every iteration:
        # a wait enqueued on a sync keeps the record it saw, and a key's next launch comes after
        # its materialise has enqueued that wait (creating them per gather cost host time)
        self._syncs = {}
        self.iteration_callbacks = []  # called by end_iteration (hook bookkeeping resets)
        self._inputs_dirty = True  # the shards may have changed since the last gather (step)
        self._streams = {}  # raw handle -> torch stream object (record_stream)
        # id(managers list) -> (that list, its _hostext.ViewPlan): the module's parameters
        # installed from its gathered allocation and released to their shards in one C++ call
        self._vplans = {}
        self.use_hostext = True  # (False: per-parameter install / release, for A/B)
        self._sync_wait = _lib.lib.zs_sync_wait  # (the bound foreign function, looked up once)
        # the host extension's one-call gather / consume (GatherFast per key; None: Python path)
        self._gfast = {}
        self._wait_fn = ctypes.cast(_lib.lib.zs_sync_wait, ctypes.c_void_p).value
        self._consume = getattr(_hostext, "consume", None) if _hostext is not None else None
        self.use_gather_fast = True  # (False: the Python gather / consume, for A/B)
        # the gather rate limit (GATHER_INFLIGHT_BYTES): on for an optimizer's side-stream runtime, whose
        # allocations are released through _release_group
        self._throttled = False
        self.max_inflight_bytes = GATHER_INFLIGHT_BYTES or None  # (default set at first use)
        self._marker_every = GATHER_MARKER_EVERY
        self._out_bytes = 0         # gathered bytes not known to be released on the GPU
        self._out_n = 0             # ... and their allocations
        self._markers = deque()     # (flag sync, epoch, bytes, allocations it covers), oldest first
        self._rel_syncs = {}        # consumer stream handle -> [flag sync, its latest epoch]
        self._rel_bytes = self._rel_n = 0  # released since the last marker
        self._counted = {}          # pending key -> its bytes counted in _out_bytes
        self._nbytes_of = {}        # id(managers list) -> (that list, its gathered bytes)
        self.n_throttle_waits = 0

    # -- the gather rate limit (GATHER_INFLIGHT_BYTES) ------------------------------------------------
    def _nbytes(self, managers) -> int:
        ent = self._nbytes_of.get(id(managers))
        if ent is None or ent[0] is not managers:
            n = sum(m.numel for m in managers) * managers[0].shard.element_size() if managers else 0
            ent = self._nbytes_of[id(managers)] = (managers, n)
        return ent[1]

    def note_release(self, managers):
        """A module's gathered parameters were released (on the current stream): every
        ``_marker_every`` releases one marker recorded there."""
        self._rel_n += 1
        self._rel_bytes += self._nbytes(managers)
        if self._rel_n >= self._marker_every:
            self._record_marker()

    def _record_marker(self):
        if not self._rel_n:
            return
        h = self._cur_h()
        ent = self._rel_syncs.get(h)
        if ent is None:  # a flag sync of its own per consumer stream: its epochs only grow
            ent = self._rel_syncs[h] = [Sync(_lib.ZS_SYNC_FLAG), 0]
        ent[0].record(h)
        ent[1] += 1
        self._markers.append((ent[0], ent[1], self._rel_bytes, self._rel_n))
        self._rel_bytes = self._rel_n = 0

    def _throttle(self, key, managers):
        """Before a new gathered allocation: while it would take the outstanding bytes past
        ``max_inflight_bytes`` (two allocations always allowed), wait on the host for the oldest
        release marker — everything before a marker on its stream is enqueued already, so it
        completes without anything this host still has to enqueue.  No marker left: go ahead."""
        nb = self._nbytes(managers)
        if self.max_inflight_bytes is None:
            self.max_inflight_bytes = torch.cuda.get_device_properties(self.device).total_memory // 8
        while (self._out_bytes + nb > self.max_inflight_bytes and self._out_n >= 2
               and self._markers):
            sy, e, b, n = self._markers.popleft()
            if sy.query()[1] < e:
                self.n_throttle_waits += 1
                while sy.query()[1] < e:
                    time.sleep(20e-6)
            self._out_bytes -= b
            self._out_n -= n
        self._out_bytes += nb
        self._out_n += 1
        self._counted[key] = nb

    def _drop_pending(self):
        """Gathers prefetched but never consumed are dropped (their memory goes back once the side
        stream is past them): no longer outstanding."""
        for key in self.pending:
            nb = self._counted.pop(key, None)
            if nb is not None:
                self._out_bytes -= nb
                self._out_n -= 1
        self._counted.clear()
        self.pending.clear()

    def _ready_sync(self, key, cur_h) -> Sync:
        """The sync the consumer stream ``cur_h`` records before ``key``'s gather (one per stream:
        a flag record from another stream would first wait for the previous stream's record)."""
        k = ("ready", key, cur_h)
        sy = self._syncs.get(k)
        if sy is None:
            sy = self._syncs[k] = Sync(self.sync_kind)
        return sy

    def _done_sync(self, key) -> Sync:
        """The sync the side stream records after ``key``'s gather, its consumers wait on."""
        k = ("done", key)
        sy = self._syncs.get(k)
        if sy is None:
            sy = self._syncs[k] = Sync(self.sync_kind)
        return sy

    def _cur_h(self) -> int:
        return torch._C._cuda_getCurrentRawStream(self._dev_idx)

    def _side_empty(self, n: int, dtype) -> torch.Tensor:
        """torch.empty on the side stream (the caching allocator's stream of the block), with the
        current stream set and restored by id — the stream context manager's host cost, per
        gather, without its Python objects."""
        prev = torch._C._cuda_getCurrentStream(self._dev_idx)
        torch._C._cuda_setStream(*self._side_ids)
        try:
            return torch.empty(n, dtype=dtype, device=self.device)
        finally:
            torch._C._cuda_setStream(*prev)

    def _stream_obj(self, h: int):
        """A torch stream object for raw handle ``h`` (cached: record_stream needs one, and
        building it per gather costs host time)."""
        st = self._streams.get(h)
        if st is None:
            cur = torch.cuda.current_stream(self.device)
            st = cur if cur.cuda_stream == h else torch.cuda.ExternalStream(h, device=self.device)
            self._streams[h] = st
        return st

    def side(self):
        """The stream collectives go to: the side stream, or (single-stream mode) the current."""
        return self.stream if self.stream is not None else torch.cuda.current_stream(self.device)

    def launch(self, key, managers, cur_h=None):
        """Enqueue the all-gather of ``managers`` on the side stream; returns immediately.
        ``cur_h``: the raw handle of the stream the gathered tensors will be read on (default:
        the current stream)."""
        if key in self.pending or not managers:
            return
        if self.ws == 1 and not any(m.fp8 for m in managers):
            # the shard is the whole parameter: nothing to gather, no stream to synchronise with
            self.pending[key] = ([(m, m._gather_prepare(None)[1]) for m in managers], None, None, None,
                                 None)
            self.n_gathers += 1
            return
        if cur_h is None:
            cur_h = self._cur_h()
        ready, done = self._ready_sync(key, cur_h), self._done_sync(key)
        ready_h, ev_h = ready.h, done.h
        self._waited.pop(ev_h, None)  # re-recorded below: no consumer has waited on this record
        timed = self.gather_events is not None and self.ws > 1
        plan = self._tables[key] if key in self._tables else self._table(key, managers)
        if self._throttled:
            self._throttle(key, managers)
        if plan is not None and plan[-1] is not None and not timed and self.stream is None:
            # single-stream mode: the RCCL group on the consumer's stream, nothing to order
            send, count, offs, total, dt, es, views, recv, raw, ordered = plan
            hold = torch.empty(total, dtype=managers[0].shard.dtype, device=self.device)
            np.add(offs, np.uint64(hold.data_ptr()), out=recv)
            ordered(cur_h, 0, cur_h, 0)
            self.pending[key] = (_Gathered(managers, hold, views, self._vplan(managers, views)),
                                 None, hold, cur_h, None)
            self.n_gathers += 1
            return
        side = self.side()
        if plan is not None and plan[-1] is not None and not timed:
            # one allocation for the module's full tensors and ONE library call: the ready sync
            # (see _take_ready), the RCCL group of all-gathers (zero-copy from the chunk-arena
            # slots), the done sync its consumers wait on.  Allocated on the side stream, which
            # writes it; the consumer records its own use (materialize)
            send, count, offs, total, dt, es, views, recv, raw, ordered = plan
            gf = self._gather_fast(key, managers, plan)
            if gf is not None:  # allocation, receive table and synced group: one C++ call
                rc, hold = gf.launch(cur_h, self._take_ready(ready_h), self._side_ids[0],
                                     self._side_h, ev_h)
                if rc:
                    _lib.check(rc, "zs_all_gather_group_synced")
            else:
                hold = self._side_empty(total, managers[0].shard.dtype)
                np.add(offs, np.uint64(hold.data_ptr()), out=recv)
                ordered(cur_h, self._take_ready(ready_h), self._side_h, ev_h)
            self.pending[key] = (_Gathered(managers, hold, views, self._vplan(managers, views)),
                                 done, hold, self._side_h, ev_h)
            self.n_gathers += 1
            return
        side_h = self._side_h if self.stream is not None else cur_h
        ready.record(cur_h)  # shards may just have been updated
        ready.wait(side_h)
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(side)
        hold = None
        fplan = None
        if plan is None:
            fplan = self._fp8_tables[key] if key in self._fp8_tables else self._fp8_plan(key, managers)
        if fplan is not None:
            # fp8 gather: one quantise launch, ONE RCCL group, one dequantise
            # launch into one allocation
            hold = self._launch_fp8(fplan, side)
            out = [(m, hold.as_strided(shape, stride, off)) for m, (shape, stride, off)
                   in zip(managers, fplan["views"])]
        elif plan is not None:
            # one allocation for the module's full tensors and ONE library call for its RCCL group
            # of all-gathers (zero-copy from the chunk-arena slots).  Allocated on the compute
            # stream (which reads it once the gather's event has passed); the side stream that
            # writes it is recorded on it, so a prefetch dropped unconsumed keeps its memory until
            # the gather has finished
            send, count, offs, total, dt, es, views, recv, raw, _ = plan
            hold = torch.empty(total, dtype=managers[0].shard.dtype, device=self.device)
            hold.record_stream(side)
            np.add(offs, np.uint64(hold.data_ptr()), out=recv)
            if raw is not None:  # cached ctypes pointers of the tables: one foreign call
                raw(side)
            else:
                self.comm.all_gather_group(send, recv, count, dt, side)
            # each manager's full tensor: one strided view of the allocation, built on install
            out = _Gathered(managers, hold, views, self._vplan(managers, views))
        else:
            with torch.cuda.stream(side):
                # kernels (fp8 quantisation) before the RCCL group, dequantisation after: an RCCL
                # group only launches its collectives at group end; every buffer a collective of
                # the group touches is referenced from `states` until the group has ended
                states = [m._gather_prepare(side) for m in managers]
                with _group_ctx(self.comm):
                    for m, st in zip(managers, states):
                        m._gather_issue(self.comm, side, st)
                out = [(m, m._gather_finish(side, st)) for m, st in zip(managers, states)]
        done.record(side_h)
        if timed:  # ring all-gather bus bytes: (ws-1)/ws of the gathered tensor, per rank
            bus = sum(m.gather_bytes() for m in managers) * (self.ws - 1)
            self.gather_events.append((e0, _timed_after(side), bus))
        self.pending[key] = (out, done, hold, cur_h, ev_h)
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

            views = []
            for off, m in zip(offs, managers):
                shape = tuple(m.full_shape)
                stride, acc = [], 1
                for d in reversed(shape):
                    stride.append(acc)
                    acc *= d
                views.append((shape, tuple(reversed(stride)), off))
            send = np.array([m.send_slot.data_ptr() for m in managers], np.uint64)
            count = np.array([m.S for m in managers], np.int64)
            recv = np.zeros(len(managers), np.uint64)  # refilled per gather (allocation + offs)
            dt = zs_dtype(managers[0].shard.dtype)
            raw = ordered = None
            bind = getattr(self.comm, "all_gather_group_bound", None)
            if bind is not None:
                raw = bind(send, recv, count, dt)
            bind = getattr(self.comm, "all_gather_group_synced_bound", None)
            if bind is not None:  # ordering through sync objects (ready / done), one call
                ordered = bind(send, recv, count, dt)
            plan = (send, count, np.array(offs, np.uint64) * np.uint64(es), max(o, 1), dt, es,
                    views, recv, raw, ordered)
        self._tables[key] = plan
        return plan

    def _gather_fast(self, key, managers, plan):
        """The key's GatherFast (csrc/zs_host_ext.cpp): its side-stream allocation, receive table
        and synced group in one call — or None (no extension, a communicator without the raw
        synced group, the per-parameter ablation)."""
        gf = self._gfast.get(key, False)
        if gf is not False:
            return gf
        gf = None
        raw_of = getattr(self.comm, "all_gather_group_synced_raw", None)
        if (self.use_hostext and self.use_gather_fast and raw_of is not None and _hostext is not None
                and hasattr(_hostext, "GatherFast") and self._side_ids is not None):
            fn, comm_h, collective = raw_of()
            send, count, offs, total, dt, es, views, recv, raw, ordered = plan
            gf = _hostext.GatherFast(int(fn), int(comm_h), bool(collective),
                                     [int(x) for x in send], [int(x) for x in count],
                                     [int(x) for x in offs], int(total), int(dt),
                                     managers[0].shard.dtype, int(self._dev_idx))
        self._gfast[key] = gf
        return gf

    def _vplan(self, managers, views):
        """The module's ViewPlan (shared by its forward and backward keys: the same managers
        list), or None — no extension, reference mode (release shrinks gradients: per parameter),
        or parameters the extension cannot rewrite in place."""
        ent = self._vplans.get(id(managers))
        if ent is not None and ent[0] is managers:
            return ent[1]
        vp = None
        if self.use_hostext and _hostext is not None and all(m.keep_full_grad for m in managers):
            try:
                vp = _hostext.ViewPlan([m.param for m in managers], [m.shard for m in managers],
                                       [list(v[0]) for v in views], [list(v[1]) for v in views],
                                       [int(v[2]) for v in views])
            except RuntimeError:
                vp = None
        self._vplans[id(managers)] = (managers, vp)
        return vp

    def _take_ready(self, ready_h: int) -> int:
        """The ready sync a fast-path gather records on the consumer stream and waits for on the
        side stream — only the first gather after the shards may have changed (construction, each
        step(): ``end_iteration`` marks them): the gathers read the chunk-arena slots, which only
        the compute stream's Adam writes, and the side stream runs its gathers in order, so one
        wait per iteration orders all of them.  Their buffers are allocated on the side stream
        (no reuse of a block the compute stream still reads: the caching allocator sees the
        consumer's recorded use), so no other ordering is needed.  Returns 0 for "no ready"."""
        if not self._inputs_dirty:
            return 0
        self._inputs_dirty = False
        return ready_h

    def _fp8_plan(self, key, managers):
        """The cached tables of a module's fp8 gather: its matrices quantised by ONE launch into
        one send buffer of concatenated rows (+ one of row scales), ONE RCCL group of two
        all-gathers (plus the plain all-gathers of its vectors, straight into place), then ONE
        dequantise launch from the rank-major gathered rows into the module's full tensors (one
        allocation, as the table path).  None: the per-parameter path (standalone managers,
        row lengths not a multiple of 8, mixed dtypes)."""
        plan = None
        fp8 = [m for m in managers if m.fp8]
        if (fp8 and all(m.send_slot is not None for m in managers)
                and len({m.shard.dtype for m in managers}) == 1
                and all(m.row % 8 == 0 and m.send_slot.data_ptr() % 16 == 0 for m in fp8)):
            ws = self.ws
            dt = managers[0].shard.dtype
            es = managers[0].shard.element_size()
            offs, o = [], 0
            for m in managers:
                offs.append(o)
                o += -(-ws * m.S // ALIGN_ELEMS) * ALIGN_ELEMS  # every full tensor 64-element aligned
            views = []
            for off, m in zip(offs, managers):
                shape = tuple(m.full_shape)
                stride, acc = [], 1
                for d in reversed(shape):
                    stride.append(acc)
                    acc *= d
                views.append((shape, tuple(reversed(stride)), off))
            q_off, sc_off, qo, so = [], [], 0, 0
            for m in fp8:  # cs * row bytes each: a multiple of 8, so every matrix's rows stay 8-B aligned
                q_off.append(qo)
                sc_off.append(so)
                qo += m.cs * m.row
                so += m.cs
            i8 = [i for i, m in enumerate(managers) if m.fp8]
            plan = {
                "n": len(fp8), "dtype": dt, "zdt": zs_dtype(dt), "total": max(o, 1), "views": views,
                "qtot": max(qo, 8), "sctot": max(so, 1),
                "src": np.array([m.send_slot.data_ptr() for m in fp8], np.uint64),
                "rows": np.array([m.r1 - m.r0 for m in fp8], np.int64),
                "cs": np.array([m.cs for m in fp8], np.int64),
                "row_len": np.array([m.row for m in fp8], np.int64),
                "q_off": np.array(q_off, np.int64), "sc_off": np.array(sc_off, np.int64),
                "dst_off": np.array([offs[i] for i in i8], np.uint64) * np.uint64(es),
                "plain": [(m, offs[i]) for i, m in enumerate(managers) if not m.fp8],
                "qptr": np.zeros(len(fp8), np.uint64), "sptr": np.zeros(len(fp8), np.uint64),
                "dst": np.zeros(len(fp8), np.uint64),
            }
        self._fp8_tables[key] = plan
        return plan

    def _launch_fp8(self, plan, side):
        ws = self.ws
        hold = torch.empty(plan["total"], dtype=plan["dtype"], device=self.device)
        hold.record_stream(side)
        h = stream_handle(side)
        with torch.cuda.stream(side):  # the temporaries live and die on the side stream
            qs = torch.empty(plan["qtot"], dtype=torch.uint8, device=self.device)
            ss = torch.empty(plan["sctot"], dtype=torch.float32, device=self.device)
            np.add(plan["q_off"].astype(np.uint64), np.uint64(qs.data_ptr()), out=plan["qptr"])
            np.add(plan["sc_off"].astype(np.uint64) * np.uint64(4), np.uint64(ss.data_ptr()),
                   out=plan["sptr"])
            _lib.call("zs_fp8_quantize_rowset", plan["n"], plan["src"].ctypes.data,
                      plan["qptr"].ctypes.data, plan["sptr"].ctypes.data, plan["rows"].ctypes.data,
                      plan["cs"].ctypes.data, plan["row_len"].ctypes.data, plan["zdt"], h)
            if ws > 1:
                qr = torch.empty(ws * plan["qtot"], dtype=torch.uint8, device=self.device)
                sr = torch.empty(ws * plan["sctot"], dtype=torch.float32, device=self.device)
                with _group_ctx(self.comm):
                    self.comm.all_gather(qs, qr, side)
                    self.comm.all_gather(ss, sr, side)
                    for m, off in plan["plain"]:
                        self.comm.all_gather(m.send_slot, hold[off:off + ws * m.S], side)
            else:
                qr, sr = qs, ss
                for m, off in plan["plain"]:
                    hold[off:off + m.S].copy_(m.send_slot)
            np.add(plan["dst_off"], np.uint64(hold.data_ptr()), out=plan["dst"])
            _lib.call("zs_fp8_dequantize_gathered", plan["n"], qr.data_ptr(), sr.data_ptr(), ws,
                      plan["qtot"], plan["sctot"], plan["q_off"].ctypes.data,
                      plan["sc_off"].ctypes.data, plan["cs"].ctypes.data,
                      plan["row_len"].ctypes.data, plan["dst"].ctypes.data, plan["zdt"], h)
        return hold

    def _fast_plan(self, key, managers):
        """The key's ordered-call table when its gather can take the one-call fast path (a chunk-
        arena module, ws > 1, no per-collective timing), else None."""
        if self.ws == 1 or not managers or self.gather_events is not None:
            return None
        plan = self._tables[key] if key in self._tables else self._table(key, managers)
        return plan if plan is not None and plan[-1] is not None else None

    def _launch_wave(self, keys, cur_h):
        """Launch the not-yet-pending groups of ``keys`` as one wave: the first gather records the
        ready event on the compute stream (``cur_h``) and makes the side stream wait for it, the
        last records the done event every member's consumer waits on.  Falls back to one launch
        per group when any of them cannot take the fast path."""
        todo = [(k, self.key_managers.get(k)) for k in keys if k not in self.pending]
        todo = [(k, ms) for k, ms in todo if ms]
        if not todo:
            return
        plans = [self._fast_plan(k, ms) for k, ms in todo]
        if len(todo) == 1 or any(pl is None for pl in plans):
            for k, ms in todo:
                self.launch(k, ms, cur_h)
            return
        single = self.stream is None
        if single:  # everything on the consumer's stream: nothing to order
            ready_h = done_h = 0
            done_ev = None
        else:
            ready_h = self._take_ready(self._ready_sync(todo[0][0], cur_h).h)
            done_ev = self._done_sync(todo[-1][0])
            done_h = done_ev.h
            self._waited.pop(done_h, None)
        last = len(todo) - 1
        side, side_h = self.stream, (cur_h if single else self._side_h)
        for j, ((k, ms), plan) in enumerate(zip(todo, plans)):
            send, count, offs, total, dt, es, views, recv, raw, ordered = plan
            gf = None
            if single:
                hold = torch.empty(total, dtype=ms[0].shard.dtype, device=self.device)
            else:  # written by the side stream: allocated there (see _take_ready)
                if self._throttled:
                    self._throttle(k, ms)
                gf = self._gather_fast(k, ms, plan)
            if gf is not None:
                rc, hold = gf.launch(cur_h, ready_h if j == 0 else 0, self._side_ids[0], side_h,
                                     done_h if j == last else 0)
                if rc:
                    _lib.check(rc, "zs_all_gather_group_synced")
            else:
                if not single:
                    hold = self._side_empty(total, ms[0].shard.dtype)
                np.add(offs, np.uint64(hold.data_ptr()), out=recv)
                ordered(cur_h, ready_h if j == 0 else 0, side_h, done_h if j == last else 0)
            self.pending[k] = (_Gathered(ms, hold, views, self._vplan(ms, views)), done_ev, hold,
                               side_h, done_h or None)
            self.n_gathers += 1

    def _ensure_wave(self, w, cur_h=None):
        """Launch wave ``w`` of the learned sequence unless it was launched this iteration."""
        G = self.wave
        if w in self._waves_launched or not 0 <= w * G < len(self.sequence):
            return
        self._waves_launched.add(w)
        if cur_h is None:
            cur_h = self._cur_h()
        self._launch_wave(self.sequence[w * G:(w + 1) * G], cur_h)

    def _prefetch(self, i, cur_h=None):
        """Make sure the wave holding sequence position ``i`` has been launched."""
        if 0 <= i < len(self.sequence):
            self._ensure_wave(i // self.wave, cur_h)

    def materialize(self, key, managers):
        cur_h = self._cur_h()
        if self.recording:
            self.sequence.append(key)
        else:
            seq = self.sequence
            if self.pos < len(seq) and seq[self.pos] == key:
                p = self.pos
            elif key in seq[self.pos:]:
                p = seq.index(key, self.pos)
            else:
                p = None
            if p is not None:
                self.pos = p + 1
                w = p // self.wave
                launched = self._waves_launched
                if w not in launched:  # (normally launched as the previous prefetch)
                    self._ensure_wave(w, cur_h)
                if w + 1 not in launched:  # the next wave, while this one computes
                    self._ensure_wave(w + 1, cur_h)
            else:
                self._prefetch(self.pos, cur_h)
        if key in self.pending:
            self.n_prefetch_hits += 1
        self.launch(key, managers, cur_h)
        out, ev, hold, alloc_h, wait_h = self.pending.pop(key)
        self._counted.pop(key, None)
        if ev is None and hold is None:  # ws == 1
            for m, full in out:
                m._install_full(full)
            return
        if (wait_h is not None and hold is not None and self._consume is not None
                and self.use_gather_fast and type(out) is _Gathered and out.vplan is not None):
            # the wait (once per wave and consuming stream), the allocator's record of this
            # stream's use, the install: one C++ call
            need = self._waited.get(wait_h) != cur_h
            rc = self._consume(self._wait_fn, wait_h if need else 0, cur_h, hold, out.vplan,
                               alloc_h is not None and alloc_h != cur_h)
            if rc:
                _lib.check(rc, "zs_sync_wait")
            if need:
                self._waited[wait_h] = cur_h
            for m in out.ms:
                m._full = True
            return
        if wait_h is not None:
            if self._waited.get(wait_h) != cur_h:  # once per wave and consuming stream
                rc = self._sync_wait(wait_h, cur_h)
                if rc:
                    _lib.check(rc, "zs_sync_wait")
                self._waited[wait_h] = cur_h
        elif alloc_h is not None and alloc_h != cur_h:
            # single-stream mode, gathered on another stream than this one: order the two
            e = torch.cuda.Event()
            e.record(torch.cuda.ExternalStream(alloc_h, device=self.device))
            torch.cuda.current_stream(self.device).wait_event(e)
        if hold is not None and alloc_h is not None and alloc_h != cur_h:
            # prefetched under another current stream (a user stream in forward, autograd's in
            # backward): the allocator must not reuse the block while THIS stream reads it
            hold.record_stream(self._stream_obj(cur_h))
        if hold is not None:  # one allocation (on this stream) behind all of the module's full
            if type(out) is _Gathered and out.vplan is not None:  # tensors: one C++ call
                out.vplan.install(hold)
                for m in out.ms:
                    m._full = True  # (full_data: the parameter's data)
                return
            for m, full in out:  # (per parameter: a strided view each)
                m.full_data = full
                m.param.data = full
            return
        cur = torch.cuda.current_stream(self.device)
        for m, full in out:
            full.record_stream(cur)
            m._install_full(full)

    def mark_inputs_changed(self):
        """The shards changed outside step()'s Adam (a checkpoint load, a caller's
        ``p.data.copy_``): the next gather waits for the compute stream again (see _take_ready),
        and gathers prefetched before the change — they read the old shards — are dropped, so
        their modules gather again on demand."""
        self._inputs_dirty = True
        self._drop_pending()

    def end_iteration(self):
        for fn in self.iteration_callbacks:
            fn()
        self._inputs_dirty = True  # step() has updated the shards
        if self.sequence:
            self.recording = False
        self._drop_pending()
        if self._throttled:  # every consumed allocation is released by now: the markers cover them
            self._record_marker()
            self._out_bytes = sum(m[2] for m in self._markers)
            self._out_n = sum(m[3] for m in self._markers)
        self._waves_launched.clear()
        self._waited.clear()
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
        if full_shape is None and shard is None and param.dim() > 0:
            # the reference's standalone manager: param.data is this rank's dim-0 shard and the
            # full tensor is the rank-ordered concatenation of ws equal shards (zero3.py:36-41)
            full_shape = (world_size * param.shape[0],) + tuple(param.shape[1:])
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
        # fp8 only for matrices (row-wise scales) whose rows are a multiple of 8 elements (the
        # vector kernels' 8-B fp8 accesses); vectors (biases, norms) and other matrices gather as
        # they are
        self.fp8 = gather_dtype == "fp8" and len(self.full_shape) >= 2 and self.row % 8 == 0
        # this manager as a one-member module (materialize()): one list object for its lifetime,
        # so the runtime's per-module caches (gather table, ViewPlan) key on it once
        self._as_group = [self]

    @property
    def full_data(self):
        """zero3.py:40: the gathered full tensor while the parameter is materialised, else None
        (a module installed through its ViewPlan marks its managers ``True``: the full tensor is
        then the parameter's data itself)."""
        f = self._full
        return self.param.data if f is True else f

    @full_data.setter
    def full_data(self, value):
        self._full = value

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
            # the module path's rowset kernel as a one-matrix set: it writes the chunk's padding
            # rows itself (q = 0, scale = 1), so nothing is pre-filled
            src = self.shard
            if rows and src.data_ptr() % 16:  # (a standalone shard at an odd offset)
                src = src.contiguous().clone()
            q = torch.empty(self.S, dtype=torch.uint8, device=dev)
            sc = torch.empty(self.cs, dtype=torch.float32, device=dev)
            ptrs = np.array([src.data_ptr() if rows else 0, q.data_ptr(), sc.data_ptr()], np.uint64)
            geom = np.array([rows, self.cs, self.row], np.int64)  # real rows, chunk rows, row length
            _lib.call("zs_fp8_quantize_rowset", 1, ptrs[0:].ctypes.data, ptrs[1:].ctypes.data,
                      ptrs[2:].ctypes.data, geom[0:].ctypes.data, geom[1:].ctypes.data,
                      geom[2:].ctypes.data, zs_dtype(self.shard.dtype), stream_handle(stream))
            return (q, sc, torch.empty(ws * self.S, dtype=torch.uint8, device=dev),
                    torch.empty(ws * self.cs, dtype=torch.float32, device=dev), src)
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
            q, sc, full_q, full_sc, _ = st
            comm.all_gather(q, full_q, stream)
            comm.all_gather(sc, full_sc, stream)
        else:
            send, full = st
            if full is not send:
                comm.all_gather(send, full, stream)

    def _gather_finish(self, stream, st):
        if not self.fp8:
            return st[1]
        _, _, full_q, full_sc, _ = st
        ws = self.world_size
        full = torch.empty(ws * self.S, dtype=self.shard.dtype, device=self.shard.device)
        # the module path's gathered kernel as a one-matrix set: rank k's rows at k * S bytes of
        # the gathered q, its scales at k * cs
        geom = np.array([0, 0, self.cs, self.row], np.int64)  # q_off, sc_off, cs, row_len
        dst = np.array([full.data_ptr()], np.uint64)
        _lib.call("zs_fp8_dequantize_gathered", 1, full_q.data_ptr(), full_sc.data_ptr(), ws, self.S,
                  self.cs, geom[0:].ctypes.data, geom[1:].ctypes.data, geom[2:].ctypes.data,
                  geom[3:].ctypes.data, dst.ctypes.data, zs_dtype(full.dtype), stream_handle(stream))
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
        rt.launch(key, self._as_group)
        out, done, hold, _, _ = rt.pending.pop(key)
        cur = torch.cuda.current_stream(self.shard.device)
        if done is not None:
            done.wait(cur.cuda_stream)
        if hold is not None:
            hold.record_stream(cur)
        for m, full in out:
            full.record_stream(cur)
            m._install_full(full)

    def release(self):
        """zero3.py:43-52: back to the local shard; shrink a full-size grad to its local rows
        (reference mode) or leave it to the reduce-scatter hook (update mode)."""
        self.param.data = self.shard
        if not self.keep_full_grad:  # update mode keeps it for the reduce-scatter: no grad lookup
            g = self.param.grad
            if g is not None and g.shape != self.shard.shape:
                self.param.grad.data = g.data.reshape(self.full_shape)[self.r0:self.r1].clone()
        self.full_data = None


class _TensorHookState:
    """Holder of the tensor-style backward bookkeeping's ``grad_ready`` / ``module_done``
    (register_zero3_hooks)."""

    grad_ready = None
    module_done = None
    counter = None


def _grad_tensors(output):
    """The tensors of a module's output (nested tuples / lists / dicts) that autograd will
    differentiate through."""
    out = []
    stack = [output]
    while stack:
        o = stack.pop()
        if torch.is_tensor(o):
            if o.requires_grad:
                out.append(o)
        elif isinstance(o, (tuple, list)):
            stack.extend(o)
        elif isinstance(o, dict):
            stack.extend(o.values())
    return out


def register_zero3_hooks(model, param_managers, units=None, reshard_after_forward=True,
                         backward_hooks=None):
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
    per step instead of two, full parameters resident between forward and backward.

    ``backward_hooks``: how the backward gather / release is attached.  "module" — the reference's
    ``register_full_backward_pre_hook`` / ``register_full_backward_hook`` (zero3.py:75-76), which
    wrap every hooked module's inputs and outputs in identity autograd nodes on each forward.
    "tensor" (default) — the same two moments without them: the forward post-hook registers a
    grad hook on the module's output tensors (fires when the first output gradient is computed,
    i.e. before the module's backward: materialise), and a post-accumulate-grad hook on each of
    its parameters counts them in (once the last has its gradient the module's backward is done:
    release); an end-of-backward callback releases whatever never counted in (frozen or unused
    parameters).  Same gathers in the same order, less host time per module.  Default (None):
    "tensor" in update mode; "module" in reference mode, whose release after backward shrinks the
    gradients already accumulated — with module hooks exactly the ones the reference shrinks (not
    Linear 0's, whose full backward hook fires before its weight gradient exists), an observable
    the reference-mode tests pin."""
    if backward_hooks is None:
        backward_hooks = "tensor" if all(m.keep_full_grad for m in param_managers.values()) \
            else "module"
    if backward_hooks not in ("tensor", "module"):
        raise ValueError(f"backward_hooks must be 'tensor' or 'module' (got {backward_hooks!r})")
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
        rt.mark_inputs_changed()  # (a new registration: nothing gathered before it is reused)
        rt.key_managers = {}
        rt._tables = {}  # a key's managers may differ from an earlier registration
        rt._gfast = {}
        rt._vplans = {}
        rt._fp8_tables = {}
        rt.iteration_callbacks = []  # (an earlier registration's bookkeeping is replaced)
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
            ms = mod_managers.get(id(module))
            if ms:
                _release_group(ms)
            return None
        return post_hook

    handles = []
    if backward_hooks == "module":
        for m in model.modules():
            # the reference hooks every module (zero3.py:73-77); a module without managed
            # parameters has nothing to gather or release, so it is left unhooked (a full backward
            # hook would only wrap its inputs and outputs in autograd nodes for nothing)
            if not mod_managers[id(m)]:
                continue
            handles.append(m.register_forward_pre_hook(make_pre("fwd")))
            handles.append(m.register_forward_hook(make_post("fwd")))
            handles.append(m.register_full_backward_pre_hook(make_pre("bwd")))
            handles.append(m.register_full_backward_hook(make_post("bwd")))
        return handles

    # backward_hooks == "tensor"
    pre_bwd = make_pre("bwd")
    pre_fwd = make_pre("fwd")
    post_fwd = make_post("fwd")
    hooked = [m for m in model.modules() if mod_managers[id(m)]]
    managed = [mg for m in hooked for mg in mod_managers[id(m)]]
    hooked_ids = [id(m) for m in hooked]
    slot_of = {mid: k for k, mid in enumerate(hooked_ids)}
    mods_of = {}  # id(param) -> the hooked modules it counts into (whatever requires grad)
    for m in hooked:
        for mg in mod_managers[id(m)]:
            mods_of.setdefault(id(mg.param), []).append(id(m))
    state = _TensorHookState()
    counter = None
    if HOSTEXT_COUNTING and _hostext is not None and hasattr(_hostext, "GradCounter"):
        # module slots count their parameters' gradients in C++; Python hears once per module
        counter = _hostext.GradCounter([0] * len(hooked), 0, False, None,
                                       WeakArgCall(state, "module_done"))
        state.counter = counter
    # per backward: how many of a module's parameters will count in (trainable ones), and which
    # modules each trainable parameter counts in; re-derived at the first backward gather of a
    # backward whenever requires_grad changed since (gradual unfreezing, frozen layers)
    n_req, param_mods, hooked_params = {}, {}, set()
    trainable_sig = [None]

    managed_params = [mg.param for mg in managed]

    def recount():
        sig = tuple([p.requires_grad for p in managed_params])
        if sig == trainable_sig[0]:
            return
        trainable_sig[0] = sig
        n_req.clear()
        param_mods.clear()
        for m in hooked:
            n_req[id(m)] = sum(1 for mg in mod_managers[id(m)] if mg.param.requires_grad)
            for mg in mod_managers[id(m)]:
                if mg.param.requires_grad:
                    param_mods.setdefault(id(mg.param), []).append(id(m))
        for mg in managed:
            p = mg.param
            if p.requires_grad and id(p) not in hooked_params:
                # newly trainable: its post-accumulate hook from now on (keyed by id, so the hook
                # the parameter holds keeps no reference to it) — a C++ count into its modules'
                # slots, or a Python hook per parameter
                hooked_params.add(id(p))
                if counter is not None:
                    for mid in mods_of[id(p)]:
                        handles.append(_CounterHandle(p, counter, -1, slot_of[mid]))
                else:
                    handles.append(_add_post_accumulate_hook(p, WeakCall(state, "grad_ready", id(p))))

    open_ = {}     # id(module) -> managers gathered for its backward, not released yet
    pending = {}   # id(module) -> parameter gradients still to come this backward
    queued = [False]
    warned = set()
    # the parameters' post-accumulate hooks (and the C++ counter's callback) reach grad_ready /
    # module_done through a weak reference to ``state`` (a strong closure would be a cycle
    # through the parameter's C++-held hook, _hooks.py); the module hooks below keep it alive as
    # long as the model has them

    def end_backward():
        queued[0] = False
        if counter is not None:
            counter.close_all()
        for ms in open_.values():
            _release_group(ms)
        open_.clear()
        pending.clear()

    def reset_stale():
        """A backward that raised before its end-of-backward callback ran leaves modules open and
        the callback flag set; the next forward (outside any backward) releases them and resets."""
        if queued[0] and torch._C._current_graph_task_id() == -1:
            end_backward()

    def backward_pre(module):
        mid = id(module)
        if not queued[0]:
            queued[0] = True
            recount()
            torch.autograd.Variable._execution_engine.queue_callback(end_backward)
        pre_bwd(module)
        open_[mid] = mod_managers[mid]
        # nothing will count in: released at the end of backward
        pending[mid] = n_req.get(mid, 0) or -1
        if counter is not None:
            counter.open(slot_of[mid], pending[mid])

    def forward_pre(module, *args):
        reset_stale()
        return pre_fwd(module, *args)

    def forward_post(module, args, output):
        post_fwd(module)
        if torch.is_grad_enabled():
            ts = _grad_tensors(output)
            if len(ts) == 1:  # one output: a plain tensor hook (cheaper than a multi-grad hook)
                ts[0].register_hook(lambda _g, module=module: backward_pre(module))
            elif ts:
                torch.autograd.graph.register_multi_grad_hook(
                    ts, lambda _g, module=module: backward_pre(module), mode="any")
            elif id(module) not in warned and any(mg.param.requires_grad
                                                   for mg in mod_managers[id(module)]):
                warned.add(id(module))
                import warnings

                warnings.warn(
                    f"zero_amd ZeRO-3: {type(module).__name__}'s output holds no tensor that "
                    "requires grad, so its parameters get no backward gather from the tensor-style "
                    "hooks; use register_zero3_hooks(..., backward_hooks='module') for such modules",
                    RuntimeWarning, stacklevel=2)
        return None

    def grad_ready(pid):
        for mid in param_mods.get(pid, ()):
            if mid in open_:
                pending[mid] -= 1
                if pending[mid] == 0:
                    _release_group(open_.pop(mid))

    def module_done(slot):  # (C++ counting: the module's last trainable gradient is in)
        ms = open_.pop(hooked_ids[slot], None)
        if ms is not None:
            _release_group(ms)

    state.grad_ready = grad_ready
    state.module_done = module_done
    forward_pre.state = state  # (the strong reference: module hook -> forward_pre -> state)
    for m in hooked:
        handles.append(m.register_forward_pre_hook(forward_pre))
        handles.append(m.register_forward_hook(forward_post))
    recount()
    for rt in runtimes:  # the end of every step() also clears what a failed backward left
        rt.iteration_callbacks.append(reset_stale)
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

    Contract (as DDP's): every rank's backward reaches the same set of parameters.  A bucket is
    launched from backward once all of its hooked parameters have fired on this rank; a parameter
    one rank reaches and another does not would put that bucket's reduce-scatter at different
    points among the ranks' collectives (and leave ``had_grad`` rank-dependent).  Parameters that
    no rank reaches are fine: their buckets are flushed, in the fixed order, at the end of backward.

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
        # per-element bookkeeping in plain lists (numpy scalar indexing costs more per hook call)
        self._size_l = [len(g) for g in groups]
        self._bucket_of_l = self.bucket_of.tolist()
        self._S_l = [int(x) for x in arena.S]
        self._N_l = [int(x) for x in arena.numel]
        self._shard_grad = [None] * n  # cached grad-arena views handed out as shard grads
        # per bucket: the sync the side stream records after its reduce-scatter (step() and the
        # shard grads wait on the last one) and, per producing stream, the one recorded before it
        kind = opt.runtime.sync_kind
        self.ev_done = [Sync(kind) for _ in range(self.K)]
        self._done_h = [e.h for e in self.ev_done]
        self._ready = {}  # (bucket, stream handle) -> Sync
        self._sync_kind = kind
        cs = opt.runtime.stream if opt.world_size > 1 else None  # (None: single-stream mode)
        if cs is not None:
            self._cs_h = cs.cuda_stream
            self._cs_id = cs.stream_id
        self.timing = None  # optional list of (start, end, bus_bytes) per launched bucket
        self._rs_tables = {}
        self.use_hostext = HOSTEXT_COUNTING  # (False: per-parameter Python hooks, for A/B)
        self.use_reduce_fast = True  # (False: every bucket launched by the Python below, for A/B)
        self._rfast = {}             # bucket -> its _hostext.ReduceFast, or None
        self._group_idx = [np.asarray(g, np.int64) for g in groups]
        self._counter = None     # the C++ gradient counter (register_hooks)
        self.reset()

    def _ready_sync(self, k: int, cur_h: int) -> Sync:
        sy = self._ready.get((k, cur_h))
        if sy is None:
            sy = self._ready[(k, cur_h)] = Sync(self._sync_kind)
        return sy

    def reset(self):
        n = len(self.opt.params)
        # buckets the last backward launched before it ended (the rest: flushed at its end)
        self.last_launched_in_backward = getattr(self, "launched_in_backward", 0)
        self.pending = list(self._size_l)
        self.marked = [False] * n
        self.had_grad = np.zeros(n, bool)
        self.local_grads = [None] * n  # ws == 1: the grad itself is the chunk's gradient
        self.next = 0
        self.callback_queued = False
        self.launched_in_backward = 0
        if getattr(self, "_counter", None) is not None:
            self._counter.reset()

    def register_hooks(self):
        """The parameters' post-accumulate-grad counting.  With the host extension: C++ hooks
        (``_hostext.GradCounter``, csrc/zs_host_ext.cpp) count each completed gradient into its
        bucket without entering Python, which hears once per completed run of buckets
        (``_launch_upto``) and once per backward (``_first_grad``) — 34 + 1 calls per C5 backward
        instead of 291.  Without it: one Python hook per parameter (``on_grad_ready``).  Either
        way the callbacks hold the reducer weakly (_hooks.py): it is owned by its optimizer."""
        params = [(i, p) for i, p in enumerate(self.opt.params) if p.requires_grad]
        if self.use_hostext and _hostext is not None and hasattr(_hostext, "GradCounter"):
            self._counter = _hostext.GradCounter(
                self._size_l, len(self.opt.params), True, WeakCall(self, "_first_grad"),
                WeakArgCall(self, "_launch_upto"),
                "zero_amd ZeRO-3: gradient accumulated twice before step(); update mode "
                "reduce-scatters each gradient once per step")
            return [_CounterHandle(p, self._counter, i, self._bucket_of_l[i]) for i, p in params]
        return [_add_post_accumulate_hook(p, WeakCall(self, "on_grad_ready", i)) for i, p in params]

    def _first_grad(self):
        """The first gradient of a backward (C++ counting): the end-of-backward flush, queued from
        inside the backward."""
        if not self.callback_queued:
            self.callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._end_backward)

    def _launch_upto(self, upto: int):
        """Buckets [next, upto) are complete (C++ counting): launch them, in order."""
        while self.next < upto:
            self._launch(self.next)
            self.launched_in_backward += 1
            self.next += 1

    def on_grad_ready(self, i: int, _param=None):
        """Parameter i's gradient is complete (its post-accumulate-grad hook, or by hand)."""
        if self._counter is not None:
            self._counter.count(i, self._bucket_of_l[i])
            return
        if self.marked[i]:
            raise RuntimeError(
                "zero_amd ZeRO-3: gradient of parameter %d accumulated twice before step(); "
                "update mode reduce-scatters each gradient once per step" % i)
        self.marked[i] = True
        self.pending[self._bucket_of_l[i]] -= 1
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
        if self.K and opt.runtime.stream is not None:
            self.ev_done[self.K - 1].wait(opt.runtime._cur_h())
        if opt._G.dtype != opt.params[0].dtype:  # a bf16 exchange's chunks stay internal
            return
        shapes, views = opt._arena.shard_shapes, self._shard_grad
        params = opt.params
        for i in np.flatnonzero(self.had_grad).tolist():
            p = params[i]
            if p.shape == shapes[i]:  # (released to its shard; p.shape: no .data tensor built)
                v = views[i]
                if v is None:
                    s, n = int(opt._arena.slot[i]), int(opt._arena.ln[i])
                    v = views[i] = opt._G[s:s + n].view(shapes[i])
                p.grad = v

    def _rs_table(self, k: int):
        """Bucket k's reduce-scatter destinations (grad chunk-arena slots) and counts, cached."""
        t = self._rs_tables.get(k)
        if t is None:
            from .comm import zs_dtype

            opt, idx = self.opt, np.asarray(self.groups[k], np.int64)
            G = opt._G
            recv = np.uint64(G.data_ptr()) + (opt._arena.slot[idx] * G.element_size()).astype(np.uint64)
            count = np.ascontiguousarray(opt._arena.S[idx], np.int64)
            send = np.zeros(len(idx), np.uint64)  # refilled per launch with the grads' addresses
            bind = getattr(opt.comm, "reduce_scatter_group_bound", None)
            raw = bind(send, recv, count, zs_dtype(G.dtype)) if bind is not None else None
            bind = getattr(opt.comm, "reduce_scatter_group_synced_bound", None)
            ordered = bind(send, recv, count, zs_dtype(G.dtype)) if bind is not None else None
            t = (recv, count, zs_dtype(G.dtype), send, raw, ordered)
            self._rs_tables[k] = t
        return t

    def _reduce_fast(self, k: int):
        """Bucket k's ReduceFast (csrc/zs_host_ext.cpp): its gradients' send table, the synced
        group, the stream records and the gradient resets in one call — or None (no extension, a
        communicator without the raw synced group, a bf16 exchange, uneven chunks)."""
        rf = self._rfast.get(k, False)
        if rf is not False:
            return rf
        rf = None
        opt = self.opt
        ar = opt._arena
        raw_of = getattr(opt.comm, "reduce_scatter_group_synced_raw", None)
        if (self.use_reduce_fast and raw_of is not None and _hostext is not None
                and hasattr(_hostext, "ReduceFast") and opt._G.dtype == ar.dtype
                and hasattr(opt.comm, "reduce_scatter_group")
                and all(self._N_l[i] == opt.world_size * self._S_l[i] for i in self.groups[k])):
            recv, count, dt, sp, raw, ordered = self._rs_table(k)
            fn, comm_h, collective = raw_of()
            rf = _hostext.ReduceFast(int(fn), int(comm_h), bool(collective),
                                     [opt.params[i] for i in self.groups[k]],
                                     [int(x) for x in recv], [int(x) for x in count], int(dt),
                                     ar.dtype, int(opt.world_size))
        self._rfast[k] = rf
        return rf

    def _launch(self, k: int):
        opt = self.opt
        ar, ws = opt._arena, opt.world_size
        rf = self._reduce_fast(k) if ws > 1 and self.timing is None else None
        if rf is not None:
            rt = opt.runtime
            cur_h = rt._cur_h()
            if rt.stream is None:  # single-stream mode: on the stream that produced the grads
                rc = rf.launch(cur_h, 0, 0, 0, cur_h, 0, False)
            else:
                rc = rf.launch(cur_h, self._ready_sync(k, cur_h).h, self._cs_id, rt._dev_idx,
                               self._cs_h, self._done_h[k] if k == self.K - 1 else 0, True)
            if rc == 0:
                self.had_grad[self._group_idx[k]] = True
                return
            if rc > 0:
                _lib.check(rc, "zs_reduce_scatter_group_synced")
            # (-1: a gradient missing or not a zero-copy send: the general path below)
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
        cur_h = opt.runtime._cur_h()
        cur = None  # the Stream object, built only on the paths that need it
        wdt = opt._G.dtype  # on the wire: the param dtype, or bf16 for grad_comm="bf16"
        sends = []  # (param index, send buffer): alive until the RCCL group has been enqueued
        S_l, N_l = self._S_l, self._N_l
        for i in self.groups[k]:
            p = opt.params[i]
            g = p.grad
            S, N = S_l[i], N_l[i]
            if g is None:
                send = torch.zeros(ws * S, dtype=wdt, device=dev)  # every rank takes part
            else:
                if g.numel() != N or g.dtype != ar.dtype:
                    raise ValueError("zero_amd ZeRO-3 update mode needs the full-size gradient "
                                     "(param %d: got %s)" % (i, tuple(g.shape)))
                self.had_grad[i] = True
                if wdt == ar.dtype and N == ws * S and g.is_contiguous():
                    send = g  # zero-copy: rows of torch.chunk are contiguous
                else:
                    flat = g.reshape(-1) if g.is_contiguous() else g.contiguous().reshape(-1)
                    if wdt != ar.dtype:  # bf16 exchange: gfx950 RNE conversion into the send buffer
                        from .kernels import convert

                        if cur is None:
                            cur = torch.cuda.current_stream(dev)
                        send = torch.empty(ws * S, dtype=wdt, device=dev) if N == ws * S else \
                            torch.zeros(ws * S, dtype=wdt, device=dev)
                        convert(flat, send[:N], cur)
                    elif N == ws * S:
                        send = flat
                    else:  # uneven chunks: every rank sends ws*S elements
                        send = torch.zeros(ws * S, dtype=wdt, device=dev)
                        send[:N].copy_(flat)
            sends.append((i, send))
        single = opt.runtime.stream is None
        tab = self._rs_tables.get(k) or (self._rs_table(k) if hasattr(opt.comm, "reduce_scatter_group")
                                         else None)
        if tab is not None and tab[5] is not None and self.timing is None:
            recv, count, dt, sp, raw, ordered = tab
            for j, (_, t) in enumerate(sends):
                sp[j] = t.data_ptr()
            params = opt.params
            if single:
                # single-stream mode: the bucket's RCCL group on the stream that produced the grads
                ordered(cur_h, 0, cur_h, 0)
                for i, _ in sends:
                    params[i].grad = None
                return
            # ONE library call: ready sync on the stream that produced the grads, the side
            # stream's wait, the bucket's RCCL group of reduce-scatters, the done sync; only the
            # last bucket's done is waited on (step(), the shard grads): the side stream runs the
            # buckets in order, so the others need no record
            ordered(cur_h, self._ready_sync(k, cur_h).h, self._cs_h,
                    self._done_h[k] if k == self.K - 1 else 0)
            cs = opt.runtime.stream
            for i, send in sends:
                send.record_stream(cs)
                params[i].grad = None
            return
        if cur is None:
            cur = torch.cuda.current_stream(dev)
        cs = cur if single else opt.runtime.stream
        cs_h = cs.cuda_stream
        ready = self._ready_sync(k, cur_h)
        ready.record(cur_h)
        ready.wait(cs_h)
        if self.timing is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(cs)
        if tab is not None:  # the bucket's RCCL group: ONE call
            recv, count, dt, sp, raw, _ = tab
            for j, (_, t) in enumerate(sends):
                sp[j] = t.data_ptr()
            if raw is not None:  # tables bound once (comm.reduce_scatter_group_bound)
                raw(cs)
            else:
                opt.comm.reduce_scatter_group(sp, recv, count, dt, cs)
        else:
            with _group_ctx(opt.comm):
                for i, send in sends:  # (a zero-copy send is the grad itself: flatten the view)
                    s = int(ar.slot[i])
                    opt.comm.reduce_scatter(send.view(-1), opt._G[s:s + int(ar.S[i])], cs)
        # the group has been enqueued: a buffer freed from here on is only reused after it
        for i, send in sends:
            send.record_stream(cs)
            opt.params[i].grad = None
        self.ev_done[k].record(cs_h)
        if self.timing is not None:
            bus = sum(int(ar.S[i]) * ws for i, _ in sends) * opt._G.element_size() * (ws - 1) / ws
            self.timing.append((e0, _timed_after(cs), bus))
        del sends


# Default reduce-scatter bucket (MB of full-size gradient), update mode.  512 rather than 128: the
# same bytes on the wire in a quarter of the RCCL launches and host bookkeeping (C5: 32 buckets per
# iteration instead of 130; rank 0 of a simulated ws=8 C5 iteration 8.9 -> 7.5 ms median, process
# CPU 16.0 -> 13.3 ms, profiles/r03_z3_bucket_ab.json), at the price of up to 512 MB of full
# gradients waiting for their collective — nothing against 288 GB of HBM.
RS_BUCKET_MB = 512.0
# Module gathers ordered (and prefetched) as waves of this many consecutive groups: one ready and
# one done event, and one consumer wait, per wave (see _GatherRuntime).  1 (per-module ordering,
# the next module prefetched while this one computes) is the default: at most two modules' full
# parameters are resident.  ``gather_wave=2`` halves the cross-stream waits, but when wave w starts
# wave w + 1 is already in flight — up to four modules' full parameters resident — and the first
# module of a wave waits for both of its gathers; its host-time win was measured on the
# compute-free parameter-set model only, which the bench now runs single-stream.
GATHER_WAVE = 1
# Cross-stream ordering of the side-stream collectives: comm.STREAM_SYNC ("flag": stream memory
# operations on a device word, resolved by the GPU; "event": HIP events, whose pending cross-stream
# waits keep a HIP runtime thread polling — profiles/r05_event_poll_probe.jsonl)


class ShardedOptimizer:
    """zero3.py:81-168 with ``update`` selecting reference (no-op) or real ZeRO-3 updates."""

    @on_param_device
    def __init__(self, optimizer: Optimizer, *, update: bool = False, comm=None, sync: bool = True,
                 gather_dtype=None, bucket_mb: float = RS_BUCKET_MB, grad_comm: str | None = None,
                 gather_wave: int = GATHER_WAVE, side_stream: bool = True,
                 stream_sync: str = STREAM_SYNC):
        if not isinstance(optimizer, torch.optim.Adam):
            raise TypeError("zero_amd ShardedOptimizer wraps torch.optim.Adam / AdamW")
        self.optimizer = optimizer
        self.original_param_groups = optimizer.param_groups
        self.params = [p for group in self.original_param_groups for p in group["params"]]
        self._param_device = self.params[0].device if self.params else None  # (on_param_device)
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
        self.runtime = _GatherRuntime(world_size, rank, comm, dev, wave=gather_wave,
                                      stream_sync=stream_sync,
                                      side_stream=side_stream)
        # the gather rate limit: the hooks release every module through _release_group
        self.runtime._throttled = self.runtime.stream is not None and world_size > 1
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
        ckpt.bind_inner_load(self)  # opt.optimizer.load_state_dict fills the flat state
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
        self._fast_sig = self._fast_sets = None
        self._step_shared = self._step_shared_sig = None
        self._retired = []
        self._expose_state()

    def _state_views(self, i: int) -> dict:
        """name -> live view of param i's chunk of the flat update state."""
        ar = self._arena
        s, n, shp = int(ar.slot[i]), int(ar.ln[i]), ar.shard_shapes[i]
        views = {"exp_avg": self._m[s:s + n].view(shp), "exp_avg_sq": self._v[s:s + n].view(shp)}
        if self._lo is not None:  # fp32 master = the bf16 chunk's bits << 16 + this residual
            views["master_residual"] = self._lo[s:s + n].view(shp)
        if self._vmax is not None:
            views["max_exp_avg_sq"] = self._vmax[s:s + n].view(shp)
        return views

    def _expose_state(self):
        """optimizer.state[p]: views of the flat state (chunk-shaped) and torch's ``step``."""
        self._step_shared_sig = None  # per-param step tensors again: the next step re-shares
        step_t = {}
        for i, p in enumerate(self.params):
            st = self.optimizer.state[p]
            st.update(self._state_views(i))
            s = int(self._steps[i])
            if s:
                t = step_t.get(s)
                if t is None:
                    t = step_t[s] = torch.tensor(float(s))
                st["step"] = t

    def _ensure_vmax(self):
        ar = self._arena
        self._vmax = torch.zeros(ar.total, dtype=torch.float32, device=ar.device)
        self._expose_state()  # (cached Adam rows gain the vmax pointer: rebuilt on their next use)

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
        cs = self.runtime.side()
        if getattr(self, "_ref_syncs", None) is None:  # (ready, done): reused every step
            self._ref_syncs = (Sync(self.runtime.sync_kind), Sync(self.runtime.sync_kind))
        ready, done_sync = self._ref_syncs
        ready.record(cur.cuda_stream)
        ready.wait(cs.cuda_stream)
        with _group_ctx(self.comm):
            for buf, _, _ in shards:
                self.comm.all_reduce(buf, cs)
        # after the group: the division runs behind the collectives on the side stream
        with torch.cuda.stream(cs):
            self.last_reduced_grads = [buf.reshape(-1)[:n].view(shp).div_(self.world_size)
                                       for buf, n, shp in shards]
        for buf, _, _ in shards:
            buf.record_stream(cs)
        done = _timed_after(cs)  # (the communication_time span's end)
        done_sync.record(cs.cuda_stream)
        done_sync.wait(cur.cuda_stream)
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
            if self.runtime.stream is None:  # single stream: the reduce-scatters are behind us
                done = torch.cuda.Event(enable_timing=True)
                done.record(cur)
            else:
                done = red.ev_done[red.K - 1]
                done.wait(cur.cuda_stream)
        idx = np.nonzero(red.had_grad & (ar.ln > 0))[0]
        self._steps[idx] += 1
        hps = {gi: adam_group_hparams(self._groups[gi], self.optimizer) for gi in set(self._group_of)}
        if any(h["amsgrad"] for h in hps.values()) and self._vmax is None:
            self._ensure_vmax()
        steps = self._steps[idx]
        uniform = len(idx) > 0 and bool((steps == steps[0]).all())
        # (ws == 1: Adam reads the local grads themselves, whose addresses change — no fast path)
        sig = (idx.tobytes(), self._vmax is None) if self.world_size > 1 else None
        fast = self._fast_sets if uniform and sig is not None and self._fast_sig == sig else None
        if fast is not None:  # the same parameters as last step, one step count: cached sets
            for gi, aset in fast:
                h = hps[gi]
                hp = adam_hparams(h["lr"], h["beta1"], h["beta2"], h["eps"], h["weight_decay"],
                                  int(steps[0]), decoupled=h["decoupled"], amsgrad=h["amsgrad"],
                                  maximize=h["maximize"], grad_div=float(self.world_size))
                if self.timing_events is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(cur)
                    aset.run(hp, cur)
                    self.timing_events.append((e0, _timed_after(cur), aset.bytes))
                else:
                    aset.run(hp, cur)
        elif len(idx):
            rows = self._adam_rows(idx)
            keys = np.stack([np.asarray(self._group_of)[idx], self._steps[idx]], axis=1)
            used = []
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
                used.append((int(key[0]), hit[1]))
            # one set per param group and one step count: next step takes the cached sets
            self._fast_sig = sig if uniform else None
            self._fast_sets = used if uniform else None
        if uniform:  # torch's state['step'] (a CPU tensor): one shared tensor, updated in place
            t = self._step_shared
            if t is None:
                t = self._step_shared = torch.tensor(float(steps[0]))
            else:
                t.fill_(float(steps[0]))
            if sig is None or self._step_shared_sig != sig:
                for i in idx.tolist():
                    self.optimizer.state[self.params[i]]["step"] = t
                self._step_shared_sig = sig
        else:
            self._step_shared_sig = None
            step_t = {}
            for i in idx:
                s_ = int(self._steps[i])
                t = step_t.get(s_)
                if t is None:
                    t = step_t[s_] = torch.tensor(float(s_))
                self.optimizer.state[self.params[i]]["step"] = t
        for p in self.params:  # zero3.py:150-153: no grad survives the step
            p.grad = None
        red.reset()
        return done

    @on_param_device
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
            if self.runtime.stream is None:  # single stream: `done` follows the last collective
                e1 = done
            else:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(self.runtime.stream)  # after the last gradient collective
            self._comm_spans.append((e0, e1))
        retired = len(self._retired) if self.update else 0
        if self._sync or retired > 64:
            torch.cuda.synchronize()
            if self.update:
                self._retired.clear()
            self._collect_comm_time()
        else:  # asynchronous steps: count the spans whose end the device has passed
            self._collect_comm_time(completed_only=True)
        self.runtime.end_iteration()
        self.step_time += time.perf_counter() - step_start
        return loss

    def _collect_comm_time(self, completed_only: bool = False):
        """zero3.py:125,158: communication_time = from step() entry until the gradient reduction is
        done.  Measured on the device: step-entry event on the compute stream → event after the
        last gradient collective on the side stream (0 when backward already finished them).
        ``completed_only`` (steps without a synchronize): only the spans the device has finished,
        so the list stays a step or two long and the counter trails by as much."""
        keep = []
        for e0, e1 in self._comm_spans:
            # both ends must have completed: e0 sits on the compute stream, which can still hold
            # queued work after every reduce-scatter on the side stream (e1) has finished, and
            # hipEventElapsedTime on an incomplete event fails
            if completed_only and not (e1.query() and e0.query()):
                keep.append((e0, e1))
                continue
            self.communication_time += max(0.0, e0.elapsed_time(e1) / 1e3)
        self._comm_spans = keep

    def zero_grad(self, set_to_none: bool = True):
        self.optimizer.zero_grad(set_to_none=set_to_none)

    def mark_params_changed(self):
        """Tell the gathers that this rank's shards (``p.data`` between gathers) were written
        outside ``step()``: the side-stream all-gathers read the shards and are ordered after the
        compute stream only at the first gather after a step, so an in-place edit between two
        steps (e.g. step → eval forward → ``p.data.copy_(...)`` → train forward) must be followed
        by this call before the next forward.  ``load_state_dict`` calls it."""
        self.runtime.mark_inputs_changed()

    # checkpointing (zero_amd/checkpoint.py) -------------------------------------------------------
    def _ckpt_header(self):
        return ckpt.header(3, self.world_size, self.rank, self.local_param_indices, update=self.update)

    @on_param_device
    def state_dict(self):
        """The inner optimizer's state dict in torch's format; update mode: every parameter's
        entry is this rank's dim-0 chunk of its state (copies of the flat state, incl. the split
        master's residual), so each rank saves its own shard.  Reference mode keeps no state
        (zero3.py:150-153), like the reference."""
        torch.cuda.synchronize(self._arena.device)
        sd = Optimizer.state_dict(self.optimizer)
        state = {}
        if self.update:
            index = {id(p): k for k, p in enumerate(ckpt.inner_params(self.optimizer))}
            for i, p in enumerate(self.params):
                entry = {k: v.detach().clone() for k, v in self._state_views(i).items()}
                entry["step"] = torch.tensor(float(self._steps[i]), dtype=torch.float32)
                state[index[id(p)]] = entry
        sd["state"] = state
        sd["zero_amd"] = self._ckpt_header()
        return sd

    @on_param_device
    def load_state_dict(self, state_dict):
        """Restore this rank's ``state_dict()``: hyper-parameters through torch's loader, the
        chunk state copied into the flat buffers.  The parameters themselves (this rank's chunks)
        are restored by the caller, e.g. ``p.data.copy_(saved_chunk)``, on the compute stream
        before the next forward.  Loading marks the shards changed (``mark_params_changed``), so
        the next gather is ordered after that copy; a caller that edits the shards at any other
        time between two steps (after an eval forward, say) calls ``mark_params_changed()``."""
        ckpt.check_header(state_dict, self._ckpt_header())
        self.mark_params_changed()
        torch.cuda.synchronize(self._arena.device)
        ckpt.load_param_groups(self.optimizer, state_dict)
        self.original_param_groups = self.optimizer.param_groups
        self._groups = list(self.optimizer.param_groups)
        self.optimizer.state.clear()
        if not self.update:
            return
        saved = state_dict.get("state", {})
        params = ckpt.inner_params(self.optimizer)
        index = {id(p): k for k, p in enumerate(params)}
        if any("max_exp_avg_sq" in e for e in saved.values()) and self._vmax is None:
            self._ensure_vmax()
        with torch.no_grad():
            for i, p in enumerate(self.params):
                entry = saved.get(index.get(id(p), -1), {})
                for name, view in self._state_views(i).items():
                    src = entry.get(name)
                    if src is not None:
                        view.copy_(src.reshape(view.shape))
                    else:  # moments 0 (fresh Adam); residual 0 (master = the bf16 chunk)
                        view.zero_()
                self._steps[i] = ckpt.step_of(entry)
        self._expose_state()
