"""Collective backends for the ZeRO step.

``RcclComm`` is the product backend: its own RCCL communicator (``zs_comm_*``, csrc/zs_comm.cpp)
bootstrapped by broadcasting an ``ncclUniqueId`` over the default ``torch.distributed`` group, and
bucketed reduce-scatter / all-gather / all-reduce enqueued on the caller's HIP stream.  It replaces
the reference's per-tensor blocking c10d calls (zero1.py:83,102; zero2.py:107,133; zero3.py:39,146).

The engine only needs the methods below (reduce_scatter / all_gather for even buckets,
reduce_v / broadcast_v for ragged ones, all_reduce for ZeRO-3), so tests can substitute a gloo-backed
implementation to exercise the multi-rank orchestration on one GPU (RCCL does not allow two ranks
of one communicator on the same device).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch
import torch.distributed as dist

from . import _lib
from .kernels import stream_handle

_DTYPES = {torch.float32: _lib.ZS_F32, torch.bfloat16: _lib.ZS_BF16, torch.uint8: _lib.ZS_U8}


def zs_dtype(dt: torch.dtype) -> int:
    try:
        return _DTYPES[dt]
    except KeyError:
        raise TypeError(f"zero_amd: unsupported dtype {dt} (float32, bfloat16, uint8)") from None


_COMM_STREAMS = {}


def comm_stream(device) -> torch.cuda.Stream:
    """THE side stream for collectives on ``device`` (one per device and process), at the highest
    priority: the compute stream's streaming kernels launch 128 workgroups per CU, and an RCCL
    kernel queued behind them would wait for CU slots while its peers spin; a high-priority queue
    gets its workgroups dispatched first.  One stream for every engine of the process — not a new
    one from torch's rotating pool per engine — so collectives of different communicators are
    never in flight at once (the ordering NCCL requires of several communicators), and a process
    that builds engine after engine keeps the same stream-to-hardware-queue mapping."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _COMM_STREAMS.get(idx)
    if s is None:
        s = _COMM_STREAMS[idx] = torch.cuda.Stream(device=idx, priority=-1)  # < 0: high priority
    return s


def rccl_version() -> int:
    v = ctypes.c_int()
    _lib.call("zs_rccl_version", ctypes.byref(v))
    return v.value


class RcclComm:
    """One RCCL communicator over the ranks of ``group`` (default: the world)."""

    def __init__(self, group=None):
        self.ws = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        uid = ctypes.create_string_buffer(_lib.ZS_UNIQUE_ID_BYTES)
        if self.rank == 0:
            _lib.call("zs_comm_unique_id", uid)
        obj = [bytes(uid.raw) if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        uid = ctypes.create_string_buffer(obj[0], _lib.ZS_UNIQUE_ID_BYTES)
        h = ctypes.c_void_p()
        _lib.call("zs_comm_init", uid, self.ws, self.rank, ctypes.byref(h))
        self._h = h

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.call("zs_comm_destroy", h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter teardown
            pass

    @contextlib.contextmanager
    def group(self):
        """RCCL group: the collectives issued inside launch together at exit."""
        _lib.call("zs_group_start")
        try:
            yield
        finally:
            _lib.call("zs_group_end")

    def reduce_scatter(self, send: torch.Tensor, recv: torch.Tensor, stream) -> None:
        """SUM-reduce ``send`` (ws*count elements) and leave chunk ``rank`` in ``recv``."""
        assert send.numel() == recv.numel() * self.ws and send.dtype == recv.dtype
        _lib.call("zs_reduce_scatter", self._h, send.data_ptr(), recv.data_ptr(), recv.numel(),
                  zs_dtype(send.dtype), stream_handle(stream))

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor, stream) -> None:
        assert recv.numel() == send.numel() * self.ws and send.dtype == recv.dtype
        _lib.call("zs_all_gather", self._h, send.data_ptr(), recv.data_ptr(), send.numel(),
                  zs_dtype(send.dtype), stream_handle(stream))

    def reduce(self, t: torch.Tensor, root: int, stream) -> None:
        """SUM-reduce ``t`` onto ``root`` in place (ZeRO overlap buckets: one owner each)."""
        _lib.call("zs_reduce", self._h, t.data_ptr(), t.data_ptr(), t.numel(), zs_dtype(t.dtype),
                  int(root), stream_handle(stream))

    def broadcast(self, t: torch.Tensor, root: int, stream) -> None:
        _lib.call("zs_broadcast", self._h, t.data_ptr(), t.data_ptr(), t.numel(),
                  zs_dtype(t.dtype), int(root), stream_handle(stream))

    def reduce_v(self, buf: torch.Tensor, win_off, win_len, stream) -> None:
        """Reduce-scatter-v in place: window r of ``buf`` (offset win_off[r], win_len[r] elements)
        is SUM-reduced onto rank r — one ncclReduce per owner, launched as one RCCL group."""
        dt, h, base, es = zs_dtype(buf.dtype), stream_handle(stream), buf.data_ptr(), buf.element_size()
        with self.group():
            for root, (off, n) in enumerate(zip(win_off, win_len)):
                if n:
                    ptr = base + int(off) * es
                    _lib.call("zs_reduce", self._h, ptr, ptr, int(n), dt, root, h)

    def broadcast_v(self, buf: torch.Tensor, win_off, win_len, stream) -> None:
        """All-gather-v in place: window r of ``buf`` is broadcast from rank r (one RCCL group)."""
        dt, h, base, es = zs_dtype(buf.dtype), stream_handle(stream), buf.data_ptr(), buf.element_size()
        with self.group():
            for root, (off, n) in enumerate(zip(win_off, win_len)):
                if n:
                    ptr = base + int(off) * es
                    _lib.call("zs_broadcast", self._h, ptr, ptr, int(n), dt, root, h)

    def all_reduce(self, t: torch.Tensor, stream) -> None:
        _lib.call("zs_all_reduce", self._h, t.data_ptr(), t.data_ptr(), t.numel(),
                  zs_dtype(t.dtype), stream_handle(stream))

    def reduce_out(self, send: torch.Tensor, recv: torch.Tensor, root: int, stream) -> None:
        """SUM-reduce ``send`` into ``recv`` on ``root`` (recv untouched elsewhere)."""
        _lib.call("zs_reduce", self._h, send.data_ptr(), recv.data_ptr(), send.numel(),
                  zs_dtype(send.dtype), int(root), stream_handle(stream))

    def reduce_group(self, send, recv, count, root, dtype: int, stream) -> None:
        """One RCCL group of reduces from device-pointer tables (flat-arena rounds): entry i sums
        ``count[i]`` elements at ``send[i]`` into ``recv[i]`` on rank ``root[i]``."""
        n = len(count)
        _lib.call("zs_reduce_group", self._h, n, send.ctypes.data_as(_PU64), recv.ctypes.data_as(_PU64),
                  count.ctypes.data_as(_PI64), root.ctypes.data_as(_PI32), int(dtype),
                  stream_handle(stream))

    def all_gather_group(self, send, recv, count, dtype: int, stream) -> None:
        """One RCCL group of all-gathers from device-pointer tables (a ZeRO-3 module's gather):
        entry i gathers ``count[i]`` elements at ``send[i]`` from every rank into ``recv[i]``."""
        _lib.call("zs_all_gather_group", self._h, len(count), send.ctypes.data_as(_PU64),
                  recv.ctypes.data_as(_PU64), count.ctypes.data_as(_PI64), int(dtype),
                  stream_handle(stream))

    def all_gather_group_bound(self, send, recv, count, dtype: int):
        """all_gather_group with its tables bound once: returns ``run(stream)``, which issues the
        group from the arrays' current contents (the caller refills ``recv`` in place) — the
        per-call ctypes conversions of the table form, paid once (ZeRO-3 gathers every module
        twice per iteration)."""
        fn = _lib.lib.zs_all_gather_group
        n = len(count)
        sp, rp, cp = send.ctypes.data_as(_PU64), recv.ctypes.data_as(_PU64), count.ctypes.data_as(_PI64)
        h, dt = self._h, int(dtype)
        keep = (send, recv, count)  # the pointers stay valid while the closure lives

        def run(stream, _keep=keep):
            _lib.check(fn(h, n, sp, rp, cp, dt, stream_handle(stream)), "zs_all_gather_group")
        return run

    def reduce_scatter_group_bound(self, send, recv, count, dtype: int):
        """reduce_scatter_group with its tables bound once (see all_gather_group_bound): the
        caller refills ``send`` in place before each ``run(stream)``."""
        fn = _lib.lib.zs_reduce_scatter_group
        n = len(count)
        sp, rp, cp = send.ctypes.data_as(_PU64), recv.ctypes.data_as(_PU64), count.ctypes.data_as(_PI64)
        h, dt = self._h, int(dtype)
        keep = (send, recv, count)

        def run(stream, _keep=keep):
            _lib.check(fn(h, n, sp, rp, cp, dt, stream_handle(stream)), "zs_reduce_scatter_group")
        return run

    def all_gather_group_ordered_bound(self, send, recv, count, dtype: int):
        """all_gather_group_bound with the stream ordering in the same library call
        (zs_all_gather_group_ordered): returns ``run(after_stream, ready_event, stream,
        done_event)`` on raw handles — record ``ready_event`` on ``after_stream``, make ``stream``
        wait for it, the group, record ``done_event`` on ``stream``: one foreign call where the
        torch event / stream API takes four."""
        return self._ordered(_lib.lib.zs_all_gather_group_ordered, send, recv, count, dtype)

    def reduce_scatter_group_ordered_bound(self, send, recv, count, dtype: int):
        """reduce_scatter_group_bound with the ordering in the same call (see
        all_gather_group_ordered_bound)."""
        return self._ordered(_lib.lib.zs_reduce_scatter_group_ordered, send, recv, count, dtype)

    def all_gather_group_synced_bound(self, send, recv, count, dtype: int):
        """all_gather_group_bound with the ordering in the same call through sync objects
        (zs_all_gather_group_synced): ``run(after_stream, ready_sync, stream, done_sync)`` on raw
        handles (a sync may be 0) — record ``ready_sync`` on ``after_stream``, make ``stream`` wait
        for it, the group, record ``done_sync`` on ``stream``.  A sync is a HIP event or a stream
        flag (``Sync``)."""
        return self._ordered(_lib.lib.zs_all_gather_group_synced, send, recv, count, dtype)

    def reduce_scatter_group_synced_bound(self, send, recv, count, dtype: int):
        """reduce_scatter_group_bound with sync-object ordering (see all_gather_group_synced_bound)."""
        return self._ordered(_lib.lib.zs_reduce_scatter_group_synced, send, recv, count, dtype)

    def all_gather_group_synced_raw(self):
        """(address of zs_all_gather_group_synced, communicator handle, True): what the host
        extension's GatherFast calls with its own tables (zero3._GatherRuntime)."""
        return (ctypes.cast(_lib.lib.zs_all_gather_group_synced, ctypes.c_void_p).value,
                int(self._h.value or 0), True)

    def reduce_scatter_group_synced_raw(self):
        """(address of zs_reduce_scatter_group_synced, communicator handle, True): what the host
        extension's ReduceFast calls with its own tables (zero3._GradReducer)."""
        return (ctypes.cast(_lib.lib.zs_reduce_scatter_group_synced, ctypes.c_void_p).value,
                int(self._h.value or 0), True)

    def _ordered(self, fn, send, recv, count, dtype):
        n = len(count)
        sp, rp, cp = send.ctypes.data_as(_PU64), recv.ctypes.data_as(_PU64), count.ctypes.data_as(_PI64)
        h, dt = self._h, int(dtype)
        keep = (send, recv, count)

        def run(after, ready, stream, done, _keep=keep):
            rc = fn(h, n, sp, rp, cp, dt, after, ready, stream, done)
            if rc:
                _lib.check(rc, fn.__name__)
        return run

    def reduce_scatter_group(self, send, recv, count, dtype: int, stream) -> None:
        """One RCCL group of SUM reduce-scatters (a ZeRO-3 gradient bucket): entry i reduces
        ``ws * count[i]`` elements at ``send[i]`` and leaves this rank's ``count[i]`` at
        ``recv[i]``."""
        _lib.call("zs_reduce_scatter_group", self._h, len(count), send.ctypes.data_as(_PU64),
                  recv.ctypes.data_as(_PU64), count.ctypes.data_as(_PI64), int(dtype),
                  stream_handle(stream))

    def broadcast_group(self, buf, count, root, dtype: int, stream) -> None:
        """One RCCL group of in-place broadcasts: ``count[i]`` elements at ``buf[i]`` from
        ``root[i]``."""
        _lib.call("zs_broadcast_group", self._h, len(count), buf.ctypes.data_as(_PU64),
                  count.ctypes.data_as(_PI64), root.ctypes.data_as(_PI32), int(dtype),
                  stream_handle(stream))


class Sync:
    """A cross-stream ordering point (``zs_sync``, include/zero_amd.h): a HIP event
    (``kind=_lib.ZS_SYNC_EVENT``) or a stream memory operation on a flag word in pinned host memory
    (``_lib.ZS_SYNC_FLAG``: a 64-bit epoch stored on the producer stream by a one-wave release-store
    kernel (round 6; ``hipStreamWriteValue64`` with zs_tune "sync_write_kernel" 0),
    a wait for >= it on the consumer (a one-wave polling kernel; ``hipStreamWaitValue64`` with
    zs_tune "sync_wait_kernel" 0); a wait whose record has already executed is
    skipped on the host; epochs never wrap).  A wait on a pending HIP event keeps one HIP
    runtime thread polling for as long as it is pending; a flag wait is resolved by the GPU and
    costs the host nothing (profiles/r05_event_poll_probe.jsonl).  ``record(stream_h)`` /
    ``wait(stream_h)`` take raw stream handles; ``h`` is the raw handle the synced group calls
    take.  A flag record from another stream than the previous record's is ordered after it (ABI
    v13), so the word's epochs only grow whichever streams record."""

    __slots__ = ("h", "kind")

    def __init__(self, kind: int):
        h = ctypes.c_void_p()
        _lib.call("zs_sync_create", int(kind), ctypes.byref(h))
        self.h, self.kind = int(h.value), int(kind)

    def record(self, stream_h: int) -> None:
        rc = _lib.lib.zs_sync_record(self.h, stream_h)
        if rc:
            _lib.check(rc, "zs_sync_record")

    def wait(self, stream_h: int) -> None:
        rc = _lib.lib.zs_sync_wait(self.h, stream_h)
        if rc:
            _lib.check(rc, "zs_sync_wait")

    def set_epoch(self, epoch: int) -> None:
        """Test hook: move a flag sync's epoch and word forward (every record must have executed)."""
        _lib.call("zs_sync_set_epoch", self.h, int(epoch))

    def query(self) -> tuple[int, int]:
        """(latest recorded epoch, current word) of a flag sync; (0, 0) for an event."""
        e, w = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.call("zs_sync_query", self.h, ctypes.byref(e), ctypes.byref(w))
        return int(e.value), int(w.value)

    def __del__(self):
        h = getattr(self, "h", 0)
        if h and _lib is not None:
            try:
                _lib.lib.zs_sync_destroy(h)
            except Exception:  # interpreter teardown
                pass
            self.h = 0


# Cross-stream ordering of every engine's collective stream (ZeRO-1/2 rounds, overlap buckets, DDP
# buckets, ZeRO-3 gathers and reduce-scatters): "flag" (stream memory operations, resolved by the
# GPU) or "event" (HIP events: a pending cross-stream wait keeps one HIP runtime thread polling —
# about one core for as long as the host runs ahead of the GPU, profiles/r05_event_poll_probe.jsonl).
# ``ZERO_AMD_STREAM_SYNC`` overrides the default (A/B runs).
STREAM_SYNC = os.environ.get("ZERO_AMD_STREAM_SYNC", "flag")


def _stream_h(stream) -> int:
    if stream is None:
        return torch._C._cuda_getCurrentRawStream(torch.cuda.current_device())
    return stream if isinstance(stream, int) else int(stream.cuda_stream)


class StreamEvent:
    """The ordering surface of a non-timing ``torch.cuda.Event`` — ``record(stream=None)``,
    ``wait(stream=None)``, so ``torch.cuda.Stream.wait_event(ev)`` takes it — over a ``Sync`` of
    the process default kind (``STREAM_SYNC``): the engines' cross-stream ordering without a HIP
    runtime thread polling.  Any stream may record (see ``Sync``)."""

    __slots__ = ("sync",)

    def __init__(self, kind: str | None = None):
        self.sync = Sync(sync_kind(kind or STREAM_SYNC))

    def record(self, stream=None) -> None:
        self.sync.record(_stream_h(stream))

    def wait(self, stream=None) -> None:
        self.sync.wait(_stream_h(stream))


def sync_kind(name: str) -> int:
    """"flag" / "event" -> the zs_sync kind."""
    kinds = {"flag": _lib.ZS_SYNC_FLAG, "event": _lib.ZS_SYNC_EVENT}
    if name not in kinds:
        raise ValueError(f"stream_sync must be 'flag' or 'event' (got {name!r})")
    return kinds[name]


_PU64 = ctypes.POINTER(ctypes.c_uint64)
_PI64 = ctypes.POINTER(ctypes.c_int64)
_PI32 = ctypes.POINTER(ctypes.c_int32)


class C10dComm:
    """The same interface over torch.distributed's own communicator of ``group`` (RCCL under the
    "nccl" backend): every call is issued with ``stream`` as torch's current stream, so c10d
    orders its internal collective stream after the caller's work and the caller's later work
    after the collective.  An A/B baseline for RcclComm (one extra stream hop per call), and the
    bench's fallback if a dedicated communicator cannot be created."""

    def __init__(self, group=None):
        self.group_ = group
        self.ws = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def _root(self, r):
        return dist.get_global_rank(self.group_, r) if self.group_ is not None else r

    @contextlib.contextmanager
    def group(self):
        yield  # c10d collectives are issued one by one

    def reduce_scatter(self, send, recv, stream):
        with torch.cuda.stream(stream):
            if recv.data_ptr() == send.data_ptr() + self.rank * recv.numel() * recv.element_size():
                out = torch.empty_like(recv)  # c10d has no in-place reduce-scatter
                dist.reduce_scatter_tensor(out, send, group=self.group_)
                recv.copy_(out)
            else:
                dist.reduce_scatter_tensor(recv, send, group=self.group_)

    def all_gather(self, send, recv, stream):
        with torch.cuda.stream(stream):
            dist.all_gather_into_tensor(recv, send.clone() if _overlaps(send, recv) else send,
                                        group=self.group_)

    def all_reduce(self, t, stream):
        with torch.cuda.stream(stream):
            dist.all_reduce(t, group=self.group_)

    def reduce(self, t, root, stream):
        with torch.cuda.stream(stream):
            dist.reduce(t, dst=self._root(root), group=self.group_)

    def broadcast(self, t, root, stream):
        with torch.cuda.stream(stream):
            dist.broadcast(t, src=self._root(root), group=self.group_)

    def reduce_out(self, send, recv, root, stream):
        with torch.cuda.stream(stream):
            if root == self.rank:
                if recv.data_ptr() != send.data_ptr():
                    recv.copy_(send)
                dist.reduce(recv, dst=self._root(root), group=self.group_)
            else:  # c10d's reduce is in place; a non-root's buffer is only read (ncclReduce)
                dist.reduce(send, dst=self._root(root), group=self.group_)

    def reduce_v(self, buf, win_off, win_len, stream):
        for root, (off, n) in enumerate(zip(win_off, win_len)):
            if n:
                self.reduce(buf[int(off):int(off) + int(n)], root, stream)

    def broadcast_v(self, buf, win_off, win_len, stream):
        for root, (off, n) in enumerate(zip(win_off, win_len)):
            if n:
                self.broadcast(buf[int(off):int(off) + int(n)], root, stream)

    def close(self):
        pass


def _overlaps(a: torch.Tensor, b: torch.Tensor) -> bool:
    a0, b0 = a.data_ptr(), b.data_ptr()
    return a0 < b0 + b.numel() * b.element_size() and b0 < a0 + a.numel() * a.element_size()
