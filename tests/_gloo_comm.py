"""TEST-ONLY communicator: GPU buffers staged through host memory and the gloo process group.

RCCL refuses two ranks of one communicator on the same GPU ("Using the same HIP device for multiple
ranks of the same Communicator is not supported", rccl.h:174-176), and the GPU box has one GPU.  To
exercise the engine's multi-rank orchestration (Layout R buckets, in-place reduce-scatter /
all-gather slices, ZeRO-1 carry, per-rank Adam windows) with the real HIP pack / Adam / unpack
kernels, ws processes share cuda:0 and exchange through this class.  Sums are done in fp32.

``group()`` behaves like an RCCL group: collectives issued inside it are held back and run at
group exit, after every kernel the caller enqueued on the stream before the exit — so a caller
that reads a collective's output, or frees one of its buffers, inside the group is caught here as
it would be on the device.
"""
import contextlib
import os

import torch
import torch.distributed as dist


class GlooStagedComm:
    def __init__(self, group=None):
        self.pg = group  # (not `group`: that name is the RCCL-like group() below)
        self.ws = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.calls = []
        self._deferred = None

    @contextlib.contextmanager
    def group(self):
        if self._deferred is not None:  # nested: the outer group runs everything
            yield
            return
        self._deferred = []
        try:
            yield
        finally:
            ops, self._deferred = self._deferred, None
            for fn, args in ops:
                fn(*args)

    def _defer(self, fn, *args):
        if self._deferred is None:
            return False
        self._deferred.append((fn, args))
        return True

    def reduce_scatter(self, send, recv, stream):
        if self._defer(self.reduce_scatter, send, recv, stream):
            return
        stream.synchronize()
        h = send.detach().to("cpu", torch.float32)
        out = torch.empty(recv.numel(), dtype=torch.float32)
        dist.reduce_scatter_tensor(out, h, group=self.pg)
        with torch.cuda.stream(stream):
            recv.copy_(out.to(recv.device).to(recv.dtype))
        self.calls.append(("rs", send.numel()))

    def all_gather(self, send, recv, stream):
        if self._defer(self.all_gather, send, recv, stream):
            return
        stream.synchronize()
        h = send.detach().to("cpu")
        if h.dtype != torch.float32:  # a gather is a byte copy: move bf16 / uint8 as int8 bytes
            h = h.view(torch.int8)
        out = torch.empty(recv.numel() * recv.element_size() // h.element_size(), dtype=h.dtype)
        dist.all_gather_into_tensor(out, h, group=self.pg)
        out = out.view(recv.dtype)
        with torch.cuda.stream(stream):
            recv.copy_(out.to(recv.device))
        self.calls.append(("ag", recv.numel()))

    def _root(self, root):
        return dist.get_global_rank(self.pg, root) if self.pg else root

    def reduce(self, t, root, stream):
        if self._defer(self.reduce, t, root, stream):
            return
        stream.synchronize()
        h = t.detach().to("cpu", torch.float32)
        dist.reduce(h, dst=self._root(root), group=self.pg)
        if root == self.rank:
            with torch.cuda.stream(stream):
                t.copy_(h.to(t.device).to(t.dtype))
        self.calls.append(("reduce", t.numel()))

    def reduce_out(self, send, recv, root, stream):
        if self._defer(self.reduce_out, send, recv, root, stream):
            return
        stream.synchronize()
        h = send.detach().to("cpu", torch.float32)
        dist.reduce(h, dst=self._root(root), group=self.pg)
        if root == self.rank:
            with torch.cuda.stream(stream):
                recv.copy_(h.to(recv.device).to(recv.dtype))
        self.calls.append(("reduce_out", send.numel()))

    def broadcast(self, t, root, stream):
        if self._defer(self.broadcast, t, root, stream):
            return
        stream.synchronize()
        h = t.detach().to("cpu")
        if h.dtype != torch.float32:
            h = h.view(torch.int8)
        dist.broadcast(h, src=self._root(root), group=self.pg)
        h = h.view(t.dtype)
        with torch.cuda.stream(stream):
            t.copy_(h.to(t.device))
        self.calls.append(("bcast", t.numel()))

    def reduce_v(self, buf, win_off, win_len, stream):
        if self._defer(self.reduce_v, buf, win_off, win_len, stream):
            return
        stream.synchronize()
        h = buf.detach().to("cpu", torch.float32)
        for root, (off, n) in enumerate(zip(win_off, win_len)):
            if n:
                part = h[int(off):int(off) + int(n)].clone()
                dist.reduce(part, dst=dist.get_global_rank(self.pg, root) if self.pg else root,
                            group=self.pg)
                if root == self.rank:
                    h[int(off):int(off) + int(n)] = part
        with torch.cuda.stream(stream):
            buf.copy_(h.to(buf.device).to(buf.dtype))
        self.calls.append(("rsv", int(sum(win_len))))

    def broadcast_v(self, buf, win_off, win_len, stream):
        if self._defer(self.broadcast_v, buf, win_off, win_len, stream):
            return
        stream.synchronize()
        h = buf.detach().to("cpu")
        for root, (off, n) in enumerate(zip(win_off, win_len)):
            if n:
                part = h[int(off):int(off) + int(n)].clone()
                raw = part if part.dtype == torch.float32 else part.view(torch.int8)
                dist.broadcast(raw, src=self._root(root), group=self.pg)
                h[int(off):int(off) + int(n)] = raw.view(part.dtype)
        with torch.cuda.stream(stream):
            buf.copy_(h.to(buf.device))
        self.calls.append(("agv", int(sum(win_len))))

    def all_reduce(self, t, stream):
        if self._defer(self.all_reduce, t, stream):
            return
        stream.synchronize()
        h = t.detach().to("cpu", torch.float32)
        dist.all_reduce(h, group=self.pg)
        with torch.cuda.stream(stream):
            t.copy_(h.to(t.device).to(t.dtype))
        self.calls.append(("ar", t.numel()))


_TYPESTR = {0: "<f4", 1: "<i2", 2: "|u1"}  # ZS_F32, ZS_BF16 (as int16 bits), ZS_U8


def _dev_view(ptr, n, dtype_code, device="cuda"):
    """TEST-ONLY: a tensor over ``n`` elements of device memory at ``ptr`` (the table-driven
    collectives take raw pointers), through ``__cuda_array_interface__``."""
    class _Arr:
        pass

    a = _Arr()
    a.__cuda_array_interface__ = {"shape": (int(n),), "typestr": _TYPESTR[int(dtype_code)],
                                  "data": (int(ptr), False), "version": 2}
    t = torch.as_tensor(a, device=device)
    return t.view(torch.bfloat16) if int(dtype_code) == 1 else t


def _add_table_methods(cls):
    """all_gather_group / reduce_scatter_group (RcclComm's table forms) over the tensor forms."""
    def all_gather_group(self, send, recv, count, dtype, stream):
        with self.group():
            for s, r, n in zip(send, recv, count):
                if int(n):
                    self.all_gather(_dev_view(s, n, dtype), _dev_view(r, int(n) * self.ws, dtype), stream)
        self.calls.append(("ag_group", len(count)))

    def reduce_scatter_group(self, send, recv, count, dtype, stream):
        with self.group():
            for s, r, n in zip(send, recv, count):
                if int(n):
                    self.reduce_scatter(_dev_view(s, int(n) * self.ws, dtype), _dev_view(r, n, dtype),
                                        stream)
        self.calls.append(("rs_group", len(count)))

    cls.all_gather_group = all_gather_group
    cls.reduce_scatter_group = reduce_scatter_group
    return cls


_add_table_methods(GlooStagedComm)


# RcclComm per (world size, rank) within ONE batch of cases (tests/_zero_run.py _run_seq opens
# and closes the scope on every rank, so every rank of a batch creates — or reuses — its
# communicator at the same case): an RCCL communicator over the socket transport costs ~1-2 s to
# bootstrap at ws = 8, and a batch runs up to a dozen cases.  The communicator is independent of
# the per-case torch.distributed group it was bootstrapped over.
_RCCL_SCOPE = [None]


def open_comm_scope():
    _RCCL_SCOPE[0] = {}  # (what an earlier, failed batch left open is not touched)


def close_comm_scope():
    comms, _RCCL_SCOPE[0] = _RCCL_SCOPE[0], None
    for c in (comms or {}).values():
        c.close()


def test_comm(group=None):
    """The multi-rank GPU workers' communicator.  Default: GlooStagedComm.  With
    ``ZS_TEST_COMM=rccl`` (tests/test_gpu_rccl.py): the PRODUCT communicator, RcclComm — every rank
    of the one-GPU box is made a separate node to RCCL by its own NCCL_HOSTID, so RCCL accepts the
    shared device and runs its real collectives (its kernels, ring order and bf16 rounding) between
    the ranks through the socket transport over loopback.  NCCL_HOSTID is read at communicator
    init, so it is set here, per rank, just before.  Inside a batch scope (open_comm_scope) the
    world group's communicator is created once and reused by the batch's later cases."""
    if os.environ.get("ZS_TEST_COMM", "") != "rccl":
        return GlooStagedComm(group)
    from zero_amd.comm import RcclComm

    scope = _RCCL_SCOPE[0]
    key = (dist.get_world_size(), dist.get_rank()) if group is None else None
    if scope is not None and key in scope:
        return scope[key]
    os.environ["NCCL_HOSTID"] = f"zs-test-rank{dist.get_rank()}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    c = RcclComm(group)
    if scope is not None and key is not None:
        scope[key] = c
    return c


class SimRankComm:
    """TEST-ONLY stand-in for rank ``rank`` of a ``ws``-rank job on one GPU, where every other rank
    contributes zeros to each sum and holds, for every gather, the same shard as this rank.  It lets
    a full-scale run exercise rank 0's real layout and kernels (arena slots, uneven chunks, Adam on
    the owned window) without peers.  ``log`` keeps, per reduce-scatter, a copy of this rank's
    chunk of the send buffer (what the sum delivers) and the receive pointer."""

    def __init__(self, ws, rank=0, keep_log=False):
        self.ws, self.rank = ws, rank
        self.log = [] if keep_log else None

    def group(self):
        return contextlib.nullcontext()

    def reduce_scatter(self, send, recv, stream):
        n = recv.numel()
        with torch.cuda.stream(stream):
            mine = send[self.rank * n:(self.rank + 1) * n]
            if self.log is not None:
                self.log.append((recv.data_ptr(), mine.clone()))
            if mine.data_ptr() != recv.data_ptr():
                recv.copy_(mine)

    def all_gather(self, send, recv, stream):
        with torch.cuda.stream(stream):
            src = send.clone()
            recv.view(self.ws, -1).copy_(src.view(1, -1).expand(self.ws, -1))

    def reduce_out(self, send, recv, root, stream):
        if root == self.rank and send.data_ptr() != recv.data_ptr():
            with torch.cuda.stream(stream):
                recv.copy_(send)

    def all_reduce(self, t, stream):
        pass

    def reduce(self, t, root, stream):
        pass

    def broadcast(self, t, root, stream):
        pass

    def reduce_v(self, buf, win_off, win_len, stream):
        pass

    def broadcast_v(self, buf, win_off, win_len, stream):
        pass
