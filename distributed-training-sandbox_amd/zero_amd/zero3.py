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

This module keeps that API.  Two modes:
  * ``update=False`` (default): reference semantics, bit-for-bit in what is observable — the
    reduced shard grads are computed (one grouped RCCL all-reduce per step, exposed as
    ``last_reduced_grads``) and then discarded; parameters stay at their initial values.
  * ``update=True``: the ZeRO-3 the reference intends — release() keeps full-size grads, step()
    reduce-scatters them (one grouped RCCL reduce-scatter) so every rank gets the summed grad of
    exactly its chunk, and the fused HIP Adam updates the chunk in place (== data-parallel Adam,
    sliced).  Optimizer state is one flat fp32 buffer over the rank's chunks.
In both modes ``materialize`` is a zero-copy RCCL all-gather from the shard straight into the full
tensor (rows of torch.chunk are contiguous: full = [chunk_0 | … | chunk_{ws-1}]), grouped per
module, launched on a side HIP stream, and the NEXT module's gather is prefetched there while the
current module computes (the order is learned on the first iteration).
"""
from __future__ import annotations

import contextlib
import time

import numpy as np
import torch
from torch.optim import Optimizer

from . import _lib
from .comm import RcclComm, comm_stream, zs_dtype
from .kernels import stream_handle
from .engine import ALIGN_ELEMS, probed_zeros
from .kernels import AdamSet, adam_hparams
from .plan import Plan
from ._sharded import adam_group_hparams
from ._lib import ZS_BF16, ZS_BF16_SPLIT, ZS_F32
from .training_utils.utils import get


def _chunk_geom(d0: int, ws: int, rank: int):
    cs = -(-d0 // ws) if d0 else 0  # torch.chunk rows per chunk
    r0, r1 = min(rank * cs, d0), min((rank + 1) * cs, d0)
    return cs, r0, r1


class _GatherRuntime:
    """Side-stream all-gathers of module parameter groups with one-ahead prefetch.

    The first iteration records the order in which module groups are materialised (forward, then
    backward); afterwards each materialise also launches the gather of the next group in that
    order, so the all-gather overlaps the current module's compute.  ``end_iteration`` (called at
    the end of step()) prefetches the first group of the next iteration."""

    def __init__(self, ws, rank, comm, device):
        self.ws, self.rank, self.comm, self.device = ws, rank, comm, device
        self.stream = comm_stream(device)
        self.pending = {}      # key -> (list[(manager, full_tensor)], event)
        self.sequence = []     # learned order of group keys
        self.pos = 0
        self.recording = True
        self.key_managers = {}
        self.n_gathers = 0
        self.n_prefetch_hits = 0

    def _group(self):
        grp = getattr(self.comm, "group", None)
        return grp() if grp is not None else contextlib.nullcontext()

    def launch(self, key, managers):
        """Enqueue the all-gather of ``managers`` on the side stream; returns immediately."""
        if key in self.pending or not managers:
            return
        ev_ready = torch.cuda.Event()
        ev_ready.record(torch.cuda.current_stream(self.device))  # shards may just have been updated
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev_ready)
            # kernels (pad copies, fp8 quantisation) before the RCCL group, dequantisation after:
            # an RCCL group only launches its collectives at group end
            states = [m._gather_prepare(self.stream) for m in managers]
            with self._group():
                for m, st in zip(managers, states):
                    m._gather_issue(self.comm, self.stream, st)
            out = [(m, m._gather_finish(self.stream, st)) for m, st in zip(managers, states)]
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.pending[key] = (out, ev)
        self.n_gathers += 1

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
        out, ev = self.pending.pop(key)
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        for m, full in out:
            full.record_stream(cur)
            m._install_full(full)

    def end_iteration(self):
        if self.sequence:
            self.recording = False
        self.pending.clear()
        self.pos = 0
        self._prefetch(0)


class Zero3ParamManager:
    """zero3.py:25-52: tracks one parameter's dim-0 shard and gathers / releases the full tensor."""

    def __init__(self, param, shard_idx, world_size, shard_dim=0, *, runtime=None, shard=None,
                 full_shape=None, keep_full_grad=False, gather_dtype=None):
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
        if gather_dtype not in (None, "fp8"):
            raise ValueError(f"gather_dtype must be None or 'fp8' (got {gather_dtype!r})")
        # fp8 only for matrices (row-wise scales); vectors (biases, norms) gather as they are
        self.fp8 = gather_dtype == "fp8" and len(self.full_shape) >= 2

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
        send = self.shard.reshape(-1)
        if ws == 1:  # the shard is the whole parameter: nothing to gather
            return (send, send)
        if send.numel() != self.S:  # short / empty last chunks: pad so every rank sends S elements
            pad = torch.zeros(self.S, dtype=send.dtype, device=dev)
            pad[:send.numel()].copy_(send)
            send = pad
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

    def materialize(self):
        """zero3.py:36-41 for this one parameter."""
        rt = self.runtime
        rt.launch(("param", id(self)), [self])
        out, ev = rt.pending.pop(("param", id(self)))
        cur = torch.cuda.current_stream(self.shard.device)
        cur.wait_event(ev)
        for m, full in out:
            full.record_stream(cur)
            m._install_full(full)

    def release(self):
        """zero3.py:43-52: back to the local shard; shrink a full-size grad to its local rows
        (reference mode) or keep it for the reduce-scatter in step() (update mode)."""
        self.param.data = self.shard
        g = self.param.grad
        if g is not None and g.shape != self.shard.shape and not self.keep_full_grad:
            self.param.grad.data = g.data.reshape(self.full_shape)[self.r0:self.r1].clone()
        self.full_data = None


def register_zero3_hooks(model, param_managers):
    """zero3.py:56-77: forward / backward pre-hooks materialise a module's direct parameters (one
    grouped all-gather, prefetched on the side stream), post-hooks release them."""
    runtimes = {m.runtime for m in param_managers.values() if m.runtime is not None}
    mod_managers = {}
    for mod in model.modules():
        ms = [param_managers[p] for _, p in mod.named_parameters(recurse=False) if p in param_managers]
        mod_managers[id(mod)] = ms
    for rt in runtimes:
        rt.key_managers = {}
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
            rt = ms[0].runtime
            if rt is None:
                for m in ms:
                    m.materialize()
            else:
                rt.materialize((phase, id(module)), ms)
            return None
        return pre_hook

    def post_hook(module, *args):
        for m in mod_managers.get(id(module)) or []:
            m.release()
        return None

    handles = []
    for m in model.modules():
        handles.append(m.register_forward_pre_hook(make_pre("fwd")))
        handles.append(m.register_forward_hook(post_hook))
        handles.append(m.register_full_backward_pre_hook(make_pre("bwd")))
        handles.append(m.register_full_backward_hook(post_hook))
    return handles


class ShardedOptimizer:
    """zero3.py:81-168 with ``update`` selecting reference (no-op) or real ZeRO-3 updates."""

    def __init__(self, optimizer: Optimizer, *, update: bool = False, comm=None, sync: bool = True,
                 gather_dtype=None):
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

        dev = self.params[0].device
        if dev.type != "cuda":
            raise RuntimeError("zero_amd: parameters must live on a GPU; there is no CPU path")
        if comm is None:
            comm = RcclComm()
        self.comm = comm
        self.runtime = _GatherRuntime(world_size, rank, comm, dev)
        # zero3.py:104-110: every param becomes its dim-0 chunk; one manager per param
        self.param_managers = {}
        self._full_shapes = []
        for param in self.params:
            full_shape = tuple(param.shape)
            self._full_shapes.append(full_shape)
            cs, r0, r1 = _chunk_geom(full_shape[0] if full_shape else 1, world_size, rank)
            shard = param.data.reshape(full_shape or (1,))[r0:r1].contiguous() if full_shape else \
                param.data.reshape(1).clone()
            param.data = shard
            self.param_managers[param] = Zero3ParamManager(
                param, rank, world_size, 0, runtime=self.runtime, shard=shard,
                full_shape=full_shape, keep_full_grad=self.update, gather_dtype=gather_dtype)
        for group in self.optimizer.param_groups:  # zero3.py:114-115
            group["params"] = [p for p in group["params"] if p in self.local_params]
        self.grad_hooks = {}
        self.communication_time = 0.0
        self.step_time = 0.0
        self.last_reduced_grads = None
        self._engine = None
        self.timing_events = None  # optional list of (start, end, bytes) around each Adam launch

    # ------------------------------------------------------------------------------------------
    def _build_update_engine(self):
        dev = self.params[0].device
        dtype = self.params[0].dtype
        numels = [int(np.prod(s)) if s else 1 for s in self._full_shapes]
        dim0 = [s[0] if s else 1 for s in self._full_shapes]
        plan = Plan(numels, self.world_size, self.rank, "chunk", dim0=dim0, align_elems=ALIGN_ELEMS)
        L = plan.stream_len(self.rank)
        pc = plan.pieces(self.rank)
        # exp_avg, exp_avg_sq (+ for bf16 params the split master's int16 residual: the fp32
        # master is the bf16 shard + residual, include/zero_amd.h ZS_BF16_SPLIT; starts at 0)
        nlo = (L + 1) // 2 if dtype == torch.bfloat16 else 0
        state, placement = probed_zeros(2 * L + nlo, torch.float32, dev)
        eng = dict(plan=plan, pieces=pc, L=L, dtype=dtype, state=state, placement=placement,
                   m=state[:L], v=state[L:2 * L],
                   vmax=None, gshard=torch.zeros(L, dtype=dtype, device=dev),
                   lo=state[2 * L:].view(torch.int16)[:L] if nlo else None,
                   steps=np.zeros(len(self.params), np.int64), cache={}, retired=[])
        self._engine = eng
        for i, so, ln in zip(pc.param, pc.stream_off, pc.length):
            p = self.params[i]
            shp = self.param_managers[p].shard.shape
            st = self.optimizer.state[p]
            st["exp_avg"] = eng["m"][so:so + ln].view(shp)
            st["exp_avg_sq"] = eng["v"][so:so + ln].view(shp)

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
                shards.append((g, n, g.shape))
        grp = getattr(self.comm, "group", None)
        with (grp() if grp is not None else contextlib.nullcontext()):
            for buf, _, _ in shards:
                self.comm.all_reduce(buf, cur)
        self.last_reduced_grads = [buf.reshape(-1)[:n].view(shp).div_(self.world_size)
                                   for buf, n, shp in shards]
        for param in self.params:  # zero3.py:150-153 for-else: every grad is dropped
            param.grad = None

    def _step_update(self):
        if self._engine is None:
            self._build_update_engine()
        eng = self._engine
        cur = torch.cuda.current_stream()
        pc, ws = eng["pieces"], self.world_size
        has = np.array([p.grad is not None for p in self.params])
        # 1. reduce-scatter every full-size grad into this rank's chunk (one RCCL group)
        grp = getattr(self.comm, "group", None)
        with (grp() if grp is not None else contextlib.nullcontext()):
            for i, so, ln in zip(pc.param, pc.stream_off, pc.length):
                p = self.params[i]
                man = self.param_managers[p]
                if p.grad is None:
                    continue
                g = p.grad.reshape(-1)
                if g.numel() != man.numel:
                    raise RuntimeError("ZeRO-3 update mode needs full-size grads at step()")
                if man.S * ws != man.numel:  # uneven chunks: pad to ws*S
                    pad = torch.zeros(man.S * ws, dtype=g.dtype, device=g.device)
                    pad[:man.numel].copy_(g)
                    g = pad
                recv = eng["gshard"][so:so + man.S] if ln == man.S else torch.empty(
                    man.S, dtype=g.dtype, device=g.device)
                self.comm.reduce_scatter(g, recv, cur)
                if ln != man.S and ln:
                    eng["gshard"][so:so + ln].copy_(recv[:ln])
        # 2. fused Adam over every chunk this rank holds
        owned = np.array([ln > 0 for ln in pc.length]) & has[pc.param]
        idx = pc.param[owned]
        eng["steps"][idx] += 1
        if any(adam_group_hparams(g, self.optimizer)["amsgrad"] for g in self._groups) and eng["vmax"] is None:
            eng["vmax"] = torch.zeros(eng["L"], dtype=torch.float32, device=eng["m"].device)
        rows = np.zeros((len(idx), 9), np.uint64)
        es = self.params[0].element_size()
        so = pc.stream_off[owned].astype(np.uint64)
        rows[:, 0] = np.uint64(eng["gshard"].data_ptr()) + so * np.uint64(es)
        shard_ptr = np.array([self.param_managers[self.params[i]].shard.data_ptr() for i in idx], np.uint64)
        if eng["lo"] is not None:  # master = bf16 shard (in and out) + residual
            rows[:, 1], rows[:, 3] = shard_ptr, shard_ptr
            rows[:, 2] = np.uint64(eng["lo"].data_ptr()) + so * np.uint64(2)
        else:
            rows[:, 1], rows[:, 2] = shard_ptr, shard_ptr
        rows[:, 4] = np.uint64(eng["m"].data_ptr()) + so * np.uint64(4)
        rows[:, 5] = np.uint64(eng["v"].data_ptr()) + so * np.uint64(4)
        if eng["vmax"] is not None:
            rows[:, 6] = np.uint64(eng["vmax"].data_ptr()) + so * np.uint64(4)
        rows[:, 8] = pc.length[owned].astype(np.uint64)
        keys = np.stack([np.asarray(self._group_of)[idx], eng["steps"][idx]], axis=1)
        for key in np.unique(keys, axis=0) if len(idx) else []:
            sel = np.nonzero((keys == key).all(axis=1))[0]
            sub = np.ascontiguousarray(rows[sel])
            ck = (int(key[0]), len(sel), int(sel[0]))
            hit = eng["cache"].get(ck)
            if hit is None or hit[0] != sub.tobytes():
                if hit is not None:  # keep until the device is idle (hipFree would sync it)
                    eng["retired"].append(hit[1])
                hit = (sub.tobytes(), AdamSet(sub, ZS_BF16, ZS_BF16_SPLIT) if eng["lo"] is not None
                       else AdamSet(sub, ZS_F32))
                eng["cache"][ck] = hit
            h = adam_group_hparams(self._groups[int(key[0])], self.optimizer)
            hp = adam_hparams(h["lr"], h["beta1"], h["beta2"], h["eps"], h["weight_decay"], int(key[1]),
                              decoupled=h["decoupled"], amsgrad=h["amsgrad"], maximize=h["maximize"],
                              grad_div=float(ws))
            if self.timing_events is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(cur)
                hit[1].run(hp, cur)
                e1.record(cur)
                self.timing_events.append((e0, e1, hit[1].bytes))
            else:
                hit[1].run(hp, cur)
        for i in idx:
            st = self.optimizer.state[self.params[i]]
            st["step"] = torch.tensor(float(eng["steps"][i]))
        for p in self.params:
            p.grad = None

    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        step_start = time.perf_counter()
        with torch.no_grad():
            if self.update:
                self._step_update()
            else:
                self._reduce_reference()
        if self._sync or (self._engine is not None and len(self._engine["retired"]) > 64):
            torch.cuda.synchronize()
            if self._engine is not None:
                self._engine["retired"].clear()
        self.communication_time += time.perf_counter() - step_start
        self.runtime.end_iteration()
        self.step_time += time.perf_counter() - step_start
        return loss

    def zero_grad(self, set_to_none: bool = True):
        self.optimizer.zero_grad(set_to_none=set_to_none)
