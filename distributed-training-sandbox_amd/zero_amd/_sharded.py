"""Shared body of the ZeRO-1 / ZeRO-2 ``ShardedOptimizer`` drop-ins.

The public surface is the reference's: ``ShardedOptimizer(optimizer)``,
``.step(closure=None)``, ``.zero_grad()``, attributes ``optimizer``, ``original_param_groups``,
``params``, ``local_param_indices``, ``local_params``, ``step_time``, ``communication_time``,
``broadcast_count``; the inner optimizer's ``param_groups`` are filtered to the owned parameters
(zero1.py:71-74) and ``optimizer.state[p]`` holds ``step`` / ``exp_avg`` / ``exp_avg_sq`` for
every owned parameter (read by memory.py:15-24).  Everything below ``step()`` is the native
engine (engine.py → libzero_amd.so); the inner torch optimizer's own ``step`` is never called.
"""
from __future__ import annotations

import time
import weakref

import torch
import torch.distributed as dist
from torch.optim import Optimizer

from . import checkpoint as ckpt
from ._hooks import on_param_device
from .engine import ShardEngine
from .training_utils.utils import get


def adam_group_hparams(group: dict, optimizer: Optimizer) -> dict:
    """Hyper-parameters of one torch.optim.Adam / AdamW param group (adam.py:38-90)."""
    lr = group["lr"]
    lr = float(lr.item()) if torch.is_tensor(lr) else float(lr)
    beta1, beta2 = group["betas"]
    decoupled = bool(group.get("decoupled_weight_decay", False)) or isinstance(
        optimizer, torch.optim.AdamW)
    return dict(lr=lr, beta1=float(beta1), beta2=float(beta2), eps=float(group["eps"]),
                weight_decay=float(group["weight_decay"]), amsgrad=bool(group.get("amsgrad", False)),
                maximize=bool(group.get("maximize", False)), decoupled=decoupled)


class ShardedOptimizerBase:
    """ZeRO-1/2 wrapper; subclasses set ``_carry`` (ZeRO-1 gradient carry) and ``_variant``."""

    _carry = False
    _variant = 2

    @on_param_device
    def __init__(self, optimizer: Optimizer, *, layout: str = "reference",
                 bucket_mb: float | None = None, comm=None, sync: bool = True, buckets: str = "ragged",
                 overlap: bool = False, overlap_bucket_mb: float = 64.0, master: str = "split",
                 arena: str = "flat", grad_comm: str | None = None):
        if arena not in ("flat", "buckets", "auto"):
            raise ValueError(f"arena must be 'flat', 'buckets' or 'auto' (got {arena!r})")
        if not isinstance(optimizer, torch.optim.Adam):
            raise TypeError("zero_amd ShardedOptimizer wraps torch.optim.Adam / AdamW "
                            f"(got {type(optimizer).__name__})")
        self.optimizer = optimizer
        self.original_param_groups = optimizer.param_groups
        self.params = [p for group in self.original_param_groups for p in group["params"]]
        self._param_device = self.params[0].device if self.params else None  # (on_param_device)
        self._group_of = [gi for gi, group in enumerate(self.original_param_groups)
                          for _ in group["params"]]
        # references to the unfiltered groups' hyper-parameter dicts (lr schedulers mutate these)
        self._groups = list(self.original_param_groups)

        world_size = get("ws")
        rank = get("rank")
        # zero1.py:55-62 / zero2.py:51-58 (the planner computes the same ranges natively)
        params_per_rank = len(self.params) // world_size
        remainder = len(self.params) % world_size
        start_idx = rank * params_per_rank + min(rank, remainder)
        end_idx = start_idx + params_per_rank + (1 if rank < remainder else 0)
        self.local_param_indices = list(range(start_idx, end_idx))
        self.local_params = set(self.params[i] for i in self.local_param_indices)
        self._shard_optimizer_params()
        ckpt.bind_inner_load(self)  # opt.optimizer.load_state_dict fills the flat state

        self.broadcast_count = 0
        self.communication_time = 0.0
        self.step_time = 0.0
        self.world_size, self.rank = world_size, rank
        self._layout = layout
        self._buckets = buckets
        self._comm = comm
        self.arena_calibration = None
        if arena == "auto":
            # measured on this job's interconnect at construction (a collective call): the flat
            # arena's grouped reduce / broadcast against the bucket arena's reduce-scatter /
            # all-gather plus its pack / unpack copies (calibrate_arena)
            arena = "flat"
            if world_size > 1 and layout == "reference" and grad_comm is None:
                self.arena_calibration = calibrate_arena(self)
                arena = self.arena_calibration["chosen"]
        # bytes per bucket (bucket arena) / per round (flat arena, all owners' windows together);
        # default 256 MiB / 1 GiB: a flat round has no pack to pipeline, so fewer, larger rounds
        # cost only the last round's Adam as exposed tail and cut the launches per step
        if bucket_mb is None:
            bucket_mb = 1024.0 if arena == "flat" else 256.0
        self._bucket_bytes = int(bucket_mb * (1 << 20))
        self._sync = sync
        self._master = master  # bf16 params: "split" (bf16 param + int16 residual) or "fp32"
        # ws > 1 exchange: "flat" = params and grads are views of one owner-major arena, rounds of
        # grouped reduce / broadcast, no pack / unpack (flat.py); "buckets" = the rank-major
        # bucket arena with pack / reduce-scatter / all-gather / unpack (engine.py)
        self._arena = arena
        # grad_comm="bf16": fp32 grads cross the interconnect as bf16 (flat
        # arena only); opt-in, since the sum is then rounded to bf16 before Adam sees it
        self._grad_comm = grad_comm
        if grad_comm is not None and arena != "flat":
            raise ValueError("grad_comm='bf16' needs the flat arena")
        self.engine: ShardEngine | None = None
        self._step_tensors = {}
        self._validated = [None] * len(self.params)
        self._overlap = bool(overlap)
        self._overlap_hooks = []
        if self._overlap:
            # hooks must exist before the first backward: build the engine (and the communicator,
            # a collective call every rank makes here) now.  Flat arena: per-owner reduces of G
            # stretches from the hooks (flat.py); bucket arena: GradBuckets views (overlap.py)
            self._build_engine()
            gb = self.engine.enable_overlap(int(overlap_bucket_mb * (1 << 20)))
            self._overlap_hooks = gb.register_hooks()
        elif self._flat():
            # params become views of the arena now, so zero_grad() can hand out grad views
            # before the first step (every rank builds it: the communicator is a collective)
            self._build_engine()
            self._overlap_hooks = self.engine.register_marks()

    def _flat(self) -> bool:
        """The flat parameter arena: the reference layout (the drop-in), or the balanced Layout F
        ablation for ZeRO-2 (the ZeRO-1 carry is per whole parameter: bucket arena there)."""
        return self._arena == "flat" and (self._layout == "reference" or
                                          (self._layout == "flat" and not self._carry))

    def _shard_optimizer_params(self):
        """zero1.py:71-74: drop non-owned params from the inner optimizer's groups."""
        for group in self.optimizer.param_groups:
            group["params"] = [p for p in group["params"] if p in self.local_params]

    # ------------------------------------------------------------------------------------------
    def _build_engine(self):
        comm = self._comm
        if self.world_size > 1 and comm is None:
            from .comm import RcclComm
            comm = RcclComm()
            self._comm = comm
        # ws=1 owns every param, so zero_grad clears them all and there is no carry
        # (zero1.py:107-108): no buffer, no 0·A term
        carry = self._carry and self.world_size > 1
        if self._flat():
            from .flat import FlatEngine

            self.engine = FlatEngine(self.params, self._group_of, self.world_size, self.rank,
                                     carry=carry, comm=comm, bucket_bytes=self._bucket_bytes,
                                     master=self._master, grad_comm=self._grad_comm,
                                     layout=self._layout)
        else:
            self.engine = ShardEngine(self.params, self._group_of, self.world_size, self.rank,
                                      layout=self._layout, carry=carry, comm=comm,
                                      bucket_bytes=self._bucket_bytes, buckets=self._buckets,
                                      master=self._master)
        if self.engine.plan.layout != 0:
            return
        self._expose_state()

    def _expose_state(self):
        """optimizer.state[p] = {'step', 'exp_avg', 'exp_avg_sq'} as views of the flat shard."""
        eng = self.engine
        for i in eng.owned_param_indices():
            p = self.params[i]
            views = eng.state_views(i)
            if views is None:
                continue
            st = self.optimizer.state[p]
            st.update(views)
            if eng.vmax is not None:
                so = int(eng.pieces.stream_off[eng.pieces.param == i][0])
                st["max_exp_avg_sq"] = eng.vmax[so:so + p.numel()].view(p.shape)

    def _hparams_of(self, gi: int) -> dict:
        return adam_group_hparams(self._groups[gi], self.optimizer)

    def _update_step_state(self):
        eng = self.engine
        for i in eng.owned_param_indices():
            s = int(eng.steps[i])
            if s == 0:
                continue
            t = self._step_tensors.get(s)
            if t is None:
                self._step_tensors.clear()
                t = self._step_tensors[s] = torch.tensor(float(s), dtype=torch.float32)
            st = self.optimizer.state[self.params[i]]
            if st.get("step") is not t:
                st["step"] = t

    # ------------------------------------------------------------------------------------------
    @on_param_device
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        step_start = time.perf_counter()
        if self.engine is None:
            self._build_engine()
        had_vmax = self.engine.vmax is not None
        grads = [p.grad for p in self.params]
        seen = self._validated
        for i, (g, p) in enumerate(zip(grads, self.params)):
            # the same grad tensor as last step: already checked (a weak reference, so a grad the
            # step releases is not kept alive by the check)
            if g is None or (seen[i] is not None and seen[i]() is g):
                continue
            # (the flat arena copies a strided / expanded gradient into its slot through torch,
            # as torch's Adam would read it; the bucket arena packs raw runs: dense only)
            if g.dtype != p.dtype or g.shape != p.shape or not (g.is_contiguous() or self._flat()):
                raise ValueError("zero_amd: grads must match their param's dtype and shape (and "
                                 "be contiguous outside the flat arena)")
            seen[i] = weakref.ref(g)
        with torch.no_grad():
            self.engine.step(grads, self._hparams_of)
        if not had_vmax and self.engine.vmax is not None:
            self._expose_state()
        self._update_step_state()
        self._release_grads()
        if self._sync:
            torch.cuda.synchronize(self.engine.device)
            if self._variant != 1:  # zero1.py:67-68: ZeRO-1 never counts communication time
                self.communication_time += self.engine.comm_time_s()
            self.engine.release_retired()
        elif self.engine.n_retired() > 64:
            torch.cuda.synchronize(self.engine.device)
            self.engine.release_retired()
        self.step_time += time.perf_counter() - step_start
        return loss

    def _release_grads(self):
        # zero2.py:113 frees non-owned grads; the reduced grads live in the bucket arena, so
        # every grad is released (the next backward allocates fresh ones).  The flat arena keeps
        # every p.grad as its view of G (this rank's local gradient).
        if self._flat():
            return
        if self._overlap:
            self.engine.gb.release()
            return
        for p in self.params:
            p.grad = None

    @on_param_device
    def zero_grad(self, set_to_none: bool = True):
        if self._flat():
            # ZeRO-2 (and ZeRO-1 at ws = 1, which has no carry): None, as the reference's —
            # backward's fresh grads are then read in place (ws = 1) or landed in the arena;
            # ZeRO-1 at ws > 1: zeroed views of the grad arena (its carry follows the views)
            self.engine.zero_grad(set_to_none=set_to_none and not (self._carry and self.world_size > 1))
            return
        if self._overlap:  # grads become zeroed views of the overlap buckets (no pack copy)
            self.engine.gb.install_views()
            return
        for p in self.params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    # convenience --------------------------------------------------------------------------------
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    # checkpointing (zero_amd/checkpoint.py) -------------------------------------------------------
    def _ckpt_header(self):
        return ckpt.header(self._variant, self.world_size, self.rank, self.local_param_indices)

    def _ckpt_views(self, i: int) -> dict:
        """name -> live view of param i's flat state (the owned params of Layout R)."""
        eng = self.engine
        views = eng.state_views(i)
        if views is None:
            raise NotImplementedError("zero_amd: state_dict() needs the reference (whole-param) layout")
        if eng.vmax is not None:
            so = int(eng.pieces.stream_off[eng.pieces.param == i][0])
            views["max_exp_avg_sq"] = eng.vmax[so:so + self.params[i].numel()].view(self.params[i].shape)
        if eng.carry is not None:
            so = int(eng.pieces.stream_off[eng.pieces.param == i][0])
            views["zero1_carry"] = eng.carry[so:so + self.params[i].numel()].view(self.params[i].shape)
        return views

    @on_param_device
    def state_dict(self):
        """The inner optimizer's state dict in torch's format (indices over the owned parameters,
        as the reference's ``opt.optimizer.state_dict()``), every tensor a copy of the engine's
        flat state, plus the split master's residual / fp32 master and ZeRO-1's carry
        (zero_amd/checkpoint.py)."""
        torch.cuda.synchronize(self.params[0].device)  # the state of every enqueued step
        sd = Optimizer.state_dict(self.optimizer)
        index = {id(p): k for k, p in enumerate(ckpt.inner_params(self.optimizer))}
        state = {}
        if self.engine is not None:
            for i in self.engine.owned_param_indices():
                p = self.params[i]
                if id(p) not in index:
                    continue
                entry = {k: v.detach().clone() for k, v in self._ckpt_views(i).items()}
                entry["step"] = torch.tensor(float(self.engine.steps[i]), dtype=torch.float32)
                state[index[id(p)]] = entry
        sd["state"] = state
        sd["zero_amd"] = self._ckpt_header()
        return sd

    @on_param_device
    def load_state_dict(self, state_dict):
        """Restore a ``state_dict()`` of this rank (or a plain torch Adam state dict over the same
        owned parameters): hyper-parameters through torch's loader, state copied into the flat
        buffers.  Parameters are the model's (load them with the model's own state dict)."""
        ckpt.check_header(state_dict, self._ckpt_header())
        if self.engine is None:
            self._build_engine()
        eng = self.engine
        torch.cuda.synchronize(eng.device)
        ckpt.load_param_groups(self.optimizer, state_dict)
        self.original_param_groups = self.optimizer.param_groups
        self._groups = list(self.optimizer.param_groups)
        saved = state_dict.get("state", {})
        params = ckpt.inner_params(self.optimizer)
        if any("max_exp_avg_sq" in saved.get(k, {}) for k in range(len(params))) and eng.vmax is None:
            eng.ensure_vmax()
            if hasattr(eng, "rebuild_rows"):
                eng.rebuild_rows()
        index = {id(p): k for k, p in enumerate(params)}
        with torch.no_grad():
            for i in eng.owned_param_indices():
                p = self.params[i]
                entry = saved.get(index.get(id(p), -1), {})
                views = self._ckpt_views(i)
                for name, view in views.items():
                    src = entry.get(name)
                    if src is not None:
                        view.copy_(src.reshape(view.shape))
                    elif name == "master_residual":  # master = the bf16 param exactly
                        view.zero_()
                    elif name == "master_param":
                        view.copy_(p.detach().reshape(view.shape))
                    else:  # no state: torch's fresh Adam (moments 0), no carry
                        view.zero_()
                eng.steps[i] = ckpt.step_of(entry)
        self.optimizer.state.clear()
        self._expose_state()
        self._update_step_state()
        ckpt.bind_inner_load(self)

    def __repr__(self):
        return (f"{type(self).__name__}(zero={self._variant}, ws={self.world_size}, rank={self.rank}, "
                f"owned={self.local_param_indices[:1]}..{self.local_param_indices[-1:]})")


CALIBRATION_BYTES = 256 << 20  # gradient bytes per calibration exchange (capped by the model's)


def _owner_bytes(opt) -> list:
    """Gradient bytes each rank owns under the reference's index ranges (zero1.py:55-62)."""
    ws, n = opt.world_size, len(opt.params)
    ppr, rem = n // ws, n % ws
    out = []
    for r in range(ws):
        a = r * ppr + min(r, rem)
        b = a + ppr + (1 if r < rem else 0)
        out.append(sum(p.numel() * p.element_size() for p in opt.params[a:b]))
    return out


def calibrate_arena(opt, iters: int = 3) -> dict:
    """``arena="auto"``: time both exchanges on this job's interconnect, at construction.

    A ``CALIBRATION_BYTES`` sample of the gradient (the model's own size if smaller) is exchanged
    the flat arena's way — one RCCL group of per-owner reduces then one of per-owner broadcasts,
    windows in proportion to what each rank owns (uneven under the reference's index ranges) — and
    the bucket arena's way — equal-chunk reduce-scatter then all-gather, plus the pack and unpack
    copies it needs (two copies of the sample through the gfx950 copy kernel) — each ``iters``
    times after one warm-up, on the collective stream.  Rank 0's times decide (a collective
    finishes on every rank together) and its choice is broadcast, so every rank builds the same
    arena.  Per-step estimates scale the sample to the model's gradient bytes; the bucket arena is
    chosen only when it is at least 5 % faster (no overlap credit to either side)."""
    import numpy as np

    from .comm import RcclComm, comm_stream
    from .kernels import CopySet

    if opt._comm is None:
        opt._comm = RcclComm()
    comm, ws = opt._comm, opt.world_size
    p0 = opt.params[0]
    dev, dt = p0.device, p0.dtype
    es = p0.element_size()
    total = sum(p.numel() for p in opt.params) * es
    align = ws * 64
    n = max(align, min(total, CALIBRATION_BYTES) // es // align * align)  # elements in the sample
    own = np.asarray(_owner_bytes(opt), np.float64)
    share = own / own.sum() if own.sum() > 0 else np.full(ws, 1.0 / ws)
    win_len = np.floor(share * n).astype(np.int64)
    win_len[-1] += n - int(win_len.sum())
    win_off = np.concatenate([[0], np.cumsum(win_len)[:-1]]).astype(np.int64)
    stream = comm_stream(dev)
    buf = torch.zeros(n, dtype=dt, device=dev)
    chunk = torch.zeros(n // ws, dtype=dt, device=dev)
    scratch = torch.empty_like(buf)
    nb = n * es
    copy = CopySet([buf.data_ptr()], [scratch.data_ptr()], [nb])

    def flat():
        comm.reduce_v(buf, win_off, win_len, stream)
        comm.broadcast_v(buf, win_off, win_len, stream)

    def buckets():
        copy.run(stream)  # pack
        comm.reduce_scatter(buf, chunk, stream)
        comm.all_gather(chunk, buf, stream)
        copy.run(stream)  # unpack

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(iters):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / iters

    torch.cuda.synchronize(dev)
    t_flat, t_buck = timed(flat), timed(buckets)
    scale = total / nb
    est = {"flat": t_flat * scale, "buckets": t_buck * scale}
    chosen = "buckets" if est["buckets"] < 0.95 * est["flat"] else "flat"
    obj = [chosen]
    dist.broadcast_object_list(obj, src=0)
    del buf, chunk, scratch, copy
    return {"chosen": obj[0], "sample_bytes": nb, "grad_bytes": total,
            "sample_ms": {"flat": t_flat, "buckets": t_buck},
            "est_ms_per_step": est, "decided_by": "rank 0"}


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()
