"""The flat-parameter-arena ZeRO-1/2 step: no pack, no unpack.

``ShardEngine``'s bucket path copies every gradient into a rank-major bucket arena (pack), runs
the collectives there and copies every parameter back (unpack): at the ws=8 SmolLM3-3B layout
those copies were 24.6 GB of HBM traffic per step, more than the Adam update itself
(profiles/r01_c4_sim8_diagnostic.json).  They exist only because parameters and gradients live
outside the arena.  ``FlatEngine`` moves them in:

* **P** — every parameter is a view of one flat buffer (``param.data`` re-pointed once, at
  construction, like an FSDP flat parameter), laid out *owner-major*: the reference's ownership
  assigns rank r the contiguous index range [start_r, end_r) (zero1.py:55-62), so rank r's
  parameters — its optimizer shard, its *stream* — are one contiguous region of P, each slot
  64-element aligned;
* **G** — the gradients, the same layout; a fresh gradient from backward is copied into its slot
  and ``p.grad`` becomes the slot's view (ZeRO-2's ``zero_grad()`` sets grads to None, as the
  reference's does); ZeRO-1's ``zero_grad()`` zeroes G and makes every ``p.grad`` a view of its
  slot, so backward accumulates straight into it (the carry needs the views to persist);
* **R** — this rank's reduced gradient, one stream long.

A step is cut into *rounds*; round j is window j (``W`` elements) of every owner's stream.  Per
round: one RCCL group of ``ncclReduce`` — owner r's window of G, summed over ranks, into R on r
(the reduce-scatter-v, zero2.py:94-113) — the fused Adam on the own window (reads R and the
master, writes the updated bf16 / fp32 parameter straight into P), and one RCCL group of in-place
``ncclBroadcast`` of every owner's window of P (the all-gather-v, zero2.py:122-133).  In a group
each rank is the root of one transfer and forwards the others', so the bus bytes per rank are
those of a ring reduce-scatter / all-gather of the round.  The reduce is out of place, so G still
holds this rank's local gradients after the step.

ZeRO-1's gradient carry (zero1.py:107-108) follows the grads the caller left:
the reference's non-owners keep last step's averaged gradient A_{t-1} in ``p.grad`` unless the
caller clears it.  Here A_{t-1} lives in the owner's carry buffer, and the owner weights it by
(ws-1) when ``p.grad`` at step() is still the arena view (cleared only by ``opt.zero_grad()``,
which in the reference clears owned grads only) and by 0 when the caller replaced the grad (e.g.
``model.zero_grad()`` → None → a fresh tensor from backward), per parameter, on the assumption
that every rank treats its grads alike.  Zeroing a view in place
(``model.zero_grad(set_to_none=False)``) cannot be told apart from ``opt.zero_grad()``.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._hooks import WeakCall
from .comm import StreamEvent
from .engine import ALIGN_ELEMS, ShardEngine, _ptr
from .kernels import check_extents, check_extents_enabled, copy_direct

_I32P = np.int32
LAND_BATCH_BYTES = 64 << 20  # fresh gradients landed per hook batch (ws > 1, no overlap)


class _Round:
    """Round j: per owner the window [lo, hi) of its stream and the device pointers of its
    reduce / broadcast; this rank's Adam rows for the window."""

    def __init__(self, j, send, recv, count, bcast, rows, idx):
        self.j = j
        self.send = np.ascontiguousarray(send, np.uint64)
        self.recv = np.ascontiguousarray(recv, np.uint64)
        self.count = np.ascontiguousarray(count, np.int64)
        self.root = np.ascontiguousarray(np.arange(len(count)), _I32P)
        self.bcast = np.ascontiguousarray(bcast, np.uint64)
        self.rows = rows
        self.idx = idx


class FlatEngine(ShardEngine):
    """``layout``: "reference" (Layout R, the reference's whole-parameter ownership, zero1.py:55-62
    — the drop-in's) or "flat" (Layout F, the ablation: balanced contiguous 1/ws slices of the
    aligned concatenation, so a parameter may straddle two owners; ZeRO-2 only, no overlap).
    Either way rank r's stream is one contiguous region of P (Layout F: P is the aligned
    concatenation itself, rank r's slice at r·S), so the rounds, the Adam rows and the grouped
    reduce / broadcast are the same code."""

    def __init__(self, params, group_of, ws: int, rank: int, *, carry=False, comm=None,
                 bucket_bytes: int = 256 << 20, master: str = "split", placement_tries: int = 8,
                 grad_comm: str | None = None, layout: str = "reference"):
        if layout not in ("reference", "flat"):
            raise ValueError(f"the flat arena takes layout 'reference' or 'flat' (got {layout!r})")
        if layout == "flat" and carry:
            raise ValueError("layout='flat' in the flat arena is ZeRO-2 only (the ZeRO-1 carry is "
                             "per whole parameter)")
        # the base class gives the layout's streams, the optimizer state and the Adam launch
        # machinery; its bucket plan (one bucket) is unused
        super().__init__(params, group_of, ws, rank, layout=layout, carry=carry, comm=comm,
                         bucket_bytes=1 << 62, buckets="ragged", placement_tries=placement_tries,
                         master=master)
        self.arena_kind = "flat"
        self.layout = layout
        plan, es, dev, dt = self.plan, self.es, self.device, self.dtype
        n = len(self.params)
        self.Ls = np.array([plan.stream_len(r) for r in range(ws)], np.int64)
        self.base = np.concatenate([[0], np.cumsum(self.Ls)[:-1]]).astype(np.int64)
        self.slot = np.zeros(n, np.int64)
        self.numel = np.array([p.numel() for p in self.params], np.int64)
        owner = np.zeros(n, np.int64)  # (Layout F: the rank holding the parameter's first element)
        for r in range(ws):
            pc = plan.pieces(r)
            first = pc.param_off == 0  # Layout R: every piece is a whole parameter
            self.slot[pc.param[first]] = self.base[r] + pc.stream_off[first]
            owner[pc.param[first]] = r
        if layout == "flat":  # every parameter one contiguous run of P (its pieces abut)
            for r in range(ws):
                pc = plan.pieces(r)
                assert np.array_equal(self.base[r] + pc.stream_off, self.slot[pc.param] + pc.param_off)
        self.owner = owner
        self.owned = np.zeros(n, bool)  # this rank updates (part of) the parameter
        self.owned[self.pieces.param[self.pieces.length > 0]] = True
        total = int(max(self.Ls.sum(), ALIGN_ELEMS))
        self.P, self.arena_placement = _zeros_placed(total, dt, dev, placement_tries)
        with torch.no_grad():
            for i, p in enumerate(self.params):
                s = int(self.slot[i])
                self.P[s:s + int(self.numel[i])].copy_(p.detach().reshape(-1))
                p.data = self.P[s:s + int(self.numel[i])].view(p.shape)
        # bf16 gradient exchange for fp32 parameters: G is converted into Gc
        # (bf16, same layout) before the reduces, which then move and sum 2 B per element; Adam
        # reads the bf16 sum (its fp32 master is the fp32 parameter itself)
        if grad_comm not in (None, "bf16"):
            raise ValueError(f"grad_comm must be None or 'bf16' (got {grad_comm!r})")
        self.grad_comm = grad_comm if dt == torch.float32 else None
        if grad_comm == "bf16" and dt != torch.float32:
            raise ValueError("grad_comm='bf16' is for fp32 parameters (bf16 grads already are)")
        # ws == 1 (no bf16 exchange): nothing to reduce, so Adam reads every gradient where it is —
        # the arena view, or the fresh tensor backward left after a set-to-None zero_grad(), in
        # place (zero2.py:120 reads p.grad as backward left it): no landing copy, and G exists
        # only once a caller asks for grad views (zero_grad(set_to_none=False), ZeRO-1's views)
        self.inplace = ws == 1 and self.grad_comm is None
        self.G, self.grad_placement = None, None
        self._total = total
        if not self.inplace:
            self._ensure_G()
        cdt = torch.bfloat16 if self.grad_comm else dt
        self.Gc = torch.zeros(total, dtype=cdt, device=dev) if self.grad_comm else self.G
        self.ces = torch.empty((), dtype=cdt).element_size()
        self.czdtype = _lib.ZS_BF16 if self.grad_comm else self.zdtype
        # ws == 1 with the bf16 exchange: Adam reads Gc (R aliases it), one round, no collective
        self.reduced_placement = None
        if ws == 1:
            self.R = self.Gc
        else:  # Adam streams R every step: placed by probe as well
            self.R, self.reduced_placement = _zeros_placed(max(int(self.Ls[rank]), ALIGN_ELEMS), cdt,
                                                           dev, placement_tries)
        self.dirty = np.zeros(n, bool)  # G slot may hold a stale gradient
        self.zero_grad_calls = 0
        W = max(ALIGN_ELEMS, (int(bucket_bytes) // (ws * es)) // ALIGN_ELEMS * ALIGN_ELEMS)
        if ws == 1:
            W = total
        self.W = W
        self.K = max(1, -(-int(self.Ls.max()) // W))
        self.rounds = [self._make_round(j) for j in range(self.K)]
        self._views = [None] * n  # the grad views handed out (identity = "still the view")
        # cross-stream ordering points (comm.StreamEvent: stream flags unless ZERO_AMD_STREAM_SYNC)
        mk = lambda: [StreamEvent() for _ in range(self.K)]  # noqa: E731
        self.ev_red, self.ev_adam, self.ev_bc = mk(), mk(), mk()
        self.ev_grads = StreamEvent()
        self.ev_c0 = torch.cuda.Event(enable_timing=True)
        self.ev_c1 = torch.cuda.Event(enable_timing=True)
        self.capture_reduced = None  # optional tensor: a copy of R after the reduces (checks)
        # which parameters backward touched since zero_grad() (post-accumulate-grad hooks): a view
        # nobody accumulated into is NO gradient (the reference's p.grad is None after zero_grad),
        # unless no backward ran at all (grads written into the views by hand)
        self.touched = np.zeros(n, bool)
        self.any_touched = False
        self._mark_hooks = []
        # parameters carrying this engine's post-accumulate-grad hook; requires_grad can change
        # after construction (gradual unfreezing), so the set is refreshed (_refresh_requires_grad)
        self.hooked = np.zeros(n, bool)
        # a fresh gradient backward hands over (p.grad was None) becomes its arena view in the
        # post-accumulate hook — except under ZeRO-1's carry, which reads "the caller replaced the
        # view" from p.grad at step() (the module docstring)
        self.adopt_fresh = self.carry is None
        self.overlap = False  # backward-overlapped reduces (enable_overlap)
        self.ov_K = 0
        self.launched_in_backward = 0
        # ws > 1 without overlap: fresh gradients are landed from the post-accumulate hooks in
        # batches of about this many bytes (and adopted), so backward never holds G plus a full
        # set of fresh gradients (the reference holds one set)
        self.land_batch_bytes = LAND_BATCH_BYTES
        self.land_pending, self.land_pending_bytes = [], 0
        self.land_marked = np.zeros(n, bool)
        self.inplace_reads = 0  # gradients the last step's Adam read in place (ws == 1)

    # ------------------------------------------------------------------------------------------
    def _ensure_G(self):
        """The gradient arena (placed by probe), allocated at construction when ws > 1 and on first
        use at ws == 1 (grad views handed out, or a gradient Adam cannot read in place)."""
        if self.G is None:
            self.G, self.grad_placement = _zeros_placed(self._total, self.dtype, self.device,
                                                        self.placement_tries)
            if getattr(self, "grad_comm", None) is None and hasattr(self, "Gc"):
                self.Gc = self.G
                if self.ws == 1:
                    self.R = self.G
        return self.G

    # ------------------------------------------------------------------------------------------
    def _make_round(self, j: int) -> _Round:
        ws, es, W, r0 = self.ws, self.es, self.W, self.rank
        lo = j * W
        count = np.clip(self.Ls - lo, 0, W)
        pb = self.P.data_ptr()
        # in place (ws == 1): the rows' gradients are bound per step (AdamSet.set_grads); 0 here
        gb = rb = 0 if self.inplace else None
        if gb is None:
            gb, rb = self.Gc.data_ptr(), self.R.data_ptr()
        ces = self.ces  # element size on the wire (bf16 exchange of fp32 grads: 2)
        send = np.uint64(gb) + ((self.base + lo) * ces).astype(np.uint64)
        recv = send.copy()
        recv[r0] = np.uint64(rb + lo * ces)
        bcast = np.uint64(pb) + ((self.base + lo) * es).astype(np.uint64)
        # this rank's Adam rows: its pieces clipped to [lo, lo + count[rank])
        pc = self.pieces
        hi = lo + int(count[r0])
        a = np.maximum(pc.stream_off, lo)
        b = np.minimum(pc.stream_off + pc.length, hi)
        keep = b > a
        idx, a, b = pc.param[keep], a[keep], b[keep]
        so = a.astype(np.int64)
        ln = (b - a).astype(np.int64)
        g = np.zeros(len(so), np.uint64) if self.inplace else np.uint64(rb) + (so * ces).astype(np.uint64)
        pslot = np.uint64(pb) + ((self.base[r0] + so) * es).astype(np.uint64)
        if self.mixed:  # master from P (split: + residual) or the fp32 master; bf16 param out to P
            rows = self._mixed_rows(idx, g, pslot, pslot, so, ln)
        else:  # fp32: P is the master, updated in place
            rows = self._adam_rows(idx, g, pslot, pslot, 0, so, ln)
        return _Round(j, send, recv, count, bcast, rows, idx)

    def slot_view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        s, n = int(self.slot[i]), int(self.numel[i])
        return buf[s:s + n].view(self.params[i].shape)

    def grad_view(self, i: int) -> torch.Tensor:
        return self.slot_view(self._ensure_G(), i)

    def grad_slot_ptrs(self, idx) -> np.ndarray:
        """Device addresses of the G slots of parameters ``idx``."""
        idx = np.asarray(idx, np.int64)
        return np.uint64(self._ensure_G().data_ptr()) + (self.slot[idx] * self.es).astype(np.uint64)

    def is_view(self, i: int, g) -> bool:
        if g is None or self.G is None:
            return False
        if g is self._views[i]:
            return True
        return (g.data_ptr() == self.G.data_ptr() + int(self.slot[i]) * self.es
                and g.shape == self.params[i].shape and g.is_contiguous())

    def install_views(self):
        for i, p in enumerate(self.params):
            if not self.is_view(i, p.grad):
                p.grad = self.grad_view(i)
            self._views[i] = p.grad

    def zero_grad(self, set_to_none: bool = False):
        """The wrapper's zero_grad().  ``set_to_none`` (ZeRO-2): every p.grad becomes None, as the
        reference's zero_grad leaves them (zero2.py:113 + the inner optimizer's zero_grad), and G
        keeps its stale values (``dirty``): backward then hands over fresh gradients.  At ws == 1
        Adam reads them in place (no copy at all); at ws > 1 they are copied into their slots and
        p.grad becomes the slot's view — from the post-accumulate hooks, per overlap bucket in
        overlap mode and in batches of ``land_batch_bytes`` otherwise — 4 B per bf16 element,
        where zeroing G and accumulating into its views costs 8 (a memset plus an in-place add).
        Otherwise (ZeRO-1 at ws > 1, whose carry needs the views to survive, or
        ``set_to_none=False``): G is zeroed and every p.grad made its arena view."""
        if set_to_none:
            for i, p in enumerate(self.params):
                p.grad = None
                self._views[i] = None
        else:
            self._ensure_G().zero_()
            self.dirty[:] = False
            self.install_views()
        self.land_pending, self.land_pending_bytes = [], 0
        self.land_marked[:] = False
        self.zero_grad_calls += 1
        self.touched[:] = False
        self.any_touched = False
        if self.overlap:
            self._ov_reset()

    def rebuild_rows(self):
        """Adam rows again (after the amsgrad buffer appeared)."""
        self.rounds = [self._make_round(j) for j in range(self.K)]

    def _static_sets(self, rd: _Round):
        """The round's Adam sets when every owned param has a grad, one per param group (the
        common case: built once, the rows never change because every pointer is the arena's)."""
        sets = getattr(rd, "sets", None)
        if sets is None:
            from .kernels import AdamSet

            groups = np.asarray(self.group_of)[rd.idx]
            sets = []
            for gi in np.unique(groups):
                sel = np.nonzero(groups == gi)[0]
                sets.append((int(gi), rd.idx[sel], AdamSet(np.ascontiguousarray(rd.rows[sel]),
                                                           self.czdtype, self.p_dtype)))
            rd.sets = sets
        return sets

    def _adam_round_fast(self, rd: _Round, hps, stream, gptr=None) -> bool:
        """Launch the round's static sets if every param in them shares its group's (step,
        carry) key this step; returns False to fall back to the general partitioning.  ``gptr``
        (in place, ws == 1): every parameter's gradient address, bound into the sets first."""
        sets = self._static_sets(rd)
        for gi, idx, aset in sets:
            hp = hps.get(gi)
            if hp is None:
                return False
        for gi, idx, aset in sets:
            if gptr is not None:
                aset.set_grads(gptr[idx], stream)
            if self.timing_events is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                aset.run(hps[gi], stream)
                e1.record(stream)
                self.timing_events.append((e0, e1, aset.bytes))
            else:
                aset.run(hps[gi], stream)
            self.last_adam_bytes += aset.bytes
        return True

    # ------------------------------------------------------------------------------------------
    def _reduce_round(self, rd: _Round, cs):
        comm = self.comm
        if hasattr(comm, "reduce_group"):
            comm.reduce_group(rd.send, rd.recv, rd.count, rd.root, self.czdtype, cs)
            return
        with _group(comm):  # tensor-level fallback (test communicators)
            for r in range(self.ws):
                c = int(rd.count[r])
                if c == 0:
                    continue
                s0 = int(self.base[r]) + rd.j * self.W
                src = self.Gc[s0:s0 + c]
                dst = self.R[rd.j * self.W:rd.j * self.W + c] if r == self.rank else src
                comm.reduce_out(src, dst, r, cs)

    def _bcast_round(self, rd: _Round, cs):
        comm = self.comm
        if hasattr(comm, "broadcast_group"):
            comm.broadcast_group(rd.bcast, rd.count, rd.root, self.zdtype, cs)
            return
        with _group(comm):
            for r in range(self.ws):
                c = int(rd.count[r])
                if c:
                    s0 = int(self.base[r]) + rd.j * self.W
                    comm.broadcast(self.P[s0:s0 + c], r, cs)

    def register_marks(self):
        """Post-accumulate-grad hooks that only record which parameters backward reached."""
        self._mark_hooks = []
        self._hook_new(self._requires_grad())
        return self._mark_hooks

    def _mark(self, i: int):
        self.touched[i] = True
        self.any_touched = True
        if self.inplace or not self.adopt_fresh:
            return  # ws == 1 reads fresh grads in place; ZeRO-1's carry needs the caller's tensors
        g = self.params[i].grad
        if g is not None and not self.is_view(i, g) and not self.land_marked[i]:  # fresh: land
            self.land_marked[i] = True  # with the next batch (once, however often accumulated)
            self.land_pending.append(i)
            self.land_pending_bytes += g.numel() * g.element_size()
            if self.land_pending_bytes >= self.land_batch_bytes:
                self._land_pending()

    def _land_pending(self, stream=None):
        """Copy the fresh gradients the hooks collected into their G slots (one zs_copy_direct on
        the stream backward produced them on) and make the slots their p.grad: the fresh tensors
        return to the allocator, stream-ordered after the copy."""
        idx = self.land_pending
        if not idx:
            return
        self.land_pending, self.land_pending_bytes = [], 0
        self.land_marked[idx] = False
        cur = torch.cuda.current_stream(self.device) if stream is None else stream
        live = [i for i in idx if self.params[i].grad is not None
                and not self.is_view(i, self.params[i].grad)]
        self._land(live, [self.params[i].grad for i in live], (), cur, adopt=True)

    def _land(self, idx, grads, zero, stream, adopt: bool):
        """Fresh gradients ``grads`` of parameters ``idx`` (not arena views: zero_grad set p.grad
        to None, or the caller assigned them) copied into their G slots, and the slots of ``zero``
        zero-filled — ONE zs_copy_direct on ``stream`` (the segments travel in the kernel
        arguments: nothing to upload for pointers that change every step).  ``adopt``: p.grad
        becomes the slot's view, so the fresh tensor returns to the allocator now (stream-ordered
        after the copy that reads it)."""
        idx = np.asarray(idx, np.int64)
        zero = np.asarray(zero, np.int64)
        if not len(idx) and not len(zero):
            return
        # the copy kernel reads numel * es contiguous bytes: anything else (strided, another dtype)
        # goes through torch's copy into the view
        dense = np.fromiter((g.is_contiguous() and g.dtype == self.dtype
                             and g.numel() == int(self.numel[i]) for i, g in zip(idx, grads)),
                            bool, len(idx))
        if not dense.all():
            for i, g in zip(idx[~dense], [g for g, d in zip(grads, dense) if not d]):
                self.grad_view(int(i)).copy_(g.reshape(self.params[i].shape))
            grads = [g for g, d in zip(grads, dense) if d]
            slow, idx = idx[~dense], idx[dense]
        else:
            slow = idx[:0]
        all_idx = np.concatenate([idx, zero])
        src = np.concatenate([np.fromiter((_ptr(g) for g in grads), np.uint64, len(idx)),
                              np.zeros(len(zero), np.uint64)])
        dst = self.grad_slot_ptrs(all_idx)
        nbytes = self.numel[all_idx] * self.es
        if check_extents_enabled():  # every segment inside its tensors (tests turn this on)
            check_extents(src[:len(idx)], nbytes[:len(idx)], grads, "grad")
            check_extents(dst, nbytes, [self.G], "G slot")
        copy_direct(src, dst, nbytes, stream)
        if adopt:
            for i in np.concatenate([idx, slow]):
                v = self.grad_view(int(i))
                self.params[i].grad = v
                self._views[i] = v

    def _requires_grad(self) -> np.ndarray:
        return np.fromiter((p.requires_grad for p in self.params), bool, len(self.params))

    def _hook_new(self, req: np.ndarray):
        """Hook every parameter that requires grad and has no hook of this engine yet."""
        name = "_ov_ready" if self.overlap else "_mark"
        for i in np.nonzero(req & ~self.hooked)[0]:
            i = int(i)
            # the engine is reached weakly: a strong closure would be a cycle through the
            # parameter's C++-held hook dict that the garbage collector cannot see (_hooks.py)
            self._mark_hooks.append(self.params[i].register_post_accumulate_grad_hook(
                WeakCall(self, name, i)))
            self.hooked[i] = True

    # ------------------------------------------------------------------------------------------
    # Backward overlap on the flat arena
    def enable_overlap(self, bucket_bytes: int):
        """Reduce gradients while backward runs: parameters grouped in reverse index order (the
        order a sequential model's backward produces them) into buckets of at most
        ``bucket_bytes`` that never mix owners, so a bucket is one contiguous stretch of its
        owner's stream in G (and in the owner's R).  A post-accumulate-grad hook counts a bucket's
        gradients; a complete bucket whose predecessors have been launched is reduced to its owner
        at once — one RCCL reduce on the comm stream behind an event on the stream that produced
        the gradient — strictly in bucket order, so every rank issues the same sequence.  step()
        reduces what backward left, runs Adam as soon as this rank's own buckets have arrived,
        and broadcasts in rounds as without overlap: no unpack, the parameters are the arena."""
        from .overlap import plan_grad_buckets

        if self.layout != "reference":
            raise ValueError("backward overlap needs the reference (owner-by-index) layout")
        groups, keys, *_ = plan_grad_buckets(self.numel.tolist(), self.owner.tolist(),
                                             int(bucket_bytes), self.ces, align=ALIGN_ELEMS)
        n = len(self.params)
        self.ov_groups = groups
        self.ov_K = len(groups)
        self.ov_owner = np.asarray(keys, np.int64)
        self.ov_lo = np.array([int(self.slot[g].min()) for g in groups], np.int64)
        self.ov_hi = np.array([int((self.slot[g] + self.numel[g]).max()) for g in groups], np.int64)
        self.ov_bucket_of = np.zeros(n, np.int64)
        for k, g in enumerate(groups):
            self.ov_bucket_of[g] = k
        # only parameters that can receive a gradient are waited for (a frozen one never fires);
        # re-counted at the first hook of a backward if requires_grad changed since
        self.ov_req = self._requires_grad()
        self.ov_size = np.array([int(self.ov_req[g].sum()) for g in groups], np.int64)
        self.ov_ev = [StreamEvent() for _ in range(self.ov_K)]
        self.ov_ev_ready = [StreamEvent() for _ in range(self.ov_K)]  # recorded where backward ran
        own = np.nonzero(self.ov_owner == self.rank)[0]
        self.ov_last_own = int(own[-1]) if len(own) else -1
        self.overlap = True
        self._ov_reset()
        return self

    def register_hooks(self):
        self._mark_hooks = []
        self._hook_new(self.ov_req)
        return self._mark_hooks

    def _ov_reset(self):
        self.ov_fresh = [[] for _ in range(self.ov_K)]  # per bucket: fresh grads to land
        self.ov_pending = self.ov_size.copy()
        self.ov_marked = np.zeros(len(self.params), bool)
        self.ov_next = 0
        self.ov_launched = 0
        self.ov_first = True

    def _ov_refresh(self):
        """First hook of a backward: if requires_grad changed since the buckets were counted, hook
        the newly trainable parameters and re-count what each bucket waits for — before any
        bucket of this backward is launched.  A newly frozen parameter's bucket no longer waits
        for it; a newly trainable one whose gradient was accumulated before this first hook is
        counted but never fires, so its bucket is reduced at step() (correct, not overlapped)."""
        req = self._requires_grad()
        if (req == self.ov_req).all():
            return
        new = req & ~self.hooked
        self._hook_new(req)
        # a newly trainable parameter may have been accumulated before its hook existed: it
        # counts as reached this backward (its view holds whatever backward put there)
        self.touched |= new
        self.any_touched = True
        self.ov_req = req
        self.ov_size = np.array([int(req[g].sum()) for g in self.ov_groups], np.int64)
        self.ov_pending = self.ov_size.copy()

    def _ov_ready(self, i: int):
        if self.ov_first:
            self.ov_first = False
            self._ov_refresh()
        if self.ov_marked[i]:
            raise RuntimeError(
                "zero_amd: gradient of parameter %d accumulated twice before step(); the "
                "backward-overlapped mode reduces each gradient once per step" % i)
        self.ov_marked[i] = True
        self.touched[i] = True
        self.any_touched = True
        g = self.params[i].grad
        # fresh (zero_grad set it to None): landed with its bucket, one copy launch (ws == 1: read
        # in place by step())
        if g is not None and not self.inplace and not self.is_view(i, g):
            self.ov_fresh[self.ov_bucket_of[i]].append(i)
        self.ov_pending[self.ov_bucket_of[i]] -= 1
        while self.ov_next < self.ov_K and self.ov_pending[self.ov_next] == 0:
            self._ov_launch(self.ov_next)
            self.ov_launched += 1
            self.ov_next += 1

    def _ov_launch(self, k: int, stream=None):
        cur = torch.cuda.current_stream(self.device) if stream is None else stream
        lo, hi, r = int(self.ov_lo[k]), int(self.ov_hi[k]), int(self.ov_owner[k])
        fresh = self.ov_fresh[k]
        if fresh:  # ZeRO-2 adopts the slots as p.grad; ZeRO-1's carry needs the caller's tensors
            self._land(fresh, [self.params[i].grad for i in fresh], (), cur, self.adopt_fresh)
            self.ov_fresh[k] = []
        if self.grad_comm:  # the bucket's grads as bf16 for the wire (gfx950 RNE kernel)
            from .kernels import convert

            convert(self.G[lo:hi], self.Gc[lo:hi], cur)
        if self.ws == 1:  # nothing to exchange: Adam reads Gc (= G unless converted)
            self.ov_ev[k].record(cur)
            return
        ev = self.ov_ev_ready[k]
        ev.record(cur)
        cs = self.comm_stream
        cs.wait_event(ev)
        e0 = self._timed_start(cs)
        b = int(self.base[r])
        if hasattr(self.comm, "reduce_group"):
            ces = self.ces
            send = np.array([self.Gc.data_ptr() + lo * ces], np.uint64)
            recv = np.array([self.R.data_ptr() + (lo - b) * ces], np.uint64) if r == self.rank else send
            self.comm.reduce_group(send, recv, np.array([hi - lo], np.int64),
                                   np.array([r], np.int32), self.czdtype, cs)
        else:  # tensor-level communicators (tests)
            src = self.Gc[lo:hi]
            self.comm.reduce_out(src, self.R[lo - b:hi - b] if r == self.rank else src, r, cs)
        self.ov_ev[k].record(cs)
        if e0 is not None:  # bus bytes of a reduce of S bytes to one root: S per rank
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(cs)
            self.comm_events.append(("rs", "flat-overlap", e0, e1, (hi - lo) * self.ces))

    def _step_overlap(self, grads, has, view, cmul, hps, hparams_of, stream):
        """step() after a backward-overlapped backward: flush, Adam, broadcast rounds."""
        n = len(self.params)
        es = self.es
        marked = self.ov_marked
        # grads assigned by hand (no hook fired) are copied in; a stale slot without a grad this
        # step is zero-filled — only in buckets not launched yet (a launched bucket is complete)
        copy = np.nonzero(has & ~view & ~marked)[0]
        zero = np.nonzero(~has & self.dirty & ~marked)[0]
        self._land(copy, [grads[i] for i in copy], zero, stream, adopt=False)
        self.dirty = has.copy()
        with _lib.phase_range("all_reduce_gradients"):  # what backward did not reduce
            while self.ov_next < self.ov_K:
                self._ov_launch(self.ov_next, stream)
                self.ov_next += 1
        self.launched_in_backward = self.ov_launched
        if self.ws > 1:
            self.ev_c1.record(self.comm_stream)
        if self.ov_last_own >= 0:  # Adam needs this rank's own buckets only
            stream.wait_event(self.ov_ev[self.ov_last_own])
        if self.capture_reduced is not None:
            self.capture_reduced.copy_(self.R[:self.capture_reduced.numel()])
        with _lib.phase_range("optimizer_step"):  # zero1.py:88
            for rd in self.rounds:
                if len(rd.idx) and not (hps and self._adam_round_fast(rd, hps, stream)):
                    live = has[rd.idx]
                    rows, idx = (rd.rows, rd.idx) if live.all() else (rd.rows[live], rd.idx[live])
                    self._run_adam(("flat", rd.j), rows, idx, hparams_of, stream,
                                   carry_mul=cmul[idx])
                self.ev_adam[rd.j].record(stream)
        if self.ws > 1:
            cs = self.comm_stream
            with _lib.phase_range("broadcast_parameters"):  # zero1.py:91-102
                for rd in self.rounds:
                    cs.wait_event(self.ev_adam[rd.j])
                    e0 = self._timed_start(cs)
                    self._bcast_round(rd, cs)
                    self.ev_bc[rd.j].record(cs)
                    self._timed_end(e0, cs, "ag", int(rd.count.sum()))
            stream.wait_event(self.ev_bc[self.K - 1])
        self._reinstall(has, view)
        self._ov_reset()

    def step(self, grads, hparams_of, stream=None):
        stream = torch.cuda.current_stream(self.device) if stream is None else stream
        n = len(self.params)
        es = self.es
        if self.land_pending:  # the hooks' last partial batch (ws > 1): land it, grads become views
            pend = list(self.land_pending)
            self._land_pending(stream)
            grads = list(grads)
            for i in pend:
                grads[i] = self.params[i].grad
        vw = self._views
        view = np.fromiter((g is not None and (g is vw[i] or self.is_view(i, g))
                            for i, g in enumerate(grads)), bool, n)
        has = np.fromiter((g is not None for g in grads), bool, n)
        req = self._requires_grad()
        if self.any_touched:  # a backward ran: an arena view it did not reach carries no gradient
            # (parameters without this engine's hook — trainable only since the last step — count
            # when they require grad; they are hooked below for the next backward)
            has &= ~view | self.touched | (~self.hooked & req)
        if (req & ~self.hooked).any() and not self.overlap:
            self._hook_new(req)
        if any(hparams_of(g)["amsgrad"] for g in set(self.group_of)) and self.vmax is None:
            self.ensure_vmax()
            self.rebuild_rows()
        self.ev_c0.record(stream)
        gptr = None
        if self.inplace:  # ws == 1: every gradient read where it is (the odd one landed first)
            gptr = self._bind_inplace(grads, has, view, stream)
        elif not self.overlap:
            # gradients not accumulated into the arena (assigned tensors, fresh grads the hooks
            # did not land) are copied in; a stale slot whose grad is gone is zero-filled
            # (overlap mode: in _step_overlap, for the parameters no hook has handled)
            copy = np.nonzero(has & ~view)[0]
            self._land(copy, [grads[i] for i in copy], np.nonzero(~has & self.dirty)[0], stream,
                       adopt=False)  # (_reinstall makes them views after the step)
            self.dirty = has.copy()
        # ZeRO-1: the carry weight per owned param (see the module docstring)
        cmul = np.where(view, self.ws - 1, 0).astype(np.int64)
        self.steps[self.owned & has] += 1
        self.last_adam_bytes = 0
        # fast path: every owned param has a grad and, per param group, one (step, carry) key
        own = self.owned
        hps = {}
        if has[own].all():
            from .kernels import adam_hparams

            gof = np.asarray(self.group_of)
            for gi in np.unique(gof[own]):
                sel = own & (gof == gi)
                st, cm = np.unique(self.steps[sel]), np.unique(cmul[sel])
                if len(st) != 1 or len(cm) != 1:
                    continue
                h = hparams_of(int(gi))
                if h["amsgrad"] and self.vmax is None:
                    continue
                hps[int(gi)] = adam_hparams(
                    h["lr"], h["beta1"], h["beta2"], h["eps"], h["weight_decay"], int(st[0]),
                    decoupled=h["decoupled"], amsgrad=h["amsgrad"], maximize=h["maximize"],
                    grad_div=float(self.ws),
                    carry_mul=float(cm[0]) if self.carry is not None else 0.0)
        if self.overlap and not self.inplace:
            self._step_overlap(grads, has, view, cmul, hps, hparams_of, stream)
            return
        if self.grad_comm:  # the exchange moves bf16: convert every local grad once (2 launches' worth
            from .kernels import convert  # of bytes: read 4 + write 2 B per element)

            convert(self.G, self.Gc, stream)
        if self.ws == 1:  # zero1.py:107-108 / zero2.py:120 at ws=1: Adam on the local grads
            with _lib.phase_range("optimizer_step"):
                for rd in self.rounds:
                    if len(rd.idx) and not (hps and self._adam_round_fast(rd, hps, stream, gptr)):
                        live = has[rd.idx]
                        rows, idx = (rd.rows, rd.idx) if live.all() else (rd.rows[live], rd.idx[live])
                        self._run_adam(("flat", rd.j), rows, idx, hparams_of, stream,
                                       carry_mul=cmul[idx],
                                       gptr=None if gptr is None else gptr[idx])
            if self.inplace:
                if self.overlap:
                    self.launched_in_backward = self.ov_launched
                    self._ov_reset()
                return  # fresh gradients stay the caller's p.grad (read in place)
            self._reinstall(has, view)
            return
        self.ev_grads.record(stream)
        cs = self.comm_stream
        cs.wait_event(self.ev_grads)
        with _lib.phase_range("all_reduce_gradients"):  # zero1.py:80-84 / zero2.py:94-113
            for rd in self.rounds:
                e0 = self._timed_start(cs)
                self._reduce_round(rd, cs)
                self.ev_red[rd.j].record(cs)
                self._timed_end(e0, cs, "rs", int(rd.count.sum()))
            self.ev_c1.record(cs)
            if self.capture_reduced is not None:
                with torch.cuda.stream(cs):
                    self.capture_reduced.copy_(self.R[:self.capture_reduced.numel()])
        with _lib.phase_range("optimizer_step"):  # zero1.py:88
            for rd in self.rounds:
                stream.wait_event(self.ev_red[rd.j])
                if len(rd.idx) and not (hps and self._adam_round_fast(rd, hps, stream)):
                    live = has[rd.idx]
                    rows, idx = (rd.rows, rd.idx) if live.all() else (rd.rows[live], rd.idx[live])
                    self._run_adam(("flat", rd.j), rows, idx, hparams_of, stream,
                                   carry_mul=cmul[idx])
                self.ev_adam[rd.j].record(stream)
        with _lib.phase_range("broadcast_parameters"):  # zero1.py:91-102
            for rd in self.rounds:
                cs.wait_event(self.ev_adam[rd.j])
                e0 = self._timed_start(cs)
                self._bcast_round(rd, cs)
                self.ev_bc[rd.j].record(cs)
                self._timed_end(e0, cs, "ag", int(rd.count.sum()))
        stream.wait_event(self.ev_bc[self.K - 1])  # the parameters are P: next forward reads it
        self._reinstall(has, view)

    def _bind_inplace(self, grads, has, view, stream) -> np.ndarray:
        """ws == 1: the gradient address Adam reads per parameter (0 = none): an arena view's slot,
        a fresh tensor itself (zero2.py:120 reads p.grad where backward left it) — or, for a
        gradient the vector kernel cannot read in place (misaligned, or not one dense run of the
        parameter's dtype: a transposed or expanded tensor a caller assigned), its G slot after a
        copy, p.grad then becoming the slot's view."""
        n = len(self.params)
        gptr = np.zeros(n, np.uint64)
        align = 8 if self.dtype == torch.bfloat16 else 16
        fresh = np.nonzero(has & ~view)[0]
        ptrs = np.fromiter((_ptr(grads[i]) for i in fresh), np.uint64, len(fresh))
        dense = np.fromiter((_dense(grads[i], self.params[i]) for i in fresh), bool, len(fresh))
        ok = ((ptrs % np.uint64(align)) == 0) & dense
        gptr[fresh[ok]] = ptrs[ok]
        odd = fresh[~ok]
        if len(odd):
            self._land(odd, [grads[i] for i in odd], (), stream, adopt=True)
        slots = np.nonzero(has & view)[0]
        if len(slots) or len(odd):
            both = np.concatenate([slots, odd]).astype(np.int64)
            gptr[both] = self.grad_slot_ptrs(both)
        self.inplace_reads = int(ok.sum())
        return gptr

    def _reinstall(self, has, view):
        """Every p.grad is (again) its arena view, holding this step's local gradient."""
        for i in np.nonzero(has & ~view)[0]:
            self.params[i].grad = self.grad_view(int(i))
            self._views[i] = self.params[i].grad

    def _timed_start(self, cs):
        if self.comm_events is None:
            return None
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(cs)
        return e0

    def _timed_end(self, e0, cs, kind, elems):
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(cs)
        # bus bytes of the round as a ring reduce-scatter / all-gather of all owners' windows
        es = self.ces if kind == "rs" else self.es
        self.comm_events.append((kind, "flat", e0, e1, elems * es * (self.ws - 1) / self.ws))

    def comm_time_s(self) -> float:
        """zero2.py:92,116: from step() entry until the gradient reduction is done."""
        if self.ws == 1:
            return 0.0
        return max(0.0, self.ev_c0.elapsed_time(self.ev_c1) / 1e3)


def _dense(g: torch.Tensor, p: torch.Tensor) -> bool:
    """``g`` is one contiguous run of ``p.numel()`` elements of ``p``'s dtype (Adam reads it as
    such); a stride-0 expand or a transpose is not."""
    return g.dtype == p.dtype and g.numel() == p.numel() and g.is_contiguous()


class _nullgroup:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _group(comm):
    grp = getattr(comm, "group", None)
    return grp() if grp is not None else _nullgroup()


def _zeros_placed(n, dtype, device, tries):
    from .engine import probed_zeros

    return probed_zeros(n, dtype, device, tries)
