"""The bucketed ZeRO step: pack → reduce-scatter → fused Adam → all-gather → unpack.

One ``ShardEngine`` per ``ShardedOptimizer``.  It owns, for this rank's optimizer shard (the
*stream* the planner assigns it), flat fp32 buffers for exp_avg / exp_avg_sq (+ max_exp_avg_sq,
the fp32 master of bf16 params, and the ZeRO-1 gradient carry), and one persistent *arena* of
bucket buffers in the parameter dtype.  A bucket buffer is one window of every rank's stream,
rank-major.  In an *even* bucket (stream positions every rank has) the windows are equal, so a
single in-place RCCL reduce-scatter hands every rank the summed gradient of its own window and a
single in-place all-gather hands every rank all updated windows.  Layout R's streams differ in
length (the reference assigns whole parameters by index); the part of the longer streams beyond
the shortest one goes into *ragged* buckets, moved by one grouped RCCL reduce (and broadcast) per
owner — the reduce-scatter-v / all-gather-v — instead of zero-padding every window to the longest
stream (SURVEY.md §7 "Uneven ownership vs equal-count reduce-scatter").

Per step and bucket k (reference loop it replaces in brackets):
  compute stream: pack(k)  — gfx950 gather of every param's grad slice into bucket k
                              [zero2.py:99-104 flatten + cat×ws; zero1.py has no copy]
  comm stream:    RS(k)     — RCCL reduce-scatter (ragged: grouped reduce), in place
                              [zero1.py:81-84 / zero2.py:107]
  compute stream: adam(k)  — fused Adam on this rank's window, grad /ws folded in, writes the
                              updated param into its bucket slot [zero1.py:88 / zero2.py:111,120]
  comm stream:    AG(k)     — RCCL all-gather (ragged: grouped broadcast), in place
                              [zero1.py:95-102 / zero2.py:126-133]
  compute stream: unpack(k) — gfx950 scatter of bucket k back into module storage
Streams are ordered by events only; adam(k) overlaps RS(k+1), unpack(k) overlaps AG(k+1).
With ws == 1 there is nothing to exchange and the step is one fused-Adam launch that reads
every grad and writes every param in place.

Segment tables are uploaded once and reused while the tensors' addresses stay the same.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from .comm import StreamEvent, comm_stream, zs_dtype
from .kernels import AdamSet, CopySet, adam_hparams
from .plan import Plan

ALIGN_ELEMS = 64  # every stream piece starts 256 B (f32) / 128 B (bf16) aligned


def _ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else int(t.data_ptr())


LAUNCH_GROWTH = 8


def launch_growth() -> int:
    """Growth factor of the copy launch groups: 8 (``ZERO_AMD_LAUNCH_GROWTH`` overrides it, for
    A/B runs).  Packing a bucket moves 2 x its bytes at ~6 TB/s; its reduce-scatter at ws = 8 moves
    7/8 of them over xGMI at <= 1.07 TB/s aggregate, so a group 8x the size of everything before it
    is packed about as fast as the collectives of what came before run — the comm stream waits at
    most once, for tens of microseconds — while 24 C4 buckets take 3 launches instead of 6:
    pack 0.70 -> 0.755 of 8 TB/s at the simulated ws=8 C4 layout (profiles/r03_launch_growth_ab.txt;
    growth 4: 0.70)."""
    try:
        g = int(os.environ.get("ZERO_AMD_LAUNCH_GROWTH", str(LAUNCH_GROWTH)))
    except ValueError:
        g = LAUNCH_GROWTH
    return max(g, 2)


def launch_groups(K: int, small_last: bool = False, growth: int | None = None):
    """Buckets 0..K-1 cut into runs whose cumulative length grows by ``growth`` — 1, 1, 2, 4, 8, …
    at 2 (1, 3, 12, … at 4) — each moved by ONE copy launch: a launch's ramp and tail are paid
    log_growth(K) times instead of K times, and the first bucket still reaches its collective after
    one bucket's copy (a group's copy overlaps the previous groups' collectives while growth stays
    below the collective : copy time ratio of a bucket).  ``small_last``: the mirror image
    (…, 4, 2, 1, 1), for the unpack after the all-gathers, so only the last bucket's copy is exposed
    after the last gather."""
    g = launch_growth() if growth is None else max(int(growth), 2)
    sizes, left, done = [], K, 0
    while left > 0:
        n = 1 if done == 0 else min(done * (g - 1), left)
        sizes.append(min(n, left))
        left -= sizes[-1]
        done += sizes[-1]
    if small_last:
        sizes = sizes[::-1]
    out, k = [], 0
    for n in sizes:
        out.append(list(range(k, k + n)))
        k += n
    return out


PROBE_MIN_BYTES = 1 << 30
# An in-place stream over an allocation in MI355X's fast VRAM region runs at ~6.2-6.3 TB/s (the
# guide's float4 copy: 6.29); in the slow regions at ~5.2 (profiles/r02_alloc/).  A candidate at or
# above this is kept at once, without allocating the remaining ones.
PROBE_ACCEPT_GBS = 5950.0
# The probe's second route (round 6): when none of the plain allocations reaches
# the acceptance rate, up to this many candidates of 1-GiB physical chunks (hipMemCreate) mapped
# side by side into one virtual range (zs_device_alloc_chunked).  Interleaved A/B at the exact
# fp32-master state size, 36 GiB, six rounds on one box (profiles/r06_vmm_modes_36g.jsonl):
# plain hipMalloc 5.45-6.19 TB/s, 3 of 6 at >= 6.0; 1-GiB chunks 5.46-6.13, 4 of 6 at >= 6.0
# (round 2's 12- and 40-GiB runs: no consistent winner) — a different draw of physical memory,
# not a cure, so it is a fallback after the plain candidates, held under the same 3-buffer bound.
PROBE_CHUNKED_TRIES = 3
PROBE_CHUNK_BYTES = 1 << 30


# device memory held by placed buffers (outside torch's cache), per device index: bytes and buffers
# held now, and the high-water mark of bytes — probe candidates included while they are held
_PLACED = {}


def _placed(dev_index: int) -> dict:
    return _PLACED.setdefault(int(dev_index), {"bytes": 0, "buffers": 0, "peak": 0})


def placed_bytes(device=None) -> int:
    """Bytes of device memory currently held by placed buffers (``probed_zeros``) on ``device``
    (None: every device).  They are hipMalloc allocations outside torch's caching allocator, so
    ``torch.cuda.memory_allocated`` does not count them; the harness memory report prints them
    beside torch's figures (training_utils/memory.py)."""
    if device is None:
        return sum(d["bytes"] for d in _PLACED.values())
    return _placed(torch.device(device).index or 0)["bytes"]


def placed_peak_bytes(device=None) -> int:
    """High-water mark of ``placed_bytes`` on ``device`` (None: the largest over devices),
    counting the placement probe's candidates while they are held."""
    if device is None:
        return max((d["peak"] for d in _PLACED.values()), default=0)
    return _placed(torch.device(device).index or 0)["peak"]


def reset_placed_peak(device=None) -> None:
    for k, d in _PLACED.items():
        if device is None or k == (torch.device(device).index or 0):
            d["peak"] = d["bytes"]


class _DeviceBuffer:
    """``nbytes`` of device memory from ``zs_device_alloc`` (hipMalloc), freed with
    ``zs_device_free`` when the last tensor viewing it is released (torch keeps this object alive
    through ``__cuda_array_interface__``).  Nothing here touches torch's caching allocator."""

    def __init__(self, nbytes: int, device, chunk_bytes: int = 0):
        import ctypes

        self.nbytes, self.device = int(nbytes), torch.device(device)
        ptr = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            if chunk_bytes:  # physical chunks side by side in one virtual range (whole chunks)
                self.nbytes = -(-self.nbytes // int(chunk_bytes)) * int(chunk_bytes)
                _lib.call("zs_device_alloc_chunked", int(nbytes), int(chunk_bytes), ctypes.byref(ptr))
            else:
                _lib.call("zs_device_alloc", self.nbytes, ctypes.byref(ptr))
        self.ptr = int(ptr.value)
        acc = _placed(self.device.index or 0)
        acc["bytes"] += self.nbytes
        acc["buffers"] += 1
        acc["peak"] = max(acc["peak"], acc["bytes"])

    @property
    def __cuda_array_interface__(self):
        return {"shape": (self.nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                "version": 2}

    def tensor(self, n: int, dtype) -> torch.Tensor:
        """The first ``n`` elements of the buffer as a 1-D ``dtype`` tensor on its device."""
        with torch.cuda.device(self.device):
            raw = torch.as_tensor(self, device=self.device)
        if raw.data_ptr() != self.ptr or raw.device != self.device:
            raise RuntimeError("zero_amd: torch did not wrap the placed buffer in place "
                               f"({raw.device}, {raw.data_ptr():#x} != {self.ptr:#x})")
        es = torch.empty((), dtype=dtype).element_size()
        return raw[:n * es].view(dtype)

    def free(self):
        if self.ptr:
            ptr, self.ptr = self.ptr, 0
            acc = _placed(self.device.index or 0)
            acc["bytes"] -= self.nbytes
            acc["buffers"] -= 1
            try:
                _lib.lib.zs_device_free(ptr)
            except Exception:  # noqa: BLE001 — interpreter shutdown: the runtime may be gone
                pass

    __del__ = free


def _stream_gbs(ptr: int, nbytes: int, stream) -> float:
    """In-place streaming GB/s of ``nbytes`` at ``ptr`` (read + write of every byte, gfx950 copy
    kernel; one warm pass first, which also touches every page)."""
    probe = CopySet([ptr], [ptr], [nbytes])  # unchanged contents
    probe.run(stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    probe.run(stream)
    e1.record(stream)
    e1.synchronize()
    return 2 * nbytes / (e0.elapsed_time(e1) / 1e3) / 1e9


def probed_zeros(n: int, dtype, device, tries: int = 8, accept_gbs: float = PROBE_ACCEPT_GBS):
    """A zero-filled buffer for a long-lived, bandwidth-bound stream, placed by measurement.

    Streaming bandwidth depends on WHERE in VRAM an allocation lands, stably per allocation:
    8-GiB buffers allocated one after another on one box streamed at 5.2 TB/s up to ~96 GiB of
    allocated VRAM, 6.3 TB/s between ~96 and ~160 GiB, 5.2 again above (profiles/r02_alloc/
    alloc_pos8.jsonl); the same launch re-measured later, or after 3 s of warm streaming, keeps its
    speed (alloc_tlb2.jsonl: not a clock effect), and the fast buffers do not translate better
    (they see MORE UTCL1 misses; identical DRAM request counts — pmc_pass*.json).  So for buffers
    of 1 GiB or more, candidates are allocated and streamed once in place by the gfx950 copy
    kernel; the first at ``accept_gbs`` or above is kept at once.  When none of ``tries`` plain
    allocations reaches it, up to ``PROBE_CHUNKED_TRIES`` more candidates take the second route —
    1-GiB physical chunks mapped side by side (``zs_device_alloc_chunked``) — and the fastest of
    all is kept.  At most THREE candidates are held at once (the best so far, the newest, and the
    last rejected one, so the next allocation cannot be handed the memory just rejected): peak
    transient memory is 3x the buffer (chunked candidates: rounded up to whole GiB).

    Candidates are device allocations of their own (``zs_device_alloc``, outside torch's caching
    allocator — round 4): a rejected one goes straight back to the device, and the caller's cached
    blocks are never touched (no ``torch.cuda.empty_cache()``).  The kept buffer is freed when its
    last tensor is; ``placed_bytes()`` counts what is held.  Skipped when free memory is short —
    then the single plain allocation is still measured.
    Returns (buffer, info dict): ``gbs`` every candidate's GB/s in allocation order,
    ``unprobed_gbs`` the first (what a plain allocation would have given), ``chosen``."""
    nbytes = n * torch.empty((), dtype=dtype).element_size()
    info = {"tries": 1, "gbs": []}
    env = os.environ.get("ZERO_AMD_PROBE_TRIES")  # diagnostics: 1 = plain allocation
    if env:
        tries = int(env)
    env = os.environ.get("ZERO_AMD_PROBE_ACCEPT_GBS")  # diagnostics: the acceptance threshold
    if env:
        accept_gbs = float(env)
    env = os.environ.get("ZERO_AMD_PROBE_MIN_BYTES")  # diagnostics: the smallest buffer probed
    if nbytes < (int(env) if env else PROBE_MIN_BYTES):
        return torch.zeros(n, dtype=dtype, device=device), info
    device = torch.device(device)
    stream = torch.cuda.current_stream(device)
    free, total = torch.cuda.mem_get_info(device)
    # three candidates are held at once: keep a quarter of the device (and 2 GiB) out of it
    room = (free - max(total // 4, 2 << 30)) // nbytes
    if tries <= 1 or room < 3:
        buf = torch.zeros(n, dtype=dtype, device=device)
        g = round(_stream_gbs(buf.data_ptr(), nbytes, stream), 1)
        info.update(gbs=[g], unprobed_gbs=g, chosen=0,
                    probe="off" if tries <= 1 else "skipped: free memory short")
        return buf, info
    best = newest_rejected = None
    chunked = PROBE_CHUNKED_TRIES if room >= 3 + (PROBE_CHUNK_BYTES * 3) // nbytes else 0
    routes = ["hipMalloc"] * tries + ["chunked"] * chunked
    info["routes"] = []
    for k, route in enumerate(routes):
        try:
            cand = _DeviceBuffer(nbytes, device, PROBE_CHUNK_BYTES if route == "chunked" else 0)
        except _lib.ZeroAmdError:
            if route == "chunked":  # the virtual-memory API refused: the plain candidates stand
                info["chunked_error"] = _lib.lib.zs_last_error().decode(errors="replace")[:200]
                break
            raise
        g = _stream_gbs(cand.ptr, nbytes, stream)
        info["gbs"].append(round(g, 1))
        info["routes"].append(route)
        if best is None or g > best[0]:
            rejected, best = best, (g, k, cand)
        else:
            rejected = (g, k, cand)
        del cand
        if newest_rejected is not None and rejected is not None:
            # the older blocker goes back to the device now; the newest stays held so the next
            # allocation cannot be handed the memory just rejected
            newest_rejected[2].free()
            newest_rejected = None
        newest_rejected = rejected if rejected is not None else newest_rejected
        rejected = None
        if best[0] >= accept_gbs:
            break
    if newest_rejected is not None:
        newest_rejected[2].free()
    keep, chosen = best[2], best[1]
    out = keep.tensor(n, dtype)
    out.zero_()
    del best, newest_rejected, keep
    route = info["routes"][chosen]
    info.update(tries=len(info["gbs"]), chosen=chosen, accept_gbs=accept_gbs,
                unprobed_gbs=info["gbs"][0], held_max=3, route=route,
                allocator="zs_device_alloc (hipMalloc)" if route == "hipMalloc" else
                "zs_device_alloc_chunked (1-GiB hipMemCreate chunks in one range)")
    return out, info


class ShardEngine:
    def __init__(self, params, group_of, ws: int, rank: int, *, layout="reference", carry=False,
                 comm=None, bucket_bytes: int = 256 << 20, align: int = ALIGN_ELEMS,
                 buckets: str = "ragged", placement_tries: int = 8, master: str = "split"):
        if not params:
            raise ValueError("ShardEngine: no parameters")
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError(f"zero_amd: parameters must live on a GPU (got {dev}); "
                               "there is no CPU path")
        dtype = params[0].dtype
        for p in params:
            if p.device != dev or p.dtype != dtype:
                raise TypeError("zero_amd: all parameters must share one device and dtype")
            if not p.is_contiguous():
                raise ValueError("zero_amd: parameters must be contiguous")
        self.zdtype = zs_dtype(dtype)
        self.params = list(params)
        self.group_of = list(group_of)
        self.ws, self.rank = ws, rank
        self.device, self.dtype = dev, dtype
        self.es = params[0].element_size()
        self.mixed = dtype == torch.bfloat16  # bf16 params → an fp32 master in the shard
        if master not in ("split", "fp32"):
            raise ValueError(f"master must be 'split' or 'fp32' (got {master!r})")
        # split: the master is the bf16 param + an int16 residual (include/zero_amd.h
        # ZS_BF16_SPLIT, 26 instead of 28 B/element per update); fp32: a separate fp32 array
        self.split = self.mixed and master == "split"
        self.p_dtype = _lib.ZS_BF16_SPLIT if self.split else _lib.ZS_BF16
        self.has_carry = bool(carry)
        self.comm = comm
        if ws > 1 and comm is None:
            raise ValueError("ShardEngine: ws > 1 needs a communicator")

        numels = [p.numel() for p in params]
        dim0 = [p.shape[0] if p.dim() > 0 else 1 for p in params]
        window = 0 if ws == 1 else max(align, int(bucket_bytes) // (ws * self.es))
        self.plan = Plan(numels, ws, rank, layout, dim0=dim0, align_elems=align, window_elems=window,
                         buckets=buckets)
        self.W, self.K = self.plan.window, self.plan.num_buckets
        self.L = self.plan.stream_len(rank)
        self.pieces = self.plan.pieces(rank)

        # exp_avg, exp_avg_sq (+ ZeRO-1 carry, + fp32 master or its int16 residual): one
        # allocation, placed by probe
        L = self.L
        nf = 2 + int(bool(carry)) + int(self.mixed and not self.split)
        nlo = (L + 1) // 2 if self.split else 0  # int16 residuals, in fp32 words
        self.state, self.placement = probed_zeros(nf * L + nlo, torch.float32, dev, placement_tries)
        views = iter([self.state[k * L:(k + 1) * L] for k in range(nf)])
        self.m, self.v = next(views), next(views)
        self.vmax = None
        self.carry = next(views) if carry else None
        self.master = next(views) if self.mixed and not self.split else None
        # residual 0 everywhere: the master starts as the bf16 param exactly
        self.lo = self.state[nf * L:].view(torch.int16)[:L] if self.split else None
        if self.master is not None:
            for i, po, so, n in zip(*self._piece_cols()):
                self.master[so:so + n].copy_(params[i].detach().reshape(-1)[po:po + n])
        self.arena = None  # allocated on the first bucketed step (not at all in overlap mode)
        self.placement_tries = placement_tries
        if ws > 1:
            self.buckets = [self.plan.bucket(k) for k in range(self.K)]
            self.segs = [self.plan.segments(k) for k in range(self.K)]
            self.comm_stream = comm_stream(dev)
            mk = lambda: [StreamEvent() for _ in range(self.K)]  # noqa: E731
            self.ev_pack, self.ev_rs, self.ev_adam, self.ev_ag = mk(), mk(), mk(), mk()
        self.ev_c0 = torch.cuda.Event(enable_timing=True)
        self.ev_c1 = torch.cuda.Event(enable_timing=True)
        self.steps = np.zeros(len(params), np.int64)  # torch's per-param state['step']
        self._cache = {}
        self.retired = []
        self.timing_events = None  # optional list of (start, end) events around each Adam launch
        self.comm_events = None    # optional list of (kind, even, start, end, bus_bytes) per collective
        self.copy_events = None    # optional list of (kind, start, end, bytes) per pack / unpack
        self.capture_reduced = None  # optional tensor (stream-long): the reduced grads, for checks
        self.last_adam_bytes = 0

    # ------------------------------------------------------------------------------------------
    def _piece_cols(self):
        pc = self.pieces
        return pc.param.tolist(), pc.param_off.tolist(), pc.stream_off.tolist(), pc.length.tolist()

    def owned_param_indices(self):
        own = getattr(self, "_owned_idx", None)
        if own is None:
            own = self._owned_idx = sorted(set(int(i) for i, n in zip(self.pieces.param,
                                                                     self.pieces.length) if n > 0))
        return own

    def state_views(self, i: int):
        """exp_avg / exp_avg_sq views of param i's shard (Layout R: the whole param)."""
        sel = np.nonzero(self.pieces.param == i)[0]
        if len(sel) != 1:
            return None
        j = int(sel[0])
        so, n = int(self.pieces.stream_off[j]), int(self.pieces.length[j])
        po = int(self.pieces.param_off[j])
        p = self.params[i]
        shape = p.shape if (po == 0 and n == p.numel()) else (n,)
        views = {"exp_avg": self.m[so:so + n].view(shape), "exp_avg_sq": self.v[so:so + n].view(shape)}
        if self.master is not None:
            views["master_param"] = self.master[so:so + n].view(shape)
        if self.lo is not None:  # the fp32 master = the bf16 param's bits << 16 + this residual
            views["master_residual"] = self.lo[so:so + n].view(shape)
        return views

    def ensure_vmax(self):
        if self.vmax is None:
            self.vmax = torch.zeros(self.L, dtype=torch.float32, device=self.device)
        return self.vmax

    def _cached(self, key, sig: bytes, build):
        hit = self._cache.get(key)
        if hit is not None and hit[0] == sig:
            return hit[1]
        obj = build()
        if hit is not None:
            # tensors moved: the old table may still be read by queued kernels, and hipFree
            # synchronises the device — keep it until the next point the device is idle
            self.retired.append(hit[1])
        self._cache[key] = (sig, obj)
        return obj

    def n_retired(self) -> int:
        gb = getattr(self, "gb", None)
        return len(self.retired) + (len(gb.retired) if gb is not None else 0)

    def release_retired(self):
        """Free replaced segment tables; call only after the device has been synchronised."""
        self.retired.clear()
        if getattr(self, "gb", None) is not None:
            self.gb.retired.clear()

    # ------------------------------------------------------------------------------------------
    def _adam_rows(self, idx, g_ptr, mst, mst_out, p_out, so, n):
        """Vectorised zs_adam_seg rows (numpy uint64 (n, 9))."""
        rows = np.zeros((len(idx), 9), np.uint64)
        so = so.astype(np.uint64)
        rows[:, 0] = g_ptr
        rows[:, 1] = mst
        rows[:, 2] = mst_out
        rows[:, 3] = p_out
        rows[:, 4] = np.uint64(self.m.data_ptr()) + so * np.uint64(4)
        rows[:, 5] = np.uint64(self.v.data_ptr()) + so * np.uint64(4)
        if self.vmax is not None:
            rows[:, 6] = np.uint64(self.vmax.data_ptr()) + so * np.uint64(4)
        if self.carry is not None:
            rows[:, 7] = np.uint64(self.carry.data_ptr()) + so * np.uint64(4)
        rows[:, 8] = n.astype(np.uint64)
        return rows

    def _mixed_rows(self, idx, g, hi, p_out, so, n):
        """Rows of a bf16-param update: master read from the bf16 param ``hi`` + its residual
        (split) or from the fp32 master array; the updated bf16 param written to ``p_out``."""
        so64 = so.astype(np.uint64)
        if self.split:
            lo = np.uint64(self.lo.data_ptr()) + so64 * np.uint64(2)
            return self._adam_rows(idx, g, hi, lo, p_out, so, n)
        mst = np.uint64(self.master.data_ptr()) + so64 * np.uint64(4)
        return self._adam_rows(idx, g, mst, mst, p_out, so, n)

    def _run_adam(self, tag, rows, param_idx, hparams_of, stream, carry_mul=None, gptr=None):
        """Partition rows by (group, step, carry multiplier) — torch's bias correction is per param,
        and the ZeRO-1 carry weight depends on which grads survived since the last step — and
        launch one fused-Adam set per part.  ``gptr`` (per row): gradient addresses bound into the
        sets before they run (AdamSet.set_grads; the rows then carry g = 0)."""
        if len(rows) == 0:
            return
        if carry_mul is None:
            carry_mul = np.full(len(param_idx), self.ws - 1 if self.carry is not None else 0, np.int64)
        keys = np.stack([np.asarray(self.group_of)[param_idx], self.steps[param_idx],
                         np.asarray(carry_mul, np.int64)], axis=1)
        for key in np.unique(keys, axis=0):
            sel = np.nonzero((keys == key).all(axis=1))[0]
            sub = np.ascontiguousarray(rows[sel])
            gidx, step, cmul = int(key[0]), int(key[1]), int(key[2])
            gz = getattr(self, "czdtype", self.zdtype)  # dtype of the reduced grad Adam reads
            aset = self._cached(("adam", tag, gidx, len(sel), int(sel[0])), sub.tobytes(),
                                lambda: AdamSet(sub, gz, self.p_dtype))
            if gptr is not None:
                aset.set_grads(np.asarray(gptr, np.uint64)[sel], stream)
            hpd = hparams_of(gidx)
            if hpd["amsgrad"] and self.vmax is None:
                raise RuntimeError("amsgrad state buffer missing")
            hp = adam_hparams(hpd["lr"], hpd["beta1"], hpd["beta2"], hpd["eps"],
                              hpd["weight_decay"], step, decoupled=hpd["decoupled"],
                              amsgrad=hpd["amsgrad"], maximize=hpd["maximize"],
                              grad_div=float(self.ws),
                              carry_mul=float(cmul) if self.carry is not None else 0.0)
            if self.timing_events is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                aset.run(hp, stream)
                e1.record(stream)
                self.timing_events.append((e0, e1, aset.bytes))
            else:
                aset.run(hp, stream)
            self.last_adam_bytes += aset.bytes

    # ------------------------------------------------------------------------------------------
    def step(self, grads, hparams_of, stream=None):
        """One optimizer step.  ``grads[i]`` is param i's local gradient (or None);
        ``hparams_of(group_index)`` returns that group's Adam hyper-parameters."""
        stream = torch.cuda.current_stream(self.device) if stream is None else stream
        n = len(self.params)
        has = np.fromiter((g is not None for g in grads), bool, n)
        gptr = np.fromiter((_ptr(g) for g in grads), np.uint64, n)
        gb = getattr(self, "gb", None)
        if gb is not None and gb.views_installed:  # a zeroed view no backward touched = no grad
            base = gb.buf.data_ptr()
            is_view = np.fromiter((g is not None and g.data_ptr() == base + int(gb.slot[i]) * self.es
                                   for i, g in enumerate(grads)), bool, n)
            has &= gb.marked | ~is_view
        if any(hparams_of(g)["amsgrad"] for g in set(self.group_of)):
            self.ensure_vmax()
        owned = getattr(self, "_owned_mask", None)
        if owned is None:
            owned = self._owned_mask = np.zeros(n, bool)
            owned[self.owned_param_indices()] = True
        self.steps[owned & has] += 1
        self.last_adam_bytes = 0
        if getattr(self, "gb", None) is not None:
            self._step_overlap(has, hparams_of, stream)
        elif self.ws == 1:
            self._step_local(gptr, has, hparams_of, stream)
        else:
            self._step_buckets(gptr, has, hparams_of, stream, grads)

    def _step_local(self, gptr, has, hparams_of, stream):
        pc = self.pieces
        sel = np.nonzero(has[pc.param] & (pc.length > 0))[0]
        idx, po, so, n = pc.param[sel], pc.param_off[sel], pc.stream_off[sel], pc.length[sel]
        pptr = np.fromiter((_ptr(self.params[i]) for i in idx), np.uint64, len(idx))
        es = np.uint64(self.es)
        g = gptr[idx] + po.astype(np.uint64) * es
        if self.mixed:
            pp = pptr + po.astype(np.uint64) * es
            rows = self._mixed_rows(idx, g, pp, pp, so, n)
        else:
            p = pptr + po.astype(np.uint64) * np.uint64(4)
            rows = self._adam_rows(idx, g, p, p, 0, so, n)
        with _lib.phase_range("optimizer_step"):  # zero1.py:88
            self._run_adam("local", rows, idx, hparams_of, stream)

    def _run_copy(self, kind, cs, stream):
        """Launch a pack / unpack CopySet; with timing on, bracket it with HIP events (algorithmic
        bytes = read + write of every byte moved)."""
        if self.copy_events is None:
            cs.run(stream)
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        cs.run(stream)
        e1.record(stream)
        self.copy_events.append((kind, e0, e1, 2 * cs.nbytes))

    def _bucket_buf(self, k):
        b = self.buckets[k]
        return b, self.arena[b.arena_off:b.arena_off + b.elems]

    def _collective(self, k, kind):
        """Reduce ("rs") or gather ("ag") bucket k in place on the comm stream."""
        b, buf = self._bucket_buf(k)
        cs, r, ws = self.comm_stream, self.rank, self.ws
        if self.comm_events is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cs)
        if b.even:
            w = int(b.win_len[0])
            mine = buf[r * w:(r + 1) * w]
            if kind == "rs":
                self.comm.reduce_scatter(buf, mine, cs)
            else:
                self.comm.all_gather(mine, buf, cs)
            bus = b.elems * self.es * (ws - 1) / ws  # ring RS / AG bus bytes
        else:
            if kind == "rs":
                self.comm.reduce_v(buf, b.win_off, b.win_len, cs)
            else:
                self.comm.broadcast_v(buf, b.win_off, b.win_len, cs)
            bus = int(b.win_len.sum()) * self.es  # reduce / broadcast bus bytes = message bytes
        if kind == "rs" and self.capture_reduced is not None and int(b.win_len[r]):
            o, n, so = int(b.win_off[r]), int(b.win_len[r]), int(b.win_stream[r])
            with torch.cuda.stream(cs):  # this rank's reduced window, in stream order
                self.capture_reduced[so:so + n].copy_(buf[o:o + n])
        if self.comm_events is not None:
            e1.record(cs)
            self.comm_events.append((kind, bool(b.even), e0, e1, bus))

    def _step_buckets(self, gptr, has, hparams_of, stream, grads=()):
        from .kernels import CHECK_EXTENTS

        if self.arena is None:
            self.arena, self.arena_placement = probed_zeros(self.plan.arena_elems, self.dtype,
                                                            self.device, self.placement_tries)
        es = np.uint64(self.es)
        pptr = np.fromiter((_ptr(p) for p in self.params), np.uint64, len(self.params))
        base = np.uint64(self.arena.data_ptr())
        r = self.rank
        cs = self.comm_stream
        self.ev_c0.record(stream)  # communication_time: step entry → last gradient reduction
        with _lib.phase_range("all_reduce_gradients"):  # zero1.py:80-84: pack + reduce-scatter
            for gi, grp in enumerate(launch_groups(self.K)):  # pack on the compute stream
                src, dst, nb = [], [], []
                for k in grp:
                    s, b = self.segs[k], self.buckets[k]
                    src.append(np.where(has[s.param], gptr[s.param] + s.param_off.astype(np.uint64) * es, 0))
                    dst.append(base + np.uint64(b.arena_off) * es + s.buf_off.astype(np.uint64) * es)
                    nb.append(s.length * self.es)
                src, dst, nb = np.concatenate(src), np.concatenate(dst), np.concatenate(nb)
                sig = src.tobytes() + dst.tobytes()
                pack = self._cached(("pack", gi), sig, lambda: CopySet(
                    src, dst, nb, bounds=(list(grads), [self.arena]) if CHECK_EXTENTS else None))
                self._run_copy("pack", pack, stream)
                for k in grp:
                    self.ev_pack[k].record(stream)
            for k in range(self.K):  # in-place reduce-scatter (-v) of each bucket
                cs.wait_event(self.ev_pack[k])
                self._collective(k, "rs")
                self.ev_rs[k].record(cs)
            self.ev_c1.record(cs)
        with _lib.phase_range("optimizer_step"):  # zero1.py:88
            for k in range(self.K):  # fused Adam on this rank's window
                stream.wait_event(self.ev_rs[k])
                s, b = self.segs[k], self.buckets[k]
                own = np.nonzero(s.rank == r)[0]
                idx = s.param[own]
                slot = base + np.uint64(b.arena_off) * es + s.buf_off[own].astype(np.uint64) * es
                so = (s.buf_off[own] - int(b.win_off[r])) + int(b.win_stream[r])
                ln = s.length[own]
                po = s.param_off[own].astype(np.uint64)
                live = has[idx]
                if self.mixed:  # master from module storage (+ residual), param out to the slot
                    rows = self._mixed_rows(idx, slot, pptr[idx] + po * es, slot, so, ln)
                else:
                    p = pptr[idx] + po * np.uint64(4)
                    rows = self._adam_rows(idx, slot, p, slot, 0, so, ln)
                self._run_adam(("bucket", k), rows[live], idx[live], hparams_of, stream)
                if not live.all():  # params without a grad keep their value: copy it into the slot
                    dead = np.nonzero(~live)[0]
                    src = pptr[idx[dead]] + po[dead] * es
                    nb = ln[dead] * self.es
                    self._cached(("pass", k), src.tobytes() + slot[dead].tobytes(),
                                 lambda: CopySet(src, slot[dead], nb)).run(stream)
                self.ev_adam[k].record(stream)
        with _lib.phase_range("broadcast_parameters"):  # zero1.py:91-102: all-gather + unpack
            for k in range(self.K):  # in-place all-gather (-v) of the updated windows
                cs.wait_event(self.ev_adam[k])
                self._collective(k, "ag")
                self.ev_ag[k].record(cs)
            # scatter the buckets back into module storage, a group per launch as their gathers
            # complete (gathers run in order on the comm stream: the group's last one suffices)
            for gi, grp in enumerate(launch_groups(self.K, small_last=True)):
                stream.wait_event(self.ev_ag[grp[-1]])
                src, dst, nb = [], [], []
                for k in grp:
                    s, b = self.segs[k], self.buckets[k]
                    src.append(base + np.uint64(b.arena_off) * es + s.buf_off.astype(np.uint64) * es)
                    dst.append(pptr[s.param] + s.param_off.astype(np.uint64) * es)
                    nb.append(s.length * self.es)
                src, dst, nb = np.concatenate(src), np.concatenate(dst), np.concatenate(nb)
                unpack = self._cached(("unpack", gi), src.tobytes() + dst.tobytes(),
                                      lambda: CopySet(src, dst, nb, bounds=(
                                          [self.arena], self.params) if CHECK_EXTENTS else None))
                self._run_copy("unpack", unpack, stream)

    # ------------------------------------------------------------------------------------------
    # backward-overlapped mode: grads reduced to their owner from
    # post-accumulate-grad hooks while backward runs; step() = Adam + broadcast + unpack.
    def enable_overlap(self, bucket_bytes: int):
        from .overlap import GradBuckets

        if self.plan.layout != 0:
            raise ValueError("backward overlap needs the reference (owner-by-index) layout")
        if self.ws > 1 and not hasattr(self.comm, "reduce"):
            raise ValueError("backward overlap needs a communicator with reduce / broadcast")
        owner = [self.plan.owner_of(i) for i in range(len(self.params))]
        self.gb = GradBuckets(self.params, owner, bucket_bytes, self._overlap_reduce)
        pc = self.pieces
        self._so_of = {int(i): int(so) for i, so, n in zip(pc.param, pc.stream_off, pc.length)}
        mk = lambda: [StreamEvent() for _ in range(self.gb.K)]  # noqa: E731
        self.ev_oadam, self.ev_obc = mk(), mk()
        return self.gb

    def _overlap_reduce(self, k, region, cs):
        if self.ws == 1:
            return
        if self.comm_events is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cs)
        self.comm.reduce(region, self.gb.key[k], cs)
        if self.comm_events is not None:
            e1.record(cs)
            self.comm_events.append(("rs", False, e0, e1, region.numel() * self.es))

    def _step_overlap(self, has, hparams_of, stream):
        gb, r, es = self.gb, self.rank, np.uint64(self.es)
        cs = gb.comm_stream
        self.ev_c0.record(stream)  # communication_time: step entry → last gradient reduction
        with _lib.phase_range("all_reduce_gradients"):  # zero1.py:80-84: reduces left by backward
            gb.flush()
        self.ev_c1.record(cs)
        base = np.uint64(gb.buf.data_ptr())
        with _lib.phase_range("optimizer_step"):  # zero1.py:88
            for k in range(gb.K):  # fused Adam on the owned buckets, reading the reduced grads
                if gb.key[k] != r:
                    continue
                stream.wait_event(gb.ev_done[k])
                idx = np.array([i for i in gb.groups[k] if has[i]], np.int64)
                if len(idx):
                    slot = base + gb.slot[idx].astype(np.uint64) * es
                    so = np.array([self._so_of[int(i)] for i in idx], np.int64)
                    ln = np.array([self.params[int(i)].numel() for i in idx], np.int64)
                    p = np.fromiter((_ptr(self.params[int(i)]) for i in idx), np.uint64, len(idx))
                    # ws > 1: the updated params go into the slot, which the broadcast
                    # sends; ws == 1: straight into module storage (no broadcast, no unpack)
                    out = slot if self.ws > 1 else p
                    if self.mixed:
                        rows = self._mixed_rows(idx, slot, p, out, so, ln)
                    else:
                        rows = self._adam_rows(idx, slot, p, out, 0, so, ln)
                    self._run_adam(("overlap", k), rows, idx, hparams_of, stream)
                dead = [i for i in gb.groups[k] if not has[i]]
                if dead and self.ws > 1:  # params without a grad keep their value: copy into the slot
                    src = [_ptr(self.params[i]) for i in dead]
                    dst = [int(base) + int(gb.slot[i]) * self.es for i in dead]
                    self._cached(("opass", k), np.array(src + dst, np.uint64).tobytes(),
                                 lambda: CopySet(src, dst, [self.params[i].numel() * self.es
                                                            for i in dead])).run(stream)
                self.ev_oadam[k].record(stream)
        with _lib.phase_range("broadcast_parameters"):  # zero1.py:91-102: broadcast + unpack
            if self.ws > 1:
                for k in range(gb.K):  # every rank, same order: broadcast each bucket from its owner
                    cs.wait_event(self.ev_oadam[k] if gb.key[k] == r else gb.ev_done[k])
                    region = gb.region(k)
                    if self.comm_events is not None:
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(cs)
                    self.comm.broadcast(region, gb.key[k], cs)
                    if self.comm_events is not None:
                        e1.record(cs)
                        self.comm_events.append(("ag", False, e0, e1, region.numel() * self.es))
                    self.ev_obc[k].record(cs)
            for k in range(gb.K if self.ws > 1 else 0):  # unpack updated params into module storage
                stream.wait_event(self.ev_obc[k])
                g = gb.groups[k]
                src = [int(base) + int(gb.slot[i]) * self.es for i in g]
                dst = [_ptr(self.params[i]) for i in g]
                self._cached(("ounpack", k), np.array(dst, np.uint64).tobytes(),
                             lambda: CopySet(src, dst, [self.params[i].numel() * self.es
                                                        for i in g])).run(stream)
        gb.reset()

    def comm_time_s(self) -> float:
        """The reference's communication_time of the last step (zero2.py:92,116): from step()
        entry until the gradient reduction is done, on the device clock (valid after a
        synchronize; 0 when backward had already finished the reductions)."""
        if self.ws == 1:
            return 0.0
        return max(0.0, self.ev_c0.elapsed_time(self.ev_c1) / 1e3)
