"""Drive the zero_amd ShardedOptimizer with a golden trajectory's exact step inputs.

Shared by the single-process GPU parity tests and the spawned multi-rank ones.  The reference's
local gradients per rank and step (tests/golden/traj_*.npz, ``r{rank}_t{t}_lg{i}``) are written into
``p.grad`` and ``step()`` runs; the returned params are compared with the reference's own.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def init_pg(rank: int, ws: int, port: int):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)


def module_for(variant: int):
    if variant == 1:
        from zero_amd import zero1 as mod
    elif variant == 2:
        from zero_amd import zero2 as mod
    else:
        from zero_amd import zero3 as mod
    return mod


def set_grad(p, g):
    """Deliver a step's local gradient the way backward does: into the existing grad (the flat
    arena's view after zero_grad(), which keeps ZeRO-1's carry as the reference's surviving grads
    do), or as a new grad when there is none."""
    if p.grad is not None and p.grad.shape == g.shape and p.grad.dtype == g.dtype:
        p.grad.copy_(g)
    else:
        p.grad = g


def check_auto_arena(opt, ws):
    """arena="auto": calibrated at construction at ws > 1, the same choice on every rank, and the
    engine built is the chosen one (the flat arena builds its engine at construction)."""
    import torch.distributed as dist

    cal = opt.arena_calibration
    if ws == 1:
        assert cal is None
        return
    assert cal["chosen"] in ("flat", "buckets") and cal["sample_bytes"] > 0
    assert all(v > 0 for v in cal["sample_ms"].values())
    every = [None] * ws
    dist.all_gather_object(every, cal["chosen"])
    assert len(set(every)) == 1, every
    kind = getattr(opt.engine, "arena_kind", "buckets") if opt.engine is not None else "buckets"
    assert kind == cal["chosen"], (kind, cal)


def run_injected(z, variant: int, rank: int, ws: int, device, comm=None, window_elems=64, tol=1e-6,
                 buckets=None, arena=None):
    """Replay the fixture's grads through ShardedOptimizer; assert params match every step."""
    mod = module_for(variant)
    steps = int(z["steps"])
    params = [torch.nn.Parameter(torch.from_numpy(z[f"init_{i}"].copy()).to(device)) for i in range(12)]
    kw = dict(bucket_mb=ws * window_elems * 4 / (1 << 20))
    if comm is not None:
        kw["comm"] = comm
    if buckets is not None:
        kw["buckets"] = buckets
    if arena is not None:
        kw["arena"] = arena
    opt = mod.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), **kw)
    if arena == "auto":
        check_auto_arena(opt, ws)
    worst = 0.0
    for t in range(steps):
        opt.zero_grad()
        for i, p in enumerate(params):
            set_grad(p, torch.from_numpy(z[f"r{rank}_t{t}_lg{i}"].copy()).to(device))
        opt.step()
        key0 = f"r{rank}_t{t}_p0"
        if key0 in z.files:
            for i, p in enumerate(params):
                e = rel(p.detach().cpu().numpy(), z[f"r{rank}_t{t}_p{i}"])
                worst = max(worst, e)
                assert e <= tol, (variant, ws, rank, t, i, e)
    # Adam state exposed through optimizer.state (memory.py:15-24 reads it)
    for i, p in enumerate(params):
        key = f"r{rank}_state_{i}_exp_avg"
        if key in z.files:
            st = opt.optimizer.state[p]
            assert int(st["step"].item()) == int(z[f"r{rank}_state_{i}_step"])
            assert rel(st["exp_avg"].cpu().numpy(), z[key]) <= tol
            assert rel(st["exp_avg_sq"].cpu().numpy(), z[f"r{rank}_state_{i}_exp_avg_sq"]) <= tol
    assert opt.local_param_indices == z[f"r{rank}_local"].tolist()
    if opt.engine is not None:  # the ZeRO-1 carry exists exactly when ws > 1 (zero1.py:107-108)
        assert (opt.engine.carry is not None) == (variant == 1 and ws > 1)
    return worst


def run_backward(z, variant: int, rank: int, ws: int, device, comm=None, tol=1e-6, overlap=True,
                 views=True, bucket_mb=None, arena=None):
    """Like run_injected, but the fixture's grads arrive through a real backward pass
    (loss = Σ_i <p_i, G_i>, so p_i.grad == G_i exactly), which fires the post-accumulate-grad
    hooks of the backward-overlapped mode.  ``views``: zero_grad() installs bucket views
    (autograd accumulates in place); otherwise grads are set to None and copied into the buckets.
    ZeRO-1 on the flat arena with ``views=False`` is the loop that clears every grad itself
    (model.zero_grad()): no carry, so the expectation is the oracle's zero_grad="model" run
    (the bucket arena keeps the reference harness's carry either way)."""
    mod = module_for(variant)
    steps = int(z["steps"])
    init = [z[f"init_{i}"] for i in range(12)]
    params = [torch.nn.Parameter(torch.from_numpy(a.copy()).to(device)) for a in init]
    kw = dict(overlap=overlap)
    if bucket_mb is not None:
        kw["overlap_bucket_mb"] = bucket_mb
    if comm is not None:
        kw["comm"] = comm
    if arena is not None:
        kw["arena"] = arena
    opt = mod.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), **kw)
    flat = getattr(opt.engine, "arena_kind", None) == "flat"
    want = None
    if flat and variant == 1 and ws > 1 and not views:
        from oracle import zero_oracle as zo

        want = zo.simulate(1, ws, init, steps=steps, zero_grad="model",
                           local_grads=lambda t, r, i: z[f"r{r}_t{t}_lg{i}"])
    for t in range(steps):
        if views:
            opt.zero_grad()
        else:
            for p in params:
                p.grad = None
        gs = [torch.from_numpy(z[f"r{rank}_t{t}_lg{i}"].copy()).to(device) for i in range(12)]
        loss = sum((p * g).sum() for p, g in zip(params, gs))
        loss.backward()
        opt.step()
        if want is not None:
            for i, p in enumerate(params):
                e = rel(p.detach().cpu().numpy(), want["params"][t][rank][i])
                assert e <= tol, (variant, ws, rank, t, i, e, "model.zero_grad")
        elif f"r{rank}_t{t}_p0" in z.files:
            for i, p in enumerate(params):
                e = rel(p.detach().cpu().numpy(), z[f"r{rank}_t{t}_p{i}"])
                assert e <= tol, (variant, ws, rank, t, i, e)
    if want is not None:
        return opt
    for i, p in enumerate(params):
        key = f"r{rank}_state_{i}_exp_avg"
        if key in z.files:
            st = opt.optimizer.state[p]
            assert int(st["step"].item()) == int(z[f"r{rank}_state_{i}_step"])
            assert rel(st["exp_avg"].cpu().numpy(), z[key]) <= tol
    return opt


def _shifted(i, fn, args, env=None):
    _apply_env(env)
    fn(i + 1, *args)


# How the ranks beside this process are started.  "forkserver" (default): forked from a server
# process that has already imported torch, numpy and zero_amd (and never touches the GPU), so a
# rank does not pay the imports — a spawned rank spent ~2-3 s of CPU importing, and the suite
# starts ~40 sets of ranks; "spawn": a fresh interpreter per rank.  A forked rank starts from the
# server's environment, so the caller's environment at start time is passed and applied first
# (GPU_MAX_HW_QUEUES, NCCL_*, ZS_TEST_COMM are read after that, at HIP / RCCL init or in the case).
START_METHOD = os.environ.get("ZS_START_METHOD", "forkserver")
_PRELOAD = ["numpy", "torch", "torch.distributed", "zero_amd", "zero_amd.zero2", "zero_amd.zero3"]


def _start_method():
    if START_METHOD == "forkserver":
        import multiprocessing as mpm

        mpm.set_forkserver_preload(_PRELOAD)  # (only read when the server starts)
    return START_METHOD


def _apply_env(env):
    if env is not None:
        os.environ.clear()
        os.environ.update(env)


# Environment of the ranks a multi-rank GPU test spawns beside this process.  Up to 8 processes
# share the box's one GPU; at HIP's default of 4 hardware queues each, an over-subscribed 8-rank
# run stalled with half the ranks inside a backward pass while the others waited in a collective.
# Two queues per spawned rank keep them within what the device schedules at once.  This process
# (rank 0 of spawn_ranks, and every single-process test) keeps the box default.
CHILD_ENV = {"GPU_MAX_HW_QUEUES": "2"}


class child_env:
    """os.environ += CHILD_ENV while child processes are started (spawned children copy the
    parent's environment at start), restored afterwards."""

    def __init__(self, extra=None):
        self.extra = dict(CHILD_ENV, **(extra or {}))

    def __enter__(self):
        self.saved = {k: os.environ.get(k) for k in self.extra}
        os.environ.update(self.extra)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        return False


def _child(i, fn, args, deadline_s, env=None):
    import faulthandler
    import sys

    _apply_env(env)
    # a rank stuck in a device-side wait (a peer died inside a collective) dumps its stack and
    # exits on its own instead of holding the GPU
    faulthandler.dump_traceback_later(deadline_s, exit=True, file=sys.stderr)
    fn(i, *args)


def spawn_all_ranks(fn, ws: int, args=(), deadline_s: float = 150.0):
    """Run ``fn(rank, *args)`` for every rank in a SPAWNED process (the caller touches no device
    and only watches): when any rank fails, the others are terminated at once — needed with RCCL,
    whose collectives never time out, so a rank whose peer died would otherwise wait on the GPU
    forever.  Every rank also exits by itself after ``deadline_s``."""
    import time

    import torch.multiprocessing as mp

    with child_env():
        ctx = mp.start_processes(_child, args=(fn, args, deadline_s, dict(os.environ)), nprocs=ws,
                                 join=False, start_method=_start_method())
    t_end = time.time() + deadline_s + 30
    try:
        while not ctx.join(timeout=1.0):  # raises (and kills the rest) when a rank fails
            if time.time() > t_end:
                raise TimeoutError(f"ranks still running after {deadline_s + 30:.0f} s")
    finally:
        for p in ctx.processes:
            if p.is_alive():
                p.kill()


def _run_seq(rank, calls):
    from _gloo_comm import close_comm_scope, open_comm_scope

    open_comm_scope()  # (every rank: the batch's cases share one RCCL communicator per rank)
    log = os.environ.get("ZS_CASE_LOG") if rank == 0 else None  # per-case seconds (suite budget)
    for fn, args in calls:
        t0 = time.perf_counter()
        fn(rank, *args)
        if log:
            with open(log, "a") as f:
                f.write(f"{time.perf_counter() - t0:8.2f} s  ws={args[0]}  {fn.__name__}{args[2:]}\n")
    # (closed only after success: a failed case may have left a collective a dead peer never joins)
    close_comm_scope()


def spawn_batch(ws: int, cases, all_spawned: bool = False, deadline_s: float = 150.0):
    """Several multi-rank cases in ONE set of ws processes, run one after another: case
    ``(fn, extra)`` runs ``fn(rank, ws, port, *extra)`` on every rank with a port of its own (each
    worker makes and destroys its own process group).  Spawning the ranks and importing torch in
    them cost more than most cases' work, so a test batches the cases of one world size."""
    from conftest import free_port

    calls, used = [], set()
    for fn, extra in cases:
        port = free_port()
        while port in used:
            port = free_port()
        used.add(port)
        calls.append((fn, (ws, port) + tuple(extra)))
    if all_spawned:
        spawn_all_ranks(_run_seq, ws, (calls,), deadline_s=deadline_s)
    else:
        spawn_ranks(_run_seq, ws, (calls,))


def spawn_ranks(fn, ws: int, args=()):
    """Run ``fn(rank, *args)`` for every rank of a ws-rank job: rank 0 in THIS process, ranks
    1..ws-1 spawned.  So a ws-rank GPU test puts exactly ws processes on the box's GPU (the
    hardware schedules up to 8 processes on a device at once; a 9th — the pytest process beside
    8 spawned ranks — over-subscribed it and stalled ws=8 runs).  A failure on any rank fails
    the test; rank 0's failure terminates the others."""
    import torch.multiprocessing as mp

    if ws == 1:
        fn(0, *args)
        return
    with child_env():
        ctx = mp.start_processes(_shifted, args=(fn, args, dict(os.environ)), nprocs=ws - 1,
                                 join=False, start_method=_start_method())
    try:
        fn(0, *args)
    except BaseException:
        try:  # a spawned rank's own failure (which broke rank 0's collective) is the real error
            ctx.join(timeout=15)
        finally:
            for p in ctx.processes:
                if p.is_alive():
                    p.terminate()
            if dist.is_initialized():
                dist.destroy_process_group()
        raise
    while not ctx.join():
        pass
