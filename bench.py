"""Benchmark: the ZeRO sharded-optimizer step on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[3]): the SmolLM3-3B-shaped synthetic
parameter set — 326 tensors, 3,075,098,624 params, bf16 params and grads, fp32 master / exp_avg /
exp_avg_sq — stepped by ``zero_amd.zero2.ShardedOptimizer(torch.optim.Adam(lr=1e-3))`` at N GPUs.
One *step* = one ``ShardedOptimizer.step()`` over the full parameter set with synthetic grads
already resident in HBM: pack → RCCL reduce-scatter → fused Adam → RCCL all-gather → unpack
(N=1: one fused Adam launch).  value = params/s = 3,075,098,624 / step time (whole job; total work
is fixed as N grows → "strong" scaling).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
N>1 runs one rank per GPU: under torch.distributed.run (WORLD_SIZE must equal N, else exit 2), or,
with no launcher, bench.py starts ``torch.distributed.run --nproc-per-node N`` itself as a child
process and relays rank 0's line.  A product communicator that cannot be created or fails its
self-check ends the run (exit 5); ``--comm c10d`` times torch.distributed's instead.
Prints ONE JSON line on rank 0 (plus diagnostics on stderr).
"""
from __future__ import annotations

import time

_T0 = time.monotonic()  # process start: the watchdog's default budget counts from here

import argparse  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import sys  # noqa: E402
from pathlib import Path  # noqa: E402

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured copy)
XGMI_LINK_GBS = 153.0  # one xGMI link, per direction (task brief: 7 links x ~153 GB/s per GPU)
XGMI_LINKS = 7


def peer_link_peak_gbs(world: int) -> float:
    """Per-rank xGMI bound for a collective over `world` ranks of one fully connected 8-GPU node:
    each rank has one direct link to every peer, so min(world-1, 7) links can carry its traffic
    (one link at N=2, all seven at N=8)."""
    return XGMI_LINK_GBS * max(1, min(world - 1, XGMI_LINKS))
HANDOFF_WHAT = {
    "default": ("every step: opt.zero_grad() (every grad None, zero2.py:138-139), fresh gradient "
                "tensors (two alternating sets), opt.step(); ws = 1: Adam reads them in place "
                "(zs_adamset_set_grads, no copy); ws > 1: no backward ran, so no hook landed them "
                "and step() copies them into the arena first"),
    "views": ("gradients resident in the flat arena's grad views (as the drop-in's hooks leave "
              "backward's gradients at ws > 1; zero_grad(set_to_none=False) at ws = 1); bucket "
              "arena: the caller's tensors"),
}

METRIC = "ZeRO step time & params/sec at 1/2/4/8 GPU; Adam HBM GB/s vs peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _cpu_sample(shapes, sample_elems: int, per_layer: int = 9, min_tensors: int = 30):
    """Indices of the tensors the CPU baseline steps: for a decoder set (C4 / C5), whole decoder
    layers from the first one (9 tensors each: q, k, v, o, gate, up, down, 2 norms) until at least
    ``min_tensors`` tensors and ``sample_elems`` parameters — the embedding is skipped, so the
    sample keeps the set's tensor-size mix and the reference's per-tensor collective count (12
    blocking calls per tensor per step, zero2.py:94-133) is represented; for the MLP sets, the
    leading tensors up to ``sample_elems``."""
    import numpy as np

    sizes = [int(np.prod(s)) for s in shapes]
    if len(shapes) > 2 * per_layer and len(shapes[1]) == 2:  # decoder set: [embed, layers..., tail]
        n_layers = (len(shapes) - 2) // per_layer
        sel, n = [], 0
        for layer in range(n_layers):
            idx = list(range(1 + layer * per_layer, 1 + (layer + 1) * per_layer))
            sel += idx
            n += sum(sizes[i] for i in idx)
            if len(sel) >= min_tensors and n >= sample_elems:
                break
        return sel, f"decoder layers 0-{layer} ({layer + 1} of {n_layers}; embedding skipped)"
    sel, n = [], 0
    for i, k in enumerate(sizes):
        if n + k > sample_elems and sel:
            break
        n += k
        sel.append(i)
    return sel, f"the {len(sel)} leading tensors"


def cpu_baseline(shapes, sample_elems: int, variant: int = 2, min_seconds: float = 10.0):
    """SURVEY.md §8(d) CPU baseline (2): the reference's own ZeRO step algorithm restated on the
    host cores — per-tensor flatten / cat x ws / gloo reduce_scatter_tensor, /ws on the owner,
    torch.optim.Adam on CPU (single-tensor path, fp32 as the reference), per-tensor broadcast
    (oracle/zero_cpu_step.py, checked against the reference's trajectories by
    tests/test_oracle.py) — on a bounded sample of whole decoder layers (``_cpu_sample``), fp32.
    The reported rate is sampled params / step time; the full-set step is extrapolated at the
    same rate per parameter AND per tensor (the sample's tensor density is the set's, minus the
    embedding), stated in the result."""
    import numpy as np
    import torch

    from oracle.zero_cpu_step import ReferenceStepCPU

    idx, what = _cpu_sample(shapes, sample_elems)
    sel = [shapes[i] for i in idx]
    n = int(sum(int(np.prod(s)) for s in sel))
    total = int(sum(int(np.prod(s)) for s in shapes))
    g = torch.Generator().manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, generator=g) * 0.02) for s in sel]
    grads = [torch.randn(s, generator=g) * 1e-3 for s in sel]
    opt = ReferenceStepCPU(ps, variant=variant if variant in (1, 2) else 2)

    def feed():  # what backward leaves (outside the timing: only step() is the reference's step)
        opt.zero_grad()
        for p, gr in zip(ps, grads):
            p.grad = gr.clone() if p.grad is None else p.grad.add_(gr)

    feed()
    opt.step()  # Adam state allocation outside the timing
    steps, el = 0, 0.0
    while el < min_seconds and steps < 100:
        feed()
        t0 = time.perf_counter()
        opt.step()
        el += time.perf_counter() - t0
        steps += 1
    rate = n * steps / el
    return dict(value=rate, unit="params/s", cores=torch.get_num_threads(), kind="port",
                tensors_sampled=len(sel), params_sampled=n, tensors_total=len(shapes),
                params_total=total, step_s_sampled=el / steps,
                extrapolated_full_step_s=total / rate,
                extrapolation=(f"full-set step ~ {total:,} params / {rate:.3g} params/s: the "
                               f"sampled layers' rate applied to the whole set ({len(shapes)} "
                               "tensors); the embedding / lm_head are single large tensors, so "
                               "per-tensor overheads weigh slightly less there"),
                sample=f"{what}: {len(sel)} tensors, {n:,} params (fp32), {steps} steps of the "
                       f"reference's ZeRO-{variant if variant in (1, 2) else 2} step restated on "
                       f"CPU (per-tensor gloo collectives + torch.optim.Adam, "
                       f"oracle/zero_cpu_step.py), {el:.1f} s of step(); torch {torch.__version__}")


def cpu_oracle_adam(shapes, sample_elems: int, min_seconds: float = 6.0, split: bool = True):
    """The C oracle (oracle/adam_oracle.c, OpenMP) doing the N=1 bf16 update on a bounded sample:
    the fastest CPU restatement of the arithmetic itself, for scale (not the baseline)."""
    import numpy as np

    from oracle import c_oracle

    n = ntens = 0
    for s in shapes:
        k = int(np.prod(s))
        if n + k > sample_elems and ntens:
            break
        n += k
        ntens += 1
    rng = np.random.default_rng(0)
    master = (rng.standard_normal(n, dtype=np.float32) * 0.02)
    g = (rng.standard_normal(n, dtype=np.float32) * 1e-3).view(np.uint32)
    g = ((g + 0x7FFF + ((g >> 16) & 1)) >> 16).astype(np.uint16)
    m = np.zeros(n, np.float32)
    v = np.zeros(n, np.float32)
    p = np.zeros(n, np.uint16)
    if split:
        p, lo = c_oracle.split_master(master)
    steps, t0 = 0, time.perf_counter()
    while True:
        steps += 1
        if split:
            c_oracle.adam_bf16_split(p, lo, g, m, v, c_oracle.hparams(step=steps))
        else:
            c_oracle.adam_bf16(master, p, g, m, v, c_oracle.hparams(step=steps))
        el = time.perf_counter() - t0
        if el >= min_seconds or steps >= 200:
            break
    return dict(value=n * steps / el, unit="params/s", cores=c_oracle.num_threads(), kind="port",
                sample=f"first {n:,} params, {steps} steps of the bf16 update by "
                       f"oracle/adam_oracle.c, {el:.1f} s")


def _busbw(bus_bytes, ms):
    return bus_bytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0


def collective_summary(events, steps, world, red_dev):
    """Per-step time and bus bandwidth of the step's collectives, from HIP events on the comm stream
    (max over ranks).  Bus bytes: ring reduce-scatter / all-gather move (ws-1)/ws of the bucket per
    rank; a reduce / broadcast (ragged buckets) moves its whole message."""
    import torch
    import torch.distributed as dist

    acc = {}
    for kind, even, e0, e1, bus in events:
        label = even if isinstance(even, str) else ("even" if even else "ragged")
        key = ("reduce" if kind == "rs" else "gather") + "_" + label
        ms, b, n = acc.get(key, (0.0, 0.0, 0))
        acc[key] = (ms + e0.elapsed_time(e1), b + bus, n + 1)
    keys = ["reduce_even", "reduce_ragged", "reduce_flat", "gather_even", "gather_ragged",
            "gather_flat"]
    t = torch.tensor([acc.get(k, (0.0, 0.0, 0))[0] for k in keys], dtype=torch.float64, device=red_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out = {"source": "HIP events around each collective on the comm stream, max over ranks",
           "link_peak_gbs": XGMI_LINK_GBS, "aggregate_peak_gbs": XGMI_LINK_GBS * XGMI_LINKS,
           "peer_links": max(1, min(world - 1, XGMI_LINKS)),
           "peer_links_peak_gbs": peer_link_peak_gbs(world)}
    tot_ms = tot_bus = 0.0
    for k, ms in zip(keys, t.tolist()):
        if k not in acc:
            continue
        _, b, n = acc[k]
        out[k] = {"calls_per_step": n / steps, "ms_per_step": ms / steps,
                  "bus_gb_per_step": b / steps / 1e9, "busbw_gbs": _busbw(b, ms)}
        tot_ms += ms
        tot_bus += b
    out["ms_per_step"] = tot_ms / steps
    out["busbw_gbs"] = _busbw(tot_bus, tot_ms)
    out["frac_of_aggregate"] = out["busbw_gbs"] / (XGMI_LINK_GBS * XGMI_LINKS)
    out["frac_of_peer_links"] = out["busbw_gbs"] / peer_link_peak_gbs(world)
    return out


def copy_summary(events, steps, world, red_dev):
    """Pack / unpack (copy_segments_kernel) achieved HBM bandwidth: algorithmic bytes (read + write
    of every byte moved) / kernel time from HIP events on the compute stream, slowest rank."""
    import torch
    import torch.distributed as dist

    out = {}
    for kind in ("pack", "unpack"):
        ev = [(e0, e1, b) for k, e0, e1, b in events if k == kind]
        if not ev:
            continue
        ms = sum(e0.elapsed_time(e1) for e0, e1, _ in ev)
        nbytes = sum(b for _, _, b in ev)
        t = torch.tensor([ms], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        gbs = nbytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        out[kind] = {"kernel": "copy_segments_kernel", "launches_per_step": len(ev) / steps,
                     "ms_per_step": ms / steps, "alg_gb_per_step": nbytes / steps / 1e9,
                     "achieved_gbs": gbs, "frac": gbs / HBM_PEAK_GBS}
    return out


def comm_selfcheck(comm, world, rank, dev):
    """Closed-form check of the RCCL communicator at this N (run before timing): in-place
    reduce-scatter / all-gather, and the ragged bucket's grouped reduce / broadcast per owner.
    Rank r contributes x_r[i] = r + i/1024 (exact in fp32); every result is an exact fp32 value."""
    import torch

    st = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    n = 4096
    i = torch.arange(world * n, device=dev, dtype=torch.float32)
    out = {}
    buf = rank + i / 1024
    # the inputs are written on the current stream and the collectives run on `st`: every call
    # waits for them (without the wait, RCCL read half-written inputs on ranks 6-7 of an N=8
    # one-GPU rehearsal and the check failed a correct communicator)
    st.wait_stream(cur)
    comm.reduce_scatter(buf, buf[rank * n:(rank + 1) * n], st)
    st.synchronize()
    want = world * (world - 1) / 2 + i[rank * n:(rank + 1) * n] * world / 1024
    out["reduce_scatter"] = bool(torch.equal(buf[rank * n:(rank + 1) * n], want))
    buf = torch.full((world * n,), -1.0, device=dev)
    buf[rank * n:(rank + 1) * n] = rank + i[:n] / 1024
    st.wait_stream(cur)
    comm.all_gather(buf[rank * n:(rank + 1) * n], buf, st)
    st.synchronize()
    out["all_gather"] = bool(torch.equal(buf, (i // n) + (i % n) / 1024))
    lens = [(r % 3 + 1) * 64 for r in range(world)]  # ragged windows, 64-element aligned
    offs = [sum(lens[:r]) for r in range(world)]
    tot = sum(lens)
    buf = rank + torch.arange(tot, device=dev, dtype=torch.float32) / 1024
    st.wait_stream(cur)
    comm.reduce_v(buf, offs, lens, st)
    st.synchronize()
    o, m = offs[rank], lens[rank]
    want = world * (world - 1) / 2 + torch.arange(o, o + m, device=dev, dtype=torch.float32) * world / 1024
    out["reduce_v"] = bool(torch.equal(buf[o:o + m], want))
    buf = torch.full((tot,), -1.0, device=dev)
    buf[o:o + m] = rank + 0.5
    st.wait_stream(cur)
    comm.broadcast_v(buf, offs, lens, st)
    st.synchronize()
    want = torch.cat([torch.full((lens[r],), r + 0.5, device=dev) for r in range(world)])
    out["broadcast_v"] = bool(torch.equal(buf, want))
    out["ok"] = all(out.values())
    return out


_PHASE = ["start"]
_REHEARSAL = [None]  # --share-gpu: set to a note that goes into the JSON line


class _stdout_to_stderr:
    """Point fd 1 at stderr for the block (native libraries write there, not to sys.stdout)."""

    def __enter__(self):
        sys.stdout.flush()
        self._saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


def _phase(name: str) -> None:
    _PHASE[0] = name
    log(f"[bench] phase: {name}")
    # test hook (a rehearsal of a hung collective): rank ZS_BENCH_INJECT_RANK stops at the first
    # phase whose name starts with ZS_BENCH_INJECT_HANG, so its peers wait in their next collective
    hang = os.environ.get("ZS_BENCH_INJECT_HANG")
    if hang and name.startswith(hang) and \
            os.environ.get("RANK", "0") == os.environ.get("ZS_BENCH_INJECT_RANK", "1"):
        log(f"[bench] ZS_BENCH_INJECT_HANG: rank {os.environ.get('RANK', '0')} stops in '{name}'")
        while True:
            time.sleep(3600)


# The driver kills a bench run after 600 s of its own clock (BENCH_r05.json run.timeout_s), and a
# run killed from outside leaves nothing.  So the watchdog's default fires inside that limit,
# counted from process start (a fresh box's first `import torch` can take a minute or two), and a
# run that dies says where it was and what it had measured: every thread's Python stack on stderr
# and, on rank 0, one JSON line with "value": null, the phase and the partial results.
WATCHDOG_BUDGET_S = 540.0
_DEADLINE = [None]  # time.monotonic() at which the watchdog fires (None: no watchdog)
_SKIPPED = {}     # optional legs left out because they would not fit before the watchdog
_PARTIAL = {}     # what this run has measured so far (dicts are shared: later updates show)
_OUT_FD = [None]  # a duplicate of the original stdout (fd 1 may be pointed at stderr for a block)
_EMITTED = [False]


def watchdog_seconds(requested, now=None) -> float:
    """The watchdog delay: ``requested`` (seconds; <= 0 disables it), or by default what is left
    of ``WATCHDOG_BUDGET_S`` since process start (at least 30 s)."""
    if requested is not None:
        return float(requested)
    elapsed = (time.monotonic() if now is None else now) - _T0
    return max(30.0, WATCHDOG_BUDGET_S - elapsed)


def _time_left() -> float:
    return float("inf") if _DEADLINE[0] is None else _DEADLINE[0] - time.monotonic()


def leg_fits(name: str, est_s: float) -> bool:
    """An optional leg (the other hand-off, the fp32-master step, the layout ablation, the sweep)
    runs only when twice its estimate plus 30 s fits in what is left before the watchdog: on a slow
    interconnect the headline line is printed without it rather than lost to the watchdog (the
    driver's K timed steps are never cut).  A skipped leg is listed in the line's
    ``skipped_legs``."""
    left = _time_left()
    if 2.0 * est_s + 30.0 <= left:
        return True
    _SKIPPED[name] = {"estimated_s": round(est_s, 1), "time_left_s": round(left, 1)}
    log(f"[bench] skipping the {name} leg: ~{est_s:.0f} s estimated, {left:.0f} s left before the "
        "watchdog")
    return False


def partial_line(failure: str, error=None) -> dict:
    """Rank 0's line for a run that did not finish: ``value`` null, the phase it died in, why, and
    whatever it had already measured (communicator self-check, exchange checks, arena calibration
    with its bus bandwidth, a timed headline if it got that far)."""
    out = {"metric": METRIC, "value": None, "unit": "params/s",
           "n_gpus": int(os.environ.get("WORLD_SIZE", "1")), "higher_is_better": True,
           "failed_phase": _PHASE[0], "failure": failure}
    if error is not None:
        out["error"] = str(error)[-2000:]
    out.update({k: v for k, v in _PARTIAL.items() if k not in out})
    return out


def _emit_partial(failure: str, error=None) -> None:
    """Print ``partial_line`` once, on rank 0 (on the original stdout)."""
    if _EMITTED[0] or int(os.environ.get("RANK", "0")) != 0:
        return
    _EMITTED[0] = True
    try:
        line = json.dumps(partial_line(failure, error), default=str) + "\n"
    except Exception as e:  # noqa: BLE001 — never lose the line to one odd value
        line = json.dumps({"metric": METRIC, "value": None, "failed_phase": _PHASE[0],
                           "failure": failure, "error": f"partial results unserialisable: {e}"}) + "\n"
    fd = _OUT_FD[0] if _OUT_FD[0] is not None else 1
    try:
        sys.stdout.flush()
    except Exception:  # noqa: BLE001
        pass
    os.write(fd, line.encode())


def _dump_stacks(why: str) -> None:
    import faulthandler

    log(f"[bench] {why}: phase '{_PHASE[0]}'; every thread's stack follows")
    try:
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
    except Exception as e:  # noqa: BLE001
        log(f"[bench] (stack dump failed: {e})")


def _start_watchdog(seconds: float) -> None:
    """A daemon timer: if the run is still going after ``seconds``, dump every thread's stack and
    the phase, print the partial line (rank 0) and end the process (os._exit(3), no exec), so a
    collective that never completes fails loudly — with evidence — before an outer limit kills the
    job silently."""
    import threading

    if seconds <= 0:
        return

    def fire():
        _dump_stacks(f"WATCHDOG after {seconds:.0f} s (rank {os.environ.get('RANK', '0')})")
        _emit_partial(f"watchdog: still in phase '{_PHASE[0]}' after {seconds:.0f} s")
        sys.stderr.flush()
        os._exit(3)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()


def _install_term_handler() -> None:
    """Under a launcher, SIGTERM is how torch.distributed.run ends the other ranks once one has
    failed.  The main thread may be blocked in a collective and would never run a Python signal
    handler, so SIGTERM is blocked in every thread and taken by a thread of its own that dumps the
    stacks, prints rank 0's partial line and exits 143."""
    import signal
    import threading

    if not hasattr(signal, "pthread_sigmask"):
        return
    signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGTERM})  # (threads started later inherit it)

    def waiter():
        signal.sigwait({signal.SIGTERM})
        _dump_stacks("SIGTERM (the launcher ends this rank: another rank failed or a limit hit)")
        _emit_partial("terminated by SIGTERM (another rank failed, or an outer limit)")
        sys.stderr.flush()
        os._exit(143)

    threading.Thread(target=waiter, name="bench-sigterm", daemon=True).start()


def _teardown(opt):
    """Drain the device and destroy the optimizer's own RCCL communicator while the HIP runtime
    and the process group are still up (not from a finaliser at interpreter exit)."""
    import torch

    torch.cuda.synchronize()
    for name in ("_comm", "comm"):
        comm = getattr(opt, name, None)
        if comm is not None and hasattr(comm, "close"):
            comm.close()


def _teardown_engine(opt):
    """Drop an optimizer built for the arena calibration (its communicator is the bench's own,
    shared, and stays open)."""
    import gc

    import torch

    torch.cuda.synchronize()
    opt.engine = None
    gc.collect()
    torch.cuda.empty_cache()


def _checked_comm(kw, world, rank, dev):
    """Run comm_selfcheck on kw["comm"] (AND-ed over ranks) before anything is measured.  A
    communicator that gets any closed-form result wrong on any rank ends the run (exit 5): a wrong
    exchange is never timed, and the run never swaps in another communicator behind the caller's
    back (``--comm c10d`` asks for torch's explicitly)."""
    import torch
    import torch.distributed as dist

    out = comm_selfcheck(kw["comm"], world, rank, dev)
    ok = torch.tensor([1.0 if out["ok"] else 0.0], device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    out["all_ranks_ok"] = bool(ok.item() == 1.0)
    if not out["all_ranks_ok"]:
        _fail_comm(rank, f"{type(kw['comm']).__name__} failed the closed-form self-check: {out}")
    return out


class CommFailed(RuntimeError):
    pass


def _fail_comm(rank: int, detail) -> None:
    """The product communicator is unusable at N>1: end the run loudly (exit 5) instead of timing
    something else.  In a test process: raise."""
    log(f"[bench] COMMUNICATOR FAILED on rank {rank}: {detail}")
    if _IN_PROCESS[0]:
        raise CommFailed(f"rank {rank}: {detail}")
    _emit_partial(f"communicator failed on rank {rank}", detail)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(5)


def _product_comm(rank: int):
    """The library's own RCCL communicator (zero_amd.comm.RcclComm); failing to create it ends
    the run (exit 5) unless the caller asked for ``--comm c10d``."""
    from zero_amd.comm import RcclComm

    try:
        return RcclComm()
    except Exception as e:  # noqa: BLE001 — reported and fatal
        _fail_comm(rank, f"RcclComm() raised {type(e).__name__}: {e} (use --comm c10d to time "
                         "torch.distributed's communicator instead)")


def _free_port() -> int:
    """A free TCP port below the ephemeral range (32768+), so no outgoing connection (gloo's pair
    sockets) can take it between this check and the rendezvous bind."""
    import random
    import socket

    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", p))
                return p
            except OSError:
                continue
    raise RuntimeError("no free port in 20000-32000")


def _self_launch_cmd(argv, n: int, port: int):
    """The command ``python bench.py --gpus N`` runs when no launcher started it: N ranks, one
    process per GPU, through torch.distributed.run on 127.0.0.1 (the driver's own form)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            str(REPO / "bench.py"), *argv]


def _launch_ranks(argv, n: int, cmd=None) -> int:
    """Run the N ranks as ONE child process (torch.distributed.run), relay rank 0's JSON line to
    stdout and everything else to stderr, and return the child's exit code.  Called before any
    GPU or torch import in this process; SIGTERM / SIGINT are forwarded to the child."""
    import signal
    import subprocess

    cmd = cmd or _self_launch_cmd(argv, n, _free_port())
    log(f"[bench] no WORLD_SIZE in the environment and --gpus {n}: launching {n} ranks: "
        + " ".join(cmd))
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    prev = {}

    def forward(sig, _frame):
        if proc.poll() is None:
            proc.send_signal(sig)

    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            prev[sig] = signal.signal(sig, forward)
        except ValueError:  # not the main thread (a test): no forwarding
            pass
    lines = 0
    try:
        for line in proc.stdout:
            s = line.strip()
            obj = None
            if s.startswith("{"):
                try:
                    obj = json.loads(s)
                except ValueError:
                    obj = None
            if isinstance(obj, dict):
                print(s, flush=True)
                lines += 1
            else:
                sys.stderr.write(line)
                sys.stderr.flush()
        rc = proc.wait()
    finally:
        for sig, h in prev.items():
            signal.signal(sig, h)
        if proc.poll() is None:
            proc.kill()
            proc.wait()
    if rc == 0 and lines != 1:
        log(f"[bench] the {n}-rank child exited 0 but printed {lines} JSON lines (expected 1)")
        return 6
    return rc


def comm_sweep(comm, arena, world, red_dev, sizes_mb=(4, 16, 64, 256), iters=5):
    """Bucket-size sweep of in-place RCCL reduce-scatter / all-gather on the bf16 arena (the C5
    sweep of BASELINE.json, run on whatever N the bench runs): busBW = bytes*(ws-1)/ws / time."""
    import torch
    import torch.distributed as dist

    st = torch.cuda.Stream(device=arena.device)
    es = arena.element_size()
    rows = []
    for mb in sizes_mb:
        n = (int(mb * (1 << 20)) // es) // world * world
        if n == 0 or n > arena.numel():
            continue
        buf = arena[:n]
        mine = buf[dist.get_rank() * (n // world):(dist.get_rank() + 1) * (n // world)]
        res = []
        for kind in ("rs", "ag"):
            op = (lambda: comm.reduce_scatter(buf, mine, st)) if kind == "rs" else \
                (lambda: comm.all_gather(mine, buf, st))
            op()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()  # nothing of ours in flight while c10d's barrier runs
            dist.barrier()
            torch.cuda.synchronize()
            e0.record(st)
            for _ in range(iters):
                op()
            e1.record(st)
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / iters)
        t = torch.tensor(res, dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        bus = n * es * (world - 1) / world
        rs_ms, ag_ms = t.tolist()
        rows.append({"bucket_mb": mb, "rs_ms": rs_ms, "rs_busbw_gbs": _busbw(bus, rs_ms),
                     "ag_ms": ag_ms, "ag_busbw_gbs": _busbw(bus, ag_ms),
                     "rs_frac_of_peer_links": _busbw(bus, rs_ms) / peer_link_peak_gbs(world),
                     "ag_frac_of_peer_links": _busbw(bus, ag_ms) / peer_link_peak_gbs(world)})
    torch.cuda.synchronize()
    arena.zero_()  # the sweep scribbled over the arena; padding must stay zero
    return rows


class _NoComm:
    """Timing-only stand-in for the collectives (--simulate-ws): leaves buffers untouched."""

    def __init__(self, ws):
        self.ws, self.rank = ws, 0

    def reduce_scatter(self, send, recv, stream):
        pass

    def all_gather(self, send, recv, stream):
        pass

    def reduce_v(self, buf, win_off, win_len, stream):
        pass

    def broadcast_v(self, buf, win_off, win_len, stream):
        pass

    def all_reduce(self, t, stream):
        pass

    def reduce_out(self, send, recv, root, stream):
        pass

    def broadcast(self, t, root, stream):
        pass

    def all_gather_group(self, send, recv, count, dtype, stream):
        pass

    def reduce_scatter_group(self, send, recv, count, dtype, stream):
        pass

    # the synced forms keep the product's host path (sync records and stream waits in one
    # library call) with the collective left out: zs_*_group_synced with no communicator, n = 0
    def all_gather_group_synced_bound(self, send, recv, count, dtype):
        return self._ordered("zs_all_gather_group_synced", dtype)

    def reduce_scatter_group_synced_bound(self, send, recv, count, dtype):
        return self._ordered("zs_reduce_scatter_group_synced", dtype)

    def all_gather_group_synced_raw(self):  # (GatherFast: the ordering alone, no collective)
        import ctypes

        from zero_amd import _lib

        return ctypes.cast(_lib.lib.zs_all_gather_group_synced, ctypes.c_void_p).value, 0, False

    def reduce_scatter_group_synced_raw(self):  # (ReduceFast: the ordering alone)
        import ctypes

        from zero_amd import _lib

        return ctypes.cast(_lib.lib.zs_reduce_scatter_group_synced, ctypes.c_void_p).value, 0, False

    # (the event-ordered forms, which earlier rounds' runtimes bind: tools/z3_host_ab.py)
    def all_gather_group_ordered_bound(self, send, recv, count, dtype):
        return self._ordered("zs_all_gather_group_ordered", dtype)

    def reduce_scatter_group_ordered_bound(self, send, recv, count, dtype):
        return self._ordered("zs_reduce_scatter_group_ordered", dtype)

    @staticmethod
    def _ordered(name, dtype):
        from zero_amd import _lib

        fn, dt = getattr(_lib.lib, name), int(dtype)

        def run(after, ready, stream, done):
            rc = fn(None, 0, None, None, None, dt, after, ready, stream, done)
            if rc:
                _lib.check(rc, name)
        return run


def _zero3_comm_summary(opt, steps, world, red_dev):
    """Per-step time and bus bandwidth of the ZeRO-3 collectives (gathers and gradient
    reduce-scatters, HIP events on the side stream), slowest rank."""
    import torch
    import torch.distributed as dist

    ge = opt.runtime.gather_events or []
    re = opt._reducer.timing or [] if opt._reducer is not None else []
    vals = [sum(a.elapsed_time(b) for a, b, _ in ge), sum(a.elapsed_time(b) for a, b, _ in re)]
    t = torch.tensor(vals, dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out = {"source": "HIP events around each gather group / reduce-scatter bucket on the side "
                     "stream, max over ranks", "peer_links_peak_gbs": peer_link_peak_gbs(world)}
    for key, ev, ms in (("all_gather", ge, float(t[0])), ("reduce_scatter", re, float(t[1]))):
        bus = sum(b for *_, b in ev)
        out[key] = {"calls_per_step": len(ev) / steps, "ms_per_step": ms / steps,
                    "bus_gb_per_step": bus / steps / 1e9, "busbw_gbs": _busbw(bus, ms),
                    "frac_of_peer_links": _busbw(bus, ms) / peer_link_peak_gbs(world)}
    return out


def _zero3_report(args, opt, world, rank, red_dev, el, total, workload, extra):
    """Time / Adam-roofline bookkeeping shared by the two ZeRO-3 benches; rank 0 prints."""
    import torch
    import torch.distributed as dist

    ev, opt.timing_events = opt.timing_events, None
    adam_ms = sum(a.elapsed_time(b) for a, b, _ in ev)
    adam_bytes = sum(nb for _, _, nb in ev)
    achieved = adam_bytes / (adam_ms / 1e3) / 1e9 if adam_ms > 0 else 0.0
    t = torch.tensor([el, -achieved], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # slowest rank's time and Adam bandwidth
    el, achieved = float(t[0]), -float(t[1])
    ms = el / args.steps * 1e3
    comm = _zero3_comm_summary(opt, args.steps, world, red_dev) if world > 1 else None
    if (comm is not None and args.comm in ("rccl", "c10d") and not args.no_comm_sweep
            and opt.grad_arena() is not None):
        # BASELINE.json configs[4]: RS / AG bus bandwidth per bucket size, on the grad chunk arena
        # (scratch between steps) after the timed region
        _phase("bucket-size sweep")
        comm["sweep"] = comm_sweep(opt.comm, opt.grad_arena(), world, red_dev,
                                   sizes_mb=(4, 8, 16, 32, 64, 128, 256))
    traffic, traffic_src, traffic_note = None, None, None
    if (args.traffic_json or world == 1) and args.gather is None \
            and getattr(args, "set_layers", None) is None:
        # PMC passes of this same configuration (profiles/README.md), matched like the ZeRO-1/2 line
        want = {"workload": args.config, "zero": 3, "param_dtype": args.dtype, "n_gpus": world,
                "master": "split"}
        traffic, traffic_src, traffic_note = match_traffic(
            want, adam_bytes / max(len(ev), 1), args.traffic_json)
    if rank == 0:
        out = {
            "metric": METRIC, "value": total / (ms / 1e3), "unit": "params/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": ("bf16 params/grads, fp32 Adam (split master)" if args.dtype == "bf16"
                      else "fp32"),
            "data": "synthetic",
            "config": dict(workload=workload, params=int(total), param_dtype=args.dtype, zero=3,
                           collective_stream=("compute (single stream)" if opt.runtime.stream is None
                                              else "side stream, prefetched in waves of "
                                              f"{opt.runtime.wave}"),
                           update="real ZeRO-3 (update=True)", bucket_mb=args.bucket_mb or 512.0,
                           gather_dtype=args.gather or args.dtype, parallelism=f"dp{world}",
                           gathers=("none at N=1: every shard is its whole parameter, no hooks "
                                    "are registered (zero3.register_zero3_hooks), so this is an "
                                    "unsharded step" if world == 1 and not args.gather
                                    else "per-layer all-gathers in forward and backward")),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "adam_segments_kernel",
                         "avg_launch_ms": adam_ms / max(len(ev), 1),
                         "alg_bytes_per_launch": adam_bytes / max(len(ev), 1),
                         "launches_per_step": len(ev) / args.steps, "traffic_source": traffic_src,
                         "traffic_note": traffic_note},
            "zero3": {"gathers_per_step": opt.runtime.n_gathers / (args.steps + args.warmup),
                      "prefetch_hits": opt.runtime.n_prefetch_hits,
                      "reduce_buckets_per_step": opt._reducer.K,
                      "reduced_in_backward": opt._reducer.last_launched_in_backward},
        }
        if comm is not None:
            out["collectives"] = comm
        if "expected" in extra:  # the slowest rank's iteration beside the prediction
            e = extra["expected"]
            e["measured_ms"] = ms
            e["measured_over_ideal"] = ms / e["ideal_ms"] if e["ideal_ms"] else None
        out.update(extra)
        if _REHEARSAL[0]:
            out["rehearsal"] = _REHEARSAL[0]
        print(json.dumps(out), flush=True)


def _zero3_timed(args, opt, step, dev, world):
    import torch
    import torch.distributed as dist

    for _ in range(args.warmup):
        step()
    opt.timing_events = []
    if world > 1:
        opt.runtime.gather_events = []
        opt._reducer.timing = []
    torch.cuda.synchronize()  # warmup drained first: no collective of ours beside c10d's barrier
    dist.barrier()
    torch.cuda.synchronize()
    _phase("timed steps")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    return time.perf_counter() - t0


def _zero3_comm(args, world, rank, dev):
    """The communicator for the ZeRO-3 benches (self-checked at N>1 like the ZeRO-1/2 one)."""
    kw = {}
    if world > 1 and args.comm == "gloo-staged":
        sys.path.insert(0, str(REPO / "tests"))
        from _gloo_comm import GlooStagedComm

        return GlooStagedComm(), None
    if world > 1:
        from zero_amd.comm import C10dComm

        kw["comm"] = C10dComm() if args.comm == "c10d" else _product_comm(rank)
        _phase("communicator self-check")
        chk = _checked_comm(kw, world, rank, dev)
        _PARTIAL["rccl_selfcheck"] = chk
        return kw["comm"], chk
    return None, None


class ExchangeCheckFailed(RuntimeError):
    pass


_IN_PROCESS = [False]  # main() called from a test process: raise instead of exiting it


NORTH_STAR_ADAM_FRAC = 0.70  # BASELINE.json north_star: fused Adam >= 70 % of peak HBM bandwidth
NORTH_STAR_BUS_FRAC = 0.60   # ... and reduce-scatter / all-gather >= 60 % of xGMI bus bandwidth


def expected_scaling(shapes, zero: int, arena: str, world: int, elem_bytes: int = 2,
                     adam_bytes_per_elem: int = 26, bucket_mb: float | None = None,
                     layout: str = "reference") -> dict:
    """The step the planner predicts on ``world`` GPUs, before it is measured, for
    the slowest rank — no overlap credit, like ``step_roofline``:

    * ZeRO-1/2 (Layout R, zero1.py:55-62): HBM = the max-rank optimizer shard x the Adam bytes per
      element (26 B bf16 split master; ZeRO-1 + 8 B carry), bucket arena + pack and unpack (read +
      write of every gradient / parameter byte); bus per rank = flat arena: a reduce and a
      broadcast group of every owner's stream, ring-equivalent 2 x sum_r L_r x es x (N-1)/N; bucket
      arena: RS / AG of the even buckets at (N-1)/N, per-owner reduce / broadcast of the ragged
      ones at their message bytes (the accounting bench.py's comm events use);
    * ZeRO-3 (Layout Z, zero3.py:105-110) hooked iteration: HBM = the max-rank chunks x Adam bytes;
      bus = forward gather + backward gather + gradient reduce-scatter of every padded chunk,
      3 x sum_i S_i x N x es x (N-1)/N.

    ``layout`` (ZeRO-1/2; VERDICT r5 #6, what the reference's ownership costs): "reference"
    (Layout R, whole parameters by index — the drop-in's, bit-exact against the reference), "flat"
    (Layout F, balanced contiguous 1/N slices of the concatenation: in the flat arena, the N > 1
    line's ``layout_ablation`` leg) or "chunk" (Layout Z, zero3.py:107-108's dim-0 chunks: bucket
    arena only, so + pack / unpack).

    ``ideal_ms`` = HBM / 8 TB/s + bus / the peer links (min(N-1, 7) x 153 GB/s);
    ``at_north_star_ms`` = HBM / (70 % of 8 TB/s) + bus / (60 % of the peer links): the step the
    north star's targets would give (Adam >= 70 % of HBM peak, RS/AG >= 60 % of xGMI busBW)."""
    import numpy as np

    from zero_amd.plan import Plan

    numels = [int(np.prod(s)) for s in shapes]
    dim0 = [int(s[0]) if len(s) else 1 for s in shapes]
    es, ws = int(elem_bytes), int(world)
    bpe = adam_bytes_per_elem + (8 if zero == 1 and ws > 1 else 0)
    total = sum(numels)
    if zero == 3:
        plan = Plan(numels, ws, 0, "chunk", dim0=dim0, align_elems=64)
        own = max(int(plan.pieces(r).length.sum()) for r in range(ws))
        padded = sum(-(-d // ws) * (n // max(d, 1)) for n, d in zip(numels, dim0)) * ws
        bus = 3 * padded * es * (ws - 1) / ws if ws > 1 else 0.0
        hbm = bpe * own
        model = "ZeRO-3: forward + backward gathers and the reduce-scatter of every padded chunk"
    else:
        if layout == "chunk" and arena != "buckets":
            raise ValueError("Layout Z (chunk) runs in the bucket arena")
        win = 0
        if arena == "buckets" and ws > 1:
            win = max(64, int((bucket_mb or 256.0) * (1 << 20)) // (ws * es))
        plan = Plan(numels, ws, 0, layout, dim0=dim0, align_elems=64, window_elems=win)
        own = max(int(plan.pieces(r).length.sum()) for r in range(ws))
        hbm = bpe * own
        if ws == 1:
            bus = 0.0
        elif arena == "flat":
            bus = 2 * sum(plan.stream_len(r) for r in range(ws)) * es * (ws - 1) / ws
        else:
            hbm += 4 * es * total  # pack + unpack: read + write of every gradient / parameter
            bus = 0.0
            for k in range(plan.num_buckets):
                b = plan.bucket(k)
                bus += 2 * (b.elems * es * (ws - 1) / ws if b.even else int(b.win_len.sum()) * es)
        model = f"ZeRO-{zero} {arena} arena" + ("" if layout == "reference" else f", layout {layout}")
    links = peer_link_peak_gbs(ws) * 1e9
    hbm_ms = hbm / (HBM_PEAK_GBS * 1e9) * 1e3
    bus_ms = bus / links * 1e3
    return {"n_gpus": ws, "model": model, "max_rank_adam_gb": bpe * own / 1e9,
            "hbm_gb_per_rank": hbm / 1e9, "bus_gb_per_rank": bus / 1e9,
            "ideal_ms": hbm_ms + bus_ms, "ideal_overlapped_ms": max(hbm_ms, bus_ms),
            "at_north_star_ms": hbm_ms / NORTH_STAR_ADAM_FRAC + bus_ms / NORTH_STAR_BUS_FRAC,
            "peer_links_gbs": links / 1e9,
            "note": "planner prediction made before the run (no overlap credit in ideal_ms; "
                    "ideal_overlapped_ms = the longer of the two)"}


def _expected_block(shapes, zero, arena, world, es, bpe, bucket_mb, measured_ms) -> dict:
    """``expected`` of a bench line: the planner's prediction for this N beside the measured step,
    and the predicted curve over N = 1, 2, 4, 8."""
    e = expected_scaling(shapes, zero, arena, world, es, bpe, bucket_mb)
    e["measured_ms"] = measured_ms
    e["measured_over_ideal"] = measured_ms / e["ideal_ms"] if e["ideal_ms"] else None
    keys = ("ideal_ms", "ideal_overlapped_ms", "at_north_star_ms", "hbm_gb_per_rank",
            "bus_gb_per_rank", "max_rank_adam_gb")
    e["curve"] = {str(n): {k: round(v, 3) for k, v in expected_scaling(
        shapes, zero, arena, n, es, bpe, bucket_mb).items() if k in keys} for n in (1, 2, 4, 8)}
    if zero in (1, 2):
        e["layouts"] = layout_costs(shapes, zero, world, es, bpe, bucket_mb)
    return e


def layout_costs(shapes, zero, world, es=2, bpe=26, bucket_mb=None) -> dict:
    """What the reference's whole-parameter ownership (Layout R) costs at ``world`` GPUs against
    the balanced layouts, predicted by the planner: the slowest rank's Adam bytes and the step's
    ideal time for Layout R / flat arena (the drop-in), Layout F / flat arena (the N > 1 line's
    ``layout_ablation`` leg) and Layout Z / bucket arena (zero3.py's chunks; + pack / unpack)."""
    rows = {"reference_flat_arena": ("flat", "reference"), "balanced_F_flat_arena": ("flat", "flat"),
            "chunk_Z_bucket_arena": ("buckets", "chunk")}
    out = {}
    for name, (arena, layout) in rows.items():
        e = expected_scaling(shapes, zero, arena, world, es, bpe,
                             bucket_mb if arena == "flat" else None, layout=layout)
        out[name] = {k: round(e[k], 3) for k in ("max_rank_adam_gb", "hbm_gb_per_rank",
                                                  "bus_gb_per_rank", "ideal_ms")}
    return out


def _placement_dependence(placement: dict) -> dict:
    """``roofline.placement_dependence``: the Adam rate is conditional on the physical memory its
    streams landed on (DESIGN §5 allocation study) — per placed buffer the candidate kept, its
    in-place stream rate, the route and what a plain single allocation gave (``unprobed_gbs``)."""
    out = {"note": "frac is conditional on placement: Adam streams at the rate of the memory its "
                   "buffers landed on (5.0-6.3 TB/s per allocation on MI355X, stable per "
                   "allocation); the probe keeps the first candidate >= accept_gbs, else the "
                   "fastest (plain hipMalloc candidates, then 1-GiB chunked ranges)"}
    for name, pl in placement.items():
        if isinstance(pl, dict) and pl.get("gbs"):
            k = int(pl.get("chosen", 0))
            out[name] = {"chosen": k, "of": len(pl["gbs"]), "chosen_gbs": pl["gbs"][k],
                         "unprobed_gbs": pl.get("unprobed_gbs"), "route": pl.get("route", "hipMalloc")}
    return out


def match_traffic(want: dict, alg_bytes_per_launch: float, traffic_json=None):
    """roofline.traffic: HBM bytes per Adam launch from a PMC summary of THIS configuration —
    ``--traffic-json`` if given, else the profiles/*_pmc.json whose ``config`` equals ``want`` — used
    only when the summary's algorithmic bytes per launch equal this run's (within 1e-6): after a
    kernel, arena or bucket change an old measurement is not reported as this run's.  Returns
    (bytes or None, source or None, note or None)."""
    # newest round's summary first (profiles are named by round: r01_, r02_, r02s2_, r03_ ...)
    cands = [Path(traffic_json)] if traffic_json else sorted((REPO / "profiles").glob("*_pmc.json"),
                                                              reverse=True)
    note = None
    for tj in cands:
        if not tj.exists():
            continue
        d = json.loads(tj.read_text())
        if not traffic_json and d.get("config") != want:
            continue
        src = str(tj.relative_to(REPO) if tj.is_absolute() and REPO in tj.parents else tj)
        alg = float(d.get("algorithmic_bytes_per_launch") or 0.0)
        if alg <= 0 or abs(alg - alg_bytes_per_launch) > 1e-6 * max(alg, alg_bytes_per_launch):
            note = (f"{src}: algorithmic bytes per launch {alg:.6g} != this run's "
                    f"{alg_bytes_per_launch:.6g}; not used")
            continue
        return d.get("hbm_bytes_per_launch"), src, None
    return None, None, note


def _fail_check(what: str, rank: int, detail) -> None:
    log(f"[bench] EXCHANGE CHECK FAILED on rank {rank}: {what}: {detail}")
    if _IN_PROCESS[0]:
        raise ExchangeCheckFailed(f"rank {rank}: {what}: {detail}")
    _emit_partial(f"exchange check failed on rank {rank}: {what}", detail)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(4)


def _bf16_sum_tolerance(world: int) -> float:
    """Bound on |RCCL bf16 sum - exact sum| relative to sum_r |g_r|: each of the (world-1) hops
    of a ring adds in fp32 and rounds the partial sum to bf16 (<= 2^-9 of its magnitude, which
    is <= sum_r |g_r|), plus the final rounding; doubled for margin."""
    return world * 2.0 ** -8


def _regen_grads(shapes, world, dev, keep, dtype=None):
    """The bench's synthetic gradients of every rank (seed = rank, N(0,1)*1e-3, one generator
    pass over the set, as generated in main / bench_zero3_paramset), reduced on the fly to the
    exact fp32 sum and sum of |g| of the tensors in ``keep`` (index -> flat element slice)."""
    import torch

    gen = torch.Generator(device=dev)
    exact = {i: None for i in keep}
    absum = {i: None for i in keep}
    for r in range(world):
        gen.manual_seed(1000 * 0 + r)
        for i, s in enumerate(shapes):
            t = (torch.empty(s, dtype=torch.float32, device=dev).normal_(generator=gen) * 1e-3)
            if i not in keep:
                continue
            v = t.to(dtype or torch.bfloat16).float().reshape(-1)[keep[i]]
            exact[i] = v.clone() if exact[i] is None else exact[i] + v
            absum[i] = v.abs() if absum[i] is None else absum[i] + v.abs()
    return exact, absum


def zero3_gather_check(opt, model, shapes, full_copies, dev, world, rank, red_dev):
    """Before timing at N>1 (BASELINE configs[4]): (1) one side-stream all-gather of a decoder
    layer through the real communicator must reproduce every full tensor bit for bit; (2) one
    hooked forward/backward: the gradient chunks the backward reduce-scatters left in p.grad must
    equal the exact fp32 sum of every rank's known synthetic gradient within the bf16 ring bound.
    AND-ed over ranks; a failure ends the run (exit 4) naming the rank and tensor."""
    import torch
    import torch.distributed as dist

    rt = opt.runtime
    layer = model.layers[1]
    idx = model.groups[1]
    ms = [opt.param_managers[getattr(layer, f"p{k}")] for k in range(layer.n)]
    rt.launch(("exchange-check",), ms)
    out, ev, _hold, _, _ = rt.pending.pop(("exchange-check",))
    if ev is not None:  # a comm.Sync (raw stream handles); single-stream mode: already in order
        ev.wait(torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    bits = lambda t: t.reshape(-1).view(torch.int16 if t.element_size() == 2 else torch.int32)  # noqa: E731
    bad = [i for (m, full), i in zip(out, idx) if not torch.equal(bits(full[:m.numel]),
                                                                   bits(full_copies[i]))]
    for m, _ in out:
        m.release()
    gather_ok = not bad
    # (2) reduce-scatter of one backward
    ar = opt._arena
    keep = {}
    for i in idx:
        r0, r1, row = ar.rows[i]
        keep[i] = slice(r0 * row, r1 * row)
    exact, absum = _regen_grads(shapes, world, dev, keep, ar.dtype)
    x = torch.zeros(1, device=dev, requires_grad=True)
    opt.zero_grad()
    model(x).sum().backward()
    torch.cuda.synchronize()
    tol = _bf16_sum_tolerance(world) if ar.dtype == torch.bfloat16 else world * 2.0 ** -22
    worst = 0.0
    rs_bad = []
    params = list(model.parameters())
    for i in idx:
        g = params[i].grad
        if g is None:
            rs_bad.append((i, "no grad chunk"))
            continue
        err = (g.float().reshape(-1) - exact[i]).abs()
        bound = tol * absum[i] + 1e-30
        ratio = float((err / bound).max()) if err.numel() else 0.0
        worst = max(worst, ratio)
        if ratio > 1.0:
            rs_bad.append((i, ratio))
    opt.step()  # completes the iteration (a warm-up step)
    torch.cuda.synchronize()
    ok = torch.tensor([1.0 if (gather_ok and not rs_bad) else 0.0], device=red_dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    res = {"gather_bit_exact": gather_ok, "gather_tensors": len(idx),
           "reduce_scatter_max_err_over_bound": worst,
           "reduce_scatter_bound": f"|sum - exact fp32 sum| <= {world} * 2^-8 * sum_r |g_r| "
                                   "(bf16 ring: one rounding per hop)",
           "all_ranks_ok": bool(ok.item() == 1.0)}
    if not gather_ok:
        _fail_check("ZeRO-3 all-gather of layer 1", rank, f"tensors {bad} differ from the full params")
    if rs_bad:
        _fail_check("ZeRO-3 backward reduce-scatter of layer 1", rank, rs_bad)
    if not res["all_ranks_ok"]:
        _fail_check("ZeRO-3 exchange", rank, "another rank failed")
    return res


def _bits(t):
    return t.reshape(-1).view(torch_int_of(t))


def torch_int_of(t):
    import torch

    return {2: torch.int16, 4: torch.int32}[t.element_size()]


def _adam_step1_restated(master, gsum, world, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
    """torch.optim.Adam's first step (adam.py:457-547, fresh state) in fp32 torch ops, in the
    fused kernel's rounding order: g = sum / ws; m = (1-b1)*g (lerp from 0); v = ((1-b2)*g)*g;
    p += (-(lr/bc1) * m) / (sqrt(v)/sqrt(bc2) + eps).  A plain-PyTorch restatement for the
    bench's exchange check (the C oracle stays in tests/)."""
    import math

    import torch

    f = lambda x: torch.tensor(x, dtype=torch.float32, device=master.device)  # noqa: E731
    g = gsum.float() / f(float(world))
    m = f(1.0 - b1) * g
    v = (f(1.0 - b2) * g) * g
    denom = torch.sqrt(v) / f(math.sqrt(1.0 - b2)) + f(eps)
    return master.float() + (f(-(lr / (1.0 - b1))) * m) / denom


def zero12_exchange_check(opt, step, params, shapes, dev, world, rank, red_dev, fatal=True):
    """Before timing at N>1: ONE real engine step on the real arena and communicator, with the
    bench's known per-rank synthetic grads (seed = rank).  Checks, on every rank:
      (1) the reduced gradient of every owned parameter (captured right after the reduce) equals
          the exact fp32 sum of all ranks' grads within the ring bound ws·2^-8·Σ|g_r| (bf16; fp32:
          ws·2^-22·Σ|g_r|);
      (2) the owned parameters after the step equal the plain-PyTorch restatement of Adam's first
          step applied to that reduced gradient, within 1 bf16 ulp (fp32: 1e-6 relative);
      (3) the all-gather / broadcast left every rank with bit-identical parameters (two checksums
          per tensor, MIN == MAX over ranks).
    A failure ends the run (exit 4) naming the rank and tensor — or, with ``fatal=False`` (the
    arena calibration, which can still measure through the other exchange), is returned in the
    result ("all_ranks_ok": False, "failure": ...) after being logged."""
    import numpy as np
    import torch
    import torch.distributed as dist

    eng = opt.engine
    pc = eng.pieces
    # this rank's pieces (param, element range, stream offset): whole parameters under the
    # reference's layout, slices of them under the balanced Layout F of the layout ablation
    own = [(int(i), int(po), int(so), int(n)) for i, po, so, n
           in zip(pc.param, pc.param_off, pc.stream_off, pc.length) if n > 0]
    cap = torch.zeros(max(eng.L, 1), dtype=eng.dtype, device=dev)
    before = {(i, po): params[i].detach().reshape(-1)[po:po + n].clone() for i, po, _, n in own}
    eng.capture_reduced = cap
    step()
    torch.cuda.synchronize()
    eng.capture_reduced = None
    exact, absum = _regen_grads(shapes, world, dev, {i: slice(None) for i, *_ in own}, eng.dtype)
    bf16 = eng.dtype == torch.bfloat16
    tol = _bf16_sum_tolerance(world) if bf16 else world * 2.0 ** -22
    worst_sum, worst_ulp, bad = 0.0, 0, []
    for i, po, so, n in own:
        got = cap[so:so + n]
        ex, ab = exact[i][po:po + n], absum[i][po:po + n]
        ratio = float(((got.float() - ex).abs() / (tol * ab + 1e-30)).max())
        worst_sum = max(worst_sum, ratio)
        if ratio > 1.0:
            bad.append(("reduced grad", i, ratio))
        want = _adam_step1_restated(before[(i, po)], got, world)
        p = params[i].detach().reshape(-1)[po:po + n]
        if bf16:
            d = (_bits(p).int() - _bits(want.to(torch.bfloat16)).int()).abs().max()
            worst_ulp = max(worst_ulp, int(d))
            if int(d) > 1:
                bad.append(("adam update (bf16 ulp)", i, int(d)))
        else:
            r = float((p - want).abs().max() / want.abs().max().clamp_min(1e-30))
            if r > 1e-6:
                bad.append(("adam update (rel)", i, r))
    del cap, before, exact, absum
    sums = []
    for p in params:
        sums += _bit_checksums(p.detach(), dev)
    t = torch.tensor(sums, dtype=torch.int64, device=red_dev)
    lo, hi = t.clone(), t.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    diverged = sorted(set(int(k) // 2 for k in np.nonzero((lo != hi).cpu().numpy())[0]))
    ok = torch.tensor([0.0 if (bad or diverged) else 1.0], device=red_dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    res = {"arena": getattr(eng, "arena_kind", "buckets"), "owned_tensors": len({i for i, *_ in own}),
           "owned_pieces": len(own),
           "reduce_max_err_over_bound": worst_sum,
           "reduce_bound": (f"|sum - exact fp32 sum| <= {world} * 2^-8 * sum_r |g_r| (bf16 ring: one "
                            "rounding per hop)") if bf16 else f"{world} * 2^-22 * sum_r |g_r|",
           "adam_max_bf16_ulp" if bf16 else "adam_rel_tol": worst_ulp if bf16 else 1e-6,
           "params_identical_across_ranks": not diverged, "all_ranks_ok": bool(ok.item() == 1.0)}
    fail = (("ZeRO step exchange", bad[:8]) if bad else
            ("ZeRO step parameter broadcast", f"tensors {diverged[:8]} differ across ranks")
            if diverged else ("ZeRO step exchange", "another rank failed")
            if not res["all_ranks_ok"] else None)
    if fail is not None:
        if fatal:
            _fail_check(fail[0], rank, fail[1])
        log(f"[bench] EXCHANGE CHECK FAILED on rank {rank} ({res['arena']} arena): {fail[0]}: "
            f"{fail[1]} — excluded from the calibration")
        res["failure"] = f"rank {rank}: {fail[0]}: {fail[1]}"[:400]
    return res


def _bit_checksums(t, dev, chunk: int = 1 << 24):
    """Two checksums of a tensor's bits (plain sum, position-weighted sum mod 65521), taken over
    16M-element chunks so the int64 temporaries stay small beside a large arena."""
    import torch

    b = _bits(t).reshape(-1)
    s0 = s1 = 0
    for o in range(0, b.numel(), chunk):
        c = b[o:o + chunk].long()
        s0 += int(c.sum())
        s1 += int((c * torch.arange(o + 1, o + c.numel() + 1, device=dev) % 65521).sum())
    return [s0, s1]


def zero3_mlp_check(opt, model, ref, x, y, step, world, rank, red_dev):
    """N>1 check of the hooked ZeRO-3 iteration before anything is timed: ONE real iteration
    (hooked all-gathers, backward reduce-scatters, update-mode step) must leave every rank's chunk
    equal to the same iteration done unsharded in plain PyTorch (the initial full weights, one
    forward / MSE / backward, torch.optim.Adam) — within 1e-5 relative (fp32; bf16: 2 ulp, i.e.
    2^-7): every rank trains on the same batch (zero3.py:186), so the mean of the reduced
    gradients is this rank's own gradient.  A failure ends the run (exit 4)."""
    import torch
    import torch.distributed as dist

    step()
    torch.cuda.synchronize()
    lin = [m for m in model if isinstance(m, torch.nn.Linear)]
    rp = [torch.nn.Parameter(t) for t in ref]
    h = x
    for k in range(len(lin)):
        h = torch.nn.functional.linear(h, rp[2 * k], rp[2 * k + 1])
        if k < len(lin) - 1:
            h = torch.relu(h)
    torch.nn.functional.mse_loss(h, y).backward()
    if ref[0].dtype != torch.float32:  # bf16 params: the update runs on fp32 masters (as ours does)
        mp = [torch.nn.Parameter(q.detach().float()) for q in rp]
        for a, q in zip(mp, rp):
            a.grad = q.grad.float()
        torch.optim.Adam(mp, lr=1e-3).step()
        for a, q in zip(mp, rp):
            q.data.copy_(a.detach())
    else:
        torch.optim.Adam(rp, lr=1e-3).step()
    torch.cuda.synchronize()
    fp32 = ref[0].dtype == torch.float32
    tol = 1e-5 if fp32 else 2.0 ** -7
    worst, bad = 0.0, []
    for i, p in enumerate(model.parameters()):
        m = opt.param_managers[p]
        want = rp[i].detach()[m.r0:m.r1].float()
        got = p.detach().reshape(want.shape).float()
        e = float((got - want).abs().max() / want.abs().max().clamp_min(1e-30)) if want.numel() else 0.0
        worst = max(worst, e)
        if e > tol:
            bad.append((i, e))
    ok = torch.tensor([0.0 if bad else 1.0], device=red_dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    res = {"what": "one hooked ZeRO-3 iteration vs the same iteration unsharded in plain PyTorch "
                   "(torch.optim.Adam), this rank's chunks", "max_rel_err": worst, "tol": tol,
           "all_ranks_ok": bool(ok.item() == 1.0)}
    if bad:
        _fail_check("ZeRO-3 iteration", rank, f"chunks of params {bad[:8]} off by more than {tol}")
    if not res["all_ranks_ok"]:
        _fail_check("ZeRO-3 iteration", rank, "another rank failed")
    return res


def bench_zero3(args, world, rank, dev, use_nccl):
    """ZeRO-3 (BASELINE.json configs[2]): one step = one training iteration of the reference
    harness loop (zero3.py:171-258: zero_grad → forward → MSE → backward → step) on the
    6×Linear(D,D)+ReLU MLP, with every parameter dim-0 sharded, the hooks' all-gathers grouped per
    module and prefetched on a side stream, the gradients reduce-scattered from backward hooks
    into the grad chunk arena, and update-mode step() = fused Adam on the local chunks.
    value = params / iteration time."""
    import torch
    import torch.distributed as dist

    from zero_amd import zero3
    from zero_amd.shapes import CONFIGS

    D = CONFIGS[args.config][1]()[0][0]
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    layers = []
    for i in range(6):
        layers += [torch.nn.Linear(D, D, device=dev, dtype=dt)] + ([torch.nn.ReLU()] if i < 5 else [])
    model = torch.nn.Sequential(*layers)
    total = sum(p.numel() for p in model.parameters())
    g = torch.Generator(device=dev).manual_seed(42)  # identical data on every rank (zero3.py:186)
    batch = args.batch or 16
    x = torch.randn(batch, D, device=dev, generator=g).to(dt)
    y = torch.randn(batch, D, device=dev, generator=g).to(dt)
    comm, chk = _zero3_comm(args, world, rank, dev)
    kw = {} if comm is None else {"comm": comm}
    ref = [p.detach().clone() for p in model.parameters()] if world > 1 and not args.gather else None
    opt = zero3.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), update=True,
                                 sync=False, gather_dtype=args.gather, bucket_mb=args.bucket_mb or 512.0, **kw)
    zero3.register_zero3_hooks(model, opt.param_managers)

    def step():
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(x), y)
        loss.backward()
        opt.step()

    red_dev = dev if use_nccl else "cpu"
    extra = {"rccl_selfcheck": chk} if chk is not None else {}
    if ref is not None:
        _phase("exchange check (ZeRO-3 training iteration)")
        extra["exchange_check"] = zero3_mlp_check(opt, model, ref, x, y, step, world, rank, red_dev)
        del ref
    _phase("warmup")
    el = _zero3_timed(args, opt, step, dev, world)
    _zero3_report(args, opt, world, rank, red_dev, el, total,
                  f"{args.config} ZeRO-3 training iteration of the reference MLP 6xLinear({D},{D})+ReLU "
                  f"(hooked all-gathers, backward reduce-scatters, update-mode step), batch {batch}",
                  extra)
    _teardown(opt)
    dist.destroy_process_group()


def bench_zero3_paramset(args, world, rank, dev, use_nccl):
    """ZeRO-3 on a synthetic parameter set (BASELINE.json configs[4]: C5 8.03e9 params; C4 also):
    one step = one hooked iteration of zero_amd.paramset.ParamSetModel — per decoder layer an
    all-gather in the forward pre-hook and again in the backward pre-hook, the synthetic full
    gradients (resident in HBM, N(0,1)·1e-3 per rank) reduce-scattered from the backward hooks into
    the grad chunk arena, then zero3.ShardedOptimizer(update=True).step() = fused Adam on the
    chunks.  value = params / iteration time (strong scaling)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from zero_amd import zero3
    from zero_amd.paramset import ParamSetModel, decoder_layer_groups
    from zero_amd.shapes import CONFIGS

    name, shape_fn = CONFIGS[args.config]
    shapes = shape_fn()
    if args.set_layers is not None:  # test-size copy of the set: fewer decoder layers
        from zero_amd import shapes as shp

        shapes = shp.decoder_shapes(args.config, args.set_layers)
        name += f" ({args.set_layers} layers)"
    total = int(sum(int(np.prod(s)) for s in shapes))
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    params = [torch.nn.Parameter(torch.empty(s, dtype=torch.float32, device=dev).normal_(
        0.0, 0.02, generator=gen).to(dt)) for s in shapes]
    gen.manual_seed(1000 * 0 + rank)
    grads = [(torch.empty(s, dtype=torch.float32, device=dev).normal_(generator=gen) * 1e-3).to(dt)
             for s in shapes]
    model = ParamSetModel(params, decoder_layer_groups(len(shapes)))
    model.set_grad_source(grads)
    full_copies = ({i: params[i].detach().clone() for i in model.groups[1]} if world > 1 else None)
    comm, chk = _zero3_comm(args, world, rank, dev)
    if args.simulate_ws > 1:  # DIAGNOSTIC: rank 0 of a simulate_ws-rank job, collectives skipped
        assert world == 1, "--simulate-ws is a single-GPU diagnostic"
        comm = _NoComm(args.simulate_ws)
        sim_ws, real_get = args.simulate_ws, zero3.get
        zero3.get = lambda what, dm=None: {"ws": sim_ws, "rank": 0}.get(what) \
            if what in ("ws", "rank") else real_get(what, dm)
    kw = {} if comm is None else {"comm": comm}
    # the synthetic layers compute nothing, so there is nothing to overlap the collectives with:
    # by default they run on the compute stream itself (no cross-stream ordering)
    opt = zero3.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), update=True,
                                 sync=False, gather_dtype=args.gather, bucket_mb=args.bucket_mb or 512.0,
                                 side_stream=args.z3_stream == "side", **kw)
    zero3.register_zero3_hooks(model, opt.param_managers)
    gather_check = None
    if world > 1:
        _phase("ZeRO-3 gather check")
        gather_check = zero3_gather_check(opt, model, shapes, full_copies, dev, world, rank,
                                          red_dev=dev if use_nccl else "cpu")
        del full_copies
    x = torch.zeros(1, device=dev, requires_grad=True)

    def step():
        opt.zero_grad()
        model(x).sum().backward()
        opt.step()

    _phase("warmup")
    el = _zero3_timed(args, opt, step, dev, world)
    if args.simulate_ws > 1:
        ev, opt.timing_events = opt.timing_events, None
        adam_ms = sum(a.elapsed_time(b) for a, b, _ in ev)
        adam_b = sum(nb for *_, nb in ev)
        if rank == 0:
            print(json.dumps({"diagnostic": f"simulate-ws {args.simulate_ws}: rank-0 compute of the "
                              "hooked ZeRO-3 iteration, collectives skipped (NOT the metric)",
                              "ms_per_step": el / args.steps * 1e3,
                              "adam_ms_per_step": adam_ms / args.steps,
                              "adam_achieved_gbs": adam_b / (adam_ms / 1e3) / 1e9 if adam_ms else 0.0,
                              "chunk_elems": int(opt._arena.ln.sum()), "layers": len(model.layers),
                              "reduce_buckets": opt._reducer.K}), flush=True)
        _teardown(opt)
        dist.destroy_process_group()
        return
    extra = {}
    # the planner's prediction beside the measured iteration
    extra["expected"] = _expected_block(shapes, 3, "chunk", world, 2 if args.dtype == "bf16" else 4,
                                        26 if args.dtype == "bf16" else 28, None, el / args.steps * 1e3)
    if chk is not None:
        extra["rccl_selfcheck"] = chk
    if gather_check is not None:
        extra["exchange_check"] = gather_check
    _zero3_report(args, opt, world, rank, dev if use_nccl else "cpu", el, total,
                  f"{args.config} {name} synthetic parameter set, ZeRO-3 through the hooks: "
                  f"{len(model.layers)} layer modules, per-layer all-gather in forward and backward, "
                  f"backward reduce-scatter of synthetic full grads, fused Adam on the chunks",
                  extra)
    _teardown(opt)
    dist.destroy_process_group()


def _fresh_buffer_gbs(dev, n=16, nbytes=64 << 20):
    """In-place copy-kernel GB/s of n buffers freshly taken from torch's allocator (diagnostic)."""
    import torch

    from zero_amd.kernels import CopySet

    bufs = [torch.empty(nbytes // 4, dtype=torch.float32, device=dev) for _ in range(n)]
    st = torch.cuda.current_stream(dev)
    out = []
    for b in bufs:
        cs = CopySet([b.data_ptr()], [b.data_ptr()], [nbytes])
        cs.run(st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(5):
            cs.run(st)
        e1.record(st)
        e1.synchronize()
        out.append(round(5 * 2 * nbytes / (e0.elapsed_time(e1) / 1e3) / 1e9))
    return out


def bench_train_smollm3(args, world, rank, dev, use_nccl):
    """SmolLM3-3B training (fsdp/train_fsdp.py's loop on random-init weights and synthetic
    tokens): tokens/s over all ranks (per-rank batch fixed → weak scaling) and the reference's
    MFU accounting.  Optimizer: zero2.ShardedOptimizer(AdamW(lr=1e-5), overlap=True) — the FSDP2
    reshard_after_forward=False analogue — or, with --zero 3, zero3.ShardedOptimizer(AdamW,
    update=True) with the gather / release hooks on every module (reshard_after_forward=True,
    train_fsdp.py:92-94)."""
    import torch
    import torch.distributed as dist

    from zero_amd import zero2, zero3
    from zero_amd.training_utils import smollm3 as sm

    cfg = sm.smollm3_config(layers=args.train_layers)
    model = sm.build_model(cfg, dev)
    params = sum(p.numel() for p in model.parameters())
    sim = args.simulate_ws > 1 and args.zero == 3
    if sim:  # DIAGNOSTIC: rank 0 of a simulate_ws-rank job, collectives skipped (buffers untouched)
        assert world == 1, "--simulate-ws is a single-GPU diagnostic"
        sim_ws, real_get = args.simulate_ws, zero3.get
        zero3.get = lambda what, dm=None: {"ws": sim_ws, "rank": 0}.get(what) \
            if what in ("ws", "rank") else real_get(what, dm)
    if args.zero == 3:
        comm, _ = _zero3_comm(args, world, rank, dev)
        if sim:
            comm = _NoComm(args.simulate_ws)
        kw = {} if comm is None else {"comm": comm}
        opt = zero3.ShardedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-5), update=True,
                                     sync=False, bucket_mb=args.bucket_mb or 512.0, **kw)
        # one gather group per decoder layer (FSDP2 fully_shard per block, train_fsdp.py:90-97)
        zero3.register_zero3_hooks(model, opt.param_managers, units=list(model.model.layers),
                                   reshard_after_forward=not args.no_reshard)
    else:
        opt = zero2.ShardedOptimizer(torch.optim.AdamW(model.parameters(), lr=1e-5),
                                     overlap=not args.no_overlap, sync=False,
                                     arena="buckets" if args.arena == "buckets" else "flat")
    batch = args.batch or 1
    g = torch.Generator(device=dev).manual_seed(42 + rank)  # each rank its own data shard
    ids = torch.randint(0, cfg.vocab_size, (batch, args.seq), device=dev, generator=g)
    opt.zero_grad()
    for _ in range(args.warmup):
        sm.train_step(model, opt, ids)
    torch.cuda.synchronize()  # warmup drained first: no collective of ours beside c10d's barrier
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = sm.train_step(model, opt, ids)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    red_dev = dev if use_nccl else "cpu"
    t = torch.tensor([el], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    ms = el / args.steps * 1e3
    tok_s = world * batch * args.seq / (ms / 1e3)
    fpt = sm.model_flops_per_token(cfg, args.seq)
    identical = None
    if world > 1 and args.zero != 3:  # ZeRO-2 broadcasts every update: replicas must agree bit for bit
        sums = []
        for p in model.parameters():
            sums += _bit_checksums(p.detach(), dev)
        lo = torch.tensor(sums, dtype=torch.int64, device=red_dev)
        hi = lo.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        identical = bool(torch.equal(lo, hi))
        if not identical:
            _fail_check("SmolLM3 ZeRO-2 replicas", rank, "parameters differ across ranks after training")
    if os.environ.get("ZERO_AMD_DIAG_BW"):  # diagnostics: streaming GB/s of fresh 64 MB buffers
        print(json.dumps({"diag_fresh_64mb_copy_gbs": _fresh_buffer_gbs(dev),
                          "segments": torch.cuda.memory_stats(dev).get("segment.all.current"),
                          "reserved_gib": torch.cuda.memory_reserved(dev) / (1 << 30)}),
              file=sys.stderr, flush=True)
    if sim:
        rt = opt.runtime
        print(json.dumps({"diagnostic": f"simulate-ws {args.simulate_ws}: rank 0's SmolLM3 ZeRO-3 "
                          "training step with every hook, gather allocation, release and bucket "
                          "launch of a ws-rank job, the collectives themselves skipped (their "
                          "buffers hold whatever memory held: the loss is meaningless; NOT the "
                          "metric)", "ms_per_step": ms, "tokens_per_s_per_rank": tok_s,
                          "gathers_per_step": rt.n_gathers / max(1, args.steps + args.warmup),
                          "reduce_buckets": opt._reducer.K, "seq": args.seq, "batch": batch,
                          "layers": cfg.num_hidden_layers,
                          "gather_throttle_waits": rt.n_throttle_waits,
                          "gather_inflight_limit_gb": (rt.max_inflight_bytes or 0) / 1e9,
                          "allocator": {k: torch.cuda.memory_stats(dev).get(k) for k in (
                              "num_alloc_retries", "num_device_alloc", "num_device_free",
                              "reserved_bytes.all.peak")}}), flush=True)
        _teardown(opt)
        dist.destroy_process_group()
        return None
    if rank == 0:
        print(json.dumps({
            "metric": f"SmolLM3-3B ZeRO-{3 if args.zero == 3 else 2} training throughput "
                      "(SURVEY §8(f) 3; not the headline)",
            "value": tok_s, "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random tokens, random init)",
            "config": {"workload": ("SmolLM3 causal-LM training step, ZeRO-3 AdamW(lr=1e-5), "
                                    "per-layer gathers" + (" (kept through backward: FSDP2 "
                                    "reshard_after_forward=False)" if args.no_reshard else "") +
                                    ", backward reduce-scatters"
                                    if args.zero == 3 else
                                    "SmolLM3 causal-LM training step, ZeRO-2 AdamW(lr=1e-5) "
                                    "backward-overlapped"), "params": int(params),
                       "layers": cfg.num_hidden_layers, "seq_len": args.seq,
                       "global_batch": world * batch, "parallelism": f"dp{world}"},
            "params_identical_across_ranks": identical, "rehearsal": _REHEARSAL[0],
            "mfu_flops_per_token": fpt,
            "tflops_per_gpu": fpt * tok_s / world / 1e12,
            "loss": float(loss.item()),
            "reference_published": "fsdp/train_fsdp.py:85-86: 1849 tok/s (ZeRO-3) / 3000 tok/s "
                                   "(ZeRO-2), 2x A100-80GB, different harness",
        }), flush=True)
    _teardown(opt)
    dist.destroy_process_group()


def main(argv=None):
    """The benchmark; returns rank 0's JSON object (None on other ranks) after printing it."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default: ~4 s of timed GPU work at N=1 (C4), long enough for an outside utilisation sampler
    ap.add_argument("--steps", type=int, default=None,
                    help="default 1500 at N=1 (~20 s of GPU time at C4, so an outside utilisation "
                         "sampler sees the timed region), 300 at N>1 (exchange-bound steps are "
                         "longer); --train: 4")
    ap.add_argument("--warmup", type=int, default=None, help="default 5 (--train: 2)")
    ap.add_argument("--config", default="C4", choices=["C2", "C3", "C4", "C5"])
    ap.add_argument("--zero", type=int, default=2, choices=[1, 2, 3],
                    help="3 on C2/C3 = a ZeRO-3 training iteration (hooked forward/backward + "
                         "update-mode step) of the MLP (BASELINE.json configs[2]); 3 on C4/C5 = the "
                         "parameter-set ZeRO-3 step (configs[4]): dim-0-chunk (Layout Z) buckets, "
                         "RS of the full grads -> fused Adam on the chunks -> AG of the updated "
                         "chunks, i.e. one parameter gather per iteration")
    ap.add_argument("--batch", type=int, default=None,
                    help="ZeRO-3 MLP batch (default 16, zero1.py:144) / --train batch (default 1)")
    ap.add_argument("--z3-stream", default="single", choices=["single", "side"],
                    help="--zero 3 on the C4/C5 parameter sets: collectives on the compute stream "
                         "(single: the synthetic layers compute nothing to overlap with) or on a "
                         "side stream with prefetch (side: what a model with compute uses)")
    ap.add_argument("--gather", default=None, choices=["fp8"],
                    help="--zero 3: all-gather parameters as row-scaled fp8 E4M3 (SURVEY §8(f) 4)")
    ap.add_argument("--train", default=None, choices=["smollm3"],
                    help="SURVEY §8(f) 3: SmolLM3-3B training step (forward + backward + ZeRO-2 "
                         "AdamW, backward-overlapped) in tokens/s; not the headline metric")
    ap.add_argument("--seq", type=int, default=8192, help="--train sequence length "
                    "(fsdp/train_fsdp.py:44: 8192)")
    ap.add_argument("--train-layers", type=int, default=None, help="--train: fewer decoder layers")
    ap.add_argument("--no-reshard", action="store_true",
                    help="--train --zero 3: keep gathered parameters from forward through backward "
                         "(FSDP2 reshard_after_forward=False, the reference's 'ZeRO-2' run)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="--train --zero 1/2: reduce in step() instead of from backward hooks")
    ap.add_argument("--set-layers", type=int, default=None,
                    help="C4/C5: a copy of the parameter set with fewer decoder layers (tests and "
                         "N=8 rehearsals on one GPU; not the metric)")
    ap.add_argument("--layout", default="reference", choices=["reference", "flat", "chunk"],
                    help="optimizer-shard layout: reference = whole params by index (zero1.py:55-62, "
                         "ZeRO-1/2); chunk = dim-0 chunks of every param (zero3.py:107-108, forced "
                         "by --zero 3 on C4/C5); flat = balanced 1/N slices (ablation)")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="MiB per bucket / flat round (default: the optimizer's own — 1024 for the "
                         "flat arena, 256 for the bucket arena, 512 for ZeRO-3 reduce buckets)")
    ap.add_argument("--arena", default="auto", choices=["auto", "flat", "buckets"],
                    help="ZeRO-1/2 exchange at N>1: flat = params and grads are views of one "
                         "owner-major arena, grouped reduce / broadcast rounds, no pack / unpack; "
                         "buckets = rank-major bucket arena, pack / RS / AG / unpack; auto = "
                         "calibrate both after their exchange checks and time the faster")
    ap.add_argument("--buckets", default="ragged", choices=["ragged", "padded"],
                    help="ragged: equal-count RS/AG over the shortest stream + one grouped "
                         "reduce/broadcast per owner for the rest; padded: every window padded")
    ap.add_argument("--no-comm-sweep", action="store_true",
                    help="skip the RS/AG bus-bandwidth sweep (N>1, after the timed region)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"],
                    help="parameter dtype; default fp32 for --zero 3 on the C2/C3 MLP (the "
                         "reference MLP is fp32, zero1.py:237-249), bf16 otherwise (C4/C5 sets)")
    ap.add_argument("--master", default="split", choices=["split", "fp32"],
                    help="bf16 params: the fp32 master as the bf16 param + an int16 residual "
                         "(split, 26 B/element per update) or a separate fp32 array (28 B)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-master-line", action="store_true",
                    help="N=1 bf16: skip timing the same step with the exact fp32 master beside "
                         "the split-master headline")
    ap.add_argument("--cpu-sample", type=int, default=256 << 20)
    ap.add_argument("--grad-handoff", default="auto", choices=["auto", "views", "default"],
                    help="ZeRO-1/2 parameter sets: how the timed step gets its gradients. views: "
                         "zero_grad(set_to_none=False) once, grads written into the arena's grad "
                         "views (resident, as a backward into the views leaves them); default: "
                         "every step opt.zero_grad() (grads None) then fresh gradient tensors "
                         "(two alternating sets), as backward leaves them after the drop-in's "
                         "default zero_grad() (zero2.py:138-139); auto: default at N=1, views "
                         "at N>1 (where the hooks land backward's grads into the views)")
    ap.add_argument("--no-layout-ablation", action="store_true",
                    help="N>1 ZeRO-2: skip timing the balanced Layout F beside the reference "
                         "layout's headline (after everything else)")
    ap.add_argument("--no-default-leg", action="store_true",
                    help="skip timing the other hand-off beside the headline's")
    ap.add_argument("--simulate-ws", type=int, default=0,
                    help="DIAGNOSTIC (N=1 only): run the ws>1 bucket path of rank 0 of a ws-rank job "
                         "with the collectives replaced by no-ops, to time pack / Adam / unpack "
                         "at that layout; prints a diagnostic line, not the metric")
    ap.add_argument("--share-gpu", action="store_true",
                    help="REHEARSAL on a one-GPU box: all ranks on one device, real RCCL between "
                         "them over its socket transport (per-rank NCCL_HOSTID); the exchange "
                         "checks and calibration run for real, the timings mean nothing")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "c10d", "gloo-staged"],
                    help="rccl: the library's own RCCL communicator; c10d: the same RCCL through "
                         "torch.distributed (A/B); gloo-staged = TEST ONLY (tests/_gloo_comm.py): "
                         "N ranks sharing one GPU")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC HBM-bytes summary for the roofline 'traffic' field (default: the "
                         "profiles/*_pmc.json whose config matches this run)")
    ap.add_argument("--watchdog-s", type=float, default=None,
                    help="end the process (exit 3) with every thread's stack and rank 0's partial "
                         "JSON line if the run has not finished after this many seconds (a "
                         "collective that never completes); default: what is left of "
                         f"{WATCHDOG_BUDGET_S:.0f} s since process start, inside the driver's 600 s; "
                         "0 disables it")
    args = ap.parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N ranks here, one process per
        # GPU, the way the reference always launches (modal_utils.py:115-120, torchrun) — before
        # anything touches the GPU, as a child process (never an exec)
        rc = _launch_ranks(sys.argv[1:] if argv is None else list(argv), args.gpus)
        if _IN_PROCESS[0]:
            return rc
        sys.exit(rc)
    if env_world is not None and int(env_world) != args.gpus:
        log(f"[bench] WORLD_SIZE={env_world} but --gpus {args.gpus}: refusing to time a job whose "
            "rank count is not the one asked for")
        if _IN_PROCESS[0]:
            raise SystemExit(2)
        sys.exit(2)
    if args.steps is None:
        args.steps = 4 if args.train else (1500 if int(os.environ.get("WORLD_SIZE", "1")) == 1 else 300)
    if args.warmup is None:
        args.warmup = 2 if args.train else 5
    if args.dtype is None:
        args.dtype = "fp32" if (args.zero == 3 and args.config in ("C2", "C3")) else "bf16"
    _DEADLINE[0] = None
    _SKIPPED.clear()
    if not _IN_PROCESS[0]:
        _OUT_FD[0] = os.dup(1)
        if env_world is not None and int(env_world) > 1:
            _install_term_handler()
        wd = watchdog_seconds(args.watchdog_s)
        _start_watchdog(wd)
        if wd > 0:
            _DEADLINE[0] = time.monotonic() + wd
    _PARTIAL.clear()
    _EMITTED[0] = False
    _PARTIAL["config"] = {"workload": args.config, "zero": args.zero, "arena_requested": args.arena,
                          "parallelism": f"dp{int(env_world or 1)}",
                          "train": args.train, "dtype": args.dtype}
    try:
        return _main(args)
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 — reported (partial line) and fatal
        import traceback

        log(f"[bench] FAILED in phase '{_PHASE[0]}': {type(e).__name__}: {e}")
        traceback.print_exc(file=sys.stderr)
        if _IN_PROCESS[0]:
            raise
        _emit_partial(f"{type(e).__name__} in phase '{_PHASE[0]}'", f"{type(e).__name__}: {e}")
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(7)


def _main(args):
    """main() after the arguments: the run itself (rank 0's JSON object, None on other ranks)."""

    import numpy as np
    import torch
    import torch.distributed as dist

    from zero_amd import zero1, zero2
    from zero_amd.shapes import CONFIGS

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.comm == "gloo-staged":  # test-only: every rank shares the box's GPUs round-robin
        local = local % torch.cuda.device_count()
    if args.share_gpu and world > 1:
        # rehearsal on a one-GPU box: every rank on the same device, each one a separate "node"
        # to RCCL (its own NCCL_HOSTID), so the real RCCL collectives run between the ranks
        # through RCCL's socket transport over loopback; read before RCCL's first init
        local = local % torch.cuda.device_count()
        os.environ["NCCL_HOSTID"] = f"zs-share-gpu-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
        # ranks probing placements on one device at once would race for its memory
        os.environ.setdefault("ZERO_AMD_PROBE_TRIES", "1")
        _REHEARSAL[0] = ("share-gpu: every rank on ONE device, RCCL between them over its socket "
                         "transport (checks are real, timings are not xGMI's)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    use_nccl = world > 1 and args.comm in ("rccl", "c10d")
    with _stdout_to_stderr():  # gloo prints a connection banner on stdout: keep ONE JSON line there
        dist.init_process_group("nccl" if use_nccl else "gloo", rank=rank, world_size=world,
                                device_id=dev if use_nccl else None)

    if args.train == "smollm3":
        return bench_train_smollm3(args, world, rank, dev, use_nccl)
    if args.zero == 3 and args.config in ("C2", "C3"):
        return bench_zero3(args, world, rank, dev, use_nccl)
    if args.zero == 3:  # parameter-set ZeRO-3 (BASELINE.json configs[4]) through the hooks
        return bench_zero3_paramset(args, world, rank, dev, use_nccl)
    name, shape_fn = CONFIGS[args.config]
    shapes = shape_fn()
    if args.set_layers is not None:  # test-size copy of the set: fewer decoder layers
        from zero_amd.shapes import decoder_shapes

        shapes = decoder_shapes(args.config, args.set_layers)
        name += f" ({args.set_layers} layers)"
    total = int(sum(int(np.prod(s)) for s in shapes))
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    params = []
    for s in shapes:
        t = torch.empty(s, dtype=torch.float32, device=dev).normal_(0.0, 0.02, generator=gen).to(dt)
        params.append(torch.nn.Parameter(t))
    gen.manual_seed(1000 * 0 + rank)
    grads = []
    for s in shapes:
        grads.append((torch.empty(s, dtype=torch.float32, device=dev).normal_(generator=gen) * 1e-3).to(dt))
    torch.cuda.synchronize()
    mod = zero1 if args.zero == 1 else zero2
    kw = {}
    comm_used = None
    if args.comm == "gloo-staged" and world > 1:
        sys.path.insert(0, str(REPO / "tests"))
        from _gloo_comm import GlooStagedComm

        kw["comm"] = GlooStagedComm()
        comm_used = "gloo-staged (test only)"
    elif world > 1:
        from zero_amd.comm import C10dComm, RcclComm

        if args.comm == "c10d":
            kw["comm"], comm_used = C10dComm(), "c10d"
        else:
            kw["comm"], comm_used = _product_comm(rank), "rccl"
    if args.simulate_ws > 1:
        assert world == 1, "--simulate-ws is a single-GPU diagnostic"
        kw["comm"] = _NoComm(args.simulate_ws)
        import zero_amd._sharded as sh
        sim_ws, real_get = args.simulate_ws, sh.get
        sh.get = lambda what, dm=None: {"ws": sim_ws, "rank": 0}.get(what) if what in ("ws", "rank") \
            else real_get(what, dm)
    selfcheck = None
    if world > 1 and args.comm in ("rccl", "c10d"):
        _phase("communicator self-check")
        selfcheck = _checked_comm(kw, world, rank, dev)
        comm_used = selfcheck.pop("comm_used", comm_used)
        _PARTIAL["rccl_selfcheck"] = selfcheck
    red_dev = dev if use_nccl else "cpu"
    multi = world > 1 or args.simulate_ws > 1
    arenas = ["flat", "buckets"] if (args.arena == "auto" and multi) else \
        [args.arena if args.arena != "auto" else "flat"]

    grad_sets = [grads]
    # what the timed step's gradients look like.  auto: what a training loop calling the drop-in's
    # default opt.zero_grad() / backward() / step() hands step() — at ws = 1 backward's fresh
    # tensors (read in place), at ws > 1 the arena's grad views (the hooks land backward's fresh
    # gradients there during backward); a hand-assigned fresh set at ws > 1 ("default") adds the
    # landing copy to step() that a real backward overlaps
    handoff_used = args.grad_handoff
    if handoff_used == "auto":
        handoff_used = "default" if not multi else "views"

    def default_step(o):
        """The drop-in's default hand-off: opt.zero_grad() sets every grad to None, then the
        step gets fresh gradient tensors (at N = 1 two sets, alternating, so every step sees new
        addresses, as backward's allocations may be: Adam reads them in place; at N > 1 one set —
        step() copies it into the arena whatever its address, and ranks sharing one GPU in a
        rehearsal have no room for a second)."""
        if len(grad_sets) == 1 and not multi:
            grad_sets.append([g.clone() for g in grads])
        k = [0]

        def st():
            o.zero_grad()
            for p, g in zip(params, grad_sets[k[0] % len(grad_sets)]):
                p.grad = g
            k[0] += 1
            o.step()
        return st

    def views_step(o):
        """Gradients resident in HBM where a backward puts them: the flat arena's grad views (at
        ws > 1 the drop-in's hooks land backward's fresh gradients there and adopt the views);
        the bucket arena takes the caller's tensors every step."""
        if getattr(o.engine, "arena_kind", None) == "flat":
            o.zero_grad(set_to_none=False)
            with torch.no_grad():
                for p, g in zip(params, grads):
                    p.grad.copy_(g)

            def st():
                o.step()
        else:
            def st():
                for p, g in zip(params, grads):
                    p.grad = g
                o.step()
        return st

    def build(arena, master=None, handoff=None):
        o = mod.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), layout=args.layout,
                                 bucket_mb=args.bucket_mb, sync=False, buckets=args.buckets,
                                 master=master or args.master, arena=arena, **kw)
        if o.engine is None:
            o._build_engine()  # (the bucket engine is otherwise built by the first step)
        return o, (default_step if (handoff or handoff_used) == "default" else views_step)(o)

    def timed(st, n):
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            st()
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()) / n * 1e3

    exchange_check, arena_ab, arena_cal = {}, {}, {}
    _PARTIAL.update(exchange_check_all_arenas=exchange_check, arena_calibration=arena_cal,
                    arena_calibration_ms_per_step=arena_ab)
    opt = step = None
    for arena in arenas:
        if opt is not None:
            _teardown_engine(opt)
            opt = step = None
        opt, step = build(arena)
        kind = getattr(opt.engine, "arena_kind", "buckets")
        if world > 1:
            _phase(f"exchange check ({kind} arena)")
            exchange_check[kind] = zero12_exchange_check(opt, step, params, shapes, dev, world, rank,
                                                         red_dev, fatal=len(arenas) == 1)
            if not exchange_check[kind]["all_ranks_ok"]:
                continue  # never time an exchange that computed a wrong step
        if len(arenas) > 1:  # calibrate: the same step through each exchange, the faster is timed
            _phase(f"arena calibration ({kind})")
            for _ in range(args.warmup):
                step()
            n_cal = max(3, min(args.steps, 5))
            opt.engine.comm_events = [] if world > 1 else None
            arena_ab[kind] = timed(step, n_cal)
            cal_ev, opt.engine.comm_events = opt.engine.comm_events, None
            # what the exchange itself moved, per arena (HIP events on the comm stream): the first
            # multi-GPU line says WHY one arena won, not only which step was shorter
            arena_cal[kind] = {"ms_per_step": arena_ab[kind], "steps": n_cal}
            if world > 1:
                cs = collective_summary(cal_ev, n_cal, world, red_dev)
                arena_cal[kind].update(
                    busbw_gbs=cs["busbw_gbs"], frac_of_peer_links=cs["frac_of_peer_links"],
                    frac_of_aggregate=cs["frac_of_aggregate"], comm_ms_per_step=cs["ms_per_step"],
                    collectives={k: v for k, v in cs.items() if isinstance(v, dict)})
    if len(arenas) > 1:
        if not arena_ab:
            _fail_check("ZeRO step exchange", rank, "every arena failed its exchange check")
        best = min(arena_ab, key=arena_ab.get)
        if best != arenas[-1] or kind != best:
            _teardown_engine(opt)
            opt, step = build(best)
    arena_used = getattr(opt.engine, "arena_kind", "buckets") if multi else "none (ws=1: no exchange)"
    lib_auto = None
    if world > 1 and len(arenas) > 1 and args.layout == "reference" and args.comm in ("rccl", "c10d"):
        # what the library's own arena="auto" (a sample exchange at construction) would pick on
        # this interconnect, beside the full-step calibration above that chose the timed arena
        from zero_amd._sharded import calibrate_arena

        _phase("library arena=auto calibration")
        lib_auto = calibrate_arena(opt)
        lib_auto["agrees_with_full_step"] = lib_auto["chosen"] == arena_used
        _PARTIAL["arena_calibration_library_auto"] = lib_auto

    _phase("warmup")
    for _ in range(args.warmup):
        step()
    eng = opt.engine
    eng.timing_events = []
    eng.comm_events = [] if world > 1 or args.simulate_ws > 1 else None
    eng.copy_events = [] if world > 1 or args.simulate_ws > 1 else None
    torch.cuda.synchronize()  # warmup drained first: no collective of ours beside c10d's barrier
    dist.barrier()
    torch.cuda.synchronize()
    _phase("timed steps")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    host_ms = (time.perf_counter() - t0) / args.steps * 1e3  # enqueue only: nothing waits
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    eng_events = eng.timing_events
    eng.timing_events = None
    comm_events, eng.comm_events = eng.comm_events, None
    copy_events, eng.copy_events = eng.copy_events, None
    headline_inplace = int(getattr(eng, "inplace_reads", 0))  # (before the other leg's steps)
    el_t = torch.tensor([el], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    ms = el / args.steps * 1e3
    _PARTIAL["timed_before_failure"] = {"ms_per_step": ms, "value": total / (ms / 1e3),
                                        "steps": args.steps, "arena": getattr(eng, "arena_kind", None)}

    # Adam roofline: algorithmic bytes / kernel time, per launch, from HIP events on the launch stream
    adam_ms = sum(a.elapsed_time(b) for a, b, _ in eng_events)
    adam_bytes = sum(nb for _, _, nb in eng_events)
    launches = len(eng_events)
    achieved = adam_bytes / (adam_ms / 1e3) / 1e9 if adam_ms > 0 else 0.0
    stats = torch.tensor([achieved, adam_ms / max(launches, 1), adam_bytes / max(launches, 1)],
                         dtype=torch.float64, device=red_dev)
    if world > 1:  # report the slowest rank's Adam
        dist.all_reduce(stats, op=dist.ReduceOp.MIN)
    achieved = float(stats[0])
    hb = torch.tensor([adam_bytes / args.steps], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(hb, op=dist.ReduceOp.MAX)
    headline_adam_gb = float(hb.item()) / 1e9  # the slowest rank's Adam bytes per step
    want = {"workload": args.config, "zero": args.zero, "param_dtype": args.dtype,
            "layout": args.layout, "n_gpus": world}
    if args.dtype == "bf16":
        want["master"] = args.master
    if world > 1 or args.simulate_ws > 1:
        want["arena"] = arena_used
    if handoff_used == "default":  # Adam reads backward's tensors in place: its own PMC summary
        want["grad_handoff"] = "default"
    traffic, traffic_src, traffic_note = match_traffic(want, float(stats[2]), args.traffic_json)

    placement = {"state": eng.placement, "arena": getattr(eng, "arena_placement", None),
                 "grads": getattr(eng, "grad_placement", None),
                 "reduced": getattr(eng, "reduced_placement", None)}
    bucket_mb, n_buckets = opt._bucket_bytes / (1 << 20), eng.K
    other_leg = None
    if not args.no_default_leg and args.simulate_ws <= 1 and \
            leg_fits("other hand-off", (args.warmup + min(args.steps, 300)) * ms / 1e3 * 1.2):
        # the same optimizer through the other gradient hand-off, beside the headline's
        other = "views" if handoff_used == "default" else "default"
        _phase(f"{other} hand-off leg")
        ostep = (default_step if other == "default" else views_step)(opt)
        for _ in range(args.warmup):
            ostep()
        eng.timing_events = []
        n_o = min(args.steps, 300)
        ms_o = timed(ostep, n_o)
        ev_o, eng.timing_events = eng.timing_events, None
        a_ms = sum(a.elapsed_time(b) for a, b, _ in ev_o)
        a_b = sum(nb for *_, nb in ev_o)
        gbs = a_b / (a_ms / 1e3) / 1e9 if a_ms > 0 else 0.0
        other_leg = {
            "handoff": other, "ms_per_step": ms_o, "value": total / (ms_o / 1e3), "steps": n_o,
            "vs_headline": ms_o / ms, "adam_achieved_gbs": gbs, "adam_frac": gbs / HBM_PEAK_GBS,
            "adam_launches_per_step": len(ev_o) / n_o,
            "grads_read_in_place": int(getattr(eng, "inplace_reads", 0)) if other == "default" else 0,
            "what": HANDOFF_WHAT[other]}
        torch.cuda.synchronize()
    fp32_master = None
    if (world == 1 and args.simulate_ws <= 1 and args.dtype == "bf16" and args.master == "split"
            and not args.no_fp32_master_line
            and leg_fits("fp32-master", 30.0 + (args.warmup + min(args.steps, 300)) * ms / 1e3 * 1.2)):
        # the same step with the exact fp32 master (28 B/elem) beside the split-master headline
        # (26 B/elem, an exact tie stored 1 ulp toward zero: DESIGN §2)
        _phase("fp32-master comparison")
        eng = None  # (its placement is kept above) so the split state can be freed
        _teardown_engine(opt)
        opt, step = build(arena_used if multi else "flat", master="fp32")
        for _ in range(args.warmup):
            step()
        opt.engine.timing_events = []
        n_fp = min(args.steps, 300)
        ms_fp = timed(step, n_fp)
        ev_fp, opt.engine.timing_events = opt.engine.timing_events, None
        a_ms = sum(a.elapsed_time(b) for a, b, _ in ev_fp)
        a_b = sum(nb for *_, nb in ev_fp)
        gbs = a_b / (a_ms / 1e3) / 1e9 if a_ms > 0 else 0.0
        fp32_master = {"ms_per_step": ms_fp, "value": total / (ms_fp / 1e3), "steps": n_fp,
                       "adam_achieved_gbs": gbs, "adam_frac": gbs / HBM_PEAK_GBS,
                       "alg_bytes_per_launch": a_b / max(len(ev_fp), 1),
                       "state_placement": opt.engine.placement,
                       "what": "the same step with master='fp32' (exact fp32 master array, "
                               "28 B/elem) instead of the split master"}
    copy_kernels = copy_summary(copy_events, args.steps, world, red_dev) if copy_events else None
    # step roofline: this rank's HBM bytes (Adam + pack + unpack) at 8 TB/s plus its bus bytes at
    # the 7-link xGMI aggregate, no overlap credit; the slowest rank's sum vs the measured step
    hbm_b = (adam_bytes + sum(b for *_, b in (copy_events or []))) / args.steps
    bus_b = sum(ev[-1] for ev in (comm_events or [])) / args.steps
    ideal = torch.tensor([hbm_b / (HBM_PEAK_GBS * 1e9) * 1e3 + bus_b / (peer_link_peak_gbs(world) * 1e9) * 1e3,
                          hbm_b, bus_b], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(ideal, op=dist.ReduceOp.MAX)
    step_roofline = {"ideal_ms": float(ideal[0]), "frac": float(ideal[0]) / ms,
                     "hbm_gb_per_step": float(ideal[1]) / 1e9, "bus_gb_per_step": float(ideal[2]) / 1e9,
                     "model": "per rank: (Adam + pack + unpack algorithmic bytes) / 8 TB/s + bus bytes "
                              "/ (min(N-1, 7) x 153 GB/s: the direct links to its peers), no overlap "
                              "credit; max over ranks"}
    collectives = None
    if world > 1:
        collectives = collective_summary(comm_events, args.steps, world, red_dev)
        if args.comm in ("rccl", "c10d") and not args.no_comm_sweep and leg_fits("bucket-size sweep", 15.0):
            _phase("bucket-size sweep")
            sweep_buf = eng.arena if getattr(eng, "arena", None) is not None else eng.R
            collectives["sweep"] = comm_sweep(opt._comm, sweep_buf, world, red_dev)

    layout_ablation = None
    if (world > 1 and args.zero == 2 and args.layout == "reference" and args.simulate_ws <= 1
            and not args.no_layout_ablation
            and leg_fits("layout ablation", 30.0 + (2 + args.warmup + min(args.steps, 50)) * ms / 1e3 * 1.5)):
        # what the reference's whole-parameter ownership costs: the same step with
        # the balanced Layout F in the flat arena — its own exchange check, then timed — after
        # everything of the headline's (its memory is freed first)
        _phase("layout ablation (balanced Layout F, flat arena)")
        eng = None
        _teardown_engine(opt)
        opt = None
        o_f = mod.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), layout="flat",
                                   bucket_mb=args.bucket_mb, sync=False, master=args.master,
                                   arena="flat", **kw)
        st_f = views_step(o_f)
        chk_f = zero12_exchange_check(o_f, st_f, params, shapes, dev, world, rank, red_dev,
                                      fatal=False)
        layout_ablation = {"layout": "flat (Layout F: balanced contiguous 1/N slices)",
                           "arena": "flat", "exchange_check": chk_f}
        if chk_f["all_ranks_ok"]:
            for _ in range(args.warmup):
                st_f()
            o_f.engine.timing_events = []
            n_f = min(args.steps, 50)
            ms_f = timed(st_f, n_f)
            ev_f, o_f.engine.timing_events = o_f.engine.timing_events, None
            a_ms = sum(a.elapsed_time(b) for a, b, _ in ev_f)
            a_b = sum(nb for *_, nb in ev_f)
            t = torch.tensor([a_b / n_f, a_b / (a_ms / 1e3) / 1e9 if a_ms > 0 else 0.0],
                             dtype=torch.float64, device=red_dev)
            mx, mn = t.clone(), t.clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(mn, op=dist.ReduceOp.MIN)
            layout_ablation.update(
                ms_per_step=ms_f, steps=n_f, vs_headline=ms_f / ms,
                max_rank_adam_gb_per_step=float(mx[0]) / 1e9,
                headline_max_rank_adam_gb_per_step=headline_adam_gb,
                min_rank_adam_achieved_gbs=float(mn[1]),
                rounds=o_f.engine.K)
        layout_ablation["expected"] = layout_costs(shapes, args.zero, world,
                                                   es=2 if args.dtype == "bf16" else 4,
                                                   bpe=26 if (args.dtype == "bf16"
                                                              and args.master == "split") else 28,
                                                   bucket_mb=bucket_mb)
        _PARTIAL["layout_ablation"] = layout_ablation
        opt = o_f  # (torn down at the end like the headline's)

    if rank == 0 and args.simulate_ws > 1:
        print(json.dumps({"diagnostic": f"simulate-ws {args.simulate_ws}: rank-0 compute of the "
                          "bucket path, collectives skipped (NOT the metric)",
                          "ms_per_step": ms, "adam_achieved_gbs": achieved,
                          "adam_ms_per_step": adam_ms / args.steps, "buckets": eng.K,
                          "window_elems": eng.W, "stream_elems": eng.L,
                          "host_enqueue_ms_per_step": host_ms,
                          "copy_kernels": copy_kernels}), flush=True)
        _teardown(opt)
        dist.destroy_process_group()
        return
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": total / (ms / 1e3),
            "unit": "params/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            # the arithmetic: bf16 params and grads, Adam in fp32 (master, exp_avg, exp_avg_sq)
            "dtype": ("bf16 params/grads, fp32 Adam" if args.dtype == "bf16" else "fp32"),
            "data": "synthetic",
            "config": {
                "workload": (f"{args.config} {name} synthetic parameter set: ZeRO-{args.zero} "
                             f"ShardedOptimizer(Adam lr=1e-3).step(), grads resident in HBM "
                             f"({handoff_used} hand-off)"),
                "params": total, "tensors": len(shapes),
                "param_dtype": args.dtype, "grad_dtype": args.dtype,
                "state_dtype": ("fp32 exp_avg, exp_avg_sq; fp32 master held as the bf16 param + "
                                "an int16 residual (include/zero_amd.h ZS_BF16_SPLIT)")
                if args.dtype == "bf16" and args.master == "split"
                else "fp32 (master, exp_avg, exp_avg_sq)",
                "master": args.master if args.dtype == "bf16" else "param",
                "zero": args.zero, "layout": args.layout,
                "bucket_mb": bucket_mb,
                "bucket_mode": args.buckets,
                "buckets": n_buckets, "parallelism": f"dp{world}", "comm": comm_used,
                "arena": arena_used,
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": "adam_segments_kernel",
                "avg_launch_ms": float(stats[1]), "alg_bytes_per_launch": float(stats[2]),
                "launches_per_step": launches / args.steps,
                "traffic_source": traffic_src, "traffic_note": traffic_note,
                "placement_dependence": _placement_dependence(placement),
            },
        }
        out["step_roofline"] = step_roofline
        if args.simulate_ws <= 1 and args.layout == "reference":
            out["expected"] = _expected_block(shapes, args.zero, arena_used if multi else "flat",
                                              world, es=2 if args.dtype == "bf16" else 4,
                                              bpe=26 if (args.dtype == "bf16" and args.master == "split")
                                              else 28, bucket_mb=bucket_mb, measured_ms=ms)
        out["placement"] = placement
        if fp32_master is not None:
            out["fp32_master_ms_per_step"] = fp32_master["ms_per_step"]
            out["fp32_master"] = fp32_master
        out["grad_handoff"] = {"handoff": handoff_used, "what": HANDOFF_WHAT[handoff_used]}
        if handoff_used == "default":
            out["grad_handoff"]["grads_read_in_place"] = headline_inplace
            out["default_zero_grad_ms_per_step"] = ms
        if other_leg is not None:
            out[f"{other_leg['handoff']}_handoff_ms_per_step"] = other_leg["ms_per_step"]
            out[f"{other_leg['handoff']}_handoff"] = other_leg
            if other_leg["handoff"] == "default":
                out["default_zero_grad_ms_per_step"] = other_leg["ms_per_step"]
        if selfcheck is not None:
            out["rccl_selfcheck"] = selfcheck
        if exchange_check:
            out["exchange_check"] = exchange_check[arena_used] if arena_used in exchange_check \
                else exchange_check
            out["exchange_check_all_arenas"] = exchange_check
        if arena_ab:
            out["arena_calibration_ms_per_step"] = arena_ab
            out["arena_calibration"] = arena_cal
        if lib_auto is not None:
            out["arena_calibration_library_auto"] = lib_auto
        if layout_ablation is not None:
            out["layout_ablation"] = layout_ablation
        out["host_enqueue_ms_per_step"] = host_ms  # rank 0's Python + launch time per step
        if handoff_used == "default" and not multi:
            out["host_enqueue_note"] = (
                "default hand-off: the host enqueues ~200 steps ahead at ~0.4 ms each, then each "
                "step waits for the GPU, so over a long run this average tends to the GPU's step "
                "time; it is not host work.  The queued depth is bounded by the kernel-argument "
                "bytes pending: each step's two gradient-pointer patch launches carry 1,808-B "
                "arguments; the same step without them (unchanged pointers) or with two "
                "small-argument launches instead never waits within 400 steps, the views step plus "
                "two 1,808-B launches waits from step 174 (profiles/r06_handoff_host.json); "
                "standalone, launches queue until ~3.7-4 MB of arguments are pending "
                "(profiles/r06_queue_depth_probe.jsonl)")
        if collectives is not None:
            out["collectives"] = collectives
        if copy_kernels is not None:
            out["copy_kernels"] = copy_kernels
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(shapes, args.cpu_sample, variant=args.zero)
            out["cpu_oracle_adam"] = cpu_oracle_adam(
                shapes, args.cpu_sample, split=args.dtype == "bf16" and args.master == "split")
        if _REHEARSAL[0]:
            out["rehearsal"] = _REHEARSAL[0]
        if _SKIPPED:
            out["skipped_legs"] = dict(_SKIPPED)
        print(json.dumps(out), flush=True)
    _teardown(opt)
    dist.destroy_process_group()
    return out if rank == 0 else None


if __name__ == "__main__":
    main()
