"""Where the host CPU of the hooked ZeRO-3 iteration goes, per thread.

Rank 0 of a simulated ws-rank job on the configs[4] parameter set (C5: 34 layer modules, 291
tensors; collectives no-ops, so the GPU runs only Adam): wall time and process CPU time per
iteration, split by thread — the main thread (forward hooks, step), autograd's device thread
(backward hooks: gathers, releases, reduce-scatter bucket launches) and every other thread of the
process (HIP runtime) — from psutil's per-thread CPU times around blocks of iterations.  Blocks
alternate nothing: this is a breakdown, not an A/B (tools/z3_host_ab.py is the A/B).

Usage: python tools/z3_host_threads.py [--config C5] [--ws 8] [--iters 20] [--blocks 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--ws", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--wave", type=int, default=None, help="gather wave (default: the library's)")
    ap.add_argument("--bucket-mb", type=float, default=None, help="reduce-scatter bucket MB")
    ap.add_argument("--stream-sync", default=None, choices=["flag", "event"],
                    help="cross-stream ordering of the side stream (default: the library's)")
    ap.add_argument("--single", action="store_true",
                    help="collectives on the compute stream (side_stream=False)")
    ap.add_argument("--no-events", action="store_true",
                    help="DIAGNOSTIC: the ordered library calls and the consumer's stream wait "
                         "become no-ops (no HIP event record / wait at all): how much of the "
                         "runtime threads' CPU the stream ordering costs")
    ap.add_argument("--device-flags", action="store_true",
                    help="stream-flag words in device memory (zs_tune sync_host_flags 0: every wait "
                         "enqueued) instead of pinned host memory")
    ap.add_argument("--no-record-stream", action="store_true",
                    help="DIAGNOSTIC (unsafe: blocks may be reused while another stream reads them; "
                         "the simulated iteration checks no data): Tensor.record_stream a no-op — "
                         "how much CPU the caching allocator's cross-stream events cost")
    ap.add_argument("--write-value", action="store_true",
                    help="flag records through hipStreamWriteValue64 (zs_tune sync_write_kernel 0) "
                         "instead of the library's one-wave store kernel")
    ap.add_argument("--alternate-write", action="store_true",
                    help="interleaved A/B in one process: even blocks record flags with the store "
                         "kernel, odd blocks with hipStreamWriteValue64")
    ap.add_argument("--alternate", default=None,
                    help="interleaved A/B of any zs_tune knob: even blocks KNOB=1, odd blocks KNOB=0")
    ap.add_argument("--stall-ms", type=float, default=0.0,
                    help="per-iteration host times; an iteration longer than this dumps every "
                         "thread's Python stack to stderr (first 4 only)")
    args = ap.parse_args()

    import faulthandler

    import psutil
    import torch
    import torch.distributed as dist

    import bench
    from zero_amd import zero3
    from zero_amd.paramset import ParamSetModel, decoder_layer_groups
    from zero_amd.shapes import CONFIGS

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    shapes = CONFIGS[args.config][1]()
    ws = args.ws
    gen = torch.Generator(device=dev).manual_seed(0)
    params = [torch.nn.Parameter(torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(
        0.0, 0.02, generator=gen)) for s in shapes]
    grads = [torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(0.0, 1e-3, generator=gen)
             for s in shapes]
    model = ParamSetModel(params, decoder_layer_groups(len(shapes)))
    model.set_grad_source(grads)
    real_get = zero3.get
    zero3.get = lambda what, dm=None: {"ws": ws, "rank": 0}.get(what) if what in ("ws", "rank") \
        else real_get(what, dm)
    comm = bench._NoComm(ws)
    if args.no_record_stream:
        torch.Tensor.record_stream = lambda self, stream: None
    if args.write_value:
        from zero_amd import _lib

        _lib.call("zs_tune", b"sync_write_kernel", 0, None)
    if args.device_flags:
        from zero_amd import _lib

        _lib.call("zs_tune", b"sync_host_flags", 0, None)
    if args.no_events:
        from zero_amd import _lib

        comm._ordered = lambda name, dtype: (lambda after, ready, stream, done: None)
        _lib.lib.zs_stream_wait_event = lambda *a: 0
        _lib.lib.zs_sync_wait = lambda *a: 0
        from zero_amd.comm import Sync

        Sync.record = Sync.wait = lambda self, h: None
    kw = {}
    if args.stream_sync is not None:
        kw["stream_sync"] = args.stream_sync
    if args.wave is not None:
        kw["gather_wave"] = args.wave
    if args.bucket_mb is not None:
        kw["bucket_mb"] = args.bucket_mb
    if args.single:
        kw["side_stream"] = False
    opt = zero3.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), update=True,
                                 sync=False, comm=comm, **kw)
    zero3.register_zero3_hooks(model, opt.param_managers)
    x = torch.zeros(1, device=dev, requires_grad=True)
    bwd_tid = set()
    params[0].register_post_accumulate_grad_hook(lambda p: bwd_tid.add(threading.get_native_id()))

    def step():
        opt.zero_grad()
        model(x).sum().backward()
        opt.step()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    proc = psutil.Process()
    main_tid = threading.get_native_id()

    def snap():
        return {t.id: t.user_time + t.system_time for t in proc.threads()}

    rows = []
    dumps = [0]
    from zero_amd import _lib as zlib
    for b in range(args.blocks):
        if args.alternate_write:
            zlib.call("zs_tune", b"sync_write_kernel", 1 - b % 2, None)
        if args.alternate:
            zlib.call("zs_tune", args.alternate.encode(), 1 - b % 2, None)
        torch.cuda.synchronize()
        s0, w0, c0 = snap(), time.perf_counter(), time.process_time()
        its = []
        for _ in range(args.iters):
            t0 = time.perf_counter()
            if args.stall_ms and dumps[0] < 4:
                faulthandler.dump_traceback_later(args.stall_ms / 1e3, exit=False)
            step()
            if args.stall_ms and dumps[0] < 4:
                faulthandler.cancel_dump_traceback_later()
            its.append((time.perf_counter() - t0) * 1e3)
            if args.stall_ms and its[-1] > args.stall_ms:
                dumps[0] += 1
        t_sync = time.perf_counter()
        torch.cuda.synchronize()
        sync_ms = (time.perf_counter() - t_sync) * 1e3
        w, c, s1 = time.perf_counter() - w0, time.process_time() - c0, snap()
        d = {tid: s1[tid] - s0.get(tid, 0.0) for tid in s1}
        n = args.iters
        main = d.get(main_tid, 0.0)
        bwd = sum(d.get(t, 0.0) for t in bwd_tid if t != main_tid)
        other = sum(v for t, v in d.items() if t != main_tid and t not in bwd_tid)
        busy = sorted(((round(v / n * 1e3, 3), t) for t, v in d.items()
                       if t != main_tid and t not in bwd_tid and v > 0), reverse=True)[:4]
        names = {}
        for t in d:
            try:
                names[t] = Path(f"/proc/self/task/{t}/comm").read_text().strip()
            except OSError:
                names[t] = "?"
        rows.append({"block": b, **({"flag_record": ("store kernel", "hipStreamWriteValue64")[b % 2]}
                                    if args.alternate_write else {}),
                     **({args.alternate: 1 - b % 2} if args.alternate else {}), "wall_ms": round(w / n * 1e3, 3), "cpu_ms": round(c / n * 1e3, 3),
                     "main_thread_ms": round(main / n * 1e3, 3),
                     "autograd_thread_ms": round(bwd / n * 1e3, 3),
                     "other_threads_ms": round(other / n * 1e3, 3),
                     "busiest_other_threads_ms": {f"{names.get(t, '?')}[{t}]": v for v, t in busy},
                     "host_iter_ms_max": round(max(its), 2),
                     "host_iter_ms_median": round(sorted(its)[len(its) // 2], 3),
                     "host_iters_over_20ms": sum(1 for v in its if v > 20), "final_sync_ms": round(sync_ms, 2)})
        print(json.dumps(rows[-1]), flush=True)
    med = lambda k: sorted(r[k] for r in rows)[len(rows) // 2]  # noqa: E731
    summ = {"config": args.config, "simulated_ws": ws, "iters_per_block": args.iters,
            "no_events": args.no_events, "side_stream": not args.single, "gather_wave": opt.runtime.wave,
            "stream_sync": "flag" if opt.runtime.sync_kind == 1 else "event",
            "device_flags": args.device_flags, "no_record_stream": args.no_record_stream,
            "flag_record": "hipStreamWriteValue64" if args.write_value else "store kernel",
            "bucket_mb": args.bucket_mb,
            "autograd_thread_is_main": bool(bwd_tid and bwd_tid <= {main_tid}),
            "median": {k: med(k) for k in ("wall_ms", "cpu_ms", "main_thread_ms",
                                           "autograd_thread_ms", "other_threads_ms")},
            "gathers_per_iteration": 2 * len(model.layers), "reduce_buckets": opt._reducer.K,
            "blocks": rows}
    if args.alternate:
        for j in (0, 1):
            sub = rows[j::2]
            summ[f"median_{args.alternate}={1 - j}"] = {
                k: sorted(r[k] for r in sub)[len(sub) // 2]
                for k in ("wall_ms", "cpu_ms", "main_thread_ms", "autograd_thread_ms", "other_threads_ms")}
    if args.alternate_write:
        for j, name in enumerate(("store kernel", "hipStreamWriteValue64")):
            sub = rows[j::2]
            summ["median_" + name.replace(" ", "_")] = {
                k: sorted(r[k] for r in sub)[len(sub) // 2]
                for k in ("wall_ms", "cpu_ms", "main_thread_ms", "autograd_thread_ms", "other_threads_ms")}
    print(json.dumps({k: v for k, v in summ.items() if k != "blocks"}), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(summ, indent=1) + "\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
