"""Host-time A/B of the hooked ZeRO-3 iteration: an earlier round's ZeRO-3 runtime
(zero_amd/zero3.py at that round's commit, loaded as a module of the zero_amd package) against the
current one, in ONE
process, alternating blocks of iterations, each on its own copy of the configs[4] parameter set as
rank 0 of a simulated ws-rank job (collectives no-ops, so the GPU runs only Adam and the rest is
host time).  Wall time per iteration and process CPU time (all threads: the backward hooks run on
autograd's device thread) per block — the box's host speed drifts by 30 % over minutes, so only
the interleaved comparison means anything.

Usage: python tools/z3_host_ab.py [--config C5] [--ws 8] [--iters 20] [--blocks 6]
       [--baseline none|r02|r03] [--events] [--single] [--no-hostext] [--no-counting]
       (extra variants of the current runtime; --no-counting: the per-parameter Python
       post-accumulate hooks instead of the C++ gradient counters, round 6)
The baseline module is ``git show <rev>:distributed-training-sandbox_amd/zero_amd/zero3.py`` (r02:
1653aab, r03: 3d19026 — the runtimes profiles/r03_z3_host_ab*.json and r04_z3_host_ab.json compare),
written to tools/_baselines/ (git-ignored, but not gpurun-ignored, so it travels to the GPU box,
which has no git history; delete it after the A/B):
run ``python tools/z3_host_ab.py --baseline r03 --extract-only`` here before the gpurun call.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))
sys.path.insert(0, str(REPO))
BASELINE_REVS = {"r02": "1653aab", "r03": "3d19026", "r06a": "994a673"}
ZERO3_PATH = "distributed-training-sandbox_amd/zero_amd/zero3.py"


def baseline_file(tag: str) -> Path:
    """tools/_baselines/_zero3_<tag>.py, extracted from git history when it is not there yet."""
    import subprocess

    out = REPO / "tools" / "_baselines" / f"_zero3_{tag}.py"
    if not out.exists():
        src = subprocess.run(["git", "-C", str(REPO), "show", f"{BASELINE_REVS[tag]}:{ZERO3_PATH}"],
                             check=True, capture_output=True, text=True).stdout
        out.parent.mkdir(exist_ok=True)
        out.write_text(f"# {ZERO3_PATH} at {BASELINE_REVS[tag]} ({tag}); extracted by "
                       "tools/z3_host_ab.py, not part of the product\n" + src)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--ws", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--baseline", default="none", choices=["none"] + sorted(BASELINE_REVS))
    ap.add_argument("--extract-only", action="store_true",
                    help="write the baseline module under tools/_baselines/ and exit (no GPU)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--events", action="store_true",
                    help="also time the current runtime with stream_sync='event'")
    ap.add_argument("--single", action="store_true",
                    help="also time the current runtime with side_stream=False")
    ap.add_argument("--no-hostext", action="store_true",
                    help="also time the current runtime without the C++ install / release")
    ap.add_argument("--no-counting", action="store_true",
                    help="also time the current runtime with per-parameter Python post-accumulate "
                         "hooks instead of the C++ gradient counters")
    ap.add_argument("--no-gather-fast", action="store_true",
                    help="also time the current runtime with the gathers issued and consumed in "
                         "Python instead of the host extension's GatherFast / consume (round 6)")
    ap.add_argument("--no-reduce-fast", action="store_true",
                    help="also time the current runtime with the gradient buckets launched in "
                         "Python instead of the host extension's ReduceFast (round 6)")
    args = ap.parse_args()
    path = baseline_file(args.baseline) if args.baseline != "none" else None
    if args.extract_only:
        print(path)
        return

    import torch
    import torch.distributed as dist

    import bench
    import zero_amd
    from zero_amd import zero3 as z3_new
    from zero_amd.paramset import ParamSetModel, decoder_layer_groups
    from zero_amd.shapes import CONFIGS

    base = {"r02": "round2", "r03": "round3"}.get(args.baseline, args.baseline)
    z3_old = None
    if path is not None:
        spec = importlib.util.spec_from_file_location(f"zero_amd._zero3_{args.baseline}", path)
        z3_old = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = z3_old
        spec.loader.exec_module(z3_old)
        assert z3_old.__package__ == zero_amd.__name__

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench._free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    shapes = CONFIGS[args.config][1]()
    ws = args.ws

    def build(mod, seed, **okw):
        gen = torch.Generator(device=dev).manual_seed(seed)
        params = [torch.nn.Parameter(torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(
            0.0, 0.02, generator=gen)) for s in shapes]
        grads = [torch.empty(s, device=dev, dtype=torch.bfloat16).normal_(0.0, 1e-3, generator=gen)
                 for s in shapes]
        model = ParamSetModel(params, decoder_layer_groups(len(shapes)))
        model.set_grad_source(grads)
        real_get = mod.get
        mod.get = lambda what, dm=None: {"ws": ws, "rank": 0}.get(what) if what in ("ws", "rank") \
            else real_get(what, dm)
        use_hostext = okw.pop("use_hostext", True)
        gather_fast = okw.pop("gather_fast", True)
        reduce_fast = okw.pop("reduce_fast", True)
        counting = okw.pop("counting", True)
        saved = getattr(mod, "HOSTEXT_COUNTING", None)
        if saved is not None:
            mod.HOSTEXT_COUNTING = counting
        try:
            opt = mod.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), update=True,
                                       sync=False, comm=bench._NoComm(ws), **okw)
            if hasattr(opt, "runtime") and opt.runtime is not None:
                opt.runtime.use_hostext = use_hostext
                if hasattr(opt.runtime, "use_gather_fast"):
                    opt.runtime.use_gather_fast = gather_fast
            red = getattr(opt, "_reducer", None)
            if red is not None and hasattr(red, "use_reduce_fast"):
                red.use_reduce_fast = reduce_fast
            mod.register_zero3_hooks(model, opt.param_managers)
        finally:
            if saved is not None:
                mod.HOSTEXT_COUNTING = saved
        x = torch.zeros(1, device=dev, requires_grad=True)

        def step():
            opt.zero_grad()
            model(x).sum().backward()
            opt.step()
        return step

    variants = {base: build(z3_old, 0)} if z3_old is not None else {}
    variants["current"] = build(z3_new, 0)
    if args.no_counting:  # the current runtime with per-parameter Python post-accumulate hooks
        variants["current_no_counting"] = build(z3_new, 0, counting=False)
    if args.events:  # the current runtime ordered by HIP events instead of stream flags
        variants["current_events"] = build(z3_new, 0, stream_sync="event")
    if args.single:  # the current runtime with its collectives on the compute stream
        variants["current_single_stream"] = build(z3_new, 0, side_stream=False)
    if args.no_gather_fast:  # the current runtime's gathers issued / consumed in Python
        variants["current_no_gather_fast"] = build(z3_new, 0, gather_fast=False)
    if args.no_reduce_fast:  # ... and its gradient buckets launched in Python
        variants["current_no_reduce_fast"] = build(z3_new, 0, reduce_fast=False)
    if args.no_gather_fast and args.no_reduce_fast:
        variants["current_neither_fast"] = build(z3_new, 0, gather_fast=False, reduce_fast=False)
    if args.no_hostext:  # the current runtime installing / releasing per parameter in Python
        variants["current_no_hostext"] = build(z3_new, 0, use_hostext=False)
        if args.single:
            variants["current_single_stream_no_hostext"] = build(z3_new, 0, side_stream=False,
                                                                 use_hostext=False)
    for st in variants.values():
        for _ in range(args.warmup):
            st()
    torch.cuda.synchronize()
    rows = []
    for b in range(args.blocks):
        names = list(variants)
        for name in (names if b % 2 == 0 else names[::-1]):
            st = variants[name]
            torch.cuda.synchronize()
            w0, c0 = time.perf_counter(), time.process_time()
            for _ in range(args.iters):
                st()
            torch.cuda.synchronize()
            w, c = time.perf_counter() - w0, time.process_time() - c0
            rows.append({"block": b, "variant": name, "wall_ms": round(w / args.iters * 1e3, 3),
                         "cpu_ms": round(c / args.iters * 1e3, 3)})
            print(json.dumps(rows[-1]), flush=True)
    summ = {}
    for name in variants:
        ws_ = sorted(r["wall_ms"] for r in rows if r["variant"] == name)
        cs_ = sorted(r["cpu_ms"] for r in rows if r["variant"] == name)
        summ[name] = {"wall_ms_median": ws_[len(ws_) // 2], "wall_ms_min": ws_[0],
                      "cpu_ms_median": cs_[len(cs_) // 2], "cpu_ms_min": cs_[0]}
    res = {"config": args.config, "simulated_ws": ws, "iters_per_block": args.iters,
           "baseline": base, "summary": summ}
    print(json.dumps(res), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(dict(res, blocks=rows), indent=1) + "\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
