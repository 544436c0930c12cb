"""The reference's experiment drivers, on the MI355X ZeRO drop-ins.

``train`` is the loop of zero1.py:111-200 / zero2.py:142-230 / zero3.py:171-258 (identical data on
every rank, batch 16, one warm-up step then 20 timed steps, MSE loss, peak memory per step, the
``record_function`` ranges "data_generation" / "zero_grad" / "forward" / "backward" /
"optimizer_step_total", and the step / communication time summary); ``run`` is ``test_zeroN()``
(zero1.py:203-320): the 6×Linear(10000,10000)+ReLU model trained with plain ``torch.optim.Adam``
and then with the variant's ``ShardedOptimizer``, each under an optional rank-0 torch.profiler
with the reference's schedule, and the peak-memory comparison.

    python -m zero_amd.harness --zero 2             # one GPU
    torchrun --nproc-per-node 8 -m zero_amd.harness --zero 2

Differences: the process group is whatever ``torchrun`` set up ("nccl" = RCCL; one GPU also works
without a launcher), and ``--width`` / ``--steps`` shrink the experiment.
"""
from __future__ import annotations

import argparse
import os
from pathlib import Path

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.profiler import ProfilerActivity, profile, record_function, schedule

from .training_utils import get, print_memory_stats, set_seed


def make_model(width: int, device, layers: int = 6) -> nn.Sequential:
    """zero1.py:237-249: Linear(width, width) blocks with ReLU in between."""
    mods = []
    for i in range(layers):
        mods.append(nn.Linear(width, width))
        if i < layers - 1:
            mods.append(nn.ReLU())
    return nn.Sequential(*mods).to(device)


def train(model, optimizer, device, is_sharded=False, profiler_context=None, *, width=10_000,
          batch_size=16, num_steps=20, verbose=True):
    """zero2.py:142-230.  Returns (model, optimizer, peak memory in MB)."""
    rank = get("rank")
    with record_function("data_generation"):
        x = torch.randn(batch_size, width, device=device)
        y = torch.randn(batch_size, width, device=device)

    optimizer.zero_grad()  # warm-up step (zero2.py:152-158)
    nn.functional.mse_loss(model(x), y).backward()
    optimizer.step()
    torch.cuda.synchronize()
    if is_sharded:
        optimizer.communication_time = 0.0
        optimizer.step_time = 0.0
    if rank == 0 and verbose:
        print_memory_stats("Initial state", model, optimizer, rank, device)
    dist.barrier()

    peak = []
    for i in range(num_steps):
        torch.cuda.reset_peak_memory_stats(device)
        with record_function("zero_grad"):
            optimizer.zero_grad()
        with record_function("forward"):
            loss = nn.functional.mse_loss(model(x), y)
        if rank == 0 and i == 0 and verbose:
            print(f"\nStep {i} memory:")
            print(f"Before backward: {torch.cuda.memory_allocated(device) / 1024**2:.2f} MB")
        with record_function("backward"):
            loss.backward()
            torch.cuda.synchronize()
        if rank == 0 and i == 0 and verbose:
            gm = sum(p.grad.numel() * p.grad.element_size() / 1024**2
                     for p in model.parameters() if p.grad is not None)
            print(f"Gradient memory after backward: {gm:.2f} MB")
        with record_function("optimizer_step_total"):
            optimizer.step()
        if profiler_context:
            profiler_context.step()
        peak.append(torch.cuda.max_memory_allocated(device) / 1024**2)
        if rank == 0 and i == 0 and verbose:
            print(f"Peak memory this step: {peak[-1]:.2f} MB")
        dist.barrier()

    if rank == 0 and verbose:
        print(f"\nFinal peak memory: {max(peak):.2f} MB")
    if is_sharded and rank == 0 and verbose:
        st = optimizer.step_time / num_steps
        ct = optimizer.communication_time / num_steps
        print("\nTiming and Communication Stats:")
        print("-" * 40)
        print(f"Average step time: {st:.3f}s")
        print(f"Average communication time: {ct:.3f}s")
        print(f"Average compute time: {st - ct:.3f}s")
        print(f"Communication overhead: {(ct / st) * 100 if st > 0 else 0.0:.1f}%")
    return model, optimizer, max(peak)


def _profiler(trace_dir: Path, name: str):
    """The reference's rank-0 profiler (zero2.py:246-262)."""
    return profile(
        activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
        schedule=schedule(skip_first=5, wait=1, warmup=2, active=5, repeat=1),
        on_trace_ready=torch.profiler.tensorboard_trace_handler(str(trace_dir / name)),
        record_shapes=True, profile_memory=True, with_stack=True, with_flops=True)


def run(variant: int, *, width: int = 10_000, num_steps: int = 20, trace_dir=None,
        verbose: bool = True):
    """test_zero{1,2,3}() (zero2.py:233-360).  Returns (peak MB plain Adam, peak MB sharded)."""
    from . import zero1, zero2, zero3

    own_pg = not dist.is_initialized()
    if own_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl")
    rank = get("rank")
    device = torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', rank))}")
    torch.cuda.set_device(device)
    set_seed(42)
    trace = Path(trace_dir) if trace_dir else None
    if trace is not None:
        trace.mkdir(parents=True, exist_ok=True)
    tag = {1: "zero1", 2: "zero2", 3: "zero3"}[variant]
    try:
        if verbose:
            print(f"\nGPU {rank} - Testing with regular Adam:")
        torch.cuda.reset_peak_memory_stats()
        model = make_model(width, device)
        opt = torch.optim.Adam(model.parameters(), lr=0.001)
        prof = _profiler(trace, "regular_adam") if (trace is not None and rank == 0) else None
        if prof:
            prof.__enter__()
        model, opt, peak_adam = train(model, opt, device, profiler_context=prof, width=width,
                                      num_steps=num_steps, verbose=verbose)
        if prof:
            prof.__exit__(None, None, None)
        del model, opt
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        dist.barrier()

        if verbose:
            print(f"\nGPU {rank} - Testing with Sharded Adam:")
        model = make_model(width, device)
        base = torch.optim.Adam(model.parameters(), lr=0.001)
        if variant == 3:
            sharded = zero3.ShardedOptimizer(base)
            zero3.register_zero3_hooks(model, sharded.param_managers)
        else:
            sharded = (zero1 if variant == 1 else zero2).ShardedOptimizer(base)
        prof = _profiler(trace, f"{tag}_adam") if (trace is not None and rank == 0) else None
        if prof:
            prof.__enter__()
        model, sharded, peak_z = train(model, sharded, device, is_sharded=True, profiler_context=prof,
                                       width=width, num_steps=num_steps, verbose=verbose)
        if prof:
            prof.__exit__(None, None, None)
        if rank == 0 and verbose:
            print("\nMemory Usage Summary:")
            print("-" * 40)
            print(f"Peak memory with regular Adam: {peak_adam:.2f} MB")
            print(f"Peak memory with ZeRO-{variant}: {peak_z:.2f} MB")
            print(f"Memory reduction: {peak_adam - peak_z:.2f} MB "
                  f"({(peak_adam - peak_z) / peak_adam * 100:.2f}%)")
        return peak_adam, peak_z
    finally:
        if own_pg:
            dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--zero", type=int, default=2, choices=[1, 2, 3])
    ap.add_argument("--width", type=int, default=10_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--trace-dir", default=os.environ.get("TRACE_DIR"))
    a = ap.parse_args(argv)
    run(a.zero, width=a.width, num_steps=a.steps, trace_dir=a.trace_dir)


if __name__ == "__main__":
    main()
