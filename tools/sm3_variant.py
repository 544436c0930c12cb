"""Diagnostic: bench.py --train smollm3 --zero 3 with parts of the ZeRO-3 machinery switched off,
to find which one makes the ws=1 step's kernels slower than ZeRO-2's.

    python tools/sm3_variant.py <variant> [bench args...]

variants: none (as is) | nohooks (no module hooks) | nobwdhooks (forward hooks only) |
          nogradhooks (no post-accumulate-grad hooks: grads collected at step()) |
          nooverlap (ZeRO-2: no backward-overlapped reduce hooks)."""
from __future__ import annotations

import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))


def main():
    variant, rest = sys.argv[1], sys.argv[2:]
    import torch

    from zero_amd import zero3

    if variant == "nohooks":
        zero3.register_zero3_hooks = lambda *a, **k: []
    elif variant == "nobwdhooks":
        real = zero3.register_zero3_hooks

        def fwd_only(*a, **k):
            pre, post = torch.nn.Module.register_full_backward_pre_hook, torch.nn.Module.register_full_backward_hook
            torch.nn.Module.register_full_backward_pre_hook = lambda self, h: None
            torch.nn.Module.register_full_backward_hook = lambda self, h: None
            try:
                return [h for h in real(*a, **k) if h is not None]
            finally:
                torch.nn.Module.register_full_backward_pre_hook = pre
                torch.nn.Module.register_full_backward_hook = post
        zero3.register_zero3_hooks = fwd_only
    elif variant == "nogradhooks":
        zero3._GradReducer.register_hooks = lambda self: []
    elif variant == "nooverlap":  # ZeRO-2 without the backward-overlapped reduce hooks
        from zero_amd import zero2

        real_init = zero2.ShardedOptimizer.__init__

        def init(self, *a, **k):
            k["overlap"] = False
            real_init(self, *a, **k)
        zero2.ShardedOptimizer.__init__ = init
    elif variant != "none":
        raise SystemExit(f"unknown variant {variant}")
    import json
    import time

    from zero_amd.training_utils import smollm3 as sm

    log = []

    def timed_step(model, optimizer, input_ids):
        """train_step with HIP events and host clocks at the phase boundaries."""
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        h = [time.perf_counter()]
        ev[0].record()
        loss = model(input_ids=input_ids, labels=input_ids).loss
        ev[1].record()
        h.append(time.perf_counter())
        loss.backward()
        ev[2].record()
        h.append(time.perf_counter())
        optimizer.step()
        optimizer.zero_grad()
        ev[3].record()
        h.append(time.perf_counter())
        log.append((ev, h))
        return loss

    sm.train_step = timed_step
    if os.environ.get("SYNC_DEBUG"):  # report host-synchronising torch calls, with their stacks
        import traceback
        import warnings

        seen = set()

        def show(message, category, filename, lineno, file=None, line=None):
            key = (filename, lineno)
            if key in seen:
                return
            seen.add(key)
            print("SYNC:", message, file=sys.stderr)
            traceback.print_stack(limit=12, file=sys.stderr)

        warnings.showwarning = show
        warnings.simplefilter("always")
        torch.cuda.set_sync_debug_mode(1)
    import bench

    sys.argv = ["bench.py"] + rest
    try:
        bench.main()
    finally:
        torch.cuda.synchronize()
        for ev, h in log[-3:]:
            print(json.dumps({"gpu_ms": [round(ev[i].elapsed_time(ev[i + 1]), 2) for i in range(3)],
                              "host_ms": [round((h[i + 1] - h[i]) * 1e3, 2) for i in range(3)]}),
                  file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
