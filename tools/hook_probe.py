"""Which part of the ZeRO-3 module hooks slows a ws=1 training step (tools/sm3_variant.py showed:
no hooks 378 ms, forward hooks only 505 ms, ZeRO-2 417 ms for SmolLM3-3B)?

A 36-layer bf16 MLP stack (Linear 2048->8192, SiLU, Linear 8192->2048, residual add), 8192 tokens,
forward + backward timed with events, under forward pre/post hooks that do
  none   — nothing;
  swap   — param.data = another view of the same storage and back (what materialize/release do at
           ws=1);
  xs     — a cross-stream round trip through a side stream (event record -> side waits -> side
           records -> current waits), as the gather runtime does per module;
  xs_hp  — the same with a high-priority side stream (comm_stream);
  both   — swap + xs_hp.
Prints one JSON line per (variant, repeat)."""
from __future__ import annotations

import json
import sys


def main():
    import torch

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    L, H, F, T = int(sys.argv[1]) if len(sys.argv) > 1 else 36, 2048, 8192, 8192
    blocks = torch.nn.ModuleList()
    for _ in range(L):
        blocks.append(torch.nn.Sequential(torch.nn.Linear(H, F, bias=False), torch.nn.SiLU(),
                                          torch.nn.Linear(F, H, bias=False)))
    blocks = blocks.to(dev, torch.bfloat16)
    x0 = torch.randn(T, H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    hp = torch.cuda.Stream(device=dev, priority=-1)
    lp = torch.cuda.Stream(device=dev)
    alt = {}
    for m in blocks.modules():
        for name, p in m.named_parameters(recurse=False):
            flat = p.data.reshape(-1)
            alt[p] = (p.data, flat.view(p.shape))  # two views of one storage

    def xs(side):
        cur = torch.cuda.current_stream(dev)
        e = torch.cuda.Event()
        e.record(cur)
        side.wait_event(e)
        e2 = torch.cuda.Event()
        e2.record(side)
        cur.wait_event(e2)

    def make(variant):
        def pre(mod, *a):
            if variant in ("xs", "xs_hp", "both"):
                xs(lp if variant == "xs" else hp)
            if variant in ("swap", "both"):
                for p in mod.parameters(recurse=False):
                    p.data = alt[p][1]

        def post(mod, *a):
            if variant in ("swap", "both"):
                for p in mod.parameters(recurse=False):
                    p.data = alt[p][0]
        return pre, post

    def step():
        h = x0
        for b in blocks:
            h = h + b(h)
        h.float().square().mean().backward()
        for b in blocks:
            for p in b.parameters():
                p.grad = None
        x0.grad = None

    for rep in range(2):
        for variant in ("none", "swap", "xs", "xs_hp", "both"):
            handles = []
            if variant != "none":
                pre, post = make(variant)
                for m in blocks.modules():
                    if any(True for _ in m.parameters(recurse=False)):
                        handles.append(m.register_forward_pre_hook(pre))
                        handles.append(m.register_forward_hook(post))
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                step()
            e1.record()
            e1.synchronize()
            print(json.dumps({"variant": variant, "rep": rep, "ms_per_step": e0.elapsed_time(e1) / 5}),
                  flush=True)
            for h in handles:
                h.remove()


if __name__ == "__main__":
    main()
