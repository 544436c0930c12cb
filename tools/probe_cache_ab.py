"""Do the placement probe's slow candidates come from torch's cached blocks?

bench.py builds the C4 set (bf16 params and grads, each made from an fp32 temporary that goes back
to torch's cache), then the optimizer probes 6-GB arena candidates: on several boxes the first
four were slow (5.4-5.5 TB/s) and the fifth fast (6.3).  This replays that allocation sequence and
probes candidates (a) as the engine does, (b) after torch.cuda.empty_cache(), in separate
processes (argv[1] = "cache" | "empty"), printing each candidate's in-place copy GB/s.

    python tools/probe_cache_ab.py cache|empty
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))


def main():
    import torch

    from zero_amd.kernels import CopySet
    from zero_amd.shapes import CONFIGS

    mode = sys.argv[1]
    dev = torch.device("cuda:0")
    _, shape_fn = CONFIGS["C4"]
    shapes = shape_fn()
    gen = torch.Generator(device=dev).manual_seed(0)
    params = [torch.empty(s, dtype=torch.float32, device=dev).normal_(generator=gen).to(torch.bfloat16)
              for s in shapes]
    grads = [torch.empty(s, dtype=torch.float32, device=dev).normal_(generator=gen).to(torch.bfloat16)
             for s in shapes]
    torch.cuda.synchronize()
    if mode == "empty":
        torch.cuda.empty_cache()
    n = sum(p.numel() for p in params)
    nbytes = n * 2 // 256 * 256
    st = torch.cuda.current_stream(dev)
    held, out = [], []
    for k in range(8):
        buf = torch.zeros(nbytes // 2, dtype=torch.bfloat16, device=dev)
        cs = CopySet([buf.data_ptr()], [buf.data_ptr()], [nbytes])
        cs.run(st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            cs.run(st)
        e1.record(st)
        e1.synchronize()
        out.append(round(3 * 2 * nbytes / (e0.elapsed_time(e1) / 1e3) / 1e9, 1))
        held.append(buf)
    print(json.dumps({"mode": mode, "candidate_gbs": out,
                      "reserved_gib": round(torch.cuda.memory_reserved(dev) / (1 << 30), 1)}), flush=True)
    del params, grads


if __name__ == "__main__":
    main()
