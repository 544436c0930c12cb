"""Dev tool: how much does WHERE the optimizer state lands change the C4 Adam launch?
One process; the model's bf16 params and grads are allocated as bench.py does; then, in turn,
the fp32 master / exp_avg / exp_avg_sq are (a) three separate allocations, (b) one allocation,
(c) one allocation made before any model tensor existed (kept from the start); each timed over
10 launches, two rounds.  Prints ms and GB/s per variant.
"""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))

from zero_amd.kernels import AdamSet, adam_hparams  # noqa: E402
from zero_amd.plan import Plan  # noqa: E402
from zero_amd.shapes import smollm3_3b_shapes  # noqa: E402
from zero_amd._lib import ZS_BF16  # noqa: E402


def timed(rows, st, hp):
    a = AdamSet(rows, ZS_BF16)
    a.run(hp, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(10):
        a.run(hp, st)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    return ms, a.bytes / ms / 1e6


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    shapes = smollm3_3b_shapes()
    numels = [int(np.prod(s)) for s in shapes]
    plan = Plan(numels, 1, 0, "reference")
    pc = plan.pieces(0)
    L = plan.stream_len(0)
    early = torch.zeros(3 * L, dtype=torch.float32, device=dev)  # (c): before the model exists
    g = torch.Generator(device=dev).manual_seed(0)
    params, grads = [], []
    for s in shapes:  # exactly bench.py's construction (fp32 temporaries included)
        params.append(torch.empty(s, dtype=torch.float32, device=dev).normal_(0.0, 0.02, generator=g)
                      .to(torch.bfloat16))
    for s in shapes:
        grads.append((torch.empty(s, dtype=torch.float32, device=dev).normal_(generator=g) * 1e-3)
                     .to(torch.bfloat16))
    torch.cuda.synchronize()
    hp = adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, 1)
    st = torch.cuda.current_stream()
    gp = np.array([grads[i].data_ptr() for i in pc.param], np.uint64)
    pp = np.array([params[i].data_ptr() for i in pc.param], np.uint64)
    so = pc.stream_off.astype(np.uint64)

    def rows_for(mb, vb, xb):
        r = np.zeros((len(pc.param), 9), np.uint64)
        mst = np.uint64(xb) + so * np.uint64(4)
        r[:, 0], r[:, 1], r[:, 2], r[:, 3] = gp, mst, mst, pp
        r[:, 4] = np.uint64(mb) + so * np.uint64(4)
        r[:, 5] = np.uint64(vb) + so * np.uint64(4)
        r[:, 8] = pc.length.astype(np.uint64)
        return r

    for rnd in range(2):
        sep = [torch.zeros(L, dtype=torch.float32, device=dev) for _ in range(3)]
        ms, gbs = timed(rows_for(*(t.data_ptr() for t in sep)), st, hp)
        print(f"round {rnd} (a) separate  {ms:7.3f} ms {gbs:7.1f} GB/s", flush=True)
        del sep
        torch.cuda.empty_cache()
        one = torch.zeros(3 * L, dtype=torch.float32, device=dev)
        ms, gbs = timed(rows_for(*(t.data_ptr() for t in one.split(L))), st, hp)
        print(f"round {rnd} (b) single    {ms:7.3f} ms {gbs:7.1f} GB/s", flush=True)
        del one
        torch.cuda.empty_cache()
        ms, gbs = timed(rows_for(*(t.data_ptr() for t in early.split(L))), st, hp)
        print(f"round {rnd} (c) early     {ms:7.3f} ms {gbs:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
