"""A/B (dev tool, not the product): does the relative placement of the fp32 optimizer-state
streams change the C4 Adam launch's bandwidth?  Same segment layout and kernel as the ws=1 step
(engine._step_local): bf16 grads and params as separate tensors, fp32 master / exp_avg /
exp_avg_sq carved out of ONE allocation at offsets L + s_k, for several staggers s (bytes).

usage: python tools/stagger_ab.py [reps]
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


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda:0")
    shapes = smollm3_3b_shapes()
    numels = [int(np.prod(s)) for s in shapes]
    plan = Plan(numels, 1, 0, "reference")
    pc = plan.pieces(0)
    L = plan.stream_len(0)
    g = torch.Generator(device=dev).manual_seed(0)
    params = [(torch.randn(s, device=dev, generator=g) * 0.02).to(torch.bfloat16) for s in shapes]
    grads = [(torch.randn(s, device=dev, generator=g) * 1e-3).to(torch.bfloat16) for s in shapes]
    staggers = [0, 4096, 65536 + 256, 1 << 20, (1 << 20) + 4096 * 3]
    big = torch.zeros(3 * L + 3 * (max(staggers) // 4 + 64), dtype=torch.float32, device=dev)
    hp = adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, 1)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = torch.cuda.current_stream()
    for rep in range(reps):
        for s in staggers:
            se = s // 4
            offs = [0, L + se, 2 * L + 2 * se]  # m, v, master element offsets
            base = np.uint64(big.data_ptr())
            so = pc.stream_off.astype(np.uint64)
            rows = np.zeros((len(pc.param), 9), np.uint64)
            gp = np.array([grads[i].data_ptr() for i in pc.param], np.uint64)
            pp = np.array([params[i].data_ptr() for i in pc.param], np.uint64)
            mst = base + (np.uint64(offs[2]) + so) * np.uint64(4)
            rows[:, 0], rows[:, 1], rows[:, 2], rows[:, 3] = gp, mst, mst, pp
            rows[:, 4] = base + (np.uint64(offs[0]) + so) * np.uint64(4)
            rows[:, 5] = base + (np.uint64(offs[1]) + so) * np.uint64(4)
            rows[:, 8] = pc.length.astype(np.uint64)
            aset = AdamSet(rows, ZS_BF16)
            aset.run(hp, st)
            torch.cuda.synchronize()
            ev0.record(st)
            for _ in range(10):
                aset.run(hp, st)
            ev1.record(st)
            torch.cuda.synchronize()
            ms = ev0.elapsed_time(ev1) / 10
            print(f"rep {rep} stagger {s:>8d} B: {ms:7.3f} ms  {aset.bytes / ms / 1e6:7.1f} GB/s",
                  flush=True)


if __name__ == "__main__":
    main()
