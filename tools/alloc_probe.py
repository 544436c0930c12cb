"""Dev tool: does an allocation's own streaming bandwidth (an in-place copy over it) predict the
C4 Adam launch's speed on it?  Several fresh state allocations after the model's tensors; for each
the in-place copy GB/s and the Adam ms."""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))

from zero_amd.kernels import AdamSet, CopySet, adam_hparams  # noqa: E402
from zero_amd.plan import Plan  # noqa: E402
from zero_amd.shapes import smollm3_3b_shapes  # noqa: E402
from zero_amd._lib import ZS_BF16  # noqa: E402


def bw(fn, nbytes, st, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms, nbytes / ms / 1e6


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    shapes = smollm3_3b_shapes()
    plan = Plan([int(np.prod(s)) for s in shapes], 1, 0, "reference")
    pc, L = plan.pieces(0), plan.stream_len(0)
    g = torch.Generator(device=dev).manual_seed(0)
    params = [torch.empty(s, device=dev).normal_(0, 0.02, generator=g).to(torch.bfloat16) for s in shapes]
    grads = [(torch.empty(s, device=dev).normal_(generator=g) * 1e-3).to(torch.bfloat16) for s in shapes]
    hp = adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, 1)
    st = torch.cuda.current_stream()
    gp = np.array([grads[i].data_ptr() for i in pc.param], np.uint64)
    pp = np.array([params[i].data_ptr() for i in pc.param], np.uint64)
    so = pc.stream_off.astype(np.uint64)
    keep = []
    for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
        buf = torch.zeros(3 * L, dtype=torch.float32, device=dev)
        keep.append(buf)  # keep it alive: the next trial gets different memory
        m, v, x = (t.data_ptr() for t in buf.split(L))
        r = np.zeros((len(pc.param), 9), np.uint64)
        r[:, 0], r[:, 1], r[:, 2], r[:, 3] = gp, np.uint64(x) + so * 4, np.uint64(x) + so * 4, pp
        r[:, 4], r[:, 5] = np.uint64(m) + so * 4, np.uint64(v) + so * 4
        r[:, 8] = pc.length.astype(np.uint64)
        a = AdamSet(r, ZS_BF16)
        ams, agbs = bw(lambda: a.run(hp, st), a.bytes, st)
        nb = buf.numel() * 4
        cs = CopySet([buf.data_ptr()], [buf.data_ptr()], [nb])  # in-place: read + write each byte
        cms, cgbs = bw(lambda: cs.run(st), 2 * nb, st)
        rms, rgbs = bw(lambda: torch.sum(buf), nb, st)
        print(f"trial {trial}: adam {ams:7.3f} ms {agbs:7.1f} GB/s | state copy-in-place {cgbs:7.1f} "
              f"GB/s | state read (torch.sum) {rgbs:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
