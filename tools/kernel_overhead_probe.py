"""Why does every kernel of the SmolLM3 ZeRO-3 step take ~30 us longer than in the ZeRO-2 step?

The ws=1 kernel traces (tools/sm3_trace.sh) show the same kernels, same grids, each ~30-35 us
longer under ZeRO-3, tiny ones included, with no idle gaps between them.  ZeRO-3 differs in three
process-wide ways: it creates a dedicated RCCL communicator even at ws=1, a high-priority side
stream, and cross-stream event waits per layer.  This probe turns them on one at a time, each
phase launching a different elementwise op so the phases separate in a kernel trace:

    rocprofv3 --kernel-trace --stats -- python3 tools/kernel_overhead_probe.py

It also prints each phase's per-launch GPU time from events (GPU-bound: the host enqueues the
whole phase before the events are read)."""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))


def main():
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    small = torch.zeros(2048, device=dev)
    big = torch.zeros(4 << 20, device=dev)
    n = 2000

    def phase(name, op, between=None):
        cur = torch.cuda.current_stream(dev)
        torch.cuda.synchronize()
        out = {}
        for label, t in (("small", small), ("big", big)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # queue work ahead so the GPU never waits on the host: a long kernel first
            big.mul_(1.0)
            e0.record(cur)
            for i in range(n):
                op(t)
                if between is not None:
                    between()
            e1.record(cur)
            e1.synchronize()
            out[label + "_us"] = round(e0.elapsed_time(e1) * 1e3 / n, 2)
        print(json.dumps({"phase": name, **out}), flush=True)

    phase("A baseline", lambda t: t.add_(1.0))
    hs = torch.cuda.Stream(device=dev, priority=-1)
    phase("B +high-priority stream (idle)", lambda t: t.sub_(1.0))
    ls = torch.cuda.Stream(device=dev)
    phase("C +normal side stream (idle)", lambda t: t.mul_(1.0))

    def xwait(stream=hs):
        cur = torch.cuda.current_stream(dev)
        ev = torch.cuda.Event()
        ev.record(cur)
        stream.wait_event(ev)
        ev2 = torch.cuda.Event()
        ev2.record(stream)
        cur.wait_event(ev2)

    phase("D cross-stream waits (high-priority) after every kernel", lambda t: t.div_(1.0), xwait)
    phase("E baseline again", lambda t: t.clamp_(-1e9, 1e9))
    phase("F cross-stream waits (normal priority)", lambda t: t.abs_(), lambda: xwait(ls))
    phase("G baseline again", lambda t: t.neg_())
    from zero_amd.comm import RcclComm

    comm = RcclComm()
    phase("H +RCCL communicator (ws=1)", lambda t: t.exp_())
    with torch.cuda.stream(hs):
        buf = torch.ones(1024, device=dev)
        comm.all_reduce(buf, hs)
    torch.cuda.synchronize()
    phase("I +one RCCL all-reduce done", lambda t: t.sqrt_())
    comm.close()
    phase("J communicator destroyed", lambda t: t.sin_())
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
