"""Feasibility probe: real RCCL collectives between ws processes that share ONE GPU.

RCCL refuses two ranks of a communicator on one device when it sees them on the same host.  Each
rank here gets its own NCCL_HOSTID, so RCCL takes every rank for a separate node and moves data
through its socket NET transport over loopback (host-staged), while the reductions and copies run
in RCCL's own kernels on the GPU buffers — the ring order and per-hop bf16 rounding of a real
ws-rank job, without a second GPU.

    python tools/rccl_net_probe.py --ws 2          (parent: spawns the ranks, checks exit codes)
"""
import argparse
import os
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def net_env(rank: int) -> dict:
    env = dict(os.environ)
    env.update(NCCL_HOSTID=f"zs-net-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    return env


def child(rank: int, ws: int, port: int) -> None:
    sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))
    import torch
    import torch.distributed as dist

    from zero_amd.comm import RcclComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    t0 = time.time()
    comm = RcclComm()
    t_init = time.time() - t0
    st = torch.cuda.current_stream()
    n = 1 << 20
    ok = True
    for dt in (torch.float32, torch.bfloat16):
        t = torch.full((n,), float(rank + 1), device=dev, dtype=dt)
        comm.all_reduce(t, st)
        torch.cuda.synchronize()
        ok &= bool((t == ws * (ws + 1) / 2).all())
        send = (torch.arange(ws * n, device=dev, dtype=torch.float32) % 251 + rank).to(dt)
        recv = torch.empty(n, device=dev, dtype=dt)
        comm.reduce_scatter(send, recv, st)
        ag = torch.empty(ws * n, device=dev, dtype=dt)
        comm.all_gather(recv, ag, st)
        torch.cuda.synchronize()
        want = sum(((torch.arange(ws * n, device=dev, dtype=torch.float32) % 251 + r).to(dt).float())
                   for r in range(ws))
        err = float((ag.float() - want).abs().max())
        ok &= err <= (0 if dt == torch.float32 else ws * 2 ** -8 * float(want.abs().max()))
        print(f"rank {rank} {dt}: rs+ag max err {err}", flush=True)
    big = torch.ones(64 << 20, device=dev, dtype=torch.bfloat16)
    comm.all_reduce(big, st)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(3):
        comm.all_reduce(big, st)
    torch.cuda.synchronize()
    dt_ar = (time.time() - t0) / 3
    print(f"rank {rank}: init {t_init:.2f} s, ok={ok}, 128 MB bf16 all-reduce {dt_ar * 1e3:.1f} ms",
          flush=True)
    comm.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", type=int, default=2)
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--port", type=int, default=29611)
    a = ap.parse_args()
    if a.rank is not None:
        return child(a.rank, a.ws, a.port)
    procs = [subprocess.Popen([sys.executable, "-u", __file__, "--ws", str(a.ws), "--rank", str(r),
                               "--port", str(a.port)], env=net_env(r)) for r in range(a.ws)]
    rcs = [p.wait() for p in procs]
    print("exit codes", rcs, flush=True)
    sys.exit(0 if all(rc == 0 for rc in rcs) else 1)


if __name__ == "__main__":
    main()
