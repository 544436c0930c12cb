"""N>1 host logic on CPU with gloo (world_size 2-4): the planner's Layout-R buckets composed with
real in-place reduce-scatter / all-gather slices reproduce the reference ZeRO-1/2 trajectories.

This emulates, with numpy and the oracle's Adam, exactly the data movement the GPU engine performs
(engine.py ShardEngine._step_buckets): pack every bucket by the plan's segments, reduce-scatter
the rank-major buffer so each rank receives its own window, Adam on the owned window (grad /ws and
the ZeRO-1 carry folded in), write the updated params into the window, all-gather, unpack.  The
device kernels themselves are covered by the -m gpu tests.
"""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, variant, name, window):
    import os

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from oracle import zero_oracle as zo
    from zero_amd.plan import Plan

    z = np.load(GOLDEN / name)
    params = [z[f"init_{i}"].copy().reshape(-1) for i in range(12)]
    shapes = [z[f"init_{i}"].shape for i in range(12)]
    plan = Plan([p.size for p in params], ws, rank, "reference", window_elems=window)
    W, BE = plan.window, plan.bucket_elems
    L = plan.stream_len(rank)
    m, v = np.zeros(L, np.float32), np.zeros(L, np.float32)
    carry = np.zeros(L, np.float32)
    steps = 0
    for t in range(int(z["steps"])):
        grads = [z[f"r{rank}_t{t}_lg{i}"].reshape(-1) for i in range(12)]
        steps += 1
        for k in range(plan.num_buckets):
            s = plan.segments(k)
            buf = np.zeros(BE, np.float32)
            for i, po, bo, ln in zip(s.param, s.param_off, s.buf_off, s.length):  # pack
                buf[bo:bo + ln] = grads[i][po:po + ln]
            out = torch.empty(W)
            dist.reduce_scatter_tensor(out, torch.from_numpy(buf))  # rank's window = summed grads
            win = out.numpy()
            for i, r, po, bo, ln in zip(s.param, s.rank, s.param_off, s.buf_off, s.length):
                if r != rank:
                    continue
                so = k * W + bo - rank * W
                gsum = win[bo - rank * W: bo - rank * W + ln]
                if variant == 1:  # A_t = (Σ G + (ws-1) A_{t-1}) / ws
                    g = ((gsum + np.float32(ws - 1) * carry[so:so + ln]) / np.float32(ws)).astype(np.float32)
                    carry[so:so + ln] = g
                else:
                    g = (gsum / np.float32(ws)).astype(np.float32)
                p, mm, vv, _ = zo.adam_update(params[i][po:po + ln], g, m[so:so + ln], v[so:so + ln], steps)
                m[so:so + ln], v[so:so + ln] = mm, vv
                win[bo - rank * W: bo - rank * W + ln] = p
            full = torch.empty(BE)
            dist.all_gather_into_tensor(full, torch.from_numpy(win))
            full = full.numpy()
            for i, po, bo, ln in zip(s.param, s.param_off, s.buf_off, s.length):  # unpack
                params[i][po:po + ln] = full[bo:bo + ln]
        if f"r{rank}_t{t}_p0" in z.files:
            for i in range(12):
                ref = z[f"r{rank}_t{t}_p{i}"].reshape(-1)
                err = np.max(np.abs(params[i] - ref)) / np.max(np.abs(ref))
                assert err <= 1e-6, (name, rank, t, i, err)
    assert [p.reshape(s).shape for p, s in zip(params, shapes)] == shapes
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("ws", [2, 3, 4])
@pytest.mark.parametrize("window", [0, 64, 192])
def test_bucketed_exchange_matches_reference(variant, ws, window):
    name = f"traj_z{variant}_ws{ws}_d16_distinct.npz"
    mp.spawn(_worker, args=(ws, _port(), variant, name, window), nprocs=ws, join=True)


def test_collective_kats_gloo():
    """02-operations.ipynb:1853-2109 known answers through the same gloo calls the tests use."""
    z = np.load(GOLDEN / "collective_kat.npz")
    mp.spawn(_kat_worker, args=(_port(), z["inputs"], z["all_reduce"], z["all_gather"]), nprocs=2,
             join=True)


def _kat_worker(rank, port, inputs, want_ar, want_ag):
    import os

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    t = torch.from_numpy(inputs[rank].copy())
    ag = torch.empty(6, dtype=t.dtype)
    dist.all_gather_into_tensor(ag, t)
    dist.all_reduce(t)
    assert t.tolist() == want_ar.tolist()
    assert ag.view(2, 3).tolist() == want_ag.tolist()
    dist.destroy_process_group()
