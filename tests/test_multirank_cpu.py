"""N>1 host logic on CPU with gloo (world_size 2-4): the planner's Layout-R buckets composed with
real in-place reduce-scatter / all-gather slices reproduce the reference ZeRO-1/2 trajectories.

This emulates, with numpy and the oracle's Adam, exactly the data movement the GPU engine performs
(engine.py ShardEngine._step_buckets): pack every bucket by the plan's segments, reduce-scatter
the rank-major buffer so each rank receives its own window (ragged buckets: one reduce per owner), Adam on the owned window (grad /ws and
the ZeRO-1 carry folded in), write the updated params into the window, all-gather, unpack.  The
device kernels themselves are covered by the -m gpu tests.
"""

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, free_port


def _port():
    return free_port()


def _worker(rank, ws, port, variant, name, window, buckets="ragged"):
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
    plan = Plan([p.size for p in params], ws, rank, "reference", window_elems=window, buckets=buckets)
    L = plan.stream_len(rank)
    m, v = np.zeros(L, np.float32), np.zeros(L, np.float32)
    carry = np.zeros(L, np.float32)
    steps = 0
    for t in range(int(z["steps"])):
        grads = [z[f"r{rank}_t{t}_lg{i}"].reshape(-1) for i in range(12)]
        steps += 1
        for k in range(plan.num_buckets):
            s, b = plan.segments(k), plan.bucket(k)
            buf = np.zeros(b.elems, np.float32)
            for i, po, bo, ln in zip(s.param, s.param_off, s.buf_off, s.length):  # pack
                buf[bo:bo + ln] = grads[i][po:po + ln]
            o0, n0 = int(b.win_off[rank]), int(b.win_len[rank])
            if b.even:  # one equal-count reduce-scatter: rank's window = summed grads
                out = torch.empty(n0)
                dist.reduce_scatter_tensor(out, torch.from_numpy(buf))
                buf[o0:o0 + n0] = out.numpy()
            else:  # ragged: one reduce per owner (reduce-scatter-v)
                for root in range(ws):
                    o, n = int(b.win_off[root]), int(b.win_len[root])
                    if n:
                        part = torch.from_numpy(buf[o:o + n].copy())
                        dist.reduce(part, dst=root)
                        if root == rank:
                            buf[o:o + n] = part.numpy()
            for i, r, po, bo, ln in zip(s.param, s.rank, s.param_off, s.buf_off, s.length):
                if r != rank:
                    continue
                so = int(b.win_stream[rank]) + bo - o0
                gsum = buf[bo:bo + ln]
                if variant == 1:  # A_t = (Σ G + (ws-1) A_{t-1}) / ws
                    g = ((gsum + np.float32(ws - 1) * carry[so:so + ln]) / np.float32(ws)).astype(np.float32)
                    carry[so:so + ln] = g
                else:
                    g = (gsum / np.float32(ws)).astype(np.float32)
                p, mm, vv, _ = zo.adam_update(params[i][po:po + ln], g, m[so:so + ln], v[so:so + ln], steps)
                m[so:so + ln], v[so:so + ln] = mm, vv
                buf[bo:bo + ln] = p
            if b.even:
                full = torch.empty(b.elems)
                dist.all_gather_into_tensor(full, torch.from_numpy(buf[o0:o0 + n0].copy()))
                buf = full.numpy()
            else:  # all-gather-v: one broadcast per owner
                for root in range(ws):
                    o, n = int(b.win_off[root]), int(b.win_len[root])
                    if n:
                        part = torch.from_numpy(buf[o:o + n].copy())
                        dist.broadcast(part, src=root)
                        buf[o:o + n] = part.numpy()
            for i, po, bo, ln in zip(s.param, s.param_off, s.buf_off, s.length):  # unpack
                params[i][po:po + ln] = buf[bo:bo + ln]
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


@pytest.mark.parametrize("variant", [1, 2])
def test_padded_buckets_match_reference(variant):
    """ZS_BUCKETS_PADDED (every window zero-padded to the longest stream) gives the same result."""
    name = f"traj_z{variant}_ws3_d16_distinct.npz"
    mp.spawn(_worker, args=(3, _port(), variant, name, 64, "padded"), nprocs=3, join=True)


def test_ws8_ragged_buckets_match_reference():
    """ws=8 with 12 params: ranks 4-7 own one param each, so most buckets are ragged."""
    mp.spawn(_worker, args=(8, _port(), 2, "traj_z2_ws8_d16_distinct.npz", 64), nprocs=8, join=True)


def _flat_worker(rank, ws, port, variant, name, window):
    """The flat-arena exchange (flat.py FlatEngine) restated with numpy + gloo: owner-major arena
    G / P (rank r's stream = its reference-owned params, 64-aligned), per round j one reduce of
    every owner's window [jW, (j+1)W) onto its owner (out of place, into R), Adam on the own
    window (ZeRO-1: carry weight ws-1, the opt.zero_grad() loop), one broadcast per owner."""
    import os

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from oracle import zero_oracle as zo
    from zero_amd.plan import Plan

    z = np.load(GOLDEN / name)
    init = [z[f"init_{i}"].copy().reshape(-1) for i in range(12)]
    n = len(init)
    plan = Plan([p.size for p in init], ws, rank, "reference")
    Ls = np.array([plan.stream_len(r) for r in range(ws)])
    base = np.concatenate([[0], np.cumsum(Ls)[:-1]])
    slot = np.zeros(n, np.int64)
    for r in range(ws):
        pc = plan.pieces(r)
        slot[pc.param] = base[r] + pc.stream_off
    P = np.zeros(int(Ls.sum()), np.float32)
    for i, a in enumerate(init):
        P[slot[i]:slot[i] + a.size] = a
    L = int(Ls[rank])
    R = np.zeros(L, np.float32)
    m, v, carry = (np.zeros(L, np.float32) for _ in range(3))
    pc = plan.pieces(rank)
    K = max(1, -(-int(Ls.max()) // window))
    for t in range(int(z["steps"])):
        G = np.zeros_like(P)
        for i in range(n):
            g = z[f"r{rank}_t{t}_lg{i}"].reshape(-1)
            G[slot[i]:slot[i] + g.size] = g
        for j in range(K):  # reduce-scatter-v: one reduce per owner window
            lo = j * window
            for r in range(ws):
                c = int(np.clip(Ls[r] - lo, 0, window))
                if c:
                    part = torch.from_numpy(G[base[r] + lo:base[r] + lo + c].copy())
                    dist.reduce(part, dst=r)
                    if r == rank:
                        R[lo:lo + c] = part.numpy()
        for i, so, ln in zip(pc.param, pc.stream_off, pc.length):  # Adam on the own stream
            gsum = R[so:so + ln]
            if variant == 1:
                g = ((gsum + np.float32(ws - 1) * carry[so:so + ln]) / np.float32(ws)).astype(np.float32)
                carry[so:so + ln] = g
            else:
                g = (gsum / np.float32(ws)).astype(np.float32)
            p, mm, vv, _ = zo.adam_update(P[base[rank] + so:base[rank] + so + ln], g, m[so:so + ln],
                                          v[so:so + ln], t + 1)
            P[base[rank] + so:base[rank] + so + ln] = p
            m[so:so + ln], v[so:so + ln] = mm, vv
        for j in range(K):  # all-gather-v: one broadcast per owner window
            lo = j * window
            for r in range(ws):
                c = int(np.clip(Ls[r] - lo, 0, window))
                if c:
                    part = torch.from_numpy(P[base[r] + lo:base[r] + lo + c].copy())
                    dist.broadcast(part, src=r)
                    P[base[r] + lo:base[r] + lo + c] = part.numpy()
        if f"r{rank}_t{t}_p0" in z.files:
            for i in range(n):
                ref = z[f"r{rank}_t{t}_p{i}"].reshape(-1)
                got = P[slot[i]:slot[i] + ref.size]
                assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) <= 1e-6, (name, rank, t, i)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("ws,window", [(2, 64), (3, 128), (4, 64), (8, 64), (4, 1 << 20)])
def test_flat_arena_exchange_matches_reference(variant, ws, window):
    name = f"traj_z{variant}_ws{ws}_d16_distinct.npz"
    mp.spawn(_flat_worker, args=(ws, _port(), variant, name, window), nprocs=ws, join=True)


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


def test_bench_xgmi_peak_counts_direct_peer_links():
    """bench.py's xGMI denominators: one direct link per peer in the 8-GPU mesh (N=2 → 1 link,
    N=8 → all 7), never more than 7."""
    import bench

    assert [bench.peer_link_peak_gbs(n) for n in (1, 2, 4, 8, 16)] == \
        [153.0, 153.0, 3 * 153.0, 7 * 153.0, 7 * 153.0]
