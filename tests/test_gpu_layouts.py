"""The bucketed engine under its two non-reference shard layouts, against the reference's ZeRO-2
trajectories (tests/golden).

Adam is elementwise, so which rank holds an element's optimizer state does not change the update:
every layout must reproduce the reference's ZeRO-2 parameters (DP-Adam, zero2.py:94-133) within
1e-6 at every step.  Layout Z ("chunk") is zero3.py:107-108's dim-0 chunking — the layout of the
ZeRO-3 parameter-set step in bench.py (BASELINE.json configs[4]) — incl. uneven chunks at ws=3;
Layout F ("flat") is the balanced contiguous 1/ws slice of the concatenated parameters — in the
bucket arena, and (round 6) in the flat parameter arena, where a parameter may straddle two
owners' streams (bench.py's N > 1 layout ablation).
ws processes share the box's GPU; the exchange goes through tests/_gloo_comm.py (and real RCCL in
tests/test_gpu_rccl.py).
"""
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, free_port
from _zero_run import spawn_batch, spawn_ranks, init_pg, rel

pytestmark = pytest.mark.gpu


def _worker(rank, ws, port, layout, name, buckets, window, arena="buckets"):
    import sys
    from conftest import PKG, REPO  # noqa: F401  (sets sys.path in the child)
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from zero_amd import zero2

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    z = np.load(GOLDEN / name)
    params = [torch.nn.Parameter(torch.from_numpy(z[f"init_{i}"].copy()).to(dev)) for i in range(12)]
    opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), comm=test_comm(),
                                 layout=layout, buckets=buckets, arena=arena,
                                 bucket_mb=ws * window * 4 / (1 << 20))
    assert opt.local_param_indices == z[f"r{rank}_local"].tolist()  # the reference's bookkeeping
    eng = opt.engine
    if arena == "flat":  # Layout F in the flat arena: params are views of P, balanced streams
        assert eng.arena_kind == "flat" and eng.layout == layout
        if ws > 1:
            assert len(set(eng.Ls.tolist())) == 1 and eng.K > 1  # equal streams; several rounds
            straddle = [i for i in range(12) if eng.owner[i] == rank and not all(
                eng.pieces.length[eng.pieces.param == i] == params[i].numel())]
            for i, p in enumerate(params):
                assert p.data_ptr() == eng.P.data_ptr() + int(eng.slot[i]) * eng.es
        else:
            straddle = []
    for t in range(int(z["steps"])):
        opt.zero_grad()
        for i, p in enumerate(params):
            p.grad = torch.from_numpy(z[f"r{rank}_t{t}_lg{i}"].copy()).to(dev)
        opt.step()
        eng = opt.engine
        if f"r{rank}_t{t}_p0" in z.files:
            for i, p in enumerate(params):
                e = rel(p.detach().cpu().numpy(), z[f"r{rank}_t{t}_p{i}"])
                assert e <= 1e-6, (layout, ws, rank, t, i, e)
    # every element's state lives on exactly one rank: the stream lengths add up to the model
    n = sum(p.numel() for p in params)
    tot = torch.tensor([eng.plan.stream_len(r) for r in range(ws)]).sum()
    assert int(tot) >= n
    owned = sum(int(ln) for ln in eng.pieces.length)
    cnt = torch.tensor([float(owned)])
    dist.all_reduce(cnt)
    assert int(cnt.item()) == n, (layout, int(cnt.item()), n)
    if arena == "flat" and ws >= 4:  # some parameter is split between two owners (at ws 2 and 3
        k = torch.tensor([float(len(straddle))])  # the d16 slices end on parameter boundaries)
        dist.all_reduce(k)
        assert k.item() > 0
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


CASES = [("chunk", 2, "ref", "ragged"), ("chunk", 3, "distinct", "ragged"),
         ("chunk", 3, "distinct", "padded"), ("chunk", 4, "distinct", "ragged"),
         ("chunk", 8, "distinct", "ragged"), ("flat", 2, "distinct", "ragged"),
         ("flat", 3, "ref", "ragged"), ("flat", 4, "distinct", "padded")]


@pytest.mark.parametrize("ws", [2, 3, 4, 8])
def test_layout_matches_reference_zero2(gpu, ws):
    """Every layout / bucket-mode case of this ws (ws = 4 adds windows smaller than most chunks:
    every parameter's chunk split across buckets), one after another in one set of processes."""
    cases = [(_worker, (layout, f"traj_z2_ws{w}_d16_{mode}.npz", buckets, 64))
             for layout, w, mode, buckets in CASES if w == ws]
    # Layout F in the flat parameter arena (128-element rounds: several rounds, straddling params;
    # every round is a gloo-staged group per owner here, so not more rounds than that)
    cases.append((_worker, ("flat", f"traj_z2_ws{ws}_d16_distinct.npz", "ragged", 128, "flat")))
    if ws == 4:
        cases.append((_worker, ("chunk", "traj_z2_ws4_d64_distinct.npz", "ragged", 64)))
    for _, (_, name, *_rest) in cases:
        assert (GOLDEN / name).exists(), name
    spawn_batch(ws, cases)
