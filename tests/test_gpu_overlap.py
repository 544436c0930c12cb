"""Backward-overlapped gradient buckets (overlap.py) on the MI355X: ZeRO-1/2 with per-owner
reduces launched from post-accumulate-grad hooks, and the DDP drop-in's bucketed all-reduce.

ZeRO: the reference trajectories (tests/golden) are replayed through a real backward pass
(loss = Σ <p_i, G_i>, so p_i.grad == G_i bit-for-bit) at 1e-6 normwise, every step.  Multi-rank
cases share the one GPU through the test-only gloo-staged communicator, as in test_gpu_parity.
DDP: every rank's averaged grads against numpy (sum over ranks in rank order, then / ws).
"""

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, free_port
from _zero_run import spawn_batch, spawn_ranks, init_pg, run_backward

pytestmark = pytest.mark.gpu


def _port():
    return free_port()


@pytest.fixture
def pg1():
    init_pg(0, 1, _port())
    yield
    dist.destroy_process_group()


def _overlap_stats(opt):
    """(buckets, buckets launched during the last backward) of either overlap implementation."""
    eng = opt.engine
    if getattr(eng, "arena_kind", None) == "flat":
        return eng.ov_K, eng.launched_in_backward
    return eng.gb.K, eng.gb.launched_in_backward


@pytest.mark.parametrize("arena", ["flat", "buckets"])
@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("views", [True, False])
def test_ws1_overlap_backward(gpu, golden, pg1, variant, views, arena):
    z = golden(f"traj_z{variant}_ws1_d16_distinct.npz")
    opt = run_backward(z, variant, 0, 1, gpu, views=views, bucket_mb=2e-3, arena=arena)
    k, launched = _overlap_stats(opt)
    assert k > 1 and launched > 0


def test_overlap_bf16_matches_bucket_engine(gpu, pg1):
    """bf16 params + fp32 master: the overlap path and the bucketed path give identical bits."""
    from zero_amd import zero2

    g = torch.Generator().manual_seed(3)
    shapes = [(96, 40), (40,), (33, 7), (7,), (128, 64), (64,)]
    init = [(torch.randn(s, generator=g) * 0.02).to(torch.bfloat16) for s in shapes]
    grads = [[(torch.randn(s, generator=g) * 1e-3).to(torch.bfloat16) for s in shapes] for _ in range(3)]
    out = []
    for overlap, arena in ((False, "flat"), (True, "flat"), (True, "buckets")):
        ps = [torch.nn.Parameter(t.clone().to(gpu)) for t in init]
        opt = zero2.ShardedOptimizer(torch.optim.Adam(ps, lr=1e-3), overlap=overlap,
                                     overlap_bucket_mb=0.01, arena=arena)
        for gs in grads:
            opt.zero_grad()
            loss = sum((p.float() * gg.to(gpu).float()).sum() for p, gg in zip(ps, gs))
            loss.backward()
            opt.step()
        out.append([p.detach().cpu().view(torch.int16) for p in ps])
    for other in out[1:]:
        for a, b in zip(out[0], other):
            assert torch.equal(a, b)


def test_overlap_unused_param_keeps_value(gpu, pg1):
    """A parameter no backward touches has no grad: Adam skips it (the reference's None grad)."""
    from zero_amd import zero2

    ps = [torch.nn.Parameter(torch.randn(64, 8, device=gpu)) for _ in range(3)]
    before = ps[1].detach().clone()
    before0 = ps[0].detach().clone()
    opt = zero2.ShardedOptimizer(torch.optim.Adam(ps, lr=1e-2), overlap=True, overlap_bucket_mb=1e-3)
    opt.zero_grad()
    (ps[0].sum() + ps[2].sum()).backward()
    opt.step()
    assert torch.equal(ps[1].detach(), before)
    assert not torch.equal(ps[0].detach(), before0)
    assert "exp_avg" in opt.optimizer.state[ps[0]]


class _NoComm:
    """Collectives as no-ops: rank 0 of a simulated two-rank job (the landing path only)."""

    def reduce_out(self, send, recv, root, stream):
        pass

    def broadcast(self, t, root, stream):
        pass

    def reduce(self, t, root, stream):
        pass


@pytest.mark.parametrize("ws", [1, 2])
@pytest.mark.parametrize("overlap", [False, True])
def test_zero2_flat_zero_grad_sets_none_then_adopts(gpu, pg1, overlap, ws, monkeypatch):
    """ZeRO-2 on the flat arena: zero_grad() leaves p.grad None (the reference's state after
    zero_grad).  ws = 1: step() reads backward's fresh gradient in place — p.grad stays backward's
    tensor and no gradient arena exists until grad views are asked for.  ws > 1 (rank 0 of a
    simulated two-rank job): the fresh gradient lands in its arena slot — with its bucket during
    backward (overlap: p.grad becomes the slot's view there), else from the hooks in batches or at
    step() — a second backward accumulating in the fresh tensor first — and p.grad is the slot's
    view after step().  zero_grad(set_to_none=False) hands out zeroed views; ZeRO-1 keeps zeroed
    views."""
    import zero_amd._sharded as sh
    from zero_amd import zero1, zero2

    kw = {}
    if ws > 1:
        monkeypatch.setattr(sh, "get", lambda what, dm=None: {"ws": ws, "rank": 0}[what])
        kw["comm"] = _NoComm()
    ps = [torch.nn.Parameter(torch.randn(64, 8, device=gpu)) for _ in range(3)]
    opt = zero2.ShardedOptimizer(torch.optim.Adam(ps, lr=1e-2), overlap=overlap,
                                 overlap_bucket_mb=1e-3, **kw)
    eng = opt.engine
    assert eng.inplace == (ws == 1) and (eng.G is None) == (ws == 1)
    opt.zero_grad()
    assert all(p.grad is None for p in ps)
    w = [torch.randn(64, 8, device=gpu) for _ in ps]
    sum((p * x).sum() for p, x in zip(ps, w)).backward()
    landed = overlap and ws > 1
    for i, (p, x) in enumerate(zip(ps, w)):
        assert eng.is_view(i, p.grad) == landed and torch.equal(p.grad, x)
    if not overlap:
        sum((p * x).sum() for p, x in zip(ps, w)).backward()
        for p, x in zip(ps, w):
            assert torch.equal(p.grad, x + x)
    fresh = [p.grad for p in ps]
    opt.step()
    for i, (p, x) in enumerate(zip(ps, w)):
        assert torch.equal(p.grad, x if overlap else x + x)
        if ws == 1:  # read in place: still backward's own tensor
            assert p.grad is fresh[i] and not eng.is_view(i, p.grad)
        else:
            assert eng.is_view(i, p.grad)
    if ws == 1:
        assert eng.G is None and eng.inplace_reads == len(ps)
    opt.zero_grad(set_to_none=False)
    assert all(eng.is_view(i, p.grad) and not p.grad.any() for i, p in enumerate(ps))
    q = torch.nn.Parameter(torch.randn(8, device=gpu))
    z1 = zero1.ShardedOptimizer(torch.optim.Adam([q], lr=1e-2), **kw)
    z1.zero_grad()
    if ws > 1:  # the carry needs the views
        assert q.grad is not None and not q.grad.any() and z1.engine.is_view(0, q.grad)
    else:  # no carry at ws = 1: None, as the reference's optimizer.zero_grad()
        assert q.grad is None


def test_overlap_double_backward_raises(gpu, pg1):
    from zero_amd import zero2

    ps = [torch.nn.Parameter(torch.randn(64, device=gpu))]
    opt = zero2.ShardedOptimizer(torch.optim.Adam(ps, lr=1e-3), overlap=True)
    opt.zero_grad()
    ps[0].sum().backward()
    with pytest.raises(RuntimeError, match="accumulated twice"):
        ps[0].sum().backward()


def _mr_worker(rank, ws, port, variant, name, views, arena):
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    z = np.load(GOLDEN / name)
    opt = run_backward(z, variant, rank, ws, torch.device("cuda:0"), comm=test_comm(),
                       views=views, bucket_mb=2e-3, arena=arena)
    k, launched = _overlap_stats(opt)
    assert k >= ws and launched > 0  # buckets reduced while backward was still running
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def _frozen_worker(rank, ws, port, variant, overlap):
    """A frozen parameter (requires_grad=False) and one the loss reaches only at step 0: without a
    gradient Adam skips a parameter (the reference's `p.grad is None`, zero2.py:99-101) — so the
    second one keeps its step-0 value although its Adam moments are non-zero — every rank ends
    bit-identical, and the frozen one does not hold back the overlapped reduces of later buckets."""
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from _zero_run import module_for, rel
    from oracle import zero_oracle as zo

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    shapes = [(40, 8), (40,), (24, 8), (24,), (16, 8), (16,)]
    frozen, unused = 2, 0  # (an unreached parameter holds back its bucket and every later one)
    g = torch.Generator().manual_seed(21)
    init = [torch.randn(s, generator=g).numpy() for s in shapes]
    steps = 3
    lg = {(t, r, i): (torch.randn(s, generator=torch.Generator().manual_seed(100 * t + 10 * r + i))
                      * 1e-2).numpy() for t in range(steps) for r in range(ws) for i, s in enumerate(shapes)}
    # ZeRO-1: the reference's owner and non-owners would disagree about a parameter that loses
    # its gradient after step 0 (the non-owners' surviving averaged grad vs the owner's None, a
    # mismatched all_reduce, zero1.py:81-84), so there the second parameter is never reached
    skip = lambda t, i: i == frozen or (i == unused and (t > 0 or variant == 1))  # noqa: E731
    grad_of = lambda t, r, i: None if skip(t, i) else lg[(t, r, i)]  # noqa: E731
    want = zo.simulate(variant, ws, init, steps=steps, local_grads=grad_of)
    params = [torch.nn.Parameter(torch.from_numpy(a.copy()).to(dev), requires_grad=i != frozen)
              for i, a in enumerate(init)]
    opt = module_for(variant).ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), comm=test_comm(),
                                               overlap=overlap, overlap_bucket_mb=1e-3)
    for t in range(steps):
        opt.zero_grad()
        loss = sum((p * torch.from_numpy(lg[(t, rank, i)].copy()).to(dev)).sum()
                   for i, p in enumerate(params) if not skip(t, i))
        loss.backward()
        opt.step()
        for i, p in enumerate(params):
            assert rel(p.detach().cpu().numpy(), want["params"][t][rank][i]) <= 1e-6, (variant, rank, t, i)
        assert torch.equal(params[frozen].detach().cpu(), torch.from_numpy(init[frozen]))
    assert not overlap or opt.engine.launched_in_backward > 0
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def test_frozen_and_unused_params(gpu):
    spawn_batch(2, [(_frozen_worker, (v, o)) for v in (1, 2) for o in (True, False)])


def _unfreeze_worker(rank, ws, port, overlap):
    """requires_grad changed after the optimizer was built (gradual unfreezing / freezing): a
    parameter frozen at construction and unfrozen at step 2 is updated from then on (hooked when
    it changes — no silent skip), one frozen at step 3 is skipped from then on, and the
    overlapped buckets re-count what they wait for.  Against the oracle, every step."""
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from _zero_run import rel
    from oracle import zero_oracle as zo
    from zero_amd import zero2

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    shapes = [(40, 8), (40,), (24, 8), (24,), (16, 8), (16,)]
    late, early = 2, 4  # trainable from step 2 on / frozen from step 3 on
    g = torch.Generator().manual_seed(23)
    init = [torch.randn(s, generator=g).numpy() for s in shapes]
    steps = 5
    lg = {(t, r, i): (torch.randn(s, generator=torch.Generator().manual_seed(100 * t + 10 * r + i))
                      * 1e-2).numpy() for t in range(steps) for r in range(ws) for i, s in enumerate(shapes)}
    skip = lambda t, i: (i == late and t < 2) or (i == early and t >= 3)  # noqa: E731
    want = zo.simulate(2, ws, init, steps=steps,
                       local_grads=lambda t, r, i: None if skip(t, i) else lg[(t, r, i)])
    params = [torch.nn.Parameter(torch.from_numpy(a.copy()).to(dev), requires_grad=i != late)
              for i, a in enumerate(init)]
    opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), comm=test_comm(),
                                 overlap=overlap, overlap_bucket_mb=1e-3)
    for t in range(steps):
        if t == 2:
            params[late].requires_grad_(True)
        if t == 3:
            params[early].requires_grad_(False)
        opt.zero_grad()
        loss = sum((p * torch.from_numpy(lg[(t, rank, i)].copy()).to(dev)).sum()
                   for i, p in enumerate(params) if not skip(t, i))
        loss.backward()
        opt.step()
        for i, p in enumerate(params):
            assert rel(p.detach().cpu().numpy(), want["params"][t][rank][i]) <= 1e-6, (overlap, rank, t, i)
    assert not torch.equal(params[late].detach().cpu(), torch.from_numpy(init[late]))
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def test_requires_grad_changes_after_construction(gpu):
    spawn_batch(2, [(_unfreeze_worker, (o,)) for o in (True, False)])


OV_CASES = [(2, True), (3, True), (3, False), (4, True)]


@pytest.mark.parametrize("ws", [2, 3, 4])
def test_multirank_overlap_backward(gpu, ws):
    """Backward-overlapped reduces against the reference's trajectories: ZeRO-1 and 2, flat and
    bucket arena, grads as bucket views or handed over (every combination of this ws)."""
    spawn_batch(ws, [(_mr_worker, (v, f"traj_z{v}_ws{ws}_d16_distinct.npz", views, arena))
                     for w, views in OV_CASES if w == ws for v in (1, 2) for arena in ("flat", "buckets")])


def test_multirank_overlap_backward_ws8_flat(gpu):
    """ws=8 (12 parameters: ranks 4-7 own one each) through a real backward on the flat arena."""
    spawn_batch(8, [(_mr_worker, (v, f"traj_z{v}_ws8_d16_distinct.npz", True, "flat")) for v in (1, 2)])


# ---------------------------------------------------------------------------------------------
# DDP
def _ddp_grads(ws, shapes, step):
    g = torch.Generator().manual_seed(1000 + step)
    return [[torch.randn(s, generator=g) for s in shapes] for _ in range(ws)]


def _ddp_worker(rank, ws, port, dtype_name):
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from zero_amd.ddp import SimpleDistributedDataParallelism

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    dt = getattr(torch, dtype_name)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(40, 24), torch.nn.ReLU(), torch.nn.Linear(24, 8),
                                torch.nn.Linear(8, 8)).to(dev).to(dt)
    ddp = SimpleDistributedDataParallelism(model, bucket_mb=1e-3,
                                           comm=test_comm() if ws > 1 else None)
    shapes = [tuple(p.shape) for p in model.parameters()]
    for step in range(3):
        allg = _ddp_grads(ws, shapes, step)
        if step == 1:
            ddp.zero_grad()          # views: autograd accumulates in place
        else:
            model.zero_grad(set_to_none=True)
        used = list(model.parameters())[:4]  # the last Linear gets no gradient
        loss = sum((p.float() * g.to(dev).to(dt).float()).sum() for p, g in zip(used, allg[rank]))
        loss.backward()
        ddp.sync_gradients()
        torch.cuda.synchronize()
        for i, p in enumerate(model.parameters()):
            if i >= 4:
                assert p.grad is None
                continue
            acc = np.zeros(shapes[i], np.float32)
            for r in range(ws):  # the staged comm sums in fp32 in rank order
                acc = acc + allg[r][i].to(dt).float().numpy()
            if dt == torch.float32:
                want = acc / np.float32(ws)
                got = p.grad.cpu().numpy()
            else:  # sum rounded to bf16 once, then / ws in fp32 rounded to bf16
                want = (torch.from_numpy(acc).to(torch.bfloat16).float() / ws).to(torch.bfloat16).float().numpy()
                got = p.grad.cpu().float().numpy()
            if ws <= 2:  # a two-term sum is order-free: bit-exact
                assert np.array_equal(got, want), (rank, step, i)
            else:  # gloo's ring may add in another order
                tol = 1e-6 if dt == torch.float32 else 2.0 ** -7
                assert np.max(np.abs(got - want)) <= tol * np.max(np.abs(want)), (rank, step, i)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def _ddp_fixture_worker(rank, ws, port, dtype_name):
    """The drop-in against the reference's own SimpleDistributedDataParallelism outputs
    (tests/golden/ddp_sync_ws*_*.npz, made by running its class on gloo): the same seeded model,
    each step's local gradients set by hand, sync_gradients().  ws = 2: bit-exact (fp32 and bf16:
    a two-term sum rounds once in any order, / 2 is exact); ws = 3: within the ring's order noise
    (fp32 1e-6, bf16 2^-7 normwise).  The last Linear gets no gradient and keeps None."""
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from zero_amd.ddp import SimpleDistributedDataParallelism

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    dt = getattr(torch, dtype_name)
    bf16 = dt == torch.bfloat16
    z = np.load(GOLDEN / f"ddp_sync_ws{ws}_{dtype_name}.npz")

    def tens(a):
        t = torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16) if bf16 else torch.from_numpy(a.copy())
        return t.to(dev)

    torch.manual_seed(0)  # the generator's model init (make_ddp_golden.py), on the CPU, then moved
    model = torch.nn.Sequential(torch.nn.Linear(40, 24), torch.nn.ReLU(), torch.nn.Linear(24, 8),
                                torch.nn.Linear(8, 8)).to(dt).to(dev)
    ddp = SimpleDistributedDataParallelism(model, bucket_mb=1e-3, comm=test_comm())
    params = list(model.parameters())
    for t in range(3):
        for i, p in enumerate(params):
            p.grad = tens(z[f"r{rank}_t{t}_in{i}"]) if bool(z[f"has{i}"]) else None
        ddp.sync_gradients()
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            if not bool(z[f"has{i}"]):
                assert p.grad is None
                continue
            got = p.grad.detach().cpu()
            want = tens(z[f"r{rank}_t{t}_out{i}"]).cpu()
            if ws == 2:
                assert torch.equal(got, want), (dtype_name, rank, t, i)
            else:
                tol = 2.0 ** -7 if bf16 else 1e-6
                d = float((got.float() - want.float()).abs().max() / want.float().abs().max())
                assert d <= tol, (dtype_name, rank, t, i, d)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


@pytest.mark.parametrize("ws", [1, 2, 3])
def test_ddp_sync_gradients(gpu, ws):
    """DDP drop-in: the numpy restatement through a real backward (every ws), and the reference's
    own sync_gradients outputs (ws 2-3)."""
    cases = [(_ddp_worker, (d,)) for d in ("float32", "bfloat16")]
    if ws > 1:
        cases += [(_ddp_fixture_worker, (d,)) for d in ("float32", "bfloat16")]
    spawn_batch(ws, cases)


# (a wave step of the vector path covers 1024 fp32 / 2048 bf16 elements; the rest is the tail)
@pytest.mark.parametrize("n", [1, 7, 1000, 1024, 2051, 4099, 5 * 2048 + 1000, 1 << 20])
@pytest.mark.parametrize("div", [2.0, 3.0, 8.0, 6.0])
@pytest.mark.parametrize("nt", [-1, 1])  # cache policy by size (here: default) / forced non-temporal
def test_scale_kernel_bit_exact(gpu, n, div, nt):
    from zero_amd import _lib
    from zero_amd.comm import zs_dtype

    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g) * 10
    for dt in (torch.float32, torch.bfloat16):
        d = x.to(dt).to(gpu)
        _lib.call("zs_tune", b"scale_nt", nt, None)
        try:
            _lib.call("zs_scale", d.data_ptr(), n, zs_dtype(dt), div,
                      torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        finally:
            _lib.call("zs_tune", b"scale_nt", -1, None)
        if dt == torch.float32:
            want = x.numpy() / np.float32(div)
            assert np.array_equal(d.cpu().numpy(), want)
        else:
            want = (x.to(dt).float() / div).to(dt)
            assert torch.equal(d.cpu(), want)
