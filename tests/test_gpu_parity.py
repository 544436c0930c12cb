"""ShardedOptimizer on the MI355X vs the reference's own trajectories (tests/golden).

Single-process cases run the product path end to end (RCCL communicator included at ws=1).
Multi-rank cases run ws processes on the one GPU of the box: pack / fused Adam / unpack are the
real HIP kernels, and the exchange goes through tests/_gloo_comm.py's gloo-staged communicator
here; tests/test_gpu_rccl.py re-runs the same workers through the product's RCCL communicator
between ranks that share the device (each rank its own RCCL node, NCCL_HOSTID).
Tolerance: 1e-6 normwise relative (north star), every step.
"""

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, free_port
from _zero_run import spawn_batch, spawn_ranks, init_pg, rel, run_injected, set_grad

pytestmark = pytest.mark.gpu


def _port():
    return free_port()


@pytest.fixture
def pg1():
    init_pg(0, 1, _port())
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("mode", ["ref", "distinct"])
def test_ws1_injected(gpu, golden, pg1, variant, mode):
    z = golden(f"traj_z{variant}_ws1_d16_{mode}.npz")
    run_injected(z, variant, 0, 1, gpu)


@pytest.mark.parametrize("variant", [1, 2])
def test_ws1_end_to_end_training(gpu, golden, pg1, variant):
    """The reference loop (zero_grad → forward → mse → backward → step) on the GPU; grads come
    from hipBLAS GEMMs, so the bound is matmul-reassociation noise, not 1e-6."""
    from _zero_run import module_for

    z = golden(f"traj_z{variant}_ws1_d16_ref.npz")
    torch.manual_seed(0)
    layers = []
    for i in range(6):
        lin = torch.nn.Linear(16, 16)
        lin.weight.data = torch.from_numpy(z[f"init_{2 * i}"].copy())
        lin.bias.data = torch.from_numpy(z[f"init_{2 * i + 1}"].copy())
        layers += [lin, torch.nn.ReLU()] if i < 5 else [lin]
    model = torch.nn.Sequential(*layers).to(gpu)
    opt = module_for(variant).ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3))
    x, y = torch.from_numpy(z["x"]).to(gpu), torch.from_numpy(z["y"]).to(gpu)
    for _ in range(int(z["steps"])):
        opt.zero_grad()
        loss = torch.nn.functional.mse_loss(model(x), y)
        loss.backward()
        opt.step()
    for i, p in enumerate(model.parameters()):
        assert rel(p.detach().cpu().numpy(), z[f"r0_t9_p{i}"]) <= 1e-4


def test_rccl_comm_ws1(gpu, pg1):
    """The RCCL communicator bootstraps and its collectives are the identity at ws=1."""
    from zero_amd.comm import RcclComm, rccl_version

    assert rccl_version() == int("".join(f"{x:02d}" if i else str(x)
                                         for i, x in enumerate(torch.cuda.nccl.version())))
    comm = RcclComm()
    t = torch.arange(1000, dtype=torch.float32, device=gpu)
    ref = t.clone()
    st = torch.cuda.current_stream()
    comm.reduce_scatter(t, t, st)
    comm.all_gather(t, t, st)
    comm.all_reduce(t, st)
    comm.reduce_v(t, [64], [900], st)      # ncclReduce / ncclBroadcast in an RCCL group
    comm.broadcast_v(t, [0], [1000], st)
    b = t.to(torch.bfloat16)
    comm.all_reduce(b, st)
    torch.cuda.synchronize()
    assert torch.equal(t, ref) and torch.equal(b, ref.to(torch.bfloat16))
    comm.close()


def test_rccl_table_collectives_ws1(gpu, pg1):
    """The table forms (zs_all_gather_group / zs_reduce_scatter_group / zs_reduce_group /
    zs_broadcast_group) are copies at ws=1: every entry lands at its own destination, zero-count
    entries are skipped, bf16 and fp32; and the GlooStagedComm adapter's raw-pointer views
    (__cuda_array_interface__) see the same memory."""
    from _gloo_comm import _dev_view
    from zero_amd import _lib
    from zero_amd.comm import RcclComm

    comm = RcclComm()
    st = torch.cuda.current_stream()
    for dt, code in ((torch.float32, _lib.ZS_F32), (torch.bfloat16, _lib.ZS_BF16)):
        counts = np.array([1000, 0, 7, 4096], np.int64)
        src = [torch.randn(int(n) or 1, device=gpu).to(dt) for n in counts]
        dst = [torch.zeros(int(n) or 1, device=gpu, dtype=dt) for n in counts]
        sp = np.array([t.data_ptr() for t in src], np.uint64)
        for fn in (comm.all_gather_group, comm.reduce_scatter_group):
            for d in dst:
                d.zero_()
            dp = np.array([t.data_ptr() for t in dst], np.uint64)
            fn(sp, dp, counts, code, st)
            torch.cuda.synchronize()
            for n, a, b in zip(counts, src, dst):
                if n:
                    assert torch.equal(a, b), (fn.__name__, dt, n)
                else:
                    assert not b.any()  # a zero-count entry touches nothing
        v = _dev_view(src[0].data_ptr(), counts[0], code)
        assert v.dtype == dt and torch.equal(v, src[0])
    buf = torch.arange(64, dtype=torch.float32, device=gpu)
    out = torch.zeros_like(buf)
    one = lambda *a: np.array(a)  # noqa: E731
    comm.reduce_group(one(buf.data_ptr()).astype(np.uint64), one(out.data_ptr()).astype(np.uint64),
                      one(64).astype(np.int64), one(0).astype(np.int32), _lib.ZS_F32, st)
    comm.broadcast_group(one(out.data_ptr()).astype(np.uint64), one(64).astype(np.int64),
                         one(0).astype(np.int32), _lib.ZS_F32, st)
    torch.cuda.synchronize()
    assert torch.equal(out, buf)
    comm.close()


def _mr_worker(rank, ws, port, variant, name, buckets="ragged", arena=None):
    import sys
    from conftest import PKG, REPO  # noqa: F401  (sets sys.path in the child)
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    z = np.load(GOLDEN / name)
    run_injected(z, variant, rank, ws, torch.device("cuda:0"), comm=test_comm(), buckets=buckets,
                 arena=arena)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


MR_CASES = [(v, f"traj_z{v}_ws{ws}_d16_{m}.npz") for v in (1, 2) for ws in (2, 3, 4, 8)
            for m in ("ref", "distinct")] + [(1, "traj_z1_ws2_d64_ref.npz"),
                                             (2, "traj_z2_ws4_d64_distinct.npz")]


def _ws_of(name):
    return int(name.split("_ws")[1].split("_")[0])


@pytest.mark.parametrize("ws", [2, 3, 4, 8])
def test_multirank_injected(gpu, ws):
    """The default ws > 1 exchange (flat parameter arena: grouped reduce / broadcast rounds, no
    pack / unpack) against the reference's trajectories, ws 2-8 incl. ZeRO-1's carry (every
    fixture of this ws, ref and distinct data, ZeRO-1 and ZeRO-2, in one set of processes)."""
    if ws == 8 and not os.environ.get("ZS_GPU_FULL"):
        pytest.skip("gloo-staged twin of tests/test_gpu_rccl.py at ws = 8 (the same cases through "
                    "the product's RCCL communicator); ZS_GPU_FULL=1 runs it too")
    spawn_batch(ws, [(_mr_worker, (v, name)) for v, name in MR_CASES if _ws_of(name) == ws])


BUCKET_CASES = [(1, 3, "ragged"), (1, 3, "padded"), (2, 3, "padded"), (2, 4, "ragged"),
                (1, 8, "ragged"), (2, 8, "ragged")]


@pytest.mark.parametrize("ws", [3, 4, 8])
def test_multirank_injected_bucket_arena(gpu, ws):
    """The rank-major bucket arena (pack / reduce-scatter / all-gather / unpack, ablation), with
    the ragged tail or the zero-padded bucket schedule."""
    spawn_batch(ws, [(_mr_worker, (v, f"traj_z{v}_ws{ws}_d16_distinct.npz", b, "buckets"))
                     for v, w, b in BUCKET_CASES if w == ws])


def _edge_worker(rank, ws, port, variant, buckets, arena="flat"):
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from _zero_run import module_for
    from oracle import zero_oracle as zo

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    shapes = [(33,), (0,), (7, 5)]  # fewer params than ranks (rank 3 owns nothing), a 0-size param
    g = torch.Generator().manual_seed(5)
    init = [torch.randn(s, generator=g).numpy() for s in shapes]
    steps = 3
    lg = {(t, r, i): (torch.randn(s, generator=torch.Generator().manual_seed(100 * t + 10 * r + i))
                      * 1e-2).numpy() for t in range(steps) for r in range(ws) for i, s in enumerate(shapes)}
    want = zo.simulate(variant, ws, init, steps=steps, local_grads=lambda t, r, i: lg[(t, r, i)])
    params = [torch.nn.Parameter(torch.from_numpy(a.copy()).to(dev)) for a in init]
    opt = module_for(variant).ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), comm=test_comm(),
                                               bucket_mb=ws * 64 * 4 / (1 << 20), buckets=buckets,
                                               arena=arena)
    if arena == "auto":
        from _zero_run import check_auto_arena

        check_auto_arena(opt, ws)
    if rank == 3:
        assert opt.local_param_indices == []
    for t in range(steps):
        opt.zero_grad()
        for i, p in enumerate(params):
            set_grad(p, torch.from_numpy(lg[(t, rank, i)].copy()).to(dev))
        opt.step()
        for i, p in enumerate(params):
            ref = want["params"][t][rank][i]
            got = p.detach().cpu().numpy()
            assert got.shape == ref.shape
            if ref.size:
                assert rel(got, ref) <= 1e-6, (variant, rank, t, i)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def test_multirank_fewer_params_than_ranks(gpu):
    """Edge cases of the reference's ownership rule on the device path: n < ws (empty ranks) and a
    zero-element parameter, against the oracle's restatement of the reference (ZeRO-1 and 2; flat
    arena, ragged and padded bucket arena, and arena="auto" calibrating with an owner of nothing)."""
    spawn_batch(4, [(_edge_worker, (v, b, a)) for v in (1, 2)
                    for b, a in (("ragged", "flat"), ("ragged", "buckets"), ("padded", "buckets"),
                                 ("ragged", "auto"))])


HP_CASES = {
    "adamw_amsgrad_2groups": (torch.optim.AdamW, [dict(lr=1e-3, weight_decay=0.05, amsgrad=True),
                                                  dict(lr=3e-3, weight_decay=0.0, amsgrad=True)]),
    "adam_l2_maximize": (torch.optim.Adam, [dict(lr=2e-3, weight_decay=0.01, maximize=True)]),
}


def _hp_worker(rank, ws, port, variant, case):
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from _zero_run import module_for
    from oracle import zero_oracle as zo

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    cls, groups = HP_CASES[case]
    shapes = [(48, 8), (48,), (20, 9), (20,), (7,), (64, 3)]
    g = torch.Generator().manual_seed(9)
    init = [torch.randn(s, generator=g).numpy() for s in shapes]
    steps = 4
    lg = {(t, r, i): (torch.randn(s, generator=torch.Generator().manual_seed(1000 * t + 10 * r + i))
                      * 1e-2).numpy() for t in range(steps) for r in range(ws) for i, s in enumerate(shapes)}
    group_of = [0 if i < 3 or len(groups) == 1 else 1 for i in range(len(shapes))]

    def kw_of(i):
        h = groups[group_of[i]]
        return dict(lr=h["lr"], weight_decay=h.get("weight_decay", 0.0), amsgrad=h.get("amsgrad", False),
                    maximize=h.get("maximize", False), decoupled=cls is torch.optim.AdamW)

    want = zo.simulate(variant, ws, init, steps=steps, local_grads=lambda t, r, i: lg[(t, r, i)],
                       adam_kw=kw_of)
    params = [torch.nn.Parameter(torch.from_numpy(a.copy()).to(dev)) for a in init]
    pg = [dict(params=[p for p, gi in zip(params, group_of) if gi == k], **h) for k, h in enumerate(groups)]
    opt = module_for(variant).ShardedOptimizer(cls(pg), comm=test_comm(),
                                               bucket_mb=ws * 128 * 4 / (1 << 20))
    for t in range(steps):
        opt.zero_grad()
        for i, p in enumerate(params):
            set_grad(p, torch.from_numpy(lg[(t, rank, i)].copy()).to(dev))
        opt.step()
        for i, p in enumerate(params):
            assert rel(p.detach().cpu().numpy(), want["params"][t][rank][i]) <= 1e-6, (case, rank, t, i)
    for i, (st, m, v, vm) in want["state"][rank].items():
        s = opt.optimizer.state[params[i]]
        assert int(s["step"].item()) == st
        assert rel(s["exp_avg"].cpu().numpy(), m) <= 1e-6
        if kw_of(i)["amsgrad"]:
            assert rel(s["max_exp_avg_sq"].cpu().numpy(), vm) <= 1e-6
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def test_multirank_hyperparameters(gpu):
    """AdamW / L2 weight decay / amsgrad / maximize and per-group lr through the ws=3 exchange
    against the oracle's restatement of the reference (ZeRO-1 and ZeRO-2, every case)."""
    spawn_batch(3, [(_hp_worker, (v, c)) for v in (1, 2) for c in sorted(HP_CASES)])


def test_profiler_ranges_match_reference_names(gpu, pg1):
    """torch.profiler shows the reference's step() ranges (zero1.py:80-91) around the native work."""
    from torch.profiler import ProfilerActivity, profile
    from zero_amd import zero2

    ps = [torch.nn.Parameter(torch.randn(256, 64, device=gpu)) for _ in range(3)]
    opt = zero2.ShardedOptimizer(torch.optim.Adam(ps, lr=1e-3))
    for p in ps:
        p.grad = torch.randn_like(p)
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        opt.step()
    names = {e.name for e in prof.events()}
    assert "optimizer_step" in names


@pytest.mark.parametrize("variant", [1, 2, 3])
def test_reference_harness_runs(gpu, variant):
    """zero_amd.harness: the reference's train() / test_zeroN() experiment (shrunken) on one GPU,
    through the same CLI a user would call; the sharded run reports its timing summary."""
    import subprocess
    import sys

    from conftest import PKG

    env = dict(__import__("os").environ, MASTER_PORT=str(_port()), PYTHONPATH=str(PKG))
    r = subprocess.run([sys.executable, "-m", "zero_amd.harness", "--zero", str(variant),
                        "--width", "512", "--steps", "3"], capture_output=True, text=True,
                       timeout=180, env=env, cwd=str(PKG))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "Memory Usage Summary" in r.stdout and "Average step time" in r.stdout


def _carry_worker(rank, ws, port, clear):
    """ZeRO-1's carry follows what the loop clears (zero1.py:107-108): opt.zero_grad() clears only
    owned grads, so the others' surviving averaged grads carry into the next all-reduce;
    model.zero_grad() clears every grad, so nothing carries.  Both against the oracle."""
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from zero_amd import zero1
    from oracle import zero_oracle as zo

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    shapes = [(40, 6), (40,), (17, 3), (5,), (64,)]
    g = torch.Generator().manual_seed(11)
    init = [torch.randn(s, generator=g).numpy() for s in shapes]
    steps = 4
    lg = {(t, r, i): (torch.randn(s, generator=torch.Generator().manual_seed(97 * t + 13 * r + i))
                      * 1e-2).numpy() for t in range(steps) for r in range(ws) for i, s in enumerate(shapes)}
    want = zo.simulate(1, ws, init, steps=steps, local_grads=lambda t, r, i: lg[(t, r, i)],
                       zero_grad=clear)
    model = torch.nn.ParameterList([torch.nn.Parameter(torch.from_numpy(a.copy()).to(dev)) for a in init])
    params = list(model)
    opt = zero1.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), comm=test_comm(),
                                 bucket_mb=ws * 64 * 4 / (1 << 20))
    for t in range(steps):
        if clear == "model":
            model.zero_grad()  # set_to_none: backward then hands over fresh grads
        else:
            opt.zero_grad()
        for i, p in enumerate(params):
            set_grad(p, torch.from_numpy(lg[(t, rank, i)].copy()).to(dev))
        opt.step()
        for i, p in enumerate(params):
            assert rel(p.detach().cpu().numpy(), want["params"][t][rank][i]) <= 1e-6, (clear, rank, t, i)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def _c1_worker(rank, ws, port, cases=(("c1", 1), ("c1", 2), ("c2", 2))):
    """BASELINE configs[0] at its real width against the reference (tests/_c1.py): the reference's
    6 × Linear(10000, 10000) (600,060,000 fp32 params, its own init) through ZeRO-1 and ZeRO-2 at
    ws = 2 for 3 steps of the exact hash gradients; every parameter's sampled elements on this
    rank after every step, and the owned parameters' Adam state, within 1e-6 of the reference's
    (tests/golden/c1_z{1,2}_ws2_sampled.npz), and every parameter's fp64 sum within 1e-6 of
    Σ|p|.  The model is built once per width (on the CPU, as the reference's).  configs[1] (c2):
    the same MLP at D = 4096 (100,687,872 params) under ZeRO-2."""
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from _zero_run import module_for
    import _c1

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    widths = {"c1": _c1.D, "c2": _c1.D_C2}
    built = {}
    for cfg, variant in cases:
        d = widths[cfg]
        if d not in built:  # the reference's init (torch.manual_seed(0), CPU)
            built.clear()
            built[d] = [p.detach() for p in _c1.make_model(d).parameters()]
        init = built[d]
        z = np.load(GOLDEN / f"{cfg}_z{variant}_ws2_sampled.npz")
        assert int(z["ws"]) == ws
        idx = [torch.from_numpy(z[f"idx_{i}"]).to(dev) for i in range(12)]
        for i, p in enumerate(init):
            assert np.array_equal(p.reshape(-1)[torch.from_numpy(z[f"idx_{i}"])].numpy(),
                                  z[f"init_{i}"]), i
        params = [torch.nn.Parameter(p.to(dev)) for p in init]
        s0 = params[0].detach().reshape(-1).double().sum().item()
        assert abs(s0 - z["initsum_0"][0]) <= 1e-9 * z["initsum_0"][1]

        def sampled(t, i):
            return t.detach().reshape(-1)[idx[i]].cpu().numpy()

        opt = module_for(variant).ShardedOptimizer(torch.optim.Adam(params, lr=1e-3),
                                                   comm=test_comm())
        assert opt.local_param_indices == z[f"r{rank}_local"].tolist()
        for t in range(int(z["steps"])):
            opt.zero_grad()
            for i, p in enumerate(params):
                set_grad(p, _c1.grad_torch(t, rank, i, p.shape, dev))
            opt.step()
            for i, p in enumerate(params):
                e = rel(sampled(p, i), z[f"r{rank}_t{t}_p{i}"])
                assert e <= 1e-6, (variant, rank, t, i, e)
                d = p.detach().reshape(-1).double()
                s, a = z[f"r{rank}_t{t}_psum{i}"]
                assert abs(d.sum().item() - s) <= 1e-6 * a, (variant, rank, t, i, d.sum().item(), s)
                del d
        for i, p in enumerate(params):
            key = f"r{rank}_state_{i}_exp_avg"
            if key in z.files:
                st = opt.optimizer.state[p]
                assert int(st["step"].item()) == int(z[f"r{rank}_state_{i}_step"])
                assert rel(sampled(st["exp_avg"], i), z[key]) <= 1e-6
                assert rel(sampled(st["exp_avg_sq"], i), z[f"r{rank}_state_{i}_exp_avg_sq"]) <= 1e-6
        del opt, params
        torch.cuda.empty_cache()
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def test_zero1_carry_follows_zero_grad(gpu):
    spawn_batch(3, [(_carry_worker, (c,)) for c in ("optimizer", "model")])


def _bf16comm_worker(rank, ws, port, which):
    """grad_comm="bf16" (SURVEY.md §8(f) 4): fp32 params, fp32 grads converted to bf16 for the
    exchange.  Every step, on every rank:
      (1) the reduced bf16 sum the exchange delivered — captured before Adam reads it (the flat
          arena's R; ZeRO-3's grad chunk arena) — is within ws·2^-8·Σ_r|bf16(g_r)| of the exact
          sum Σ_r bf16(g_r), element by element (RCCL's ring adds in fp32 and rounds each of its
          ws-1 partial sums to bf16: one rounding of at most 2^-9 of Σ|g| per hop, doubled);
      (2) the updated parameters, exp_avg and exp_avg_sq equal the C oracle's Adam applied to that
          captured sum and the state before the step, bit for bit;
      (3) the trajectory stays within 2e-2 of the reference's fp32 trajectory (the price of bf16
          gradients; opt-in).
    Where the exchange rounds the fp32 sum once (the gloo-staged communicator, and any ring at
    ws = 2) the trajectory also follows the oracle's emulation of the exchange within 1e-4."""
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from oracle import c_oracle
    from oracle import zero_oracle as zo
    from zero_amd import zero2, zero3

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    z = np.load(GOLDEN / f"traj_z2_ws{ws}_d16_distinct.npz")
    init = [z[f"init_{i}"] for i in range(12)]
    params = [torch.nn.Parameter(torch.from_numpy(a.copy()).to(dev)) for a in init]
    rccl = os.environ.get("ZS_TEST_COMM") == "rccl"
    want = None
    if not rccl or ws == 2:
        want = zo.simulate(2, ws, init, local_grads=lambda t, r, i: z[f"r{r}_t{t}_lg{i}"],
                           grad_comm="bf16")
    if which in ("zero2", "zero2_overlap"):
        opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), comm=test_comm(),
                                     bucket_mb=ws * 64 * 4 / (1 << 20), grad_comm="bf16",
                                     overlap=which == "zero2_overlap", overlap_bucket_mb=2e-3)
        eng = opt.engine
        assert eng.R.dtype == torch.bfloat16
        cap = torch.zeros(max(eng.L, 1), dtype=torch.bfloat16, device=dev)
        pc = eng.pieces
        # param index -> (captured sum, rows of the full tensor) of every param this rank updates
        own = {int(i): (slice(int(so), int(so) + int(n)), slice(None))
               for i, so, n in zip(pc.param, pc.stream_off, pc.length) if n > 0}
        reduced = lambda i: cap[own[i][0]]  # noqa: E731
    else:
        opt = zero3.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), update=True,
                                     comm=test_comm(), grad_comm="bf16")
        assert opt.grad_arena().dtype == torch.bfloat16
        ar = opt._arena
        own = {}
        for i in range(12):
            r0, r1, row = ar.rows[i]
            if r1 > r0:
                own[i] = (slice(int(ar.slot[i]), int(ar.slot[i]) + int(ar.ln[i])), slice(r0, r1))
        reduced = lambda i: opt.grad_arena()[own[i][0]]  # noqa: E731
    cs = lambda a: a if which != "zero3" else a[rank * -(-a.shape[0] // ws):(rank + 1) * -(-a.shape[0] // ws)]  # noqa: E731
    bf = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(torch.bfloat16).double()  # noqa: E731
    worst = 0.0
    for t in range(int(z["steps"])):
        opt.zero_grad()
        before = {}
        for i, p in enumerate(params):
            if i in own:
                st = opt.optimizer.state[p]
                before[i] = [p.detach().cpu().numpy().reshape(-1).copy(),
                             st["exp_avg"].cpu().numpy().reshape(-1).copy(),
                             st["exp_avg_sq"].cpu().numpy().reshape(-1).copy()]
            g = torch.from_numpy(z[f"r{rank}_t{t}_lg{i}"].copy()).to(dev)
            if which != "zero3":
                set_grad(p, g)
            else:  # a full-size grad on a sharded param, as autograd leaves it
                shard = p.data
                p.data = torch.empty(g.shape, device=dev)
                p.grad = g
                p.data = shard
        if which != "zero3":
            opt.engine.capture_reduced = cap
        opt.step()
        torch.cuda.synchronize()
        hp = c_oracle.hparams(step=t + 1, grad_div=float(ws))
        for i, (_, rows) in own.items():
            got = reduced(i).double().cpu().reshape(-1)
            parts = [bf(z[f"r{r}_t{t}_lg{i}"])[rows].reshape(-1) for r in range(ws)]
            exact = sum(parts)
            bound = ws * 2.0 ** -8 * sum(q.abs() for q in parts)
            err = (got - exact).abs()
            over = err > bound
            assert not bool(over.any()), (which, rank, t, i, "reduced sum outside the ring bound",
                                          int(over.nonzero()[0]), float(err.max()))
            worst = max(worst, float((err / bound.clamp_min(1e-300)).max()))
            # (2) Adam on exactly that sum: bit for bit against the C oracle
            p0, m0, v0 = before[i]
            c_oracle.adam_f32(p0, got.float().numpy().copy(), m0, v0, hp)
            st = opt.optimizer.state[params[i]]
            for name, mine, ref in (("param", params[i].detach(), p0), ("exp_avg", st["exp_avg"], m0),
                                    ("exp_avg_sq", st["exp_avg_sq"], v0)):
                mb = mine.cpu().numpy().reshape(-1).view(np.uint32)
                assert np.array_equal(mb, ref.view(np.uint32)), (which, rank, t, i, name)
        for i, p in enumerate(params):
            got = p.detach().cpu().numpy()
            if want is not None:
                e = rel(got, cs(want["params"][t][rank][i]))
                assert e <= 1e-4, (which, rank, t, i, e)
            assert rel(got, cs(z[f"r{rank}_t{t}_p{i}"])) <= 2e-2, (which, rank, t, i)
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


@pytest.mark.parametrize("ws,whiches", [(3, ("zero2", "zero2_overlap", "zero3")), (4, ("zero2", "zero3"))])
def test_bf16_gradient_exchange_for_fp32_params(gpu, ws, whiches):
    spawn_batch(ws, [(_bf16comm_worker, (w,)) for w in whiches])


def _comm_time_worker(rank, ws, port):
    """The counters mean what the reference's mean: ZeRO-1 never counts
    communication (zero1.py:67-68); ZeRO-2 counts from step() entry to the end of the gradient
    reduction (zero2.py:92,116) — part of, never more than, step_time; ZeRO-3 likewise for its
    shard all-reduce (zero3.py:125,158)."""
    import sys
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from zero_amd import zero1, zero2, zero3

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    dev = torch.device("cuda:0")
    shapes = [(256, 64), (256,), (64, 32)]

    def run(make, steps=3, full_grads=False):
        g = torch.Generator().manual_seed(3)
        params = [torch.nn.Parameter(torch.randn(s, generator=g).to(dev)) for s in shapes]
        opt = make(params)
        for _ in range(steps):
            opt.zero_grad()
            for p, s in zip(params, shapes):
                gr = torch.randn(s, generator=g).to(dev)
                if full_grads and gr.shape != p.shape:
                    shard = p.data
                    p.data = torch.empty(gr.shape, device=dev)
                    p.grad = gr
                    p.data = shard
                else:
                    set_grad(p, gr)
            opt.step()
        torch.cuda.synchronize()
        return opt

    o1 = run(lambda ps: zero1.ShardedOptimizer(torch.optim.Adam(ps), comm=test_comm()))
    assert o1.communication_time == 0.0 and o1.step_time > 0
    for arena in ("flat", "buckets"):
        o2 = run(lambda ps: zero2.ShardedOptimizer(torch.optim.Adam(ps), comm=test_comm(),
                                                   arena=arena))
        assert 0.0 < o2.communication_time <= o2.step_time, (arena, o2.communication_time, o2.step_time)
    o3 = run(lambda ps: zero3.ShardedOptimizer(torch.optim.Adam(ps), comm=test_comm()),
             full_grads=True)
    assert 0.0 < o3.communication_time <= o3.step_time
    dist.barrier()
    dist.destroy_process_group()
    sys.stdout.flush()


def test_timing_counters_follow_reference(gpu):
    spawn_ranks(_comm_time_worker, 2, (2, _port()))
