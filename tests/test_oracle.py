"""Pin the CPU oracle (numpy + C restatements) against the reference's own outputs."""
import numpy as np
import pytest

from conftest import GOLDEN
from oracle import c_oracle
from oracle import zero_oracle as zo

CASES = ["default", "wd", "amsgrad", "maximize", "adamw", "hyper"]
CFG = {
    "default": dict(),
    "wd": dict(weight_decay=1e-2),
    "amsgrad": dict(amsgrad=True),
    "maximize": dict(maximize=True),
    "adamw": dict(weight_decay=1e-2, decoupled=True),
    "hyper": dict(lr=1e-2, betas=(0.8, 0.99), eps=1e-6),
}


def rel(a, b):
    return float(np.max(np.abs(a.astype(np.float64) - b)) / max(np.max(np.abs(b)), 1e-30))


@pytest.mark.parametrize("case", CASES)
def test_numpy_adam_vs_torch_kat(golden, case):
    """adam_update restates torch.optim.Adam/AdamW (adam.py:394-547) within 1e-6 over 10 steps."""
    z = golden("adam_kat.npz")
    cfg = CFG[case]
    p = z[f"{case}_p0"].copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    vmax = np.zeros_like(p)
    for t, g in enumerate(z[f"{case}_grads"]):
        p, m, v, vmax = zo.adam_update(p, g, m, v, t + 1, vmax=vmax, **cfg)
    assert rel(p, z[f"{case}_p"]) <= 1e-6
    assert rel(m, z[f"{case}_m"]) <= 1e-6
    assert rel(v, z[f"{case}_v"]) <= 1e-6


@pytest.mark.parametrize("case", CASES)
def test_c_adam_vs_torch_kat(golden, case):
    z = golden("adam_kat.npz")
    cfg = dict(CFG[case])
    betas = cfg.pop("betas", (0.9, 0.999))
    p = z[f"{case}_p0"].copy()
    m, v, vmax = np.zeros_like(p), np.zeros_like(p), np.zeros_like(p)
    for t, g in enumerate(z[f"{case}_grads"]):
        hp = c_oracle.hparams(beta1=betas[0], beta2=betas[1], step=t + 1, **cfg)
        c_oracle.adam_f32(p, np.ascontiguousarray(g), m, v, hp, vmax=vmax if cfg.get("amsgrad") else None)
    assert rel(p, z[f"{case}_p"]) <= 1e-6
    assert rel(m, z[f"{case}_m"]) <= 1e-6
    assert rel(v, z[f"{case}_v"]) <= 1e-6
    if case == "amsgrad":
        assert rel(vmax, z["amsgrad_vmax"]) <= 1e-6


def test_c_and_numpy_oracles_agree_bitwise():
    rng = np.random.default_rng(0)
    p = rng.standard_normal(10001).astype(np.float32)
    m, v = np.zeros_like(p), np.zeros_like(p)
    pn, mn, vn = p.copy(), m.copy(), v.copy()
    for t in range(1, 6):
        g = rng.standard_normal(p.size).astype(np.float32) * 1e-3
        c_oracle.adam_f32(p, g, m, v, c_oracle.hparams(step=t))
        pn, mn, vn, _ = zo.adam_update(pn, g, mn, vn, t)
    # the numpy fma emulation double-rounds in rare cases: allow 1 ulp on a handful
    assert np.mean(p != pn) < 1e-3
    assert rel(p, pn) < 1e-7


def test_bf16_rounding_helpers():
    x = np.array([1.0, 1.00390625, 1.005859375, -2.5, np.inf, np.nan, 3.0e38], np.float32)
    bits = zo.f32_to_bf16_bits(x)
    import torch

    ref = torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    assert (bits[:5] == ref[:5]).all() and (bits[6] == ref[6])
    assert np.isnan(zo.bf16_bits_to_f32(bits)[5])


def _traj_files(variant):
    return sorted(p.name for p in GOLDEN.glob(f"traj_z{variant}_*.npz"))


def _load_case(z):
    ws, steps = int(z["ws"]), int(z["steps"])
    init = [z[f"init_{i}"] for i in range(12)]
    return ws, steps, init


@pytest.mark.parametrize("variant", [1, 2])
def test_simulate_with_fixture_grads(golden, variant):
    """The restated ZeRO-1 (incl. the carry) / ZeRO-2 step, fed the reference's own local grads,
    reproduces every rank's params after every step within 1e-6 (normwise)."""
    for name in _traj_files(variant):
        z = golden(name)
        ws, steps, init = _load_case(z)
        lg = lambda t, r, i: z[f"r{r}_t{t}_lg{i}"]  # noqa: E731
        out = zo.simulate(variant, ws, init, steps=steps, local_grads=lg)
        for t in range(steps):
            for r in range(ws):
                if f"r{r}_t{t}_p0" not in z.files:
                    continue
                for i in range(12):
                    assert rel(out["params"][t][r][i], z[f"r{r}_t{t}_p{i}"]) <= 1e-6, (name, t, r, i)
        for r in range(ws):  # final Adam state of owned params
            for i, (st, m, v, _) in out["state"][r].items():
                assert int(z[f"r{r}_state_{i}_step"]) == st
                assert rel(m, z[f"r{r}_state_{i}_exp_avg"]) <= 1e-6
                assert rel(v, z[f"r{r}_state_{i}_exp_avg_sq"]) <= 1e-6


@pytest.mark.parametrize("cfg,variant", [("c1", 1), ("c1", 2), ("c2", 2)])
def test_simulate_c1_full_width_samples(golden, cfg, variant):
    """BASELINE configs[0] at its real width (6 × Linear(10000, 10000), ws = 2, 3 steps of the
    exact hash gradients, tests/_c1.py): the restated step run on the fixture's sampled elements
    alone reproduces the reference's sampled params on both ranks after every step (incl. ZeRO-1's
    carry) and the owned params' Adam state, within 1e-6 — and the hash gradients themselves are
    the ones the reference consumed (their sampled values, recomputed here, drive the match).
    configs[1] (c2): the same MLP at D = 4096 under ZeRO-2."""
    import _c1

    z = golden(f"{cfg}_z{variant}_ws2_sampled.npz")
    ws, steps, d = int(z["ws"]), int(z["steps"]), int(z["D"])
    assert (ws, steps, d) == (_c1.WS, _c1.STEPS, {"c1": _c1.D, "c2": _c1.D_C2}[cfg])
    idx = [z[f"idx_{i}"] for i in range(12)]
    for i, s in enumerate(_c1.shapes(d)):  # the fixture's sample is the one tests/_c1.py draws
        assert np.array_equal(idx[i], _c1.sample_idx(i, int(np.prod(s))))
    init = [z[f"init_{i}"] for i in range(12)]
    out = zo.simulate(variant, ws, init, steps=steps,
                      local_grads=lambda t, r, i: _c1.grad_np(t, r, i, idx[i]))
    for t in range(steps):
        for r in range(ws):
            for i in range(12):
                assert rel(out["params"][t][r][i], z[f"r{r}_t{t}_p{i}"]) <= 1e-6, (t, r, i)
    for r in range(ws):
        assert z[f"r{r}_local"].tolist() == list(range(*zo.owner_range(12, ws, r)))
        for i, (st, m, v, _) in out["state"][r].items():
            assert int(z[f"r{r}_state_{i}_step"]) == st == steps
            assert rel(m, z[f"r{r}_state_{i}_exp_avg"]) <= 1e-6
            assert rel(v, z[f"r{r}_state_{i}_exp_avg_sq"]) <= 1e-6
    # the update moved every parameter (a fixture of unchanged params would pin nothing)
    assert all(not np.array_equal(z[f"r0_t{steps - 1}_p{i}"], init[i]) for i in range(12))


def test_simulate_zero3_reference_mode(golden):
    """ZeRO-3 reference: params never change (zero3.py:150-153 for-else) and the reduced shards
    are Σ_r chunk_r(grad_r)/ws, bit-compatible within 1e-6 of the reference's all_reduce."""
    for name in _traj_files(3):
        z = golden(name)
        ws, steps, init = _load_case(z)
        g = lambda t, r, i: z[f"r{r}_t{t}_g{i}"]  # noqa: E731  (grads as step() saw them)
        out = zo.simulate(3, ws, init, steps=steps, local_grads=g)
        for t in range(steps):
            for r in range(ws):
                if f"r{r}_t{t}_red0" not in z.files:
                    continue
                for k in range(12):
                    assert rel(out["reduced"][t][r][k], z[f"r{r}_t{t}_red{k}"]) <= 1e-6, (name, t, r, k)
                for i in range(12):  # the rank's (shard) params are the init chunk, unchanged
                    p = z[f"r{r}_t{t}_p{i}"]
                    a, b = zo.chunk_rows(init[i].shape[0], ws, r)
                    assert np.array_equal(p, init[i][a:b])


@pytest.mark.parametrize("name", ["traj_z1_ws2_d16_distinct.npz", "traj_z2_ws4_d16_distinct.npz",
                                  "traj_z2_ws1_d16_ref.npz"])
def test_simulate_end_to_end_mlp(golden, name):
    """Full restatement (numpy forward/backward + ZeRO semantics) tracks the reference within
    matmul-reassociation noise."""
    z = golden(name)
    ws, steps, init = _load_case(z)
    variant = int(name[6])
    xs = [z["x"] if "x" in z.files else z[f"r{r}_x"] for r in range(ws)]
    ys = [z["y"] if "y" in z.files else z[f"r{r}_y"] for r in range(ws)]
    out = zo.simulate(variant, ws, init, xs, ys, steps=steps)
    for i in range(12):
        assert rel(out["params"][-1][0][i], z[f"r0_t{steps - 1}_p{i}"]) <= 1e-4


def test_split_master_encoding():
    """The split master (include/zero_amd.h ZS_BF16_SPLIT) as the C oracle states it: hi is the RNE
    bf16 of the master; (hi, lo) gives the master back bit for bit, except an exact tie that rounds
    down to an even hi, which comes back 1 ulp toward zero (hi unchanged); NaN stays NaN."""
    from oracle import c_oracle

    rng = np.random.default_rng(7)
    x = (rng.standard_normal(1 << 20) * 0.02).astype(np.float32)
    u = x.view(np.uint32)
    u[:4] = [0x3C808000, 0x3C818000, 0xBC808000, 0x00008000]  # even tie, odd tie, -even, denormal
    u[4:8] = [0x7F7FFFFF, 0x7F7F8000, 0x7F800000, 0x7FC00001]  # overflow to inf, inf, NaN
    hi, lo = c_oracle.split_master(x)
    assert np.array_equal(hi[:7], zo.f32_to_bf16_bits(x[:7]))
    back = c_oracle.join_master(hi, lo).view(np.uint32)
    tie_even = ((u & 0xFFFF) == 0x8000) & (((u >> 16) & 1) == 0)
    ok = ~tie_even
    ok[7] = False
    assert np.array_equal(back[ok], u[ok])
    assert np.array_equal(back[tie_even], u[tie_even] - 1)
    assert np.array_equal(c_oracle.split_master(back[tie_even].view(np.float32))[0], hi[tie_even])
    assert np.isnan(back[7:8].view(np.float32)).all()
    assert 0 < tie_even.sum() < 64  # ~2^-17 of uniformly random masters (+ the planted one)


def test_split_master_adam_tracks_fp32_master():
    """Adam on the split master follows the fp32-master oracle: identical bf16 params and state
    over 20 steps except where a tie nudge (1 ulp of the master) propagated."""
    from oracle import c_oracle

    rng = np.random.default_rng(3)
    n = 1 << 16
    master = (rng.standard_normal(n) * 0.02).astype(np.float32)
    hi, lo = c_oracle.split_master(master)
    master = c_oracle.join_master(hi, lo)  # start from a representable master
    m1, v1, m2, v2 = (np.zeros(n, np.float32) for _ in range(4))
    p_ref = np.zeros(n, np.uint16)
    for t in range(1, 21):
        g = zo.f32_to_bf16_bits((rng.standard_normal(n) * 1e-2).astype(np.float32))
        hp = c_oracle.hparams(step=t, grad_div=2.0)
        c_oracle.adam_bf16(master, p_ref, g, m1, v1, hp)
        c_oracle.adam_bf16_split(hi, lo, g, m2, v2, hp)
    joined = c_oracle.join_master(hi, lo)
    diff = joined.view(np.uint32) != master.view(np.uint32)
    assert diff.mean() < 1e-3
    assert np.max(np.abs(joined - master)) <= 4 * np.max(np.spacing(np.abs(master)))
    assert np.mean(hi != p_ref) < 1e-3


def _cpu_step_worker(rank, ws, port, variant, name):
    import os

    import torch
    import torch.distributed as dist

    from oracle.zero_cpu_step import ReferenceStepCPU

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    z = np.load(GOLDEN / name)
    params = [torch.nn.Parameter(torch.from_numpy(z[f"init_{i}"].copy())) for i in range(12)]
    opt = ReferenceStepCPU(params, variant=variant)
    for t in range(int(z["steps"])):
        opt.zero_grad()
        for i, p in enumerate(params):  # backward accumulates into a surviving grad (carry)
            g = torch.from_numpy(z[f"r{rank}_t{t}_lg{i}"].copy())
            p.grad = g if p.grad is None else p.grad + g
        opt.step()
        if f"r{rank}_t{t}_p0" in z.files:
            for i, p in enumerate(params):
                ref = z[f"r{rank}_t{t}_p{i}"]
                assert np.max(np.abs(p.detach().numpy() - ref)) <= 1e-6 * np.max(np.abs(ref)), (t, i)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("variant,ws", [(1, 2), (2, 2), (1, 3), (2, 4)])
def test_cpu_reference_step_restatement(variant, ws):
    """oracle/zero_cpu_step.py (bench.py's cpu_baseline: the reference's per-tensor gloo step +
    torch.optim.Adam on the host cores) reproduces the reference's own trajectories."""
    import torch.multiprocessing as mp

    from conftest import free_port

    mp.spawn(_cpu_step_worker, args=(ws, free_port(), variant, f"traj_z{variant}_ws{ws}_d16_distinct.npz"),
             nprocs=ws, join=True)


@pytest.mark.parametrize("ws", [2, 3])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_ddp_sync_restatement_vs_reference(golden, ws, dtype):
    """zero_oracle.ddp_sync against the reference's own SimpleDistributedDataParallelism
    (tests/golden/make_ddp_golden.py: its class, run on gloo): bit-exact for fp32 at ws=2 and
    for bf16 at ws=2 (a two-term sum rounds once in any order); at ws=3 within the ring's
    summation-order noise (fp32 1e-6, bf16 2^-7 normwise)."""
    z = golden(f"ddp_sync_ws{ws}_{dtype}.npz")
    bf16 = dtype == "bfloat16"

    def val(a):
        return zo.bf16_bits_to_f32(a).reshape(a.shape) if bf16 else a

    for t in range(3):
        for i in range(6):
            if not bool(z[f"has{i}"]):
                assert f"r0_t{t}_out{i}" not in z.files  # no gradient: skipped, stays None
                continue
            want = zo.ddp_sync([val(z[f"r{r}_t{t}_in{i}"]) for r in range(ws)], bf16=bf16)
            for r in range(ws):
                got = val(z[f"r{r}_t{t}_out{i}"])
                if ws == 2:
                    assert np.array_equal(got, want), (ws, dtype, t, i, r)
                else:
                    tol = 2.0 ** -7 if bf16 else 1e-6
                    assert np.max(np.abs(got - want)) <= tol * np.max(np.abs(want)), (ws, dtype, t, i, r)
