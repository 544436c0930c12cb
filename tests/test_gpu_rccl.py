"""The multi-rank GPU workers again, through the PRODUCT communicator (RcclComm) instead of the
gloo-staged test one: real RCCL collectives between ws ranks that share the box's one GPU.

RCCL refuses two ranks of a communicator on one device when it sees them on one host; each rank
gets its own NCCL_HOSTID (tests/_gloo_comm.py ``test_comm``), so RCCL takes every rank for a
separate node and connects them through its socket transport over loopback.  The reductions,
copies, ring order, group semantics and bf16 rounding are RCCL's own, on the same device buffers
the engine hands to it on a real 8-GPU node — only the wire between ranks differs (sockets
instead of xGMI).  So these tests pin the ws > 1 calls of the product path: grouped
ncclReduce / ncclBroadcast rounds of the flat arena, in-place reduce-scatter / all-gather of the
bucket arena, the overlapped reduces from backward hooks, the ZeRO-3 table gathers and
reduce-scatters from module hooks, DDP's all-reduce.

Bounds are the workers' own (1e-6 against the reference's trajectories for fp32).  Cases whose
worker compares bit for bit against a rank-ordered fp32 sum stay at ws = 2, where every order of
a two-term sum is the same; ws 3-4 cases compare within tolerances that allow RCCL's ring order.
Finally bench.py runs at N = 2 with ``--share-gpu`` (same trick): its exchange checks, arena
calibration and ZeRO-3 gather check pass against real RCCL.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO, free_port
from _zero_run import CHILD_ENV, spawn_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl_env(monkeypatch):
    monkeypatch.setenv("ZS_TEST_COMM", "rccl")
    monkeypatch.setenv("NCCL_HOSTID", "zs-test-rank0")  # (restored after the test)
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    monkeypatch.setenv("NCCL_IB_DISABLE", "1")
    yield


def _batch(ws, cases):
    """The cases of one ws in one set of processes: every rank spawned (a failing rank takes the
    others down) up to ws = 4; at ws = 8 rank 0 runs here, as in the gloo-staged tests (9
    processes on the device stalled those)."""
    spawn_batch(ws, cases, all_spawned=ws <= 4)


def _zero12_cases(ws):
    from test_gpu_layouts import _worker as layout_worker
    from test_gpu_overlap import _ddp_fixture_worker, _ddp_worker, _frozen_worker, _mr_worker as ov_worker
    from test_gpu_parity import (_bf16comm_worker, _carry_worker, _comm_time_worker, _edge_worker,
                                 _hp_worker, _mr_worker)

    inj = {2: [(1, "distinct", None), (2, "distinct", None), (2, "distinct", "auto")],
           3: [(1, "distinct", "buckets")],
           4: [(1, "ref", None), (2, "distinct", None), (2, "distinct", "buckets")],
           8: [(2, "distinct", None), (1, "distinct", None), (2, "distinct", "buckets"),
               (1, "distinct", "buckets"), (1, "ref", None), (2, "ref", None),
               (1, "distinct", "auto")]}[ws]
    cases = [(_mr_worker, (v, f"traj_z{v}_ws{ws}_d16_{m}.npz", "ragged", a)) for v, m, a in inj]
    if ws == 2:
        from test_gpu_checkpoint import _ckpt_worker

        cases += [(_ckpt_worker, ("z1_fp32",)), (_ckpt_worker, ("z2_bf16_split",))]
        cases += [(_bf16comm_worker, ("zero2",)), (_comm_time_worker, ()),
                  (ov_worker, (1, "traj_z1_ws2_d16_distinct.npz", True, "flat")),
                  (_frozen_worker, (2, True)), (_ddp_worker, ("float32",)), (_ddp_worker, ("bfloat16",)),
                  (_ddp_fixture_worker, ("float32",)), (_ddp_fixture_worker, ("bfloat16",))]
    if ws == 3:
        cases += [(_hp_worker, (2, "adamw_amsgrad_2groups")), (_carry_worker, ("optimizer",)),
                  (_bf16comm_worker, ("zero2_overlap",)),
                  (ov_worker, (2, "traj_z2_ws3_d16_distinct.npz", True, "buckets")),
                  (_ddp_worker, ("float32",))]
    if ws == 4:
        cases += [(_edge_worker, (1, "ragged", "flat")), (_edge_worker, (2, "ragged", "flat")),
                  (_bf16comm_worker, ("zero2",)),
                  (ov_worker, (2, "traj_z2_ws4_d16_distinct.npz", True, "flat")),
                  (layout_worker, ("chunk", "traj_z2_ws4_d64_distinct.npz", "ragged", 64))]
    if ws in (2, 8):  # the layout ablation's balanced Layout F in the flat arena (bench.py N > 1)
        cases += [(layout_worker, ("flat", f"traj_z2_ws{ws}_d16_distinct.npz", "ragged", 128, "flat"))]
    if ws == 8:
        cases += [(_bf16comm_worker, ("zero2",))]
    return cases


@pytest.mark.parametrize("ws", [2, 3, 4])
def test_rccl_zero12(gpu, rccl_env, ws):
    """ZeRO-1/2 through real RCCL: the reference's trajectories on the flat arena (grouped reduce /
    broadcast rounds) and the bucket arena (in-place RS / AG); ws 2-4 add the overlapped backward,
    bf16 gradient exchange, hyper-parameters, the ZeRO-1 carry, empty ranks, the timing counters,
    DDP and the chunk layout."""
    _batch(ws, _zero12_cases(ws))


def test_rccl_c1_full_width(gpu, rccl_env):
    """BASELINE configs[0] at its real width (6 × Linear(10000, 10000), 600M fp32 params) at
    ws = 2 through real RCCL, ZeRO-1 (carry) and ZeRO-2, against the reference's sampled run
    (tests/_c1.py, test_gpu_parity._c1_worker): 2.4 GB reduced and broadcast per step; and
    configs[1] (D = 4096, 100M params) under ZeRO-2."""
    from test_gpu_parity import _c1_worker

    spawn_batch(2, [(_c1_worker, ())], all_spawned=True, deadline_s=300)


def _zero3_cases(ws):
    from test_gpu_fp8 import _mr as fp8_worker
    from test_gpu_parity import _bf16comm_worker
    from test_gpu_train import _mr_zero3
    from test_gpu_zero3 import _mem_worker, _mr

    cases = {2: [("_ref_mode", "traj_z3_ws2_d16_distinct.npz"),
                 ("_update_hooks", "traj_z2_ws2_d16_distinct.npz"),
                 ("_update_hooks_single", "traj_z2_ws2_d16_distinct.npz"),
                 ("_update_hooks_wave3", "traj_z2_ws2_d16_distinct.npz"),
                 ("_update_hooks_events", "traj_z2_ws2_d16_distinct.npz"),
                 ("_update_hooks_throttled", "traj_z2_ws2_d16_distinct.npz"),
                 ("_ref_mode_single", "traj_z3_ws2_d16_distinct.npz"),
                 ("_shards_changed", "traj_z2_ws2_d16_distinct.npz")],
             3: [("_update_injected", "traj_z2_ws3_d16_distinct.npz"),
                 ("_update_hooks_single", "traj_z2_ws3_d16_distinct.npz")],
             4: [("_ref_mode", "traj_z3_ws4_d16_distinct.npz"), ("_ref_injected", "traj_z3_ws4_d16_ref.npz"),
                 ("_update_hooks", "traj_z2_ws4_d16_distinct.npz"),
                 ("_update_hooks_single", "traj_z2_ws4_d16_distinct.npz"),
                 ("_update_hooks_throttled", "traj_z2_ws4_d16_distinct.npz")],
             # ws = 8: the exchanges the first 8-GPU run executes — table gathers from the module
             # hooks in forward and backward, backward reduce-scatters, the shard all-reduce
             8: [("_ref_mode", "traj_z3_ws8_d16_distinct.npz"), ("_ref_injected", "traj_z3_ws8_d16_ref.npz"),
                 ("_update_hooks", "traj_z2_ws8_d16_ref.npz"), ("_update_hooks", "traj_z2_ws8_d16_distinct.npz"),
                 ("_update_injected", "traj_z2_ws8_d16_distinct.npz"),
                 ("_update_hooks_single", "traj_z2_ws8_d16_distinct.npz")]}[ws]
    cases = [(_mr, c) for c in cases]
    if ws == 2:  # SmolLM3 ZeRO-3 AdamW bit-exact against the C oracle; fp8 gathers; checkpoint
        from test_gpu_checkpoint import _ckpt_worker

        cases += [(_ckpt_worker, ("z3_bf16",))]
        cases += [(_mr_zero3, (False, True)), (_mr_zero3, (True, False)),
                  (fp8_worker, (True,)), (fp8_worker, (False,))]
    if ws == 4:
        cases += [(_bf16comm_worker, ("zero3",)), (_mem_worker, ())]
    if ws == 8:
        cases += [(_bf16comm_worker, ("zero3",))]
    return cases


@pytest.mark.parametrize("ws", [2, 3, 4])
def test_rccl_zero3(gpu, rccl_env, ws):
    """ZeRO-3 through real RCCL: table gathers from the module hooks (reference and update mode),
    backward reduce-scatters, uneven chunks (ws = 3), bf16 gradient exchange, sharded gradient
    memory, fp8 gathers, SmolLM3 ZeRO-3 AdamW bit for bit against the C oracle, checkpointing."""
    _batch(ws, _zero3_cases(ws))


def test_rccl_ws8(gpu, rccl_env):
    """Every ws = 8 case through real RCCL in ONE set of eight processes sharing one communicator
    per rank (round 6: test_rccl_zero12[8] and test_rccl_zero3[8] merged — the same cases, one
    spawn and one RCCL bootstrap instead of two): ZeRO-1/2 trajectories on both arenas, the
    reference's injected step, arena="auto", the balanced Layout F, the bf16 exchange; then every
    ZeRO-3 exchange the 8-GPU run executes (hooked gathers in forward and backward, backward
    reduce-scatters, the reference mode's shard all-reduce, the bf16 exchange)."""
    _batch(8, _zero12_cases(8) + _zero3_cases(8))


# --- bench.py at N = 2 on the shared GPU ------------------------------------------------
def _bench2(args, timeout=300, launcher=True):
    """bench.py at N = 2 on the shared GPU, under torch.distributed.run (the driver's SCALE form)
    or, with ``launcher=False``, as plain ``python bench.py --gpus 2`` (bench.py starts the two
    ranks itself)."""
    env = dict(os.environ, **CHILD_ENV)
    for k in ("ZS_TEST_COMM", "NCCL_HOSTID", "WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)  # (bench --share-gpu sets NCCL_HOSTID per rank)
    launch = ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
              "127.0.0.1", "--master-port", str(free_port())] if launcher else []
    cmd = [sys.executable, *launch, "bench.py", "--gpus", "2",
           "--share-gpu", "--no-cpu-baseline", "--watchdog-s", str(timeout - 30)] + args
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("zero", [1, 2])
def test_bench_share_gpu_exchange_check(gpu, zero):
    """The N>1 bench path against real RCCL: communicator self-check, the exchange check of BOTH
    arenas (one real engine step on the bf16 arena vs the exact fp32 sum and a PyTorch Adam
    restatement; bit-identical parameters on every rank), calibration, timed steps.  ZeRO-2 runs
    as plain ``python bench.py --gpus 2`` (no launcher: bench.py starts the two ranks itself)."""
    out = _bench2(["--config", "C2", "--dtype", "bf16", "--zero", str(zero), "--steps", "3",
                   "--warmup", "1", "--no-comm-sweep"], launcher=zero == 1)
    assert out["n_gpus"] == 2 and out["rccl_selfcheck"]["all_ranks_ok"]
    assert out["config"]["parallelism"] == "dp2"
    for kind in ("flat", "buckets"):
        assert out["arena_calibration"][kind]["busbw_gbs"] > 0, out["arena_calibration"]
    assert out["config"]["comm"] == "rccl", out["config"]["comm"]
    assert out["rehearsal"].startswith("share-gpu")
    checks = out["exchange_check_all_arenas"]
    assert set(checks) == {"flat", "buckets"} and set(out["arena_calibration_ms_per_step"]) == set(checks)
    for kind, c in checks.items():
        assert c["all_ranks_ok"], (kind, c)
    if zero == 2:  # the balanced Layout F timed beside the reference layout
        lab = out["layout_ablation"]
        assert lab["exchange_check"]["all_ranks_ok"] and lab["ms_per_step"] > 0, lab
        assert lab["exchange_check"]["owned_pieces"] >= 1 and lab["rounds"] >= 1
        assert set(lab["expected"]) == {"reference_flat_arena", "balanced_F_flat_arena",
                                        "chunk_Z_bucket_arena"}


def test_bench_share_gpu_zero3_paramset(gpu):
    """configs[4]'s ZeRO-3 parameter-set step at N = 2 (2 layers): the gather check and a short
    bucket sweep through real RCCL."""
    out = _bench2(["--zero", "3", "--config", "C5", "--set-layers", "2", "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == 2
    assert out["exchange_check"]["all_ranks_ok"], out["exchange_check"]
    assert out["rehearsal"].startswith("share-gpu")


def test_bench_share_gpu_zero3_mlp(gpu):
    """configs[2]'s hooked ZeRO-3 training iteration (the reference MLP, here C2-wide) at N = 2:
    one real iteration through RCCL equals the unsharded plain-PyTorch iteration (fp32, the
    reference MLP's dtype and the bench's default here: within 1e-5; bf16 params: 2^-7)."""
    for dt, tol in (("fp32", 1e-5), ("bf16", 2.0 ** -7)):
        out = _bench2(["--zero", "3", "--config", "C2", "--dtype", dt, "--steps", "2", "--warmup", "1"])
        assert out["n_gpus"] == 2 and out["rehearsal"].startswith("share-gpu")
        assert out["config"]["param_dtype"] == dt
        chk = out["exchange_check"]
        assert chk["all_ranks_ok"] and chk["max_rel_err"] <= chk["tol"] == tol, (dt, chk)


@pytest.mark.parametrize("zero", [2, 3])
def test_bench_share_gpu_smollm3(gpu, zero):
    """§8(f) 3 at N = 2 through real RCCL: SmolLM3 (2 decoder layers, full vocabulary) trains
    with ZeRO-2 (backward-overlapped reduces; replicas bit-identical afterwards) or ZeRO-3
    (per-layer gathers, backward reduce-scatters)."""
    out = _bench2(["--train", "smollm3", "--zero", str(zero), "--train-layers", "2", "--seq", "256",
                   "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == 2 and out["rehearsal"].startswith("share-gpu")
    assert out["loss"] == out["loss"] and out["value"] > 0  # finite loss
    if zero == 2:
        assert out["params_identical_across_ranks"] is True


# --- bench.py at N = 8 on the shared GPU: every exchange the 8-GPU run can pick ---------------
def _bench_rank(rank, ws, port, argv):
    """One rank of ``bench.main(argv)`` with the environment torch.distributed.run gives it (rank 0
    runs in this process, as every ws = 8 test here: 8 processes on the one GPU, not 9)."""
    import sys

    from conftest import REPO

    if str(REPO) not in sys.path:
        sys.path.insert(0, str(REPO))
    import bench

    env = {"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(ws),
           "LOCAL_WORLD_SIZE": str(ws), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
           "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1"}
    keys = list(env) + ["NCCL_HOSTID", "ZERO_AMD_PROBE_TRIES", "ZS_TEST_COMM"]
    saved = {k: os.environ.get(k) for k in keys}
    os.environ.update(env)
    os.environ.pop("ZS_TEST_COMM", None)
    bench._IN_PROCESS[0] = True
    try:
        out = bench.main(argv)
    finally:
        bench._IN_PROCESS[0] = False
        bench._REHEARSAL[0] = None
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    if rank == 0:
        checks = out["exchange_check_all_arenas"]
        assert set(checks) == {"flat", "buckets"}, checks
        for kind, c in checks.items():
            assert c["all_ranks_ok"] and "failure" not in c, (kind, c)
            assert c["reduce_max_err_over_bound"] <= 1.0 and c["adam_max_bf16_ulp"] <= 1, (kind, c)
            assert c["params_identical_across_ranks"], (kind, c)
        assert set(out["arena_calibration_ms_per_step"]) == {"flat", "buckets"}
        cal = out["arena_calibration"]
        for kind in ("flat", "buckets"):  # each exchange's own bus bandwidth, not only its step
            assert cal[kind]["busbw_gbs"] > 0 and cal[kind]["frac_of_peer_links"] > 0, cal
            assert cal[kind]["ms_per_step"] == out["arena_calibration_ms_per_step"][kind]
        assert out["rccl_selfcheck"]["all_ranks_ok"] and out["config"]["comm"] == "rccl"
        lib = out["arena_calibration_library_auto"]  # the library's arena="auto" on the same wire
        assert lib["chosen"] in ("flat", "buckets") and lib["sample_bytes"] > 0, lib
        assert lib["agrees_with_full_step"] == (lib["chosen"] == out["config"]["arena"]), lib


@pytest.mark.timeout(600)
def test_bench_share_gpu_n8_both_arenas(gpu):
    """The driver's default N=8 run (C4 ZeRO-2, ``--arena auto``) rehearsed through real RCCL on a
    4-layer copy of the SmolLM3-3B set (the full set at N = 8 takes minutes over sockets:
    tools/r06.sh rehearsal8, profiles/r04_rccl_net/c4_n8_full.json): communicator
    self-check, then BOTH arenas the calibration can pick — the flat arena's grouped reduce /
    broadcast rounds and the bucket arena's pack / RS / AG / unpack — each exchange-checked (reduced
    grads within the ring bound, Adam within 1 bf16 ulp of the restatement, ranks bit-identical),
    calibrated and timed; the library's own arena="auto" choice is reported beside it."""
    from _zero_run import spawn_ranks

    argv = ["--gpus", "8", "--share-gpu", "--no-cpu-baseline", "--watchdog-s", "0", "--config", "C4",
            "--set-layers", "4", "--zero", "2", "--arena", "auto", "--steps", "2", "--warmup", "1",
            "--no-comm-sweep", "--no-layout-ablation"]  # (the ablation leg: the N = 2 test)
    spawn_ranks(_bench_rank, 8, (8, free_port(), argv))
