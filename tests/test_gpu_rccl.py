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
from _zero_run import spawn_all_ranks, spawn_ranks

pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl_env(monkeypatch):
    monkeypatch.setenv("ZS_TEST_COMM", "rccl")
    monkeypatch.setenv("NCCL_HOSTID", "zs-test-rank0")  # (restored after the test)
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    monkeypatch.setenv("NCCL_IB_DISABLE", "1")
    yield


def _run(fn, ws, *args):
    """Every rank spawned (a failing rank takes the others down) up to ws = 4; at ws = 8 rank 0
    runs here, as in the gloo-staged tests (9 processes on the device stalled those)."""
    if ws <= 4:
        spawn_all_ranks(fn, ws, (ws, free_port()) + args)
    else:
        spawn_ranks(fn, ws, (ws, free_port()) + args)


# --- ZeRO-1/2 against the reference's trajectories ------------------------------------------
@pytest.mark.parametrize("variant,ws,mode,arena", [
    (1, 2, "distinct", None), (2, 2, "distinct", None), (1, 4, "ref", None), (2, 4, "distinct", None),
    (1, 3, "distinct", "buckets"), (2, 4, "distinct", "buckets"), (2, 8, "distinct", None)])
def test_rccl_injected_trajectories(gpu, rccl_env, variant, ws, mode, arena):
    """Flat arena (grouped reduce / broadcast rounds) and bucket arena (in-place RS / AG)."""
    from test_gpu_parity import _mr_worker

    _run(_mr_worker, ws, variant, f"traj_z{variant}_ws{ws}_d16_{mode}.npz", "ragged", arena)


@pytest.mark.parametrize("variant", [1, 2])
def test_rccl_fewer_params_than_ranks(gpu, rccl_env, variant):
    from test_gpu_parity import _edge_worker

    _run(_edge_worker, 4, variant, "ragged", "flat")


def test_rccl_hyperparameters(gpu, rccl_env):
    from test_gpu_parity import _hp_worker

    _run(_hp_worker, 3, 2, "adamw_amsgrad_2groups")


def test_rccl_zero1_carry(gpu, rccl_env):
    from test_gpu_parity import _carry_worker

    _run(_carry_worker, 3, "optimizer")


@pytest.mark.parametrize("which,ws", [("zero2", 2), ("zero2", 4), ("zero2_overlap", 3), ("zero3", 4)])
def test_rccl_bf16_gradient_exchange(gpu, rccl_env, which, ws):
    """bf16 sums inside RCCL (ring order, per-hop rounding) vs the oracle's emulation (1e-4)."""
    from test_gpu_parity import _bf16comm_worker

    _run(_bf16comm_worker, ws, which)


def test_rccl_timing_counters(gpu, rccl_env):
    from test_gpu_parity import _comm_time_worker

    _run(_comm_time_worker, 2)


# --- backward-overlapped reduces, DDP ------------------------------------------------------
@pytest.mark.parametrize("variant,ws,arena", [(1, 2, "flat"), (2, 4, "flat"), (2, 3, "buckets")])
def test_rccl_overlap_backward(gpu, rccl_env, variant, ws, arena):
    from test_gpu_overlap import _mr_worker

    _run(_mr_worker, ws, variant, f"traj_z{variant}_ws{ws}_d16_distinct.npz", True, arena)


def test_rccl_frozen_and_unused(gpu, rccl_env):
    from test_gpu_overlap import _frozen_worker

    _run(_frozen_worker, 2, 2, True)


@pytest.mark.parametrize("ws,dtype_name", [(2, "float32"), (2, "bfloat16"), (3, "float32")])
def test_rccl_ddp_sync_gradients(gpu, rccl_env, ws, dtype_name):
    from test_gpu_overlap import _ddp_worker

    _run(_ddp_worker, ws, dtype_name)


# --- ZeRO-3 -------------------------------------------------------------------------------
@pytest.mark.parametrize("fn,ws,name", [
    ("_ref_mode", 2, "traj_z3_ws2_d16_distinct.npz"), ("_ref_mode", 4, "traj_z3_ws4_d16_distinct.npz"),
    ("_ref_injected", 4, "traj_z3_ws4_d16_ref.npz"),
    ("_update_injected", 3, "traj_z2_ws3_d16_distinct.npz"),
    ("_update_hooks", 2, "traj_z2_ws2_d16_distinct.npz"), ("_update_hooks", 4, "traj_z2_ws4_d16_distinct.npz")])
def test_rccl_zero3(gpu, rccl_env, fn, ws, name):
    from test_gpu_zero3 import _mr

    _run(_mr, ws, fn, name)


def test_rccl_zero3_gradient_memory(gpu, rccl_env):
    from test_gpu_zero3 import _mem_worker

    _run(_mem_worker, 4)


@pytest.mark.parametrize("reshard", [True, False])
def test_rccl_zero3_fp8_gather(gpu, rccl_env, reshard):
    from test_gpu_fp8 import _mr

    _run(_mr, 2, reshard)


@pytest.mark.parametrize("units,reshard", [(False, True), (True, False)])
def test_rccl_smollm3_zero3_bit_exact(gpu, rccl_env, units, reshard):
    """SmolLM3 ZeRO-3 AdamW at ws=2, bit-exact against the C oracle every step."""
    from test_gpu_train import _mr_zero3

    _run(_mr_zero3, 2, units, reshard)


def test_rccl_chunk_layout(gpu, rccl_env):
    from test_gpu_layouts import _worker

    _run(_worker, 4, "chunk", "traj_z2_ws4_d64_distinct.npz", "ragged", 64)


# --- bench.py at N = 2 on the shared GPU ------------------------------------------------
def _bench2(args, timeout=300):
    env = dict(os.environ)
    env.pop("ZS_TEST_COMM", None)
    env.pop("NCCL_HOSTID", None)  # bench --share-gpu sets it per rank
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2",
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
    restatement; bit-identical parameters on every rank), calibration, timed steps."""
    out = _bench2(["--config", "C2", "--dtype", "bf16", "--zero", str(zero), "--steps", "3",
                   "--warmup", "1", "--no-comm-sweep"])
    assert out["n_gpus"] == 2 and out["rccl_selfcheck"]["all_ranks_ok"]
    assert out["config"]["comm"] == "rccl", out["config"]["comm"]
    assert out["rehearsal"].startswith("share-gpu")
    checks = out["exchange_check_all_arenas"]
    assert set(checks) == {"flat", "buckets"} and set(out["arena_calibration_ms_per_step"]) == set(checks)
    for kind, c in checks.items():
        assert c["all_ranks_ok"], (kind, c)


def test_bench_share_gpu_zero3_paramset(gpu):
    """configs[4]'s ZeRO-3 parameter-set step at N = 2 (2 layers): the gather check and a short
    bucket sweep through real RCCL."""
    out = _bench2(["--zero", "3", "--config", "C5", "--set-layers", "2", "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == 2
    assert out["exchange_check"]["all_ranks_ok"], out["exchange_check"]
    assert out["rehearsal"].startswith("share-gpu")


def test_bench_share_gpu_zero3_mlp(gpu):
    """configs[2]'s hooked ZeRO-3 training iteration (the reference MLP, here C2-wide) at N = 2:
    one real iteration through RCCL equals the unsharded plain-PyTorch iteration (bf16 params:
    within 2^-7 of the largest element; fp32: 1e-5)."""
    out = _bench2(["--zero", "3", "--config", "C2", "--steps", "2", "--warmup", "1"])
    assert out["n_gpus"] == 2 and out["rehearsal"].startswith("share-gpu")
    chk = out["exchange_check"]
    assert chk["all_ranks_ok"] and chk["max_rel_err"] <= chk["tol"] == 2.0 ** -7
