"""bench.py's contract on the GPU box: the JSON line (N=1), the N>1 harness (2 ranks sharing the
one GPU through the test-only gloo-staged communicator) and the ws=8 bucket path at scale."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO, free_port
from _zero_run import spawn_ranks

pytestmark = pytest.mark.gpu

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "roofline"}


def _run(cmd, timeout=240):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def _port():
    return free_port()


def test_bench_json_line_n1(gpu):
    out = _run([sys.executable, "bench.py", "--config", "C2", "--dtype", "fp32", "--steps", "3",
                "--warmup", "1", "--no-cpu-baseline"])
    assert KEYS <= set(out) and out["n_gpus"] == 1 and out["value"] > 0
    rf = out["roofline"]
    # above 1 the timed kernel would not be doing its algorithmic work: fail
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1.0 and rf["achieved"] > 0
    assert "fp32_master" not in out  # fp32 parameters: the master is the parameter


def test_bench_fp32_master_line_beside_split_headline(gpu):
    """bf16 parameters at N=1: the split-master line carries the same step with the exact fp32
    master beside it, measured after the headline's timed region."""
    out = _run([sys.executable, "bench.py", "--config", "C2", "--steps", "3", "--warmup", "1",
                "--no-cpu-baseline"])
    assert out["config"]["master"] == "split"
    fm = out["fp32_master"]
    assert out["fp32_master_ms_per_step"] == fm["ms_per_step"] > 0 and fm["steps"] == 3
    # 28 vs 26 B per element over the same elements
    ratio = fm["alg_bytes_per_launch"] / out["roofline"]["alg_bytes_per_launch"]
    assert abs(ratio - 28 / 26) < 1e-3, ratio
    # N=1 times the default hand-off (zero_grad() -> None, fresh grads): Adam read every one of
    # C2's 12 gradient tensors in place; the views hand-off is timed beside it
    gh = out["grad_handoff"]
    assert gh["handoff"] == "default" and gh["grads_read_in_place"] == 12, gh
    assert out["default_zero_grad_ms_per_step"] == out["ms_per_step"]
    assert out["views_handoff_ms_per_step"] > 0


def test_bench_harness_two_ranks_gloo_staged(gpu):
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                "--config", "C2", "--dtype", "fp32", "--steps", "2", "--warmup", "1",
                "--comm", "gloo-staged", "--bucket-mb", "64"], timeout=600)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["value"] > 0
    assert out["config"]["buckets"] > 1 and out["roofline"]["launches_per_step"] >= 1
    coll = out["collectives"]
    assert coll["peer_links"] == 1 and coll["peer_links_peak_gbs"] == 153.0  # N=2: one direct link
    assert coll["frac_of_peer_links"] == pytest.approx(coll["busbw_gbs"] / 153.0)


def test_bench_simulated_ws8_bucket_path(gpu):
    """The ws=8 Layout-R bucket path (pack / Adam / unpack over all buckets) at C4 scale."""
    out = _run([sys.executable, "bench.py", "--config", "C4", "--steps", "3", "--warmup", "1",
                "--simulate-ws", "8", "--no-cpu-baseline"])
    assert "diagnostic" in out and out["buckets"] > 1 and out["ms_per_step"] > 0


def test_bench_zero3_parameter_set_n1(gpu):
    """--zero 3 on C4 (configs[4]'s step on the 3B set), update mode, one rank: every shard is its
    whole parameter, so no hooks are registered and nothing is gathered (the backward still hands
    each gradient to the reducer, and one fused Adam runs over the chunk arena)."""
    out = _run([sys.executable, "bench.py", "--config", "C4", "--zero", "3", "--steps", "3",
                "--warmup", "1", "--no-cpu-baseline"])
    assert out["config"]["zero"] == 3 and out["value"] > 0 and out["n_gpus"] == 1
    assert out["zero3"]["gathers_per_step"] == 0 and out["roofline"]["frac"] > 0
    assert out["roofline"]["launches_per_step"] == 1


def test_bench_zero3_parameter_set_simulated_ws8(gpu):
    """Rank 0's compute of the hooked ZeRO-3 C5 iteration at ws=8 (collectives skipped)."""
    out = _run([sys.executable, "bench.py", "--config", "C5", "--zero", "3", "--steps", "2",
                "--warmup", "1", "--simulate-ws", "8", "--no-cpu-baseline"])
    assert "diagnostic" in out and out["layers"] == 34
    # Layout Z is balanced: rank 0 holds 1/8 of every parameter (C5 dims divide by 8)
    assert out["chunk_elems"] * 8 == 8_030_261_248


def test_bench_zero3_parameter_set_two_ranks_gloo_staged(gpu):
    """The N>1 ZeRO-3 parameter-set path incl. its exchange check (gather bit-exact, backward
    reduce-scatter within the bf16 bound), 2 ranks on the one GPU through the gloo-staged comm."""
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                "--config", "C4", "--zero", "3", "--set-layers", "2", "--steps", "2", "--warmup", "1",
                "--comm", "gloo-staged"], timeout=600)
    assert out["n_gpus"] == 2 and out["exchange_check"]["all_ranks_ok"]
    assert out["exchange_check"]["gather_bit_exact"]
    assert out["collectives"]["all_gather"]["calls_per_step"] > 0


def test_bench_zero3_training_iteration(gpu):
    """--zero 3: hooked forward/backward + update-mode step of the C2 MLP (configs[2] harness)."""
    out = _run([sys.executable, "bench.py", "--config", "C2", "--zero", "3", "--dtype", "fp32",
                "--steps", "3", "--warmup", "1", "--no-cpu-baseline"])
    assert out["config"]["zero"] == 3 and out["value"] > 0
    assert out["roofline"]["launches_per_step"] >= 1 and out["zero3"]["gathers_per_step"] == 0


def _selfcheck_worker(rank, ws, port):
    import torch
    import torch.distributed as dist

    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401
    from _zero_run import init_pg
    import bench

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    out = bench.comm_selfcheck(GlooStagedComm(), ws, rank, torch.device("cuda:0"))
    assert out["ok"], out
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_comm_selfcheck_logic(gpu, ws):
    """bench.comm_selfcheck's closed-form expectations hold for a correct communicator (the
    test-only gloo-staged one here; RCCL at N>1 in the driver's multi-GPU runs)."""
    import torch.multiprocessing as mp

    spawn_ranks(_selfcheck_worker, ws, (ws, _port()))


def test_comm_backends_selfcheck_ws1(gpu):
    """RcclComm and the C10dComm A/B backend pass the bench's closed-form self-check on an "nccl"
    (RCCL) process group of one rank."""
    import torch
    import torch.distributed as dist

    import bench
    from zero_amd.comm import C10dComm, RcclComm

    import os
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        for comm in (RcclComm(), C10dComm()):
            out = bench.comm_selfcheck(comm, 1, 0, torch.device("cuda:0"))
            assert out["ok"], (type(comm).__name__, out)
            comm.close()
    finally:
        dist.destroy_process_group()
