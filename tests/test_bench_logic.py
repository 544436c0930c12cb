"""bench.py's host-side logic on the CPU: the exchange check's bit checksums (chunked, so a large
arena needs no full-size int64 temporaries) and the xGMI denominators of the busBW fractions."""
import pytest
import numpy as np
import torch

import bench


def _plain_checksums(t):
    b = bench._bits(t).reshape(-1).long()
    return [int(b.sum()), int((b * torch.arange(1, b.numel() + 1) % 65521).sum())]


def test_bit_checksums_chunked_equal_plain():
    g = torch.Generator().manual_seed(3)
    for dt in (torch.bfloat16, torch.float32):
        for n in (1, 63, 1000, 4097):
            t = torch.randn(n, generator=g).to(dt)
            want = _plain_checksums(t)
            for chunk in (1, 7, 64, 1 << 24):
                assert bench._bit_checksums(t, "cpu", chunk=chunk) == want, (dt, n, chunk)


def test_bit_checksums_see_one_flipped_bit():
    t = torch.randn(5000).to(torch.bfloat16)
    u = t.clone()
    u.view(torch.int16)[4321] ^= 1
    assert bench._bit_checksums(t, "cpu", chunk=1000) != bench._bit_checksums(u, "cpu", chunk=1000)


def test_peer_link_denominators():
    assert bench.peer_link_peak_gbs(1) == bench.XGMI_LINK_GBS
    assert bench.peer_link_peak_gbs(2) == bench.XGMI_LINK_GBS
    assert bench.peer_link_peak_gbs(8) == 7 * bench.XGMI_LINK_GBS
    assert np.isclose(bench.peer_link_peak_gbs(8), 1071.0)


def test_bf16_sum_tolerance_grows_with_ranks():
    assert bench._bf16_sum_tolerance(2) < bench._bf16_sum_tolerance(8) == 8 * 2.0 ** -8


def test_copy_launch_groups_cover_buckets_in_order():
    """Pack / unpack launch groups (zero_amd/engine.py launch_groups): every bucket exactly once,
    in order; growing runs (pack: the first bucket alone, unpack: the last bucket alone)."""
    import sys

    sys.path.insert(0, str(bench.REPO / "distributed-training-sandbox_amd"))
    from zero_amd.engine import launch_groups

    for growth in (2, 4, 8):
        for K in range(1, 70):
            for small_last in (False, True):
                g = launch_groups(K, small_last=small_last, growth=growth)
                assert [k for grp in g for k in grp] == list(range(K))
                assert len(g) <= 2 + int(np.log(K) / np.log(growth)) if K > 1 else len(g) == 1
                assert len(g[-1 if small_last else 0]) == 1
    assert [len(x) for x in launch_groups(24, growth=2)] == [1, 1, 2, 4, 8, 8]
    assert [len(x) for x in launch_groups(24, growth=8)] == [1, 7, 16]
    assert [len(x) for x in launch_groups(24)] == [1, 7, 16]  # the default growth
    assert [len(x) for x in launch_groups(24, small_last=True)] == [16, 7, 1]


def test_traffic_matcher_needs_equal_algorithmic_bytes(tmp_path):
    """roofline.traffic is taken from a PMC summary only when the summary's algorithmic bytes per
    launch are this run's: a stale measurement is reported as a note, not as traffic."""
    import json

    f = tmp_path / "x_pmc.json"
    f.write_text(json.dumps({"config": {"workload": "C4"}, "hbm_bytes_per_launch": 100.0,
                             "algorithmic_bytes_per_launch": 99}))
    t, src, note = bench.match_traffic({"workload": "C4"}, 99.0, str(f))
    assert t == 100.0 and src and note is None
    t, src, note = bench.match_traffic({"workload": "C4"}, 120.0, str(f))
    assert t is None and src is None and "not used" in note
    # the committed summaries: the C4 split-master headline matches its own algorithmic bytes
    want = {"workload": "C4", "zero": 2, "param_dtype": "bf16", "layout": "reference", "n_gpus": 1,
            "master": "split"}
    t, src, _ = bench.match_traffic(want, 79952564224.0)
    assert t is not None and src.startswith("profiles/")


def test_self_launch_command_is_one_rank_per_gpu_on_loopback():
    """`python bench.py --gpus N` without a launcher starts torch.distributed.run with N ranks on
    127.0.0.1 and the same arguments (modal_utils.py:115-120)."""
    import sys

    argv = ["--gpus", "8", "--steps", "3"]
    cmd = bench._self_launch_cmd(argv, 8, 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29999"
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv


def test_world_size_mismatch_exits_nonzero():
    """WORLD_SIZE set and different from --gpus: exit 2 before anything is timed (it used to log a
    note and time WORLD_SIZE ranks)."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(bench.REPO / "bench.py"), "--gpus", "8"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=1 but --gpus 8" in r.stderr and r.stdout == ""


def test_launch_ranks_relays_one_json_line_and_exit_code(tmp_path, capsys):
    """The self-launch relay: the child's JSON line goes to stdout, everything else to stderr, and
    the child's exit code is returned (a crash is not hidden; a 0 exit without the line is 6)."""
    import sys

    script = tmp_path / "child.py"
    script.write_text("import sys, json\nprint('banner')\nprint(json.dumps({'metric': 'm', 'value': 1}))\n"
                      "print('noise', file=sys.stderr)\nsys.exit(int(sys.argv[1]))\n")
    assert bench._launch_ranks([], 2, cmd=[sys.executable, str(script), "0"]) == 0
    out = capsys.readouterr()
    assert out.out.strip().splitlines() == ['{"metric": "m", "value": 1}']
    assert "banner" in out.err
    assert bench._launch_ranks([], 2, cmd=[sys.executable, str(script), "7"]) == 7
    script.write_text("print('no json')\n")
    assert bench._launch_ranks([], 2, cmd=[sys.executable, str(script)]) == 6


def test_product_comm_failure_is_fatal(monkeypatch):
    """RcclComm() failing at N>1 ends the run (in a test process: raises) instead of timing
    torch's communicator under the product's name."""
    import pytest

    import zero_amd.comm as comm_mod

    def boom():
        raise OSError("no RCCL")

    monkeypatch.setattr(comm_mod, "RcclComm", boom)
    bench._IN_PROCESS[0] = True
    try:
        with pytest.raises(bench.CommFailed, match="RcclComm"):
            bench._product_comm(3)
    finally:
        bench._IN_PROCESS[0] = False


def test_cpu_baseline_sample_is_whole_decoder_layers():
    """the CPU baseline steps whole decoder layers (>= 30 tensors), not the
    leading 3 tensors dominated by the embedding."""
    import sys

    sys.path.insert(0, str(bench.REPO / "distributed-training-sandbox_amd"))
    from zero_amd.shapes import llama31_8b_shapes, mlp_shapes, smollm3_3b_shapes

    for shapes in (smollm3_3b_shapes(), llama31_8b_shapes()):
        idx, what = bench._cpu_sample(shapes, 256 << 20)
        assert len(idx) >= 30 and len(idx) % 9 == 0 and 0 not in idx, (len(idx), what)
        assert idx == list(range(1, 1 + len(idx)))  # layers 0..k, in order
        assert sum(int(np.prod(shapes[i])) for i in idx) >= 256 << 20
    idx, _ = bench._cpu_sample(mlp_shapes(4096), 64 << 20)
    assert idx == list(range(len(idx))) and len(idx) >= 1


def test_expected_scaling_matches_the_planner_at_c4_n8():
    """the prediction committed before the first 8-GPU line.  C4 ZeRO-2 on the flat
    arena at N = 8: the slowest rank's Adam streams 15.23 GB of HBM and the exchange moves 10.76 GB
    of bus bytes per rank — 11.95 ms at 8 TB/s + 7 x 153 GB/s, no overlap credit."""
    import sys

    sys.path.insert(0, str(bench.REPO / "distributed-training-sandbox_amd"))
    from zero_amd.shapes import CONFIGS

    c4 = CONFIGS["C4"][1]()
    e = bench.expected_scaling(c4, 2, "flat", 8)
    assert abs(e["hbm_gb_per_rank"] - 15.23) < 0.01 and abs(e["bus_gb_per_rank"] - 10.76) < 0.01
    assert abs(e["ideal_ms"] - 11.95) < 0.01
    assert e["at_north_star_ms"] > e["ideal_ms"] > e["ideal_overlapped_ms"]
    # N = 1: no exchange, the whole 26 B x 3.075e9 Adam stream (the headline's 79.95 GB)
    e1 = bench.expected_scaling(c4, 2, "flat", 1)
    assert e1["bus_gb_per_rank"] == 0 and abs(e1["hbm_gb_per_rank"] - 79.9526) < 1e-3
    # strong scaling of C4 is exchange-bound: at most ~1.1x over the measured N=1 step (13.05 ms)
    assert 13.05 / e["ideal_ms"] < 1.15
    # the bucket arena adds pack + unpack (4 B per bf16 element) and pays RS/AG bus bytes
    b = bench.expected_scaling(c4, 2, "buckets", 8)
    assert abs(b["hbm_gb_per_rank"] - e["hbm_gb_per_rank"] - 4 * 2 * 3075098624 / 1e9) < 1e-6
    # ZeRO-3 on C5: three exchanges of the padded chunks per iteration
    c5 = CONFIGS["C5"][1]()
    z = bench.expected_scaling(c5, 3, "chunk", 8)
    assert 3 * 8.03 * 2 * 7 / 8 <= z["bus_gb_per_rank"] < 3 * 8.1 * 2 * 7 / 8


# --- a run that dies leaves evidence -----------------------------------------
def test_default_watchdog_fires_inside_the_drivers_limit():
    """The driver kills a bench run at 600 s; the default watchdog fires before, counted from
    process start (the first import torch on a fresh box is part of the driver's clock)."""
    assert bench.WATCHDOG_BUDGET_S <= 540.0
    assert bench.watchdog_seconds(None, now=bench._T0) == bench.WATCHDOG_BUDGET_S < 600.0
    assert bench.watchdog_seconds(None, now=bench._T0 + 120.0) == pytest.approx(bench.WATCHDOG_BUDGET_S - 120.0)
    assert bench.watchdog_seconds(None, now=bench._T0 + 1e4) == 30.0  # (late start: still fires)
    assert bench.watchdog_seconds(250.0) == 250.0 and bench.watchdog_seconds(0) == 0.0


_STUCK = r"""
import sys, time
sys.path.insert(0, {repo!r})
import bench
bench._PARTIAL["rccl_selfcheck"] = {{"ok": True, "all_ranks_ok": True}}
bench._PARTIAL["arena_calibration"] = {{"flat": {{"busbw_gbs": 123.5, "ms_per_step": 40.0}}}}
bench._PARTIAL["exchange_check_all_arenas"] = {{"flat": {{"all_ranks_ok": True}}}}
{setup}
bench._phase("exchange check (buckets arena)")
print("ready", file=sys.stderr, flush=True)
def stuck_in_a_collective():
    time.sleep(120)
stuck_in_a_collective()
"""


def _run_stuck(setup, env=None, signal_after=None):
    import os
    import signal
    import subprocess
    import sys
    import time

    code = _STUCK.format(repo=str(bench.REPO), setup=setup)
    p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, env=dict(os.environ, **(env or {})))
    if signal_after is not None:
        line = ""
        while "ready" not in line:
            line = p.stderr.readline()
            assert line, "the child ended before it was ready"
        time.sleep(signal_after)
        p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=60)
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    return p.returncode, lines, err


def _check_partial(lines, err, phase="exchange check (buckets arena)"):
    import json

    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["value"] is None and d["metric"] == bench.METRIC and d["failed_phase"] == phase
    assert d["rccl_selfcheck"]["all_ranks_ok"] and d["arena_calibration"]["flat"]["busbw_gbs"] == 123.5
    assert d["exchange_check_all_arenas"]["flat"]["all_ranks_ok"]
    # every thread's Python stack, down to the frame that was stuck
    assert "stuck_in_a_collective" in err and "Thread 0x" in err, err[-2000:]
    return d


def test_watchdog_dumps_stacks_and_prints_the_partial_line():
    """An injected stuck phase: exit 3, every thread's stack on stderr, rank 0's JSON line with
    value null, the phase and what was measured before it."""
    rc, lines, err = _run_stuck("bench._start_watchdog(3.0)")
    assert rc == 3, (rc, err[-2000:])
    d = _check_partial(lines, err)
    assert d["failure"].startswith("watchdog")


def test_watchdog_on_a_nonzero_rank_prints_no_line():
    rc, lines, err = _run_stuck("bench._start_watchdog(2.0)", env={"RANK": "3"})
    assert rc == 3 and lines == [] and "stuck_in_a_collective" in err


def test_sigterm_from_the_launcher_leaves_the_partial_line():
    """torch.distributed.run ends the surviving ranks with SIGTERM once one rank has failed: the
    rank blocked in a collective still dumps its stacks and prints the partial line (exit 143)."""
    rc, lines, err = _run_stuck("bench._install_term_handler()", signal_after=1.0)
    assert rc == 143, (rc, err[-2000:])
    d = _check_partial(lines, err)
    assert "SIGTERM" in d["failure"]


def test_a_run_that_raises_prints_the_partial_line(tmp_path):
    """main() on a machine without a GPU raises in its first device call: the run ends with exit
    7 and ONE JSON line (value null, the phase, the error), not a bare traceback."""
    import json
    import os
    import subprocess
    import sys

    if torch.cuda.is_available():
        import pytest

        pytest.skip("needs a machine without a GPU (the raise is the device call)")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(bench.REPO / "bench.py"), "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--watchdog-s", "0"], capture_output=True, text=True,
                       timeout=300, env=env, cwd=tmp_path)
    assert r.returncode == 7, (r.returncode, r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] is None and d["error"] and d["config"]["workload"] == "C4"


def test_layout_costs_of_reference_ownership_at_c4_n8():
    """what the reference's whole-parameter ownership (Layout R) costs at N = 8 on
    C4, from the planner: the slowest rank's Adam traffic is 15.23 GB against the balanced 1/8 of
    79.95 GB = 9.99 GB for Layout Z (zero3.py's chunks) and Layout F (the flat arena's balanced
    slices, the N > 1 line's layout_ablation leg); the exchange is the same, so the balanced flat
    arena's ideal step is ~0.65 ms shorter, while Layout Z's bucket arena adds pack / unpack."""
    import sys

    sys.path.insert(0, str(bench.REPO / "distributed-training-sandbox_amd"))
    from zero_amd.plan import Plan
    from zero_amd.shapes import CONFIGS

    c4 = CONFIGS["C4"][1]()
    lc = bench.layout_costs(c4, 2, 8)
    r, f, z = lc["reference_flat_arena"], lc["balanced_F_flat_arena"], lc["chunk_Z_bucket_arena"]
    assert abs(r["max_rank_adam_gb"] - 15.23) < 0.01
    assert abs(f["max_rank_adam_gb"] - 79.9526 / 8) < 0.01 and abs(z["max_rank_adam_gb"] - 9.99) < 0.01
    # ... against the planner itself: 26 B per element of the longest Layout Z / F stream
    numels = [int(np.prod(s)) for s in c4]
    dim0 = [int(s[0]) for s in c4]
    for layout, row in (("chunk", z), ("flat", f)):
        pl = Plan(numels, 8, 0, layout, dim0=dim0, align_elems=64)
        own = max(int(pl.pieces(k).length.sum()) for k in range(8))
        assert abs(26 * own / 1e9 - row["max_rank_adam_gb"]) < 1e-3, layout
    assert f["bus_gb_per_rank"] == r["bus_gb_per_rank"]
    assert 0.5 < r["ideal_ms"] - f["ideal_ms"] < 0.8
    assert z["hbm_gb_per_rank"] > r["hbm_gb_per_rank"]  # pack + unpack outweigh the balance
    e = bench._expected_block(c4, 2, "flat", 8, 2, 26, 1024.0, measured_ms=20.0)
    assert e["layouts"] == lc and e["curve"]["8"]["max_rank_adam_gb"] == r["max_rank_adam_gb"]


def test_optional_legs_yield_to_the_watchdog(monkeypatch):
    """On a slow interconnect the optional legs are skipped (and listed) rather than letting the
    watchdog kill the run before the headline line is printed; without a watchdog they all run."""
    import time

    monkeypatch.setattr(bench, "_SKIPPED", {})
    monkeypatch.setattr(bench, "_DEADLINE", [None])
    assert bench.leg_fits("layout ablation", 1e6) and not bench._SKIPPED
    monkeypatch.setattr(bench, "_DEADLINE", [time.monotonic() + 200.0])
    assert bench.leg_fits("bucket-size sweep", 15.0)           # 2 x 15 + 30 <= 200
    assert not bench.leg_fits("other hand-off", 90.0)           # 2 x 90 + 30 > 200
    assert set(bench._SKIPPED) == {"other hand-off"}
    assert bench._SKIPPED["other hand-off"]["estimated_s"] == 90.0
