"""bench.py's host-side logic on the CPU: the exchange check's bit checksums (chunked, so a large
arena needs no full-size int64 temporaries) and the xGMI denominators of the busBW fractions."""
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
