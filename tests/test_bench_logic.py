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
