"""BASELINE.json configs[0] at its real width: the reference MLP 6 × Linear(10000, 10000)
(600,060,000 fp32 params, zero1.py:237-249) at ws = 2, for the sampled full-width fixtures
``tests/golden/c1_z{1,2}_ws2_sampled.npz`` (made by ``make_golden.py c1`` from the reference's own
ShardedOptimizer on gloo) — and configs[1], the same MLP at D = 4096 (100,687,872 params) under
ZeRO-2, ``c2_z2_ws2_sampled.npz``.

The full tensors are too large to commit, so a fixture keeps, per parameter, a fixed sample of
element indices and the values there (initial, after every step on every rank, final Adam state),
plus fp64 sums over every element.  ZeRO-1/2's arithmetic is elementwise per parameter (sums over
ranks, Adam), so the oracle reproduces the sampled values from the sampled inputs alone.

The step inputs are gradients every side computes exactly: an integer hash of (step, rank, param,
element) mapped to fp32 by exact operations (a 24-bit integer, × 2^-24, − 0.5, × 2^-9), so the
reference on CPU, numpy at the sample indices and torch on the GPU produce the same bits with no
2.4 GB gradient file.  (The reference harness's gradients come from a backward of random data;
those would differ by GEMM rounding between CPU and GPU — the d16 / d64 fixtures cover real
backwards.)"""
from __future__ import annotations

import numpy as np

D = 10000      # configs[0]
D_C2 = 4096    # configs[1]
WS = 2
STEPS = 3
N_SAMPLE = 2048
MUL = 2654435761  # odd: k -> k·MUL mod 2^24 is a permutation of the 24-bit residues


def shapes(d: int = D):
    out = []
    for _ in range(6):
        out += [(d, d), (d,)]
    return out


def _seed(t: int, r: int, i: int) -> int:
    return 40503 * (1000 * t + 10 * r + i + 1)


def grad_np(t: int, r: int, i: int, idx: np.ndarray) -> np.ndarray:
    """Rank r's local gradient of param i at step t, at flat element indices ``idx`` (fp32)."""
    h = (np.asarray(idx, np.int64) * MUL + _seed(t, r, i)) & 0xFFFFFF
    x = h.astype(np.float32) * np.float32(2.0 ** -24) - np.float32(0.5)
    return (x * np.float32(2.0 ** -9)).astype(np.float32)


def grad_torch(t: int, r: int, i: int, shape, device=None):
    """The same gradient as a whole tensor (torch, any device)."""
    import torch

    n = int(np.prod(shape))
    k = torch.arange(n, dtype=torch.int64, device=device)
    h = (k * MUL + _seed(t, r, i)) & 0xFFFFFF
    del k
    x = h.to(torch.float32)
    del h
    x.mul_(2.0 ** -24).sub_(0.5).mul_(2.0 ** -9)
    return x.reshape(shape)


def sample_idx(i: int, n: int) -> np.ndarray:
    """The fixture's element sample of param i (n elements): both ends plus N_SAMPLE draws."""
    rng = np.random.default_rng(1000 + i)
    return np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, N_SAMPLE)])).astype(np.int64)


def make_model(d: int = D):
    """The reference's model (zero1.py:237-249) with the fixture's init (torch.manual_seed(0))."""
    import torch
    import torch.nn as nn

    torch.manual_seed(0)
    layers = []
    for li in range(6):
        layers.append(nn.Linear(d, d))
        if li < 5:
            layers.append(nn.ReLU())
    return nn.Sequential(*layers)
