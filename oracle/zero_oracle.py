"""TEST INFRASTRUCTURE — numpy restatement of the reference ZeRO step (checker only).

Every function cites the reference file:line it restates (paths relative to the reference repo,
xo-toybox/distributed-training-sandbox @ 2025-11-28).  The Adam arithmetic lives in a third-party
dependency of the reference, ``torch.optim.Adam`` (pinned torch==2.4.1, pyproject.toml:13; the
non-capturable single-tensor algorithm is unchanged in the torch 2.10 used to capture fixtures,
torch/optim/adam.py:394-547); it is restated here from that published algorithm.

Pinned by tests/test_oracle.py against tests/golden/*.npz (outputs of the reference itself).
Never imported by the product (zero_amd).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
F64 = np.float64


# ----------------------------------------------------------------------------------------------
# ownership
# ----------------------------------------------------------------------------------------------
def owner_range(n: int, ws: int, rank: int) -> tuple[int, int]:
    """zero1.py:55-59 (identical in zero2.py:51-55, zero3.py:93-97)."""
    ppr, rem = n // ws, n % ws
    start = rank * ppr + min(rank, rem)
    return start, start + ppr + (1 if rank < rem else 0)


def owner_of(n: int, ws: int, i: int) -> int:
    """zero1.py:92-100 (zero2.py:123-131): broadcast source of param index i."""
    ppr, rem = n // ws, n % ws
    if i < (ppr + 1) * rem:
        return i // (ppr + 1)
    return (i - rem) // ppr


def chunk_rows(d0: int, ws: int, rank: int) -> tuple[int, int]:
    """torch.chunk(ws, dim=0)[rank] row range, as used by zero3.py:44,107,142."""
    cs = -(-d0 // ws)
    return min(rank * cs, d0), min((rank + 1) * cs, d0)


# ----------------------------------------------------------------------------------------------
# Adam (torch.optim.Adam / AdamW, non-capturable single-tensor path)
# ----------------------------------------------------------------------------------------------
def fma32(a, b, c):
    """fp32 fused multiply-add emulated in fp64 (the product of two fp32 is exact in fp64)."""
    return (np.asarray(a, F64) * np.asarray(b, F64) + np.asarray(c, F64)).astype(F32)


def adam_update(p, g, m, v, step, *, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                amsgrad=False, maximize=False, decoupled=False, vmax=None):
    """One update of adam.py:394-547; returns new (p, m, v, vmax).  All arrays fp32.

    Rounding order follows torch's CPU kernels: lerp_ → fma(1-β1, g-m, m) (ATen Lerp.h,
    weight < 0.5 branch); mul_(β2).addcmul_(g, g, 1-β2) → fma((1-β2)·g, g, v·β2);
    denom = sqrt(v)/sqrt(bc2) + eps; addcdiv_(m, denom, -step_size) → p + (-step_size·m)/denom.
    """
    beta1, beta2 = betas
    p = np.asarray(p, F32).copy()
    g = np.asarray(g, F32)
    if maximize:  # adam.py:402
        g = -g
    if weight_decay != 0:
        if decoupled:  # adam.py:421-423
            p = (p * F32(1 - lr * weight_decay)).astype(F32)
        else:  # adam.py:433 grad.add(param, alpha=wd)
            g = fma32(F32(weight_decay), p, g)
    m = fma32(F32(1 - beta1), (g - m).astype(F32), m)  # adam.py:463 exp_avg.lerp_(grad, 1-β1)
    v = fma32((F32(1 - beta2) * g).astype(F32), g, (np.asarray(v, F32) * F32(beta2)).astype(F32))
    bc1 = 1 - beta1 ** step  # adam.py:532-537 (python floats)
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    bc2_sqrt = bc2 ** 0.5
    vv = v
    if amsgrad:  # adam.py:539-543
        vmax = np.maximum(vmax, v).astype(F32)
        vv = vmax
    denom = (np.sqrt(vv) / F32(bc2_sqrt)).astype(F32) + F32(eps)
    p = (p + (F32(-step_size) * m).astype(F32) / denom.astype(F32)).astype(F32)
    return p, m.astype(F32), v.astype(F32), vmax


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 → bf16 bit pattern (NaN kept quiet)."""
    u = np.asarray(x, F32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_bits_to_f32(h: np.ndarray) -> np.ndarray:
    return (np.asarray(h, np.uint16).astype(np.uint32) << 16).view(F32)


# ----------------------------------------------------------------------------------------------
# the reference harness model: 6 × Linear(D, D) with ReLU between, MSE loss (zero1.py:237-249,
# zero1.py:150-161)
# ----------------------------------------------------------------------------------------------
def mlp_grads(params, x, y):
    """Loss and grads of nn.Sequential(Linear,ReLU,…,Linear) + mse_loss (mean reduction)."""
    Ws, bs = params[0::2], params[1::2]
    hs, zs = [np.asarray(x, F32)], []
    h = hs[0]
    for li, (W, b) in enumerate(zip(Ws, bs)):
        z = (h @ W.T + b).astype(F32)
        zs.append(z)
        h = np.maximum(z, 0).astype(F32) if li < len(Ws) - 1 else z
        hs.append(h)
    out = hs[-1]
    diff = (out - y).astype(F32)
    loss = float(np.mean(diff.astype(F64) ** 2))
    d = (F32(2.0 / diff.size) * diff).astype(F32)
    grads = [None] * len(params)
    for li in range(len(Ws) - 1, -1, -1):
        grads[2 * li] = (d.T @ hs[li]).astype(F32)
        grads[2 * li + 1] = d.sum(axis=0, dtype=F32)
        if li > 0:
            d = ((d @ Ws[li]) * (zs[li - 1] > 0)).astype(F32)
    return loss, grads


def _sum_ranks(arrs):
    """Sum over ranks in rank order in fp32 (a ring's order is unspecified; tolerance covers it)."""
    acc = np.asarray(arrs[0], F32).copy()
    for a in arrs[1:]:
        acc = (acc + a).astype(F32)
    return acc


def ddp_sync(local_by_rank, bf16: bool = False):
    """DDP/ddp.py:43-47 ``sync_gradients``: every rank's gradient all-reduced (SUM) then divided
    in place by the world size.  fp32: the sum in rank order, then ``/ ws`` in fp32.  bf16: the
    sum rounded to bf16 once (a ring rounds per hop — within tolerance of this), then ``/ ws``
    rounded to bf16.  Returns fp32 values."""
    ws = len(local_by_rank)
    acc = _sum_ranks([np.asarray(a, F32) for a in local_by_rank])
    if bf16:
        acc = bf16_round(acc)
        return bf16_round((acc / F32(ws)).astype(F32))
    return (acc / F32(ws)).astype(F32)


def bf16_round(x):
    """fp32 → bf16 (round to nearest even) → fp32."""
    return bf16_bits_to_f32(f32_to_bf16_bits(np.asarray(x, F32))).reshape(np.shape(x))


def simulate(variant: int, ws: int, init, xs=None, ys=None, steps: int = 10, lr: float = 1e-3,
             local_grads=None, adam_kw=None, zero_grad: str = "optimizer", grad_comm=None):
    """Restate a ``steps``-long run of reference ZeRO-``variant`` at world size ``ws``.

    init: list of fp32 param arrays (identical on every rank, torch.manual_seed(0) in the fixture).
    xs, ys: per-rank inputs (used when local_grads is None: grads come from ``mlp_grads``).
    local_grads: optional callable (t, rank, i) -> that rank's local grad of param i at step t
                 (from the fixture), replacing the forward/backward.
    adam_kw: optional callable i -> keyword arguments of ``adam_update`` for param i (its param
             group's lr / betas / eps / weight_decay / amsgrad / maximize / decoupled).
    zero_grad: what the training loop clears before each backward — "optimizer" (the
             reference harness: ShardedOptimizer.zero_grad(), owned grads only, zero1.py:107-108)
             or "model" (model.zero_grad(): every grad, so nothing carries over).
    grad_comm: None, or "bf16" (variant 2 only): the build's bf16 gradient exchange of fp32
             params — every rank's grad rounded to bf16, summed in fp32, the sum rounded to bf16
             (a reduce that accumulates in fp32 and delivers bf16).  Not a reference behaviour.
    Returns dict with per-step params per rank, per-step reduced grads per rank (list in the
    reference's collective order), and final Adam state per rank.
    """
    n = len(init)
    params = [[np.array(p, F32) for p in init] for _ in range(ws)]
    held = [[None] * n for _ in range(ws)]  # p.grad per rank
    state = [dict() for _ in range(ws)]     # owned param index -> (step, m, v)
    out = {"params": [], "reduced": [], "state": state}
    for t in range(steps):
        # zero_grad: inner optimizer only holds owned params (zero1.py:107-108, 71-74)
        for r in range(ws):
            s, e = (0, n) if zero_grad == "model" else owner_range(n, ws, r)
            for i in range(s, e):
                held[r][i] = None
        for r in range(ws):
            if local_grads is None:
                _, g = mlp_grads(params[r] if variant != 3 else [np.array(p, F32) for p in init],
                                 xs[r], ys[r])
            else:
                g = [local_grads(t, r, i) for i in range(n)]
            for i in range(n):
                if g[i] is None:  # no gradient this step (frozen or unused parameter)
                    continue
                if variant == 3:
                    held[r][i] = np.array(g[i], F32)
                else:  # backward accumulates into a surviving grad (ZeRO-1 carry)
                    held[r][i] = g[i].copy() if held[r][i] is None else (held[r][i] + g[i]).astype(F32)
        reduced = [[] for _ in range(ws)]
        if variant == 1:  # zero1.py:80-84: all_reduce(SUM) then /ws on every param, every rank
            for i in range(n):
                if all(held[r][i] is None for r in range(ws)):  # `if p.grad is not None` everywhere
                    for r in range(ws):
                        reduced[r].append(None)
                    continue
                a = (_sum_ranks([held[r][i] for r in range(ws)]) / F32(ws)).astype(F32)
                for r in range(ws):
                    held[r][i] = a.copy()
                    reduced[r].append(a.copy())
            grads_for = lambda r, i: held[r][i]  # noqa: E731
        elif variant == 2:  # zero2.py:94-113: reduce_scatter of ws copies == all-reduce; owner /ws
            own_grad = [dict() for _ in range(ws)]
            for i in range(n):
                if all(held[r][i] is None for r in range(ws)):  # no grad anywhere: no collective
                    for r in range(ws):
                        own_grad[r][i] = None
                        reduced[r].append(None)
                    continue
                if grad_comm == "bf16":
                    ssum = bf16_round(_sum_ranks([bf16_round(held[r][i].reshape(-1))
                                                  for r in range(ws)]))
                else:
                    ssum = _sum_ranks([held[r][i].reshape(-1) for r in range(ws)])
                for r in range(ws):
                    s, e = owner_range(n, ws, r)
                    if s <= i < e:
                        own_grad[r][i] = (ssum / F32(ws)).astype(F32).reshape(held[r][i].shape)
                        held[r][i] = own_grad[r][i]
                    else:
                        held[r][i] = None
                    reduced[r].append(ssum.copy())
            grads_for = lambda r, i: own_grad[r][i]  # noqa: E731
        else:  # zero3.py:131-153: chunk own rows, all_reduce, /ws, then every grad discarded
            for i in range(n):
                shards = []
                for r in range(ws):
                    g = held[r][i]
                    if g.shape[0] == init[i].shape[0]:  # full-size grad: chunk (zero3.py:141-143)
                        a, b = chunk_rows(g.shape[0], ws, r)  # (release() already did this for
                        g = g[a:b]                            #  modules whose bwd hook fired)
                    shards.append(g)
                red = (_sum_ranks(shards) / F32(ws)).astype(F32)
                for r in range(ws):
                    reduced[r].append(red.copy())
                    held[r][i] = None
            grads_for = None
        if variant in (1, 2):  # Adam on owned params (zero1.py:88 / zero2.py:120)
            for r in range(ws):
                s, e = owner_range(n, ws, r)
                for i in range(s, e):
                    if grads_for(r, i) is None:  # torch Adam skips a parameter without a grad
                        continue
                    z0 = np.zeros_like(init[i])
                    st, m, v, vm = state[r].get(i, (0, z0, z0, z0))
                    st += 1
                    kw = dict(lr=lr) if adam_kw is None else dict(adam_kw(i))
                    p, m, v, vm = adam_update(params[r][i], grads_for(r, i), m, v, st, vmax=vm, **kw)
                    params[r][i] = p
                    state[r][i] = (st, m, v, vm)
            for i in range(n):  # broadcast from owner (zero1.py:91-102 / zero2.py:122-133)
                o = owner_of(n, ws, i)
                for r in range(ws):
                    params[r][i] = params[o][i].copy()
        out["params"].append([[p.copy() for p in params[r]] for r in range(ws)])
        out["reduced"].append(reduced)
    return out
