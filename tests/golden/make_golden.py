"""Generate the golden fixtures that pin the oracle and the HIP path.

Runs ONLY in the build container (it imports the reference from /root/reference, which never
travels to the GPU box).  Outputs are small ``.npz`` files next to this script; the reference's
source is never copied — only inputs and the outputs the reference computed from them.

What it captures (SURVEY.md §8(c) "Golden vectors to capture"):

1. ``ownership.npz`` — the ZeRO-1/2/3 parameter-index ownership ranges computed by the
   reference's own ``ShardedOptimizer.__init__`` (zero1.py:51-62, zero2.py:47-58, zero3.py:89-100)
   and the owner rank each parameter is broadcast from (zero1.py:91-102, zero2.py:122-133), for
   n in 1..64 ∪ {291, 326, 400} and ws in 1..16 ∪ {32, 64}.  Collected with a fake ``dist``/``get``
   injected into the reference module namespace, so no process group is needed.
2. ``traj_z{1,2,3}_ws{W}_d{D}_{mode}.npz`` — real gloo multi-process runs of the reference
   ``ShardedOptimizer`` (torch.cuda.synchronize stubbed: zero1.py:104 calls it unconditionally):
   6×Linear(D,D)+ReLU, ``torch.manual_seed(0)`` init, 10 steps of zero_grad → forward → MSE →
   backward → step (the loop of zero1.py:140-174), lr=1e-3.  Saved: inputs per rank, initial
   params, each rank's local gradients entering every ``step()`` (so a test can inject exactly the
   step's inputs), params after every step per rank, every reduced gradient the reference's
   collectives produced (after the in-place ``/ws``), final Adam state per owned param, and for
   ZeRO-3 the grad shapes seen at ``step()`` plus the all_gather call count.
3. ``adam_kat.npz`` — ``torch.optim.Adam`` / ``AdamW`` CPU (single-tensor path, torch 2.10;
   the reference pins 2.4.1 whose non-capturable math is the same, adam.py:457-547)
   known-answer trajectories for several hyper-parameter sets.
2b. ``c1_z{1,2}_ws2_sampled.npz`` (``make_golden.py c1``) — BASELINE configs[0] at its real
   width: the reference's 6 × Linear(10000, 10000) model and ShardedOptimizer at ws = 2 on gloo,
   3 steps of the exact hash gradients of tests/_c1.py; sampled elements and fp64 sums per
   parameter (tests/_c1.py says why).
4. ``collective_kat.npz`` — the 2-rank known answers from 02-operations.ipynb:1853-2109
   (rank r holds [0+r, 1+r, 2+r]): all_reduce → [1,3,5], all_gather → [[0,1,2],[1,2,3]].

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent
REF_ZERO = Path("/root/reference/zero")
STEPS = 10


def _load_ref(variant: int):
    """Import the reference zeroN.py as a fresh module (read-only mount: no bytecode)."""
    sys.dont_write_bytecode = True
    if str(REF_ZERO) not in sys.path:
        sys.path.insert(0, str(REF_ZERO))
    import torch

    torch.cuda.synchronize = lambda *a, **k: None  # zero1.py:104 etc. call it unconditionally
    spec = importlib.util.spec_from_file_location(f"ref_zero{variant}", REF_ZERO / f"zero{variant}.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# ----------------------------------------------------------------------------------------------
# 1. ownership tables
# ----------------------------------------------------------------------------------------------
class _FakeDist:
    """Stands in for torch.distributed inside the reference module to observe owner ranks."""

    class ReduceOp:
        SUM = "sum"

    def __init__(self):
        self.bcast_src = []

    def all_reduce(self, t, op=None):
        pass

    def reduce_scatter_tensor(self, out, inp, op=None):
        out.copy_(inp[: out.numel()])

    def broadcast(self, t, src):
        self.bcast_src.append(int(src))


def make_ownership():
    import torch

    mods = {v: _load_ref(v) for v in (1, 2, 3)}
    ns = list(range(1, 65)) + [291, 326, 400]
    wss = list(range(1, 17)) + [32, 64]
    out = {"ns": np.array(ns), "wss": np.array(wss)}
    for n in ns:
        for ws in wss:
            starts, ends = [], []
            owner_from_bcast = None
            for rank in range(ws):
                per_variant = []
                for v, mod in mods.items():
                    mod.get = (lambda ws_, rank_: (lambda s, dm=None: {"ws": ws_, "rank": rank_}[s]))(ws, rank)
                    params = [torch.nn.Parameter(torch.zeros(2)) for _ in range(n)]
                    if v == 3:
                        # zero3 chunks every param along dim 0; a 2-element param cannot be chunked
                        # ws>2 ways, so observe only the index ranges via a 1-row-per-rank param.
                        params = [torch.nn.Parameter(torch.zeros(ws, 1)) for _ in range(n)]
                    opt = mod.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3))
                    per_variant.append(tuple(opt.local_param_indices))
                    if v == 1 and rank == 0:
                        fake = _FakeDist()
                        mod.dist = fake
                        for p in params:
                            p.grad = torch.zeros_like(p)
                        opt.step()
                        owner_from_bcast = fake.bcast_src
                        mod.dist = torch.distributed
                assert per_variant[0] == per_variant[1] == per_variant[2], (n, ws, rank, per_variant)
                idx = per_variant[0]
                starts.append(idx[0] if idx else None)
                ends.append(idx[-1] + 1 if idx else None)
            # empty ranges: the reference's list(range(start,end)) is empty; record start=end from
            # the formula's neighbours (start of the next non-empty range or n)
            s_arr = np.zeros(ws, np.int64)
            e_arr = np.zeros(ws, np.int64)
            for r in range(ws):
                if starts[r] is None:
                    s_arr[r] = e_arr[r] = n if r == 0 or e_arr[r - 1] == n else e_arr[r - 1]
                else:
                    s_arr[r], e_arr[r] = starts[r], ends[r]
            out[f"n{n}_ws{ws}_start"] = s_arr
            out[f"n{n}_ws{ws}_end"] = e_arr
            out[f"n{n}_ws{ws}_owner"] = np.array(owner_from_bcast, np.int64)
    np.savez_compressed(OUT / "ownership.npz", **out)
    print("ownership.npz:", len(out), "arrays")


# ----------------------------------------------------------------------------------------------
# 2. trajectories
# ----------------------------------------------------------------------------------------------
def _make_model(D):
    import torch.nn as nn

    layers = []
    for i in range(6):
        layers.append(nn.Linear(D, D))
        if i < 5:
            layers.append(nn.ReLU())
    return nn.Sequential(*layers)


class _RecDist(types.SimpleNamespace):
    """Pass-through torch.distributed that remembers the tensors reduced by the reference."""

    def __init__(self, real):
        super().__init__()
        self._real = real
        self.reduced = []
        self.n_all_gather = 0
        self.ReduceOp = real.ReduceOp

    def __getattr__(self, name):
        return getattr(self._real, name)

    def all_reduce(self, t, op=None, **kw):
        self._real.all_reduce(t, op=op, **kw)
        self.reduced.append(t)

    def reduce_scatter_tensor(self, out, inp, op=None, **kw):
        self._real.reduce_scatter_tensor(out, inp, op=op, **kw)
        self.reduced.append(out)

    def broadcast(self, t, src, **kw):
        self._real.broadcast(t, src=src, **kw)

    def all_gather(self, outs, t, **kw):
        self._real.all_gather(outs, t, **kw)
        self.n_all_gather += 1


def _traj_worker(rank, ws, port, variant, D, mode, tmpdir):
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    mod = _load_ref(variant)
    rec = _RecDist(dist)
    mod.dist = rec

    torch.manual_seed(0)
    model = _make_model(D)
    params = list(model.parameters())
    init = [p.detach().clone() for p in params]
    gen = torch.Generator().manual_seed(42 if mode == "ref" else 100 + rank)
    x = torch.randn(16, D, generator=gen)
    y = torch.randn(16, D, generator=gen)

    opt = mod.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3))
    if variant == 3:
        mod.register_zero3_hooks(model, opt.param_managers)
    raw = {}  # raw local grads as autograd produces them (before accumulation into p.grad)
    for i, p in enumerate(params):
        p.register_hook(lambda g, i=i: raw.__setitem__(i, g.detach().clone()))
    rec_out = {"x": x.numpy(), "y": y.numpy(),
               "local": np.array(opt.local_param_indices, np.int64)}
    for i, t in enumerate(init):
        rec_out[f"init_{i}"] = t.numpy()
    keep = (lambda t: True) if D <= 16 else (lambda t: t in (0, STEPS - 1))
    for step in range(STEPS):
        rec.n_all_gather = 0
        raw.clear()
        opt.zero_grad()
        out = model(x)
        loss = F.mse_loss(out, y)
        loss.backward()
        if variant == 3:
            rec_out[f"t{step}_gradshape"] = np.array(
                [list(p.grad.shape) + [0] * (2 - p.grad.dim()) if p.grad is not None else [-1, -1]
                 for p in params], np.int64)
            rec_out[f"t{step}_pshape"] = np.array(
                [list(p.data.shape) + [0] * (2 - p.data.dim()) for p in params], np.int64)
        for i, g in raw.items():  # the step's inputs: this rank's raw local grads
            rec_out[f"t{step}_lg{i}"] = g.numpy()
        for i, p in enumerate(params):  # p.grad as step() sees it (ZeRO-1 carry / ZeRO-3 chunks)
            if p.grad is not None and variant == 3:
                rec_out[f"t{step}_g{i}"] = p.grad.detach().clone().numpy()
        rec.reduced = []
        opt.step()
        rec_out[f"t{step}_loss"] = np.array(loss.item(), np.float64)
        rec_out[f"t{step}_nred"] = np.array(len(rec.reduced))
        rec_out[f"t{step}_nallgather"] = np.array(rec.n_all_gather)
        if not keep(step):
            continue
        for k, t in enumerate(rec.reduced):
            rec_out[f"t{step}_red{k}"] = t.detach().clone().numpy()
        for i, p in enumerate(params):
            rec_out[f"t{step}_p{i}"] = p.detach().clone().numpy()
    # final Adam state for the params this rank's inner optimizer holds
    for i, p in enumerate(params):
        st = opt.optimizer.state.get(p, {})
        if st:
            rec_out[f"state_{i}_step"] = np.array(float(st["step"]))
            rec_out[f"state_{i}_exp_avg"] = st["exp_avg"].numpy()
            rec_out[f"state_{i}_exp_avg_sq"] = st["exp_avg_sq"].numpy()
    np.savez(Path(tmpdir) / f"rank{rank}.npz", **rec_out)
    dist.barrier()
    dist.destroy_process_group()


_PORT = [29600]


def make_traj(variant, ws, D, mode):
    import torch.multiprocessing as mp

    _PORT[0] += 1
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_traj_worker, args=(ws, _PORT[0], variant, D, mode, td), nprocs=ws, join=True)
        merged = {"ws": np.array(ws), "D": np.array(D), "steps": np.array(STEPS)}
        for r in range(ws):
            with np.load(Path(td) / f"rank{r}.npz") as z:
                for k in z.files:
                    if k.startswith("init_") or k in ("x", "y") and mode == "ref":
                        if r == 0:
                            merged[k] = z[k]
                        continue
                    merged[f"r{r}_{k}"] = z[k]
    name = f"traj_z{variant}_ws{ws}_d{D}_{mode}.npz"
    np.savez_compressed(OUT / name, **merged)
    print(name, len(merged), "arrays")


# ----------------------------------------------------------------------------------------------
# 2b. configs[0] at its real width, sampled (tests/_c1.py)
# ----------------------------------------------------------------------------------------------
def _c1_worker(rank, ws, port, variant, tmpdir, d=None):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, str(OUT.parent))
    import _c1

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(4)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    mod = _load_ref(variant)
    model = _c1.make_model(d or _c1.D)
    params = list(model.parameters())
    idx = [_c1.sample_idx(i, p.numel()) for i, p in enumerate(params)]
    rec = {}

    def sample(t, i):
        return t.detach().reshape(-1)[torch.from_numpy(idx[i])].numpy().copy()

    def sums(t):
        a = t.detach().reshape(-1).double()
        return np.array([a.sum().item(), a.abs().sum().item()], np.float64)

    for i, p in enumerate(params):
        rec[f"idx_{i}"] = idx[i]
        rec[f"init_{i}"] = sample(p, i)
        rec[f"initsum_{i}"] = sums(p)
    opt = mod.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3))
    rec["local"] = np.array(opt.local_param_indices, np.int64)
    for t in range(_c1.STEPS):
        opt.zero_grad()
        for i, p in enumerate(params):  # what backward's AccumulateGrad does with these grads
            g = _c1.grad_torch(t, rank, i, p.shape)
            if p.grad is None:
                p.grad = g
            else:
                p.grad.add_(g)
        opt.step()
        for i, p in enumerate(params):
            rec[f"t{t}_p{i}"] = sample(p, i)
            rec[f"t{t}_psum{i}"] = sums(p)
    for i, p in enumerate(params):
        st = opt.optimizer.state.get(p, {})
        if st:
            rec[f"state_{i}_step"] = np.array(float(st["step"]))
            rec[f"state_{i}_exp_avg"] = sample(st["exp_avg"], i)
            rec[f"state_{i}_exp_avg_sq"] = sample(st["exp_avg_sq"], i)
    np.savez(Path(tmpdir) / f"rank{rank}.npz", **rec)
    dist.barrier()
    dist.destroy_process_group()


def make_c1(variant, cfg="c1"):
    import torch.multiprocessing as mp

    sys.path.insert(0, str(OUT.parent))
    import _c1

    d = {"c1": _c1.D, "c2": _c1.D_C2}[cfg]
    _PORT[0] += 1
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_c1_worker, args=(_c1.WS, _PORT[0], variant, td, d), nprocs=_c1.WS, join=True)
        merged = {"ws": np.array(_c1.WS), "D": np.array(d), "steps": np.array(_c1.STEPS)}
        for r in range(_c1.WS):
            with np.load(Path(td) / f"rank{r}.npz") as z:
                for k in z.files:
                    if k.startswith(("idx_", "init_", "initsum_")):
                        if r == 0:
                            merged[k] = z[k]
                        else:  # every rank built the same model
                            assert np.array_equal(merged[k], z[k]), k
                        continue
                    merged[f"r{r}_{k}"] = z[k]
    name = f"{cfg}_z{variant}_ws{_c1.WS}_sampled.npz"
    np.savez_compressed(OUT / name, **merged)
    print(name, len(merged), "arrays")


# ----------------------------------------------------------------------------------------------
# 3. Adam known answers
# ----------------------------------------------------------------------------------------------
ADAM_CASES = {
    "default": dict(cls="Adam", lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0),
    "wd": dict(cls="Adam", lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2),
    "amsgrad": dict(cls="Adam", lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=True),
    "maximize": dict(cls="Adam", lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, maximize=True),
    "adamw": dict(cls="AdamW", lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2),
    "hyper": dict(cls="Adam", lr=1e-2, betas=(0.8, 0.99), eps=1e-6, weight_decay=0.0),
}


def make_adam_kat():
    import torch

    out = {}
    n = 4099  # odd: exercises vector tails
    rng = np.random.default_rng(1234)
    for name, cfg in ADAM_CASES.items():
        cfg = dict(cfg)
        cls = getattr(torch.optim, cfg.pop("cls"))
        p0 = rng.standard_normal(n).astype(np.float32) * 0.05
        grads = rng.standard_normal((STEPS, n)).astype(np.float32) * 1e-2
        grads[:, :7] = 0.0  # exact zeros
        grads[:, 7:11] *= 1e5  # large
        grads[:, 11:15] *= 1e-18  # tiny (below sqrt(eps) scale)
        grads[3, 15:40] = 0.0  # a zero step in the middle
        p = torch.nn.Parameter(torch.from_numpy(p0.copy()))
        opt = cls([p], foreach=False, **cfg)
        for t in range(STEPS):
            p.grad = torch.from_numpy(grads[t].copy())
            opt.step()
        st = opt.state[p]
        out[f"{name}_p0"] = p0
        out[f"{name}_grads"] = grads
        out[f"{name}_p"] = p.detach().numpy().copy()
        out[f"{name}_m"] = st["exp_avg"].numpy().copy()
        out[f"{name}_v"] = st["exp_avg_sq"].numpy().copy()
        if "max_exp_avg_sq" in st:
            out[f"{name}_vmax"] = st["max_exp_avg_sq"].numpy().copy()
    np.savez_compressed(OUT / "adam_kat.npz", **out)
    print("adam_kat.npz", len(out), "arrays")


def make_collective_kat():
    # 02-operations.ipynb:1853,1867 (all_reduce SUM), :2006,2021 (reduce dst 0), :2062,2109 (all_gather)
    np.savez(OUT / "collective_kat.npz",
             inputs=np.array([[0, 1, 2], [1, 2, 3]], np.int64),
             all_reduce=np.array([1, 3, 5], np.int64),
             reduce_dst0=np.array([1, 3, 5], np.int64),
             all_gather=np.array([[0, 1, 2], [1, 2, 3]], np.int64))
    print("collective_kat.npz")


def main():
    which = sys.argv[1:] or ["ownership", "traj", "adam", "coll"]
    if "ownership" in which:
        make_ownership()
    if "adam" in which:
        make_adam_kat()
    if "coll" in which:
        make_collective_kat()
    if "c1" in which:  # not in the default set: two 600M-parameter ranks, ~20 GB of host memory
        make_c1(1)
        make_c1(2)
    if "c2" in which:  # configs[1]: the same MLP at D = 4096 under ZeRO-2
        make_c1(2, "c2")
    if "traj" in which:
        for variant in (1, 2, 3):
            for ws in (1, 2, 3, 4, 8):
                if variant == 3 and 16 % ws:
                    continue  # uneven chunks deadlock the reference all_gather (zero3.py:38-39)
                for mode in ("ref", "distinct"):
                    make_traj(variant, ws, 16, mode)
            if variant in (1, 2):
                make_traj(variant, 2, 64, "ref")
            if variant == 2:
                make_traj(variant, 4, 64, "distinct")


if __name__ == "__main__":
    main()
