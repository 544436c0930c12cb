"""SmolLM3 training step through the ZeRO-2 drop-in: a shrunken SmolLM3
(transformers, random init) trains with zero2.ShardedOptimizer(AdamW) in backward-overlapped mode;
after every step every parameter's bf16 bits equal the C oracle's AdamW (decoupled weight decay,
split fp32 master = bf16 param + int16 residual) applied to the gradients the backward produced."""
import numpy as np
import pytest
import torch
import torch.distributed as dist

from _zero_run import init_pg

pytestmark = pytest.mark.gpu


def test_smollm3_zero2_adamw_overlap_bit_exact(gpu):
    from oracle import c_oracle
    from zero_amd import zero2
    from zero_amd.training_utils import smollm3 as sm

    init_pg(0, 1, 29655)
    try:
        cfg = sm.smollm3_config(layers=2, hidden=128, intermediate=256, heads=4, kv_heads=2, vocab=512)
        model = sm.build_model(cfg, gpu)
        params = list(model.parameters())
        lr, wd = 1e-3, 0.01
        opt = zero2.ShardedOptimizer(torch.optim.AdamW(params, lr=lr, weight_decay=wd), overlap=True,
                                     overlap_bucket_mb=0.05)
        assert opt.engine.arena_kind == "flat" and opt.engine.ov_K > 1
        hi = [p.detach().reshape(-1).view(torch.int16).cpu().numpy().view(np.uint16).copy()
              for p in params]
        lo = [np.zeros_like(x) for x in hi]  # the master starts as the bf16 param exactly
        m = [np.zeros(x.size, np.float32) for x in hi]
        v = [np.zeros(x.size, np.float32) for x in hi]
        g = torch.Generator(device=gpu).manual_seed(1)
        ids = torch.randint(0, cfg.vocab_size, (2, 64), device=gpu, generator=g)
        opt.zero_grad()
        for t in range(1, 5):
            loss = model(input_ids=ids, labels=ids).loss
            loss.backward()
            grads = [p.grad.detach().reshape(-1).view(torch.int16).cpu().numpy().view(np.uint16).copy()
                     for p in params]
            opt.step()
            opt.zero_grad()
            hp = c_oracle.hparams(lr=lr, weight_decay=wd, step=t, decoupled=True)
            for i, p in enumerate(params):
                c_oracle.adam_bf16_split(hi[i], lo[i], grads[i], m[i], v[i], hp)
                got = p.detach().reshape(-1).view(torch.int16).cpu().numpy().view(np.uint16)
                assert np.array_equal(got, hi[i]), (t, i)
                res = opt.optimizer.state[p].get("master_residual")
                if res is not None:  # owned params expose the residual: equal to the oracle's
                    assert np.array_equal(res.reshape(-1).cpu().numpy().view(np.uint16), lo[i]), (t, i)
            assert torch.isfinite(loss)
    finally:
        dist.destroy_process_group()


def _zero3_smollm3(rank, ws, port, dev, units=False, reshard=True):
    """One rank of a SmolLM3 ZeRO-3 run (update mode, AdamW, hooks on every module with
    parameters).  Every rank trains on the SAME batch, so the reduce-scattered sum of a chunk is
    exactly ws times this rank's own gradient and the mean is exact: each rank's chunks then equal
    the C oracle's split-master AdamW of its own full gradient (captured by a hook registered
    before the optimizer's), bit for bit, every step."""
    from oracle import c_oracle
    from zero_amd import zero3
    from zero_amd.training_utils import smollm3 as sm

    cfg = sm.smollm3_config(layers=2, hidden=128, intermediate=256, heads=4, kv_heads=2, vocab=512)
    model = sm.build_model(cfg, dev)
    params = list(model.parameters())
    full = {}  # full gradient of every param as backward produced it (before the reduce-scatter)
    for i, p in enumerate(params):
        p.register_post_accumulate_grad_hook(
            lambda q, i=i: full.__setitem__(i, q.grad.detach().reshape(-1).view(torch.int16)
                                            .cpu().numpy().view(np.uint16).copy()))
    lr, wd = 1e-3, 0.01
    kw = {}
    if ws > 1:
        from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401

        kw["comm"] = test_comm()
    opt = zero3.ShardedOptimizer(torch.optim.AdamW(params, lr=lr, weight_decay=wd), update=True,
                                 bucket_mb=0.05, **kw)
    zero3.register_zero3_hooks(model, opt.param_managers,
                               units=list(model.model.layers) if units else None,
                               reshard_after_forward=reshard)
    ar = opt._arena
    hi, lo, m, v = [], [], [], []
    for i, p in enumerate(params):
        x = p.detach().reshape(-1).view(torch.int16).cpu().numpy().view(np.uint16).copy()
        hi.append(x)
        lo.append(np.zeros_like(x))
        m.append(np.zeros(x.size, np.float32))
        v.append(np.zeros(x.size, np.float32))
    g = torch.Generator(device=dev).manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), device=dev, generator=g)
    for t in range(1, 4):
        full.clear()
        loss = sm.train_step(model, opt, ids)
        assert torch.isfinite(loss) and len(full) == len(params)
        hp = c_oracle.hparams(lr=lr, weight_decay=wd, step=t, decoupled=True)
        for i, p in enumerate(params):
            r0, r1, row = ar.rows[i]
            gch = full[i][r0 * row:r1 * row].copy()
            c_oracle.adam_bf16_split(hi[i], lo[i], gch, m[i], v[i], hp)
            got = p.detach().reshape(-1).view(torch.int16).cpu().numpy().view(np.uint16)
            assert np.array_equal(got, hi[i]), (rank, t, i)
    assert ws == 1 or opt.runtime.n_prefetch_hits > 0  # (ws=1: no hooks, nothing to gather)
    if ws > 1:  # gather groups per iteration: forward AND backward, or forward only (FSDP2 ZeRO-2)
        groups = len(set(k[1] for k in opt.runtime.key_managers))
        # over 3 iterations, + the prefetch of the 4th iteration's first wave (wave groups)
        n, w = opt.runtime.n_gathers, opt.runtime.wave
        if reshard:
            assert 6 * groups <= n <= 6 * groups + w, (n, groups, w)
        else:  # forward gathers only — except the tied embedding, which lm_head's backward
            # releases before the embedding's backward needs it again
            assert 3 * groups <= n <= 3 * (groups + 1) + w, (n, groups, w)


def test_smollm3_zero3_adamw_bit_exact(gpu):
    """SURVEY.md §8(f) 3, the ZeRO-3 half (fsdp/train_fsdp.py:92-94 reshard_after_forward=True)."""
    init_pg(0, 1, 29657)
    try:
        _zero3_smollm3(0, 1, None, gpu)
    finally:
        dist.destroy_process_group()


def _mr_zero3(rank, ws, port, units, reshard=True):
    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    try:
        _zero3_smollm3(rank, ws, port, torch.device("cuda:0"), units, reshard)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_smollm3_zero3_two_ranks_bit_exact(gpu):
    """Per-module groups; units=True: one gather group per decoder layer (FSDP2's per-block
    fully_shard); reshard=False: parameters stay gathered from forward through backward (FSDP2's
    reshard_after_forward=False, the reference's "ZeRO-2" run, fsdp/train_fsdp.py:84-86)."""
    from _zero_run import spawn_batch

    spawn_batch(2, [(_mr_zero3, (u, r)) for u, r in ((False, True), (True, True), (True, False))])
