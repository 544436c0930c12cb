"""Full-scale (BASELINE.json configs[3], SmolLM3-3B set, 3.08e9 bf16 params) properties of the
bucketed ZeRO-2 step, size-independent so no full-size oracle run is needed.  ws = 1 is the
headline's own step (one 3.08e9-element stream: offsets past 2^31).

Rank 0 of a ws-rank job runs on the one GPU with an identity communicator (nothing arrives from
the other ranks, nothing leaves): after one step every parameter rank 0 owns must equal the C
oracle's Adam of (own grad / ws) — checked bit-exactly on a random sample of every owned tensor —
and every parameter it does not own must equal its own packed grad, bit for bit (pack → the
untouched window → unpack is a round trip through the even and the ragged buckets).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class IdentityComm:
    def __init__(self, ws):
        self.ws, self.rank = ws, 0

    def reduce_scatter(self, send, recv, stream):
        pass

    def all_gather(self, send, recv, stream):
        pass

    def reduce_v(self, buf, win_off, win_len, stream):
        pass

    def broadcast_v(self, buf, win_off, win_len, stream):
        pass

    def reduce_out(self, send, recv, root, stream):  # flat arena: the sum of own + zeros
        if root == self.rank and send.data_ptr() != recv.data_ptr():
            with torch.cuda.stream(stream):
                recv.copy_(send)

    def broadcast(self, t, root, stream):
        pass


@pytest.mark.parametrize("ws,buckets,arena", [(8, "ragged", "buckets"), (4, "padded", "buckets"),
                                              (8, "ragged", "flat"), (3, "ragged", "flat"),
                                              (1, "ragged", "flat")])
def test_c4_rank0_bucket_path_full_scale(gpu, monkeypatch, ws, buckets, arena):
    import torch.distributed as dist

    import zero_amd._sharded as sh
    from _zero_run import init_pg
    from oracle import c_oracle
    from zero_amd import zero2
    from zero_amd.shapes import smollm3_3b_shapes

    from conftest import free_port

    init_pg(0, 1, free_port())
    real_get = sh.get
    monkeypatch.setattr(sh, "get", lambda what, dm=None: {"ws": ws, "rank": 0}[what]
                        if what in ("ws", "rank") else real_get(what, dm))
    try:
        shapes = smollm3_3b_shapes()
        gen = torch.Generator(device=gpu).manual_seed(0)
        params, grads = [], []
        for s in shapes:
            params.append(torch.nn.Parameter(
                (torch.randn(s, device=gpu, generator=gen) * 0.02).to(torch.bfloat16)))
            grads.append((torch.randn(s, device=gpu, generator=gen) * 1e-3).to(torch.bfloat16))
        init = [p.detach().clone() for p in params]
        opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), comm=IdentityComm(ws),
                                     buckets=buckets, arena=arena)
        if arena == "flat":  # into the arena views, as bench.py (set_to_none=False keeps them)
            opt.zero_grad(set_to_none=False)
            for p, g in zip(params, grads):
                p.grad.copy_(g)
        else:
            for p, g in zip(params, grads):
                p.grad = g
        opt.step()
        torch.cuda.synchronize()
        eng = opt.engine
        if arena == "flat" and ws == 1:  # the headline's layout: ONE stream of 3.08e9 elements,
            # so arena offsets, Adam chunk indices and segment offsets run past 2^31 (int64 paths)
            assert getattr(eng, "arena_kind", None) == "flat" and eng.P.numel() > 2 ** 31
        elif arena == "flat":
            assert getattr(eng, "arena_kind", None) == "flat" and eng.K > 1
            for p in params:  # every parameter is a view of the arena
                assert p.data.untyped_storage().data_ptr() == eng.P.untyped_storage().data_ptr()
        else:
            assert eng.K > 1 and (buckets == "padded" or eng.plan.num_even < eng.K)
        owned = set(opt.local_param_indices)
        hp = c_oracle.hparams(step=1, grad_div=float(ws))
        rng = np.random.default_rng(0)
        for i, (p, g, p0) in enumerate(zip(params, grads, init)):
            bits = p.detach().view(torch.int16).reshape(-1)
            if i not in owned:
                if arena == "flat":  # nothing arrives from the absent owner: unchanged
                    assert torch.equal(bits, p0.view(torch.int16).reshape(-1)), i
                else:  # pack -> window -> unpack round trip
                    assert torch.equal(bits, g.view(torch.int16).reshape(-1)), i
                continue
            n = p.numel()
            idx = torch.from_numpy(np.unique(rng.integers(0, n, min(n, 4096)))).to(gpu)
            master = p0.reshape(-1)[idx].float().cpu().numpy()
            gb = g.reshape(-1)[idx].view(torch.int16).cpu().numpy().view(np.uint16).copy()
            out = np.zeros(len(idx), np.uint16)
            c_oracle.adam_bf16(master, out, gb, np.zeros(len(idx), np.float32),
                               np.zeros(len(idx), np.float32), hp)
            got = bits[idx].cpu().numpy().view(np.uint16)
            assert np.array_equal(got, out), i
            # exp_avg (a view of the flat shard) after step 1: fma(1-b1, g/ws - 0, 0)
            gf = (gb.astype(np.uint32) << 16).view(np.float32) / np.float32(ws)
            m_want = np.float32(1.0 - 0.9) * gf
            m_got = opt.optimizer.state[p]["exp_avg"].reshape(-1)[idx].cpu().numpy()
            assert np.array_equal(m_got, m_want), i
    finally:
        dist.destroy_process_group()
