"""The drop-in's DEFAULT gradient hand-off.

The reference's step() reads ``p.grad`` wherever backward left it after ``zero_grad()`` set every
grad to None (zero2.py:94-120, 138-139).  At world size 1 the ZeRO-2 drop-in now does the same:
Adam reads backward's fresh gradient tensors in place (``zs_adamset_set_grads`` re-points the
fused-Adam tables in stream order), with no landing copy and no gradient arena.  At ws > 1 the
fresh gradients are landed into the arena from the post-accumulate hooks in batches, so backward
never holds the arena plus a whole set of fresh gradients.  Every check below is bit-exact against
the C oracle on the gradients the real backward produced."""
import numpy as np
import pytest
import torch
import torch.distributed as dist

from _zero_run import init_pg
from conftest import free_port

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.detach().reshape(-1).contiguous().view(torch.int16).cpu().numpy().view(np.uint16).copy()


def _mlp(dev, dtype, widths=(96, 160, 64, 40), seed=0):
    torch.manual_seed(seed)
    layers = []
    for a, b in zip(widths[:-1], widths[1:]):
        layers += [torch.nn.Linear(a, b), torch.nn.GELU()]
    return torch.nn.Sequential(*layers[:-1]).to(dev, dtype)


def _oracle_state(params, dtype):
    if dtype == torch.bfloat16:
        hi = [_bits(p) for p in params]
        return dict(hi=hi, lo=[np.zeros_like(x) for x in hi],
                    m=[np.zeros(x.size, np.float32) for x in hi],
                    v=[np.zeros(x.size, np.float32) for x in hi])
    p32 = [p.detach().reshape(-1).cpu().numpy().copy() for p in params]
    return dict(p=p32, m=[np.zeros_like(x) for x in p32], v=[np.zeros_like(x) for x in p32])


def _oracle_step(st, grads, hp, dtype):
    from oracle import c_oracle

    for i, g in enumerate(grads):
        if dtype == torch.bfloat16:
            c_oracle.adam_bf16_split(st["hi"][i], st["lo"][i], _bits(g), st["m"][i], st["v"][i], hp)
        else:
            c_oracle.adam_f32(st["p"][i], g.detach().reshape(-1).cpu().numpy().copy(), st["m"][i],
                              st["v"][i], hp)


def _assert_params(params, st, dtype, t):
    for i, p in enumerate(params):
        if dtype == torch.bfloat16:
            assert np.array_equal(_bits(p), st["hi"][i]), (t, i)
        else:
            got = p.detach().reshape(-1).cpu().numpy()
            assert np.array_equal(got.view(np.uint32), st["p"][i].view(np.uint32)), (t, i)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("overlap", [False, True])
def test_zero2_ws1_default_zero_grad_reads_fresh_grads_in_place(gpu, dtype, overlap):
    """opt.zero_grad() → backward → opt.step() at ws = 1: bit-exact vs the C oracle every step,
    no gradient arena allocated, p.grad still backward's own tensor after the step."""
    from oracle import c_oracle
    from zero_amd import zero2

    init_pg(0, 1, free_port())
    try:
        model = _mlp(gpu, dtype)
        params = list(model.parameters())
        opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), overlap=overlap,
                                     overlap_bucket_mb=0.02)
        eng = opt.engine
        assert eng.inplace and eng.G is None
        st = _oracle_state(params, dtype)
        gen = torch.Generator(device=gpu).manual_seed(3)
        for t in range(1, 6):
            x = torch.randn(32, 96, device=gpu, generator=gen).to(dtype)
            opt.zero_grad()
            assert all(p.grad is None for p in params)
            model(x).float().square().mean().backward()
            grads = [p.grad for p in params]
            ptrs = [g.data_ptr() for g in grads]
            opt.step()
            _oracle_step(st, grads, c_oracle.hparams(step=t), dtype)
            _assert_params(params, st, dtype, t)
            # read in place: no arena, no copy, the caller's tensors untouched as p.grad
            assert eng.G is None and eng.inplace_reads == len(params)
            assert [p.grad.data_ptr() for p in params] == ptrs
    finally:
        dist.destroy_process_group()


def test_zero2_ws1_mixed_handoffs_bit_exact(gpu):
    """Within one optimizer: fresh grads (in place), then grad views (zero_grad(set_to_none=False):
    the arena appears), then a misaligned hand-assigned grad (landed into its slot: the vector
    kernel cannot read it in place), then fresh again — every step bit-exact vs the oracle."""
    from oracle import c_oracle
    from zero_amd import zero2

    init_pg(0, 1, free_port())
    try:
        dtype = torch.bfloat16
        model = _mlp(gpu, dtype, seed=1)
        params = list(model.parameters())
        opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3))
        eng = opt.engine
        st = _oracle_state(params, dtype)
        gen = torch.Generator(device=gpu).manual_seed(5)
        for t, mode in enumerate(["fresh", "views", "odd", "fresh", "views"], start=1):
            x = torch.randn(16, 96, device=gpu, generator=gen).to(dtype)
            opt.zero_grad(set_to_none=mode != "views")
            model(x).float().square().mean().backward()
            if mode == "odd":  # param 0's gradient as a 2-byte-offset view of a bigger buffer
                g0 = params[0].grad
                buf = torch.empty(g0.numel() + 1, dtype=dtype, device=gpu)
                buf[1:].copy_(g0.reshape(-1))
                params[0].grad = buf[1:].view(g0.shape)
                assert params[0].grad.data_ptr() % 8 != 0
            grads = [p.grad.detach().clone() for p in params]
            opt.step()
            _oracle_step(st, grads, c_oracle.hparams(step=t), dtype)
            _assert_params(params, st, dtype, t)
            if mode == "views":
                assert eng.G is not None and all(eng.is_view(i, p.grad) for i, p in enumerate(params))
            if mode == "odd":
                assert eng.is_view(0, params[0].grad) and eng.inplace_reads == len(params) - 1
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_zero2_ws1_strided_assigned_grads_are_landed(gpu, dtype):
    """a gradient the caller assigns that is not one dense run — a transpose
    (``p.grad = x.t()``) or a stride-0 ``expand`` — has the parameter's shape and dtype, so torch
    accepts it, but Adam would read ``numel`` contiguous elements from its pointer.  It must be
    copied into its slot through torch (``_land``'s non-dense path) and read from there; the step
    stays bit-exact against the oracle on the gradient's logical values."""
    from oracle import c_oracle
    from zero_amd import zero2

    init_pg(0, 1, free_port())
    try:
        torch.manual_seed(2)
        w = torch.nn.Parameter(torch.randn(64, 96, device=gpu).to(dtype))  # transposed grad
        r = torch.nn.Parameter(torch.randn(48, 80, device=gpu).to(dtype))  # expanded row grad
        c = torch.nn.Parameter(torch.randn(40, 64, device=gpu).to(dtype))  # expanded column grad
        d = torch.nn.Parameter(torch.randn(256, device=gpu).to(dtype))     # dense, read in place
        params = [w, r, c, d]
        opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3))
        eng = opt.engine
        st = _oracle_state(params, dtype)
        for t in range(1, 5):
            opt.zero_grad()
            w.grad = (torch.randn(96, 64, device=gpu) * 1e-2).to(dtype).t()
            r.grad = (torch.randn(1, 80, device=gpu) * 1e-2).to(dtype).expand(48, 80)
            c.grad = (torch.randn(40, 1, device=gpu) * 1e-2).to(dtype).expand(40, 64)
            d.grad = (torch.randn(256, device=gpu) * 1e-2).to(dtype)
            assert not any(p.grad.is_contiguous() for p in params[:3])
            grads = [p.grad.detach().contiguous().clone() for p in params]
            dptr = d.grad.data_ptr()
            opt.step()
            _oracle_step(st, grads, c_oracle.hparams(step=t), dtype)
            _assert_params(params, st, dtype, t)
            assert all(eng.is_view(i, params[i].grad) for i in range(3))  # landed and adopted
            assert d.grad.data_ptr() == dptr and eng.inplace_reads == 1
    finally:
        dist.destroy_process_group()


def test_adamset_set_grads_rebinds_in_stream_order(gpu):
    """zs_adamset_set_grads: the same set run over two gradient buffers in turn (segments with
    vector parts and scalar tails) equals the oracle bit for bit; a misaligned pointer for a
    segment with a vector part is refused and leaves the binding as it was; 0 = zero gradient."""
    from oracle import c_oracle
    from zero_amd._lib import ZS_F32, ZeroAmdError
    from zero_amd.kernels import AdamSet, adam_hparams

    rng = np.random.default_rng(7)
    lens = [1000, 4099, 3, 65536 + 5]
    p0 = [rng.standard_normal(n).astype(np.float32) * 0.1 for n in lens]
    P = [torch.from_numpy(x.copy()).to(gpu) for x in p0]
    M = [torch.zeros_like(x) for x in P]
    V = [torch.zeros_like(x) for x in P]
    GA = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(gpu) for n in lens]
    GB = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(gpu) for n in lens]
    rows = np.array([[0, p.data_ptr(), p.data_ptr(), 0, m.data_ptr(), v.data_ptr(), 0, 0, p.numel()]
                     for p, m, v in zip(P, M, V)], np.uint64)
    aset = AdamSet(rows, ZS_F32)
    assert aset.bytes == sum(lens) * 24  # no gradient bound yet: no gradient bytes
    cp, cm, cv = [x.copy() for x in p0], [np.zeros_like(x) for x in p0], [np.zeros_like(x) for x in p0]
    st = torch.cuda.current_stream()
    for t in range(1, 6):
        gs = GA if t % 2 else GB
        ptr = np.array([g.data_ptr() for g in gs], np.uint64)
        if t == 4:
            ptr[1] = 0  # segment 1 gets no gradient this step (zero gradient)
        aset.set_grads(ptr, st)
        assert aset.bytes == sum(lens) * 24 + 4 * sum(n for n, q in zip(lens, ptr) if q)
        aset.run(adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, t), st)
        for i in range(len(lens)):
            g = gs[i].cpu().numpy() if ptr[i] else np.zeros(lens[i], np.float32)
            c_oracle.adam_f32(cp[i], np.ascontiguousarray(g), cm[i], cv[i], c_oracle.hparams(step=t))
    bad = np.array([g.data_ptr() for g in GA], np.uint64)
    bad[3] += 4  # 4-byte aligned only: segment 3 has a vector part
    with pytest.raises(ZeroAmdError):
        aset.set_grads(bad, st)
    torch.cuda.synchronize()
    for i in range(len(lens)):
        assert np.array_equal(P[i].cpu().numpy().view(np.uint32), cp[i].view(np.uint32)), i
        assert np.array_equal(M[i].cpu().numpy().view(np.uint32), cm[i].view(np.uint32)), i


class _NoComm:
    """Collectives as no-ops: rank 0 of a simulated ws-rank job (the landing path only)."""

    def reduce_out(self, send, recv, root, stream):
        pass

    def broadcast(self, t, root, stream):
        pass


def test_zero2_ws2_hook_landing_bounds_peak_memory(gpu, monkeypatch):
    """ZeRO-2 at ws > 1 without overlap keeps the full-size gradient arena G,
    so backward's fresh gradients are landed from the post-accumulate hooks in batches and
    adopted (p.grad = the slot's view): the peak of torch's allocations across zero_grad(),
    backward and step() stays near one batch, not a whole second set of gradients."""
    import zero_amd._sharded as sh
    from zero_amd import zero2

    init_pg(0, 1, free_port())
    try:
        monkeypatch.setattr(sh, "get", lambda what, dm=None: {"ws": 2, "rank": 0}[what])
        dtype = torch.bfloat16
        torch.manual_seed(0)
        model = torch.nn.Sequential(*[torch.nn.Linear(1024, 1024, bias=False)
                                      for _ in range(16)]).to(gpu, dtype)  # 2 MiB of grad each
        params = list(model.parameters())
        opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), comm=_NoComm())
        eng = opt.engine
        eng.land_batch_bytes = 4 << 20
        grad_bytes = sum(p.numel() * p.element_size() for p in params)  # 32 MiB
        x = torch.randn(8, 1024, device=gpu, dtype=dtype)
        for t in range(3):
            opt.zero_grad()
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats(gpu)
            base = torch.cuda.memory_allocated(gpu)
            model(x).float().square().mean().backward()
            # landed from the hooks, batch by batch (at most the last partial batch is left)
            assert sum(eng.is_view(i, p.grad) for i, p in enumerate(params)) >= len(params) - 1
            opt.step()
            torch.cuda.synchronize()
            peak = torch.cuda.max_memory_allocated(gpu) - base
            # a batch (4 MiB) + the gradient that completes it + activations: far below 32 MiB
            assert peak < grad_bytes // 3, (t, peak, grad_bytes)
            assert all(eng.is_view(i, p.grad) for i, p in enumerate(params))
    finally:
        dist.destroy_process_group()
