"""Low-precision (fp8 E4M3, row-wise scaled) ZeRO-3 parameter all-gather.

Kernels: bit-exact against a numpy/torch restatement (float32 scaling in the same order, torch's
float8_e4m3fn round-to-nearest-even for the cast).  ZeRO-3: every rank's materialised full
parameter equals that restatement applied row by row to the full original parameter — rows are
scaled independently, so where the dim-0 chunk boundaries fall does not matter.
"""

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port
from _zero_run import spawn_batch, spawn_ranks, init_pg

pytestmark = pytest.mark.gpu


def fp8_rows_oracle(x: torch.Tensor):
    """(q bytes, scales, dequantised float32) of a 2-D float tensor (CPU)."""
    x = x.float().numpy()
    amax = np.max(np.abs(x), axis=1).astype(np.float32)
    inv = np.where(amax > 0, np.float32(448.0) / np.where(amax > 0, amax, 1), np.float32(1)).astype(np.float32)
    v = np.clip((x * inv[:, None]).astype(np.float32), np.float32(-448), np.float32(448))
    q = torch.from_numpy(v).to(torch.float8_e4m3fn)
    sc = np.where(amax > 0, amax / np.float32(448.0), np.float32(1)).astype(np.float32)
    deq = (q.float().numpy() * sc[:, None]).astype(np.float32)
    return q.view(torch.uint8).numpy(), sc, deq


def _port():
    return free_port()


# (the vector path keeps rows in registers in 8, 16 or 32 16-B chunks per lane — up to 4096 / 8192
# / 16384 bf16 or 2048 / 4096 / 8192 fp32 elements — longer rows are streamed twice in batches of 8;
# 37 takes the scalar fallback; dequantisation items are (row, segment) pairs of 2048 bf16 / 1024
# fp32 elements, so most row lengths here end in a partial segment)
@pytest.mark.parametrize("rows,row_len", [(5, 64), (3, 37), (17, 12800), (4, 8), (1, 11008),
                                          (9, 4096), (6, 2048), (5, 14336), (7, 4104), (4, 8192),
                                          (3, 16392), (2, 40968), (1031, 24)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fp8_rows_kernels_bit_exact(gpu, rows, row_len, dtype):
    from zero_amd import _lib
    from zero_amd.comm import zs_dtype

    g = torch.Generator().manual_seed(rows * row_len)
    x = (torch.randn(rows, row_len, generator=g) * torch.logspace(-3, 2, rows)[:, None]).to(dtype)
    if rows >= 4:
        x[2] = 0  # all-zero row: scale 1
        x[3, : min(5, row_len)] = 1e-30  # deep subnormal territory after scaling
    q_want, sc_want, deq_want = fp8_rows_oracle(x)
    d = x.to(gpu)
    q = torch.empty(rows, row_len, dtype=torch.uint8, device=gpu)
    sc = torch.empty(rows, dtype=torch.float32, device=gpu)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("zs_fp8_quantize_rows", d.data_ptr(), zs_dtype(dtype), q.data_ptr(), sc.data_ptr(),
              rows, row_len, st)
    y = torch.empty(rows, row_len, dtype=dtype, device=gpu)
    _lib.call("zs_fp8_dequantize_rows", q.data_ptr(), sc.data_ptr(), y.data_ptr(), zs_dtype(dtype),
              rows, row_len, st)
    torch.cuda.synchronize()
    assert np.array_equal(sc.cpu().numpy(), sc_want)
    assert np.array_equal(q.cpu().numpy(), q_want)
    want = torch.from_numpy(deq_want).to(dtype)
    assert torch.equal(y.cpu(), want)


@pytest.mark.parametrize("ws", [1, 3, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fp8_rowset_and_gathered_bit_exact(gpu, ws, dtype):
    """The gather group's fused forms: zs_fp8_quantize_rowset over several matrices of one module
    (each rank its dim-0 chunk, padding rows past the real ones) and zs_fp8_dequantize_gathered
    from the rank-major concatenation the all-gather produces, against the row oracle on the
    full matrices (padding rows come back as zeros)."""
    from zero_amd import _lib
    from zero_amd.comm import zs_dtype

    # (d0, row_len): uneven chunks, a row longer than 16384 bf16 (non-resident path), 17 matrices
    # (> 16 per launch: two launches), short matrices
    shapes = [(37, 64), (40, 2048), (9, 4104), (5, 16392), (3, 8)] + [(ws + 2, 24)] * 12
    g = torch.Generator().manual_seed(ws)
    fulls = [(torch.randn(d0, rl, generator=g) * 10.0 ** torch.randint(-3, 3, (d0, 1), generator=g)
              ).to(dtype) for d0, rl in shapes]
    fulls[0][4] = 0  # all-zero row: scale 1
    cs = [-(-d0 // ws) for d0, _ in shapes]
    n = len(shapes)
    q_off = np.cumsum([0] + [c * rl for c, (_, rl) in zip(cs, shapes)])[:-1].astype(np.int64)
    sc_off = np.cumsum([0] + cs)[:-1].astype(np.int64)
    qtot = int(sum(c * rl for c, (_, rl) in zip(cs, shapes)))
    sctot = int(sum(cs))
    st = torch.cuda.current_stream().cuda_stream
    qr = torch.empty(ws * qtot, dtype=torch.uint8, device=gpu)
    sr = torch.empty(ws * sctot, dtype=torch.float32, device=gpu)
    keep = []
    for k in range(ws):  # every rank's send side, straight into its place in the gathered buffer
        chunks = [f[k * c:(k + 1) * c].contiguous().to(gpu) for f, c in zip(fulls, cs)]
        keep += chunks
        src = np.array([t.data_ptr() for t in chunks], np.uint64)
        qp = np.uint64(qr.data_ptr() + k * qtot) + q_off.astype(np.uint64)
        sp = np.uint64(sr.data_ptr() + 4 * k * sctot) + (sc_off * 4).astype(np.uint64)
        rows = np.array([t.shape[0] for t in chunks], np.int64)
        cs_a = np.array(cs, np.int64)
        rl = np.array([r for _, r in shapes], np.int64)
        _lib.call("zs_fp8_quantize_rowset", n, src.ctypes.data, qp.ctypes.data, sp.ctypes.data,
                  rows.ctypes.data, cs_a.ctypes.data, rl.ctypes.data, zs_dtype(dtype), st)
    outs = [torch.full((ws * c, r), 7.0, dtype=dtype, device=gpu) for c, (_, r) in zip(cs, shapes)]
    dst = np.array([o.data_ptr() for o in outs], np.uint64)
    # (every table a named array: a temporary's .ctypes.data would point at freed memory)
    cs_t = np.array(cs, np.int64)
    len_t = np.array([r for _, r in shapes], np.int64)
    _lib.call("zs_fp8_dequantize_gathered", n, qr.data_ptr(), sr.data_ptr(), ws, qtot, sctot,
              q_off.ctypes.data, sc_off.ctypes.data, cs_t.ctypes.data, len_t.ctypes.data,
              dst.ctypes.data, zs_dtype(dtype), st)
    torch.cuda.synchronize()
    qh, sh = qr.cpu().numpy(), sr.cpu().numpy()
    for m, (f, c, o) in enumerate(zip(fulls, cs, outs)):
        q_want, sc_want, deq_want = fp8_rows_oracle(f)
        d0, rl = f.shape
        for k in range(ws):  # the send side, rank by rank (padding rows: q = 0, scale = 1)
            real = max(0, min(c, d0 - k * c))
            qk = qh[k * qtot + q_off[m]: k * qtot + q_off[m] + c * rl].reshape(c, rl)
            sk = sh[k * sctot + sc_off[m]: k * sctot + sc_off[m] + c]
            assert np.array_equal(qk[:real], q_want[k * c:k * c + real]), (m, k)
            assert np.array_equal(sk[:real], sc_want[k * c:k * c + real]), (m, k)
            assert not qk[real:].any() and np.all(sk[real:] == 1.0), (m, k)
        got = o.cpu()
        assert torch.equal(got[:d0], torch.from_numpy(deq_want).to(dtype)), m
        assert not got[d0:].float().any(), m


def _check_materialize(rank, ws, dtype, comm=None, reshard=True):
    from zero_amd import zero3

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(40, 24), torch.nn.ReLU(), torch.nn.Linear(24, 10)).to(dev).to(dtype)
    full = [p.detach().cpu().clone() for p in model.parameters()]
    kw = {"comm": comm} if comm is not None else {}
    opt = zero3.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), gather_dtype="fp8", **kw)
    for p, f in zip(model.parameters(), full):
        man = opt.param_managers[p]
        man.materialize()
        torch.cuda.synchronize()
        got = p.detach().cpu()
        if f.dim() >= 2:
            assert man.fp8
            want = torch.from_numpy(fp8_rows_oracle(f)[2]).to(dtype)
        else:
            want = f
        assert torch.equal(got, want), (rank, tuple(f.shape))
        man.release()
    # a hooked training iteration runs on fp8-gathered weights (reshard=False: gathered once,
    # kept from forward through backward)
    zero3.register_zero3_hooks(model, opt.param_managers, reshard_after_forward=reshard)
    x = torch.randn(8, 40, device=dev).to(dtype)
    n0 = opt.runtime.n_gathers
    loss = model(x).float().pow(2).mean()
    loss.backward()
    opt.step()
    assert torch.isfinite(loss)
    if ws > 1:  # two Linear modules: gathered in forward, and again in backward unless kept,
        # plus the prefetch of the next iteration's first wave (up to `wave` groups)
        base, w = (4 if reshard else 2), opt.runtime.wave
        assert base <= opt.runtime.n_gathers - n0 <= base + w
    assert all(m.full_data is None for m in opt.param_managers.values())  # released after backward


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_zero3_fp8_gather_ws1(gpu, dtype):
    init_pg(0, 1, _port())
    try:
        _check_materialize(0, 1, dtype)
    finally:
        dist.destroy_process_group()


def _mr(rank, ws, port, reshard=True):
    from conftest import PKG, REPO  # noqa: F401
    from _gloo_comm import GlooStagedComm, test_comm  # noqa: F401

    torch.cuda.set_device(0)
    init_pg(rank, ws, port)
    _check_materialize(rank, ws, torch.bfloat16, comm=test_comm(), reshard=reshard)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws,reshards", [(2, (True, False)), (3, (True,))])
def test_zero3_fp8_gather_multirank(gpu, ws, reshards):
    spawn_batch(ws, [(_mr, (r,)) for r in reshards])


@pytest.mark.parametrize("ws", [1, 3])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_zero3_fp8_standalone_manager_uses_set_kernels(gpu, ws, dtype, monkeypatch):
    """a standalone Zero3ParamManager's fp8 gather runs the module path's set
    kernels as a one-matrix set (zs_fp8_quantize_rowset / zs_fp8_dequantize_gathered), never the
    per-matrix zs_fp8_*_rows forms.  Every rank's send side is built by the manager itself; the
    all-gather is emulated by concatenating them rank-major; the full tensor (the reference's
    torch.cat of ws equal shards, zero3.py:36-41) equals the row oracle.  A matrix whose rows are
    not a multiple of 8 elements gathers unquantised."""
    from zero_amd import _lib, zero3

    called = []
    real_call = _lib.call
    monkeypatch.setattr(_lib, "call", lambda name, *a: (called.append(name), real_call(name, *a))[1])
    g = torch.Generator().manual_seed(ws)
    d0 = 13 * ws
    full = (torch.randn(d0, 64, generator=g) * 10.0 ** torch.randint(-3, 3, (d0, 1), generator=g)).to(dtype)
    full[5] = 0
    cs = 13
    st = torch.cuda.current_stream()
    states, mans = [], []
    for k in range(ws):
        p = torch.nn.Parameter(full[k * cs:(k + 1) * cs].contiguous().to(gpu))
        m = zero3.Zero3ParamManager(p, k, ws, gather_dtype="fp8")
        assert m.fp8 and m.full_shape == (d0, 64) and m.cs == cs
        states.append(m._gather_prepare(st))
        mans.append(m)
    fq = torch.cat([s[0] for s in states])
    fsc = torch.cat([s[1] for s in states])
    out = mans[0]._gather_finish(st, (None, None, fq, fsc, None))
    torch.cuda.synchronize()
    want = torch.from_numpy(fp8_rows_oracle(full)[2]).to(dtype)
    assert torch.equal(out[:full.numel()].view(d0, 64).cpu(), want)
    assert "zs_fp8_quantize_rows" not in called and "zs_fp8_dequantize_rows" not in called
    assert called.count("zs_fp8_quantize_rowset") == ws and called.count("zs_fp8_dequantize_gathered") == 1
    odd = zero3.Zero3ParamManager(torch.nn.Parameter(torch.zeros(5, 12, device=gpu, dtype=dtype)), 0, 1,
                                  gather_dtype="fp8")
    assert not odd.fp8  # row of 12 elements: gathered as it is
