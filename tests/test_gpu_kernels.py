"""gfx950 kernels through the C ABI: segment copy (bit-exact) and fused Adam (vs the C oracle
bit-exact, vs torch.optim.Adam's known answers within 1e-6)."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import zero_oracle as zo

pytestmark = pytest.mark.gpu


def _seed(n):
    return np.random.default_rng(n)


@pytest.mark.parametrize("nt", [-1, 1])  # cache policy by size (here: default) / non-temporal
def test_copy_segments_bit_exact(gpu, nt):
    from zero_amd import _lib

    _lib.call("zs_tune", b"copy_nt", nt, None)
    try:
        _copy_case(gpu)
    finally:
        _lib.call("zs_tune", b"copy_nt", -1, None)


def _copy_case(gpu):
    from zero_amd.kernels import CopySet

    rng = _seed(1)
    src = torch.randint(0, 256, (1 << 20,), dtype=torch.uint8, device=gpu)
    dst = torch.zeros(1 << 21, dtype=torch.uint8, device=gpu)
    want = torch.zeros_like(dst).cpu()
    s_cpu = src.cpu()
    srcs, dsts, nbs = [], [], []
    doff = 0
    lens = [0, 1, 2, 15, 16, 17, 31, 64, 1000, 16384, 16385, 100_000, 65536 * 3 + 7]
    for k, ln in enumerate(lens * 2):
        align = k % 2 == 0
        so = int(rng.integers(0, 1000)) * (16 if align else 1)
        doff = (doff + 15) // 16 * 16 if align else doff + 3
        zero = (k % 7) == 3
        srcs.append(0 if zero else src.data_ptr() + so)
        dsts.append(dst.data_ptr() + doff)
        nbs.append(ln)
        want[doff:doff + ln] = 0 if zero else s_cpu[so:so + ln]
        doff += ln
    dst.fill_(0)
    CopySet(srcs, dsts, nbs).run(torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert torch.equal(dst.cpu(), want)


def test_copy_zero_fill_overwrites(gpu):
    from zero_amd.kernels import CopySet

    dst = torch.full((4096,), 7, dtype=torch.float32, device=gpu)
    CopySet([0], [dst.data_ptr() + 64], [1024]).run(torch.cuda.current_stream())
    torch.cuda.synchronize()
    h = dst.cpu()
    assert (h[16:16 + 256] == 0).all() and (h[:16] == 7).all() and (h[272:] == 7).all()


def _adam_rows(g, master, master_out, p_out, m, v, vmax=None, carry=None, n=None):
    ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    n = master.numel() if n is None else n
    return np.array([[ptr(g), ptr(master), ptr(master_out), ptr(p_out), ptr(m), ptr(v),
                      ptr(vmax), ptr(carry), n]], dtype=np.uint64)


CASES = {
    "default": dict(),
    "wd": dict(weight_decay=1e-2),
    "amsgrad": dict(amsgrad=True),
    "maximize": dict(maximize=True),
    "adamw": dict(weight_decay=1e-2, decoupled=True),
    "hyper": dict(lr=1e-2, beta1=0.8, beta2=0.99, eps=1e-6),
}


@pytest.mark.parametrize("case", list(CASES))
def test_adam_fp32_vs_torch_kat_and_oracle(gpu, golden, case):
    from zero_amd._lib import ZS_F32
    from zero_amd.kernels import AdamSet, adam_hparams

    z = golden("adam_kat.npz")
    cfg = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0)
    cfg.update(CASES[case])
    flags = {k: cfg.pop(k) for k in ("decoupled", "amsgrad", "maximize") if k in cfg}
    p0 = z[f"{case}_p0"]
    p = torch.from_numpy(p0.copy()).to(gpu)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    vmax = torch.zeros_like(p) if flags.get("amsgrad") else None
    g = torch.empty_like(p)
    aset = AdamSet(_adam_rows(g, p, p, None, m, v, vmax), ZS_F32)
    # C oracle in lock-step
    cp, cm, cv, cx = p0.copy(), np.zeros_like(p0), np.zeros_like(p0), np.zeros_like(p0)
    for t, gt in enumerate(z[f"{case}_grads"]):
        g.copy_(torch.from_numpy(gt))
        aset.run(adam_hparams(cfg["lr"], cfg["beta1"], cfg["beta2"], cfg["eps"], cfg["weight_decay"],
                              t + 1, **flags), torch.cuda.current_stream())
        c_oracle.adam_f32(cp, np.ascontiguousarray(gt), cm, cv,
                          c_oracle.hparams(step=t + 1, **cfg, **flags),
                          vmax=cx if flags.get("amsgrad") else None)
    torch.cuda.synchronize()
    hp_, hm, hv = p.cpu().numpy(), m.cpu().numpy(), v.cpu().numpy()
    # bit-exact against the C restatement (same rounding order, IEEE sqrt/div on both sides)
    assert np.array_equal(hp_.view(np.uint32), cp.view(np.uint32))
    assert np.array_equal(hm.view(np.uint32), cm.view(np.uint32))
    assert np.array_equal(hv.view(np.uint32), cv.view(np.uint32))
    # within 1e-6 of torch.optim.Adam itself (north-star tolerance)
    for a, key in ((hp_, "p"), (hm, "m"), (hv, "v")):
        ref = z[f"{case}_{key}"]
        assert np.max(np.abs(a - ref)) / np.max(np.abs(ref)) <= 1e-6


@pytest.mark.parametrize("ws,carry", [(1, False), (3, False), (4, False), (3, True), (8, True)])
def test_adam_bf16_master_and_carry_vs_oracle(gpu, ws, carry):
    """bf16 grads + fp32 master/m/v + bf16 param out; grad/ws and the ZeRO-1 carry folded in."""
    from zero_amd._lib import ZS_BF16
    from zero_amd.kernels import AdamSet, adam_hparams

    rng = _seed(ws)
    n = 100_003
    master0 = (rng.standard_normal(n) * 0.02).astype(np.float32)
    master = torch.from_numpy(master0.copy()).to(gpu)
    pbf = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
    m, v = torch.zeros_like(master), torch.zeros_like(master)
    cr = torch.zeros_like(master) if carry else None
    g = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
    aset = AdamSet(_adam_rows(g, master, master, pbf, m, v, carry=cr), ZS_BF16)
    cm_, cp_, cmm, cvv = master0.copy(), np.zeros(n, np.uint16), np.zeros(n, np.float32), np.zeros(n, np.float32)
    ccr = np.zeros(n, np.float32) if carry else None
    for t in range(1, 6):
        gt = torch.from_numpy((rng.standard_normal(n) * 1e-2).astype(np.float32)).to(torch.bfloat16)
        g.copy_(gt)
        kw = dict(grad_div=float(ws), carry_mul=float(ws - 1) if carry else 0.0)
        aset.run(adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, t, **kw), torch.cuda.current_stream())
        c_oracle.adam_bf16(cm_, cp_, gt.view(torch.int16).numpy().view(np.uint16).copy(), cmm, cvv,
                           c_oracle.hparams(step=t, **kw), carry=ccr)
    torch.cuda.synchronize()
    assert np.array_equal(master.cpu().numpy().view(np.uint32), cm_.view(np.uint32))
    assert np.array_equal(pbf.cpu().view(torch.int16).numpy().view(np.uint16), cp_)
    assert np.array_equal(pbf.cpu().view(torch.int16).numpy().view(np.uint16),
                          zo.f32_to_bf16_bits(cm_))
    if carry:
        assert np.array_equal(cr.cpu().numpy().view(np.uint32), ccr.view(np.uint32))


@pytest.mark.parametrize("ws,carry,ams", [(1, False, False), (4, False, True), (3, True, False)])
def test_adam_split_master_vs_oracle(gpu, ws, carry, ams):
    """ZS_BF16_SPLIT: the fp32 master held as the bf16 param + an int16 residual, updated in place,
    bit-exact against the C oracle over 6 steps (vector path and a scalar tail: n % 4 == 3).
    The start state holds every tie class of the encoding: exact ties under an even and an odd
    bf16 param, both signs, a denormal tie, and values next to the bf16 overflow threshold."""
    from zero_amd._lib import ZS_BF16, ZS_BF16_SPLIT
    from zero_amd.kernels import AdamSet, adam_hparams

    rng = _seed(10 * ws + carry)
    n = 65_539
    master0 = (rng.standard_normal(n) * 0.02).astype(np.float32)
    special = np.array([0x3C808000, 0x3C818000, 0xBC808000, 0xBC818000, 0x00008000, 0x80008000,
                        0x7F7F7FFF, 0x7F7F8000, 0x3F80FFFF, 0x00000000], np.uint32)
    u = master0.view(np.uint32)
    u[:len(special)] = special
    u[-len(special):] = special  # and in the scalar tail
    hi0, lo0 = c_oracle.split_master(master0)
    # the encoding itself: exact except an even-hi tie, which moves 1 ulp toward zero
    back = c_oracle.join_master(hi0, lo0).view(np.uint32)
    tie_even = ((u & 0xFFFF) == 0x8000) & (((u >> 16) & 1) == 0)
    assert np.array_equal(back[~tie_even], u[~tie_even]) and np.array_equal(back[tie_even], u[tie_even] - 1)
    assert np.array_equal(hi0, zo.f32_to_bf16_bits(master0))
    hi = torch.from_numpy(hi0.view(np.int16).copy()).to(gpu).view(torch.bfloat16)
    lo = torch.from_numpy(lo0.view(np.int16).copy()).to(gpu)
    m, v = torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    vm = torch.zeros(n, device=gpu) if ams else None
    cr = torch.zeros(n, device=gpu) if carry else None
    g = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
    aset = AdamSet(_adam_rows(g, hi, lo, hi, m, v, vmax=vm, carry=cr, n=n), ZS_BF16, ZS_BF16_SPLIT)
    assert aset.bytes == n * (2 + 2 + 4 + 8 + 8 + 2 + (8 if ams else 0) + (8 if carry else 0))
    chi, clo = hi0.copy(), lo0.copy()
    cm_, cv_ = np.zeros(n, np.float32), np.zeros(n, np.float32)
    cvm = np.zeros(n, np.float32) if ams else None
    ccr = np.zeros(n, np.float32) if carry else None
    for t in range(1, 7):
        gt = torch.from_numpy((rng.standard_normal(n) * 1e-2).astype(np.float32)).to(torch.bfloat16)
        g.copy_(gt)
        kw = dict(grad_div=float(ws), carry_mul=float(ws - 1) if carry else 0.0)
        aset.run(adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, t, amsgrad=ams, **kw),
                 torch.cuda.current_stream())
        c_oracle.adam_bf16_split(chi, clo, gt.view(torch.int16).numpy().view(np.uint16).copy(), cm_,
                                 cv_, c_oracle.hparams(step=t, amsgrad=ams, **kw), vmax=cvm, carry=ccr)
    torch.cuda.synchronize()
    assert np.array_equal(hi.cpu().view(torch.int16).numpy().view(np.uint16), chi)
    assert np.array_equal(lo.cpu().numpy().view(np.uint16), clo)
    assert np.array_equal(m.cpu().numpy().view(np.uint32), cm_.view(np.uint32))
    assert np.array_equal(v.cpu().numpy().view(np.uint32), cv_.view(np.uint32))
    if carry:
        assert np.array_equal(cr.cpu().numpy().view(np.uint32), ccr.view(np.uint32))


def test_adam_split_master_rejects_bad_tables(gpu):
    from zero_amd._lib import ZS_BF16_SPLIT, ZS_F32, ZeroAmdError
    from zero_amd.kernels import AdamSet

    n = 64
    hi = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
    m, v = torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    with pytest.raises(ZeroAmdError, match="master_out"):  # no residual buffer
        AdamSet(_adam_rows(hi, hi, None, hi, m, v, n=n), 1, ZS_BF16_SPLIT)
    lo = torch.zeros(n, dtype=torch.int16, device=gpu)
    with pytest.raises(ZeroAmdError, match="bf16 grads"):
        AdamSet(_adam_rows(m, hi, lo, hi, m, v, n=n), ZS_F32, ZS_BF16_SPLIT)


def test_adam_many_segments_unaligned_and_tails(gpu):
    """Segment table with tails, unaligned (scalar-path) segments, null grads and 1-elem segs."""
    from zero_amd._lib import ZS_F32
    from zero_amd.kernels import AdamSet, adam_hparams

    rng = _seed(7)
    N = 300_000
    P = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).to(gpu)
    G = torch.from_numpy(rng.standard_normal(N).astype(np.float32) * 1e-3).to(gpu)
    M, V = torch.zeros_like(P), torch.zeros_like(P)
    rows, off = [], 0
    for k, ln in enumerate([1, 3, 4, 5, 2047, 2048, 2049, 4096 + 13, 70_001, 1, 999]):
        off += k % 3  # k%3 != 0 → unaligned (scalar path)
        gp = 0 if k == 4 else G.data_ptr() + 4 * off
        r = [gp] + [P.data_ptr() + 4 * off] * 2 + [0, M.data_ptr() + 4 * off, V.data_ptr() + 4 * off,
                                                   0, 0, ln]
        rows.append(r)
        off += ln
    rows = np.array(rows, dtype=np.uint64)
    p_ref, g_ref = P.cpu().numpy().copy(), G.cpu().numpy().copy()
    m_ref, v_ref = np.zeros(N, np.float32), np.zeros(N, np.float32)
    AdamSet(rows, ZS_F32).run(adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, 1), torch.cuda.current_stream())
    torch.cuda.synchronize()
    for r in rows:
        o = (int(r[1]) - P.data_ptr()) // 4
        ln = int(r[8])
        gg = np.zeros(ln, np.float32) if int(r[0]) == 0 else g_ref[o:o + ln].copy()
        pp, mm, vv = p_ref[o:o + ln].copy(), m_ref[o:o + ln].copy(), v_ref[o:o + ln].copy()
        c_oracle.adam_f32(pp, gg, mm, vv, c_oracle.hparams(step=1))
        p_ref[o:o + ln], m_ref[o:o + ln], v_ref[o:o + ln] = pp, mm, vv
    assert np.array_equal(P.cpu().numpy().view(np.uint32), p_ref.view(np.uint32))
    assert np.array_equal(M.cpu().numpy().view(np.uint32), m_ref.view(np.uint32))


def test_pack_unpack_round_trip_c2(gpu):
    """Size-independent property at C2 scale (100.7M fp32 params): pack every Layout-R bucket at
    ws=4, unpack into fresh tensors, get the params back bit-for-bit."""
    from zero_amd.kernels import CopySet
    from zero_amd.plan import Plan
    from zero_amd.shapes import mlp_shapes

    shapes = mlp_shapes(4096)
    ps = [torch.randn(s, device=gpu) for s in shapes]
    outs = [torch.empty_like(p) for p in ps]
    plan = Plan([p.numel() for p in ps], 4, 0, "reference", window_elems=4 << 20)
    arena = torch.zeros(plan.arena_elems, device=gpu)
    st = torch.cuda.current_stream()
    assert plan.num_even < plan.num_buckets  # ranks own 33.6M / 16.8M elements: ragged tail
    for k in range(plan.num_buckets):
        s, b = plan.segments(k), plan.bucket(k)
        src = [ps[i].data_ptr() + 4 * po for i, po in zip(s.param, s.param_off)]
        dst = [arena.data_ptr() + 4 * (b.arena_off + bo) for bo in s.buf_off]
        CopySet(src, dst, s.length * 4).run(st)
        CopySet(dst, [outs[i].data_ptr() + 4 * po for i, po in zip(s.param, s.param_off)],
                s.length * 4).run(st)
    torch.cuda.synchronize()
    for p, o in zip(ps, outs):
        assert torch.equal(p, o)


@pytest.mark.parametrize("case", ["f32_l2_ws3", "bf16_out_carry_ws4", "adamw_f32", "unaligned_bf16"])
def test_adam_step_single_range_vs_oracle(gpu, case):
    """zs_adam_step (SURVEY.md §8(b)'s single-range form) is bit-exact against the C oracle over
    3 steps: vector body + scalar tail (n = 100,003), grad / ws for ws = 3 and 4, ZeRO-1 carry,
    L2 / AdamW decay, and a range offset by one element (scalar path throughout)."""
    from zero_amd.kernels import adam_step

    rng = _seed(["f32_l2_ws3", "bf16_out_carry_ws4", "adamw_f32", "unaligned_bf16"].index(case) + 40)
    n = 100_003
    bf16 = case in ("bf16_out_carry_ws4", "unaligned_bf16")
    ws = {"f32_l2_ws3": 3, "bf16_out_carry_ws4": 4}.get(case, 1)
    carry = case == "bf16_out_carry_ws4"
    kw = dict(weight_decay=1e-2 if case in ("f32_l2_ws3", "adamw_f32") else 0.0,
              decoupled=case == "adamw_f32")
    off = 1 if case == "unaligned_bf16" else 0
    p0 = (rng.standard_normal(n) * 0.02).astype(np.float32)
    P = torch.zeros(n + off, device=gpu)[off:]
    P.copy_(torch.from_numpy(p0))
    M, V = torch.zeros(n + off, device=gpu)[off:], torch.zeros(n + off, device=gpu)[off:]
    C = torch.zeros(n, device=gpu) if carry else None
    PB = torch.zeros(n + off, dtype=torch.bfloat16, device=gpu)[off:] if bf16 else None
    G = torch.zeros(n + off, dtype=torch.bfloat16 if bf16 else torch.float32, device=gpu)[off:]
    rp, rm, rv = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    rb, rc = np.zeros(n, np.uint16), (np.zeros(n, np.float32) if carry else None)
    for t in range(1, 4):
        gt = torch.from_numpy((rng.standard_normal(n) * 1e-2).astype(np.float32))
        gt = gt.to(torch.bfloat16) if bf16 else gt
        G.copy_(gt)
        adam_step(P, G, M, V, step=t, grad_div=float(ws), p_bf16=PB, carry=C,
                  carry_mul=float(ws - 1) if carry else 0.0, **kw)
        hp = c_oracle.hparams(step=t, grad_div=float(ws), carry_mul=float(ws - 1) if carry else 0.0,
                              **kw)
        if bf16:
            c_oracle.adam_bf16(rp, rb, gt.view(torch.int16).numpy().view(np.uint16).copy(), rm, rv,
                               hp, carry=rc)
        else:
            c_oracle.adam_f32(rp, gt.numpy().copy(), rm, rv, hp)
    torch.cuda.synchronize()
    assert np.array_equal(P.cpu().numpy().view(np.uint32), rp.view(np.uint32))
    assert np.array_equal(M.cpu().numpy().view(np.uint32), rm.view(np.uint32))
    assert np.array_equal(V.cpu().numpy().view(np.uint32), rv.view(np.uint32))
    if bf16:
        assert np.array_equal(PB.cpu().view(torch.int16).numpy().view(np.uint16), rb)
    if carry:
        assert np.array_equal(C.cpu().numpy().view(np.uint32), rc.view(np.uint32))


@pytest.mark.parametrize("ws", [1, 3, 4, 7])
def test_adam_step_literal_signature_vs_oracle(gpu, ws):
    """SURVEY.md §8(b)'s literal zs_adam_step (float scalars, grad_scale = 1/ws, const carry):
    with hyper-parameters exactly representable in fp32 the scalars it derives are torch's, so
    it is bit-exact against the C oracle with the same double scalars — grad / ws (ws = 7: the
    divisor is recovered from float(1/7)), ZeRO-1 carry with carry_scale = ws - 1, bf16 copy."""
    import ctypes

    from zero_amd import _lib
    from zero_amd.kernels import stream_handle

    rng = _seed(70 + ws)
    n = 50_001
    lr, b1, b2, eps, wd = 2.0 ** -10, 0.875, 1 - 2.0 ** -10, 2.0 ** -27, 2.0 ** -7
    p0 = (rng.standard_normal(n) * 0.02).astype(np.float32)
    P = torch.from_numpy(p0.copy()).to(gpu)
    M, V = torch.zeros(n, device=gpu), torch.zeros(n, device=gpu)
    C = torch.zeros(n, device=gpu) if ws > 1 else None
    PB = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
    G = torch.zeros(n, device=gpu)
    rp, rm, rv = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    rc = np.zeros(n, np.float32) if ws > 1 else None
    f = ctypes.c_float
    st = torch.cuda.current_stream(gpu)
    for t in range(1, 4):
        gt = (rng.standard_normal(n) * 1e-2).astype(np.float32)
        G.copy_(torch.from_numpy(gt))
        _lib.call("zs_adam_step", P.data_ptr(), PB.data_ptr(), G.data_ptr(), _lib.ZS_F32,
                  M.data_ptr(), V.data_ptr(), n, f(lr), f(b1), f(b2), f(eps), f(wd), 1, t,
                  f(np.float32(1.0 / ws)), None if C is None else C.data_ptr(), f(ws - 1),
                  stream_handle(st))
        hp = c_oracle.hparams(lr, b1, b2, eps, wd, step=t, decoupled=True, grad_div=float(ws),
                              carry_mul=float(ws - 1))
        c_oracle.adam_f32(rp, gt.copy(), rm, rv, hp, carry=rc)
    torch.cuda.synchronize()
    assert np.array_equal(P.cpu().numpy().view(np.uint32), rp.view(np.uint32))
    assert np.array_equal(M.cpu().numpy().view(np.uint32), rm.view(np.uint32))
    assert np.array_equal(V.cpu().numpy().view(np.uint32), rv.view(np.uint32))
    want_b = torch.from_numpy(rp).to(torch.bfloat16).view(torch.int16).numpy()
    assert np.array_equal(PB.cpu().view(torch.int16).numpy(), want_b)
    if C is not None:
        assert np.array_equal(C.cpu().numpy().view(np.uint32), rc.view(np.uint32))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_pack_unpack_through_plan_bit_exact(gpu, dtype):
    """zs_pack / zs_unpack against the plan's own segment table, bit-exact, at
    ws=3 with even and ragged buckets: a missing grad packs as zeros, re-pointed grads rebuild the
    cached tables, and unpacking every bucket returns every grad element to its parameter."""
    from zero_amd import _lib
    from zero_amd.plan import Plan

    zdt = _lib.ZS_F32 if dtype == torch.float32 else _lib.ZS_BF16
    es = 4 if dtype == torch.float32 else 2
    shapes = [(257, 129), (3000,), (64, 64), (5,), (1000, 33), (1,), (4096, 7)]
    numels = [int(np.prod(s)) for s in shapes]
    plan = Plan(numels, 3, 1, "reference", window_elems=6000)
    assert 0 < plan.num_even < plan.num_buckets
    st = torch.cuda.current_stream().cuda_stream
    rounds = [[torch.randn(n, device=gpu).to(dtype) for n in numels] for _ in range(2)]
    rounds[1][3] = None  # a param without a grad: its slots pack as zeros
    for grads in rounds:
        ptrs = [0 if g is None else g.data_ptr() for g in grads]
        host = [None if g is None else g.view(torch.int16 if es == 2 else torch.int32).cpu().numpy()
                for g in grads]
        outs = [torch.zeros(n, dtype=dtype, device=gpu) for n in numels]
        for k in range(plan.num_buckets):
            b, s = plan.bucket(k), plan.segments(k)
            assert plan.bucket_bytes(k, zdt) == b.elems * es
            buf = torch.full((b.elems,), 7, dtype=dtype, device=gpu)
            plan.pack(k, ptrs, buf.data_ptr(), zdt, st)
            want = buf.view(torch.int16 if es == 2 else torch.int32).cpu().numpy().copy()
            for i, po, bo, ln in zip(s.param, s.param_off, s.buf_off, s.length):
                want[bo:bo + ln] = 0 if host[i] is None else host[i][po:po + ln]
            got = buf.view(torch.int16 if es == 2 else torch.int32).cpu().numpy()
            assert np.array_equal(got, want), k
            plan.unpack(k, buf.data_ptr(), [o.data_ptr() for o in outs], zdt, st)
        torch.cuda.synchronize()
        for g, o in zip(grads, outs):
            assert torch.equal(o, torch.zeros_like(o) if g is None else g)


@pytest.mark.parametrize("n", [1, 7, 8, 1000, 1024, 1025, 4099, 3 * 1024 + 517, 1 << 20])
@pytest.mark.parametrize("offset,nt", [(0, -1), (0, 1), (1, -1)])
def test_convert_fp32_bf16_bit_exact(gpu, n, offset, nt):
    """zs_convert fp32 → bf16 is round-to-nearest-even bit for bit (numpy restatement), including
    ties, subnormals, the overflow edge and infinities; NaN stays NaN; bf16 → fp32 is exact.
    offset 1 makes the buffers unaligned (scalar path); nt 1 forces the vector path's non-temporal
    policy (by size, these buffers take the default one)."""
    from oracle import zero_oracle as zo
    from zero_amd import _lib
    from zero_amd.kernels import convert

    _lib.call("zs_tune", b"convert_nt", nt, None)
    try:
        _convert_case(gpu, n, offset, zo, convert)
    finally:
        _lib.call("zs_tune", b"convert_nt", -1, None)


def _convert_case(gpu, n, offset, zo, convert):

    rng = np.random.default_rng(n + offset)
    x = (rng.standard_normal(n + offset) * 10.0 ** rng.integers(-40, 39, n + offset)).astype(np.float32)
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 3.3895314e38, 3.4028235e38, 1e-45,
                        -1e-40, 1.0 + 2.0 ** -8, 1.0 + 3 * 2.0 ** -8, 1.0 + 2.0 ** -8 + 2.0 ** -20],
                       np.float32)
    k = min(len(special), n)
    x[offset:offset + k] = special[:k]
    src = torch.from_numpy(x).to(gpu)[offset:]
    dst = torch.empty(n + offset, dtype=torch.bfloat16, device=gpu)[offset:]
    convert(src, dst)
    torch.cuda.synchronize()
    got = dst.view(torch.int16).cpu().numpy().view(np.uint16)
    want = zo.f32_to_bf16_bits(x[offset:])
    nan = np.isnan(x[offset:])
    assert np.array_equal(got[~nan], want[~nan])
    assert np.isnan(zo.bf16_bits_to_f32(got[nan])).all()
    back = torch.empty(n + offset, dtype=torch.float32, device=gpu)[offset:]
    convert(dst, back)
    torch.cuda.synchronize()
    b = back.cpu().numpy()
    assert np.array_equal(b[~nan].view(np.uint32), zo.bf16_bits_to_f32(got[~nan]).view(np.uint32))


@pytest.mark.parametrize("nt", [-1, 1])
def test_copy_direct_matches_copyset(gpu, nt):
    """zs_copy_direct (segments in the kernel arguments, ABI v11) writes exactly what the table
    copy writes: > 64 segments (several launches), empty and zero-fill segments, unaligned ones."""
    from zero_amd import _lib
    from zero_amd.kernels import CopySet, copy_direct

    rng = _seed(7)
    src = torch.randint(0, 256, (1 << 21,), dtype=torch.uint8, device=gpu)
    segs, doff = [], 0
    for k in range(150):
        ln = int(rng.choice([0, 1, 15, 16, 17, 4096, 65537]))
        align = k % 3 != 0
        so = int(rng.integers(0, 1000)) * (16 if align else 1)  # so + ln < 16000 + 65537 < 2 MiB
        doff = (doff + 15) // 16 * 16 if align else doff + 5
        segs.append((None if k % 11 == 4 else so, doff, ln))
        doff += ln
    size = doff + 64  # every destination byte in bounds (the host checks what the kernel assumes)
    assert all(b + c <= size for _, b, c in segs)
    assert all(a is None or a + c <= src.numel() for a, _, c in segs)
    outs = [torch.full((size,), 7, dtype=torch.uint8, device=gpu) for _ in range(2)]
    _lib.call("zs_tune", b"copy_nt", nt, None)
    try:
        for out, fn in zip(outs, ("set", "direct")):
            s = [0 if a is None else src.data_ptr() + a for a, _, _ in segs]
            d = [out.data_ptr() + b for _, b, _ in segs]
            n = [c for _, _, c in segs]
            if fn == "set":
                CopySet(s, d, n).run(torch.cuda.current_stream())
            else:
                copy_direct(s, d, n, torch.cuda.current_stream())
        torch.cuda.synchronize()
    finally:
        _lib.call("zs_tune", b"copy_nt", -1, None)
    assert torch.equal(outs[0], outs[1])
    want = torch.full((size,), 7, dtype=torch.uint8)
    sc = src.cpu()
    for a, b, c in segs:
        want[b:b + c] = 0 if a is None else sc[a:a + c]
    assert torch.equal(outs[1].cpu(), want)
