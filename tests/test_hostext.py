"""The ZeRO-3 hooks' host helper (csrc/zs_host_ext.cpp, zero_amd/_hostext*.so): a module's
parameters installed from its gathered allocation and put back to their shards in one call.  CPU
tensors: the helper only rewrites tensor metadata, so its semantics are checked here against the
per-parameter Python it replaces (``param.data = hold.as_strided(...)`` / ``param.data = shard``,
zero3.py:36-52)."""
import pytest
import torch


def _ext():
    from zero_amd import zero3

    assert zero3._hostext is not None, "zero_amd/_hostext*.so missing: run __graft_entry__.build()"
    return zero3._hostext


def _plan(ext, dtype=torch.float32):
    shapes = [(64, 64), (128,), (32, 8)]
    params = [torch.nn.Parameter(torch.randn(s[0] // 4, *s[1:]).to(dtype)) if len(s) > 1
              else torch.nn.Parameter(torch.randn(s[0] // 4).to(dtype)) for s in shapes]
    shards = [p.data for p in params]
    views, off = [], 0
    for s in shapes:
        stride, acc = [], 1
        for d in reversed(s):
            stride.append(acc)
            acc *= d
        views.append((s, tuple(reversed(stride)), off))
        off += -(-acc // 64) * 64
    vp = ext.ViewPlan(params, shards, [list(v[0]) for v in views], [list(v[1]) for v in views],
                      [v[2] for v in views])
    return vp, params, shards, views, off


def test_install_release_match_per_parameter_python():
    ext = _ext()
    vp, params, shards, views, total = _plan(ext)
    assert vp.size == 3 and vp.extent <= total
    hold = torch.randn(total)
    vp.install(hold)
    for p, (shape, stride, off) in zip(params, views):
        want = hold.as_strided(shape, stride, off)
        assert p.shape == want.shape and p.stride() == want.stride()
        assert p.data_ptr() == want.data_ptr() and torch.equal(p.detach(), want)
        assert p.requires_grad and p.is_leaf
    v0 = [p._version for p in params]
    # autograd through the installed parameters: full-shape gradients
    x = torch.randn(5, 64)
    ((x @ params[0]).sum() + params[1].sum() + params[2].sum()).backward()
    assert params[0].grad.shape == (64, 64) and params[1].grad.shape == (128,)
    vp.release()
    for p, sh in zip(params, shards):
        assert p.shape == sh.shape and p.data_ptr() == sh.data_ptr() and torch.equal(p.detach(), sh)
    assert [p._version for p in params] == v0  # as `param.data = x`: no version bump
    assert params[0].grad.shape == (64, 64)  # release leaves the gradient alone (update mode)
    # the views alone, parameters untouched
    vs = vp.views(hold)
    assert all(torch.equal(v, hold.as_strided(*spec)) for v, spec in zip(vs, views))
    assert params[0].shape == shards[0].shape


def test_install_refuses_a_short_or_foreign_allocation():
    ext = _ext()
    vp, params, shards, _, total = _plan(ext)
    with pytest.raises(RuntimeError, match="views reach"):
        vp.install(torch.zeros(vp.extent - 1))
    with pytest.raises(RuntimeError, match="dtype"):
        vp.install(torch.zeros(total, dtype=torch.float64))
    with pytest.raises(RuntimeError, match="1-D"):
        vp.install(torch.zeros(2, total))
    assert all(p.data_ptr() == s.data_ptr() for p, s in zip(params, shards))  # nothing touched
    with pytest.raises(RuntimeError, match="differ in length"):
        ext.ViewPlan(params, shards[:2], [[1]] * 3, [[1]] * 3, [0] * 3)


def test_release_group_uses_the_module_plan_or_falls_back():
    from zero_amd import zero3

    class M:  # the manager surface _release_group touches (full_data stored as _full, as
        # Zero3ParamManager's property does: the plan path clears _full directly)
        def __init__(self, p, rt):
            self.param, self.shard, self.runtime, self._full = p, p.data, rt, None
            self.released = 0

        @property
        def full_data(self):
            return self._full

        @full_data.setter
        def full_data(self, v):
            self._full = v

        def release(self):
            self.released += 1
            self.param.data = self.shard
            self.full_data = None

    class RT:
        _throttled = False  # (the runtime's gather rate limit: not exercised here)

    ext = _ext()
    vp, params, shards, _, total = _plan(ext)
    rt = RT()
    ms = [M(p, rt) for p in params]
    for m, s in zip(ms, shards):
        m.shard = s
    rt._vplans = {id(ms): (ms, vp)}
    hold = torch.zeros(total)
    vp.install(hold)
    for m in ms:
        m.full_data = hold
    zero3._release_group(ms)
    assert all(m.full_data is None and m.released == 0 for m in ms)
    assert all(p.data_ptr() == s.data_ptr() for p, s in zip(params, shards))
    other = list(ms)  # another list object: no plan of its own -> per parameter
    zero3._release_group(other)
    assert all(m.released == 1 for m in ms)
    rt._vplans[id(other)] = (other, None)  # a module the extension could not take: per parameter
    zero3._release_group(other)
    assert all(m.released == 2 for m in ms)


def test_manager_full_data_is_the_parameters_full_tensor():
    """zero3.py:40 exposes the gathered tensor as ``full_data``; a module installed through its
    ViewPlan marks its managers, and full_data is then the parameter's (full) data."""
    from zero_amd import zero3

    p = torch.nn.Parameter(torch.randn(4, 8))
    m = zero3.Zero3ParamManager(p, 0, 2)
    assert m.full_data is None and m.full_shape == (8, 8)
    full = torch.randn(8, 8)
    p.data = full
    m._full = True  # as _GatherRuntime.materialize after ViewPlan.install
    assert m.full_data.shape == (8, 8) and m.full_data.data_ptr() == full.data_ptr()
    m.full_data = None
    assert m.full_data is None


def test_gathered_pairs_with_and_without_a_plan():
    """_Gathered (a module's pending gather) yields the same (manager, full tensor) pairs through
    its ViewPlan's views as through per-parameter strided views."""
    from zero_amd import zero3

    ext = _ext()
    vp, params, shards, views, total = _plan(ext)
    hold = torch.randn(total)
    ms = [object() for _ in params]
    a = list(zero3._Gathered(ms, hold, views, vp))
    b = list(zero3._Gathered(ms, hold, views, None))
    assert [m for m, _ in a] == ms == [m for m, _ in b]
    for (_, x), (_, y), (shape, stride, off) in zip(a, b, views):
        assert x.shape == y.shape == shape and x.stride() == y.stride() == stride
        assert x.data_ptr() == y.data_ptr() == hold.data_ptr() + off * hold.element_size()


# --- GradCounter: the ZeRO-3 backward's per-parameter gradient counting in C++ (round 6) ------
def _chain(n=5, width=8):
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(width, width) * 0.1) for _ in range(n)]

    def loss():
        h = torch.ones(2, width)
        for p in ps:
            h = torch.tanh(h @ p)
        return h.sum()
    return ps, loss


def test_ordered_counter_calls_python_once_per_completed_run_of_buckets():
    """Backward produces the chain's gradients last parameter first; buckets (in backward order)
    [4, 3] [2] [1, 0]: Python hears 'next = 1' after parameter 3, 'next = 2' after 2 and 'next =
    3' after 0 — three calls for five gradients — plus one on_first at the first gradient; the
    Python post-accumulate hooks registered before and after the counter still run, in order, and
    BEFORE the count (a bucket launch drops p.grad: every Python hook still sees the gradient)."""
    ext = _ext()
    ps, loss = _chain()
    bucket_of = [2, 2, 1, 0, 0]
    log = []
    ps[2].register_post_accumulate_grad_hook(lambda p: log.append("py-before"))
    c = ext.GradCounter([2, 1, 2], len(ps), True, lambda: log.append("first"),
                        lambda nxt: log.append(("ready", nxt)), "twice")
    for i, p in enumerate(ps):
        ext.attach(p, c, i, bucket_of[i])
    ps[2].register_post_accumulate_grad_hook(lambda p: log.append("py-after"))
    loss().backward()
    assert log == ["first", ("ready", 1), "py-before", "py-after", ("ready", 2), ("ready", 3)], log
    assert c.next == 3 and c.counted == 5 and c.pending() == [0, 0, 0]
    assert [ext.attached(p) for p in ps] == [1] * 5
    # a second backward before reset(): every gradient would be reduced twice
    with pytest.raises(RuntimeError, match="twice"):
        loss().backward()
    c.reset()
    log.clear()
    for p in ps:
        p.grad = None
    loss().backward()
    assert log[0] == "first" and log[-1] == ("ready", 3)


def test_unordered_counter_counts_open_slots_only_and_detaches():
    """Module counting: a slot counts only while open (from its backward gather), fires once when
    its last trainable parameter's gradient is in, and a detached counter hears nothing."""
    ext = _ext()
    ps, loss = _chain(4)
    fired = []
    c = ext.GradCounter([0, 0], 0, False, None, lambda slot: fired.append(slot))
    slot_of = [0, 0, 1, 1]
    for i, p in enumerate(ps):
        ext.attach(p, c, -1, slot_of[i])
    c.open(1, 2)  # module 1 (params 2, 3) open; module 0 never opened
    loss().backward()
    assert fired == [1]
    c.reset()
    c.open(0, 2)
    c.open(1, -1)  # nothing will count in: never fires (released at the end of backward)
    for p in ps:
        p.grad = None
    loss().backward()
    assert fired == [1, 0]
    for p in ps:
        ext.detach(p, c)
        p.grad = None
    c.reset()
    c.open(0, 2)
    c.open(1, 2)
    loss().backward()
    assert fired == [1, 0] and [ext.attached(p) for p in ps] == [0] * 4
    with pytest.raises(RuntimeError, match="out of range"):
        c.open(2, 1)


def test_counter_callbacks_hold_their_owner_weakly():
    """The counter lives on the parameters' hooks; its callbacks must not keep the reducer alive
    (zero_amd/_hooks.py): a WeakArgCall to a dropped owner is a no-op."""
    import gc
    import weakref

    from zero_amd._hooks import WeakArgCall

    ext = _ext()
    ps, loss = _chain(2)

    class Owner:
        def __init__(self):
            self.seen = []

        def ready(self, k):
            self.seen.append(k)

    o = Owner()
    c = ext.GradCounter([2], 2, True, None, WeakArgCall(o, "ready"))
    for i, p in enumerate(ps):
        ext.attach(p, c, i, 0)
    loss().backward()
    assert o.seen == [1]
    ref = weakref.ref(o)
    del o
    gc.collect()
    assert ref() is None
    c.reset()
    for p in ps:
        p.grad = None
    loss().backward()  # the owner is gone: nothing happens


# --- GatherFast / ReduceFast: a module gather and a gradient bucket in one call (round 6) -------
def test_gather_fast_validates_its_tables():
    ext = _ext()
    assert ext.GatherFast(1, 0, False, [1, 2], [3, 4], [0, 64], 128, 0, torch.float32, 0).size == 2
    with pytest.raises(RuntimeError, match="differ in length"):
        ext.GatherFast(1, 0, False, [1, 2], [3], [0, 64], 128, 0, torch.float32, 0)
    with pytest.raises(RuntimeError, match="total"):
        ext.GatherFast(1, 0, False, [1], [3], [0], 0, 0, torch.float32, 0)
    with pytest.raises(RuntimeError, match="NULL"):
        ext.GatherFast(0, 0, False, [1], [3], [0], 8, 0, torch.float32, 0)


def test_reduce_fast_declines_what_is_not_a_zero_copy_send():
    """launch() returns -1 and touches nothing (no library call: the function address here is
    bogus) unless every gradient is present, dense, of the bucket's dtype and exactly ws chunks
    long — the caller's general path then handles (or refuses) it."""
    ext = _ext()
    ws = 2
    ps = [torch.nn.Parameter(torch.zeros(4, 3)), torch.nn.Parameter(torch.zeros(6))]
    rf = ext.ReduceFast(12345, 0, True, ps, [0, 0], [6, 3], 0, torch.float32, ws)
    assert rf.launch(0, 0, 0, 0, 0, 0, False) == -1  # no gradients at all
    ps[0].grad = torch.ones(4, 3)
    assert rf.launch(0, 0, 0, 0, 0, 0, False) == -1  # one missing
    ps[1].grad = torch.ones(6)
    ps[0].grad = torch.ones(3, 4).t()  # not dense
    assert rf.launch(0, 0, 0, 0, 0, 0, False) == -1
    ps[0].grad = torch.ones(4, 3)
    uneven = ext.ReduceFast(12345, 0, True, ps, [0, 0], [6, 4], 0, torch.float32, ws)
    assert uneven.launch(0, 0, 0, 0, 0, 0, False) == -1  # 6 elements are not 2 chunks of 4
    bf = ext.ReduceFast(12345, 0, True, ps, [0, 0], [6, 3], 1, torch.bfloat16, ws)
    assert bf.launch(0, 0, 0, 0, 0, 0, False) == -1  # fp32 gradients, a bf16 bucket
    assert ps[0].grad is not None and ps[1].grad is not None  # nothing reset
    with pytest.raises(RuntimeError, match="differ in length"):
        ext.ReduceFast(12345, 0, True, ps, [0], [6, 3], 0, torch.float32, ws)
