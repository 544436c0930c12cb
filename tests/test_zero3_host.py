"""Host logic of the ZeRO-3 runtime that needs no GPU: the per-parameter post-accumulate-grad
dispatcher (zero3._add_post_accumulate_hook) — one autograd hook per parameter running every
registered callback in registration order, handles that remove one callback each, the autograd
hook gone with the last one, nothing kept alive by the dispatcher's table."""
import gc
import weakref

import torch


def _zero3():
    from zero_amd import zero3
    return zero3


def test_dispatch_order_and_removal():
    z3 = _zero3()
    p = torch.nn.Parameter(torch.ones(3))
    calls = []
    h1 = z3._add_post_accumulate_hook(p, lambda q: calls.append(("a", q is p)))
    h2 = z3._add_post_accumulate_hook(p, lambda q: calls.append(("b", q is p)))
    assert len(p._post_accumulate_grad_hooks) == 1  # one autograd hook for both callbacks
    (p * 2).sum().backward()
    assert calls == [("a", True), ("b", True)]
    h1.remove()
    h1.remove()  # idempotent
    calls.clear()
    p.grad = None
    (p * 2).sum().backward()
    assert calls == [("b", True)]
    h2.remove()
    assert not p._post_accumulate_grad_hooks and p not in z3._post_acc
    calls.clear()
    p.grad = None
    (p * 2).sum().backward()
    assert calls == []


def test_callback_may_remove_itself_during_dispatch():
    z3 = _zero3()
    p = torch.nn.Parameter(torch.ones(2))
    calls = []
    handles = []
    handles.append(z3._add_post_accumulate_hook(p, lambda q: (calls.append(1), handles[0].remove())))
    z3._add_post_accumulate_hook(p, lambda q: calls.append(2))
    (p * 1).sum().backward()
    assert calls == [1, 2]  # the second still runs in the backward that removed the first
    calls.clear()
    p.grad = None
    (p * 1).sum().backward()
    assert calls == [2]


def test_table_keeps_nothing_alive():
    z3 = _zero3()

    class Owner:
        pass

    o = Owner()
    o.p = torch.nn.Parameter(torch.ones(2))
    h = z3._add_post_accumulate_hook(o.p, lambda q: None)
    ref = weakref.ref(o)
    h.remove()  # with the hook gone, only the table's weak entry could still reach the owner
    del o, h
    gc.collect()
    assert ref() is None


# --- register_zero3_hooks' tensor-style backward bookkeeping on the CPU (fake managers) ---------
class _FakeRuntime:
    def __init__(self, log):
        self.log, self.iteration_callbacks = log, []

    def materialize(self, key, ms):
        self.log.append(("gather", key[0], ms[0].name))
        for m in ms:
            m.full_data = True

    def end_iteration(self):
        for fn in self.iteration_callbacks:
            fn()

    def mark_inputs_changed(self):  # (register_zero3_hooks: nothing gathered before is reused)
        self.log.append(("inputs changed",))


class _FakeManager:
    """What register_zero3_hooks reads of a Zero3ParamManager (update mode: keep_full_grad)."""

    def __init__(self, param, name, rt, log):
        self.param, self.name, self.runtime, self.log = param, name, rt, log
        self.keep_full_grad, self.world_size, self.fp8, self.full_data = True, 2, False, None

    def release(self):
        self.log.append(("release", self.name))
        self.full_data = None
        self.grad_at_release = self.param.grad is not None


_MGRS = {}


def _managers_of(model):
    return _MGRS[id(model)]


def _hooked_mlp():
    z3 = _zero3()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(4, 4, bias=False), torch.nn.Linear(4, 4, bias=False))
    log = []
    rt = _FakeRuntime(log)
    names = {model[0].weight: "w0", model[1].weight: "w1"}
    mgrs = {p: _FakeManager(p, n, rt, log) for p, n in names.items()}
    z3.register_zero3_hooks(model, mgrs, backward_hooks="tensor")
    _MGRS[id(model)] = list(mgrs.values())
    return model, rt, log


def test_tensor_hooks_backward_that_raises_is_cleaned_up():
    """a backward that raises before its end-of-backward callback must not leave the
    callback flag set — later backwards would never queue it, so a module none of whose
    parameters counts in (here: module 1, frozen) would stay gathered after every backward."""
    z3 = _zero3()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(4, 4, bias=False), torch.nn.Linear(4, 4, bias=False))
    model[1].weight.requires_grad_(False)
    log = []
    rt = _FakeRuntime(log)
    mgrs = {model[0].weight: _FakeManager(model[0].weight, "w0", rt, log),
            model[1].weight: _FakeManager(model[1].weight, "w1", rt, log)}
    z3.register_zero3_hooks(model, mgrs, backward_hooks="tensor")
    x = torch.randn(2, 4, requires_grad=True)
    h = model(x)
    h.register_hook(lambda g: (_ for _ in ()).throw(RuntimeError("boom")))  # raises in backward
    import pytest

    with pytest.raises(RuntimeError, match="boom"):
        (h * 1).sum().backward()
    for _ in range(2):  # later iterations: every module released by the end of each backward
        model[0].weight.grad = None
        model(x).sum().backward()
        assert mgrs[model[1].weight].full_data is None, "module 1 left gathered after backward"
        assert mgrs[model[0].weight].full_data is None
        rt.end_iteration()


def test_tensor_hooks_follow_requires_grad_changes():
    """the per-module count of gradients to wait for is re-derived when requires_grad
    changes after registration.  Module 1 (weight + bias): with its bias frozen after
    registration it must be released by its weight's gradient — before module 0's backward — not
    held gathered until the end of backward; unfrozen again, it must not be released before the
    bias gradient is accumulated."""
    z3 = _zero3()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
    log = []
    rt = _FakeRuntime(log)
    names = {model[0].weight: "w0", model[0].bias: "b0", model[1].weight: "w1", model[1].bias: "b1"}
    mgrs = {p: _FakeManager(p, n, rt, log) for p, n in names.items()}
    z3.register_zero3_hooks(model, mgrs, backward_hooks="tensor")
    x = torch.randn(2, 4, requires_grad=True)
    model(x).sum().backward()
    log.clear()
    model[1].bias.requires_grad_(False)  # frozen after registration
    for p in model.parameters():
        p.grad = None
    model(x).sum().backward()
    bwd = log[[i for i, e in enumerate(log) if e[:2] == ("gather", "bwd")][0]:]
    rel = [e[1] for e in bwd if e[0] == "release"]
    assert rel.index("w1") < rel.index("w0"), bwd  # module 1 released by w1's gradient
    assert [e for e in bwd if e[0] == "gather"][1][2] == "w0"
    i_gather0 = bwd.index(("gather", "bwd", "w0"))
    assert ("release", "w1") in bwd[:i_gather0], bwd  # ... before module 0 was even gathered
    log.clear()
    model[1].bias.requires_grad_(True)  # unfrozen: counted in again
    for p in model.parameters():
        p.grad = None
    model(x).sum().backward()
    assert mgrs[model[1].bias].grad_at_release and mgrs[model[1].weight].grad_at_release, log
    assert model[1].bias.grad is not None


def test_comm_time_waits_for_both_events():
    """an asynchronous step adds a span only when BOTH of its events have completed
    (elapsed_time on an incomplete compute-stream event raises)."""
    z3 = _zero3()

    class Ev:
        def __init__(self, done):
            self.done = done

        def query(self):
            return self.done

        def elapsed_time(self, other):
            assert self.done and other.done, "elapsed_time on an incomplete event"
            return 2.0

    opt = z3.ShardedOptimizer.__new__(z3.ShardedOptimizer)
    opt.communication_time = 0.0
    opt._comm_spans = [(Ev(False), Ev(True)), (Ev(True), Ev(True))]
    opt._collect_comm_time(completed_only=True)
    assert len(opt._comm_spans) == 1 and opt.communication_time == 2.0 / 1e3


def test_weak_post_accumulate_callbacks_do_not_leak():
    """torch does not let the garbage collector traverse a tensor's post-accumulate-grad hooks,
    so a hook closure that reaches its parameter again is an uncollectable cycle; the package's
    post-accumulate hooks call their owners through zero_amd._hooks.WeakCall instead."""
    from zero_amd._hooks import WeakCall

    class Owner:
        def __init__(self):
            self.p = torch.nn.Parameter(torch.zeros(3))
            self.calls = []
            self.p.register_post_accumulate_grad_hook(WeakCall(self, "hit", 7))

        def hit(self, i):
            self.calls.append(i)

    o = Owner()
    (o.p * 2).sum().backward()
    assert o.calls == [7]
    ref = weakref.ref(o)
    del o
    gc.collect()
    assert ref() is None  # (a plain `lambda _p: self.hit(7)` keeps it alive forever)


def test_tensor_hooks_release_their_managers():
    """register_zero3_hooks' tensor-style bookkeeping: once the model and the managers are dropped,
    nothing the parameters' hooks hold keeps the managers alive."""
    z3 = _zero3()
    model = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
    log = []
    rt = _FakeRuntime(log)
    mgrs = {p: _FakeManager(p, str(i), rt, log) for i, p in enumerate(model.parameters())}
    z3.register_zero3_hooks(model, mgrs, backward_hooks="tensor")
    model(torch.randn(2, 4)).sum().backward()
    ref = weakref.ref(next(iter(mgrs.values())))
    params = list(model.parameters())  # the parameters outlive the model, as a user's may
    del model, mgrs, rt
    gc.collect()
    assert ref() is None
    del params


def test_on_param_device_switches_to_the_parameters_gpu(monkeypatch):
    """The optimizers' entry points run with the parameters' GPU current (the library's tables,
    RCCL communicator and events are created on the current device): a wrapper whose parameters
    sit on cuda:3 while cuda:0 is current enters torch.cuda.device(cuda:3); no switch when it is
    already current, none for CPU tensors."""
    import contextlib

    from zero_amd._hooks import on_param_device

    entered = []

    @contextlib.contextmanager
    def fake_device(dev):
        entered.append(dev)
        yield

    cur = [0]
    monkeypatch.setattr(torch.cuda, "current_device", lambda: cur[0])
    monkeypatch.setattr(torch.cuda, "device", fake_device)

    class Opt:
        @on_param_device
        def __init__(self, optimizer):
            self.optimizer = optimizer

        @on_param_device
        def step(self):
            return "stepped"

    class FakeParam:
        device = torch.device("cuda", 3)

    inner = type("Inner", (), {"param_groups": [{"params": [FakeParam()]}]})()
    o = Opt(inner)
    assert entered == [torch.device("cuda", 3)]
    o._param_device = torch.device("cuda", 3)
    assert o.step() == "stepped" and len(entered) == 2
    cur[0] = 3
    assert o.step() == "stepped" and len(entered) == 2  # already current: no switch
    o._param_device = torch.device("cpu")
    assert o.step() == "stepped" and len(entered) == 2
