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
