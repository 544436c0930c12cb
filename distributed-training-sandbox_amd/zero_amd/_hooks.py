"""Post-accumulate-grad hook callbacks that hold their owner weakly.

torch keeps a tensor's post-accumulate-grad hooks in a dict referenced from C++ (the autograd
meta), and the garbage collector does not traverse that edge: a hook whose closure reaches the
parameter again (hook -> optimizer -> its parameter list -> the parameter -> hook) is a cycle the
collector cannot see, so dropping the optimizer and the model would never free them — nor the
flat arenas and optimizer state they hold (tests/test_gpu_placement.py).  Every post-accumulate
hook of the package therefore calls its owner through ``WeakCall``: the owner (an engine, a
reducer, a hook state) is kept alive by whoever uses it, and the hook left on a parameter after
its owner is gone is a no-op.
"""
from __future__ import annotations

import functools
import weakref


class WeakCall:
    """``owner.<name>(*args)`` through a weak reference to ``owner``; the tensor the hook passes is
    dropped.  A no-op once the owner is gone."""

    __slots__ = ("_ref", "_name", "_args")

    def __init__(self, owner, name: str, *args):
        self._ref = weakref.ref(owner)
        self._name = name
        self._args = args

    def __call__(self, _tensor=None):
        owner = self._ref()
        if owner is not None:
            getattr(owner, self._name)(*self._args)

    def alive(self) -> bool:
        return self._ref() is not None


class WeakArgCall:
    """``owner.<name>(*args, *call_args)`` through a weak reference to ``owner`` — the callbacks of
    the C++ gradient counters (zero_amd/_hostext ``GradCounter``), which pass a bucket or module
    index.  A no-op once the owner is gone."""

    __slots__ = ("_ref", "_name", "_args")

    def __init__(self, owner, name: str, *args):
        self._ref = weakref.ref(owner)
        self._name = name
        self._args = args

    def __call__(self, *call_args):
        owner = self._ref()
        if owner is not None:
            getattr(owner, self._name)(*self._args, *call_args)


def _first_param_device(obj):
    """The device of the first parameter a wrapper (or its optimizer) manages, or None."""
    opt = obj if hasattr(obj, "param_groups") else getattr(obj, "optimizer", None)
    if opt is None:
        return None
    for g in opt.param_groups:
        for p in g["params"]:
            return p.device
    return None


def on_param_device(fn):
    """Run a wrapper's method with the parameters' GPU as the current device.  The library
    allocates its device tables (hipMalloc), creates its RCCL communicator (ncclCommInitRank) and
    its HIP events on the *current* device; a caller that keeps its parameters on cuda:k without
    ``torch.cuda.set_device(k)`` (the reference always sets it, zero1.py:206-207) would otherwise
    put them on cuda:0.  No device switch when it already is the current one."""
    import torch

    @functools.wraps(fn)
    def wrapped(self, *args, **kw):
        dev = getattr(self, "_param_device", None)
        if dev is None:
            src = (args[0] if args else kw.get("optimizer")) if fn.__name__ == "__init__" else self
            dev = _first_param_device(src) if src is not None else None
        if dev is None or dev.type != "cuda" or dev.index is None or \
                dev.index == torch.cuda.current_device():
            return fn(self, *args, **kw)
        with torch.cuda.device(dev):
            return fn(self, *args, **kw)
    return wrapped
