"""Python handles for the gfx950 kernels behind the C ABI (csrc/zs_kernels.hip).

``CopySet``  — one launch of the descriptor-driven gather/scatter copy (pack / unpack).
``copy_direct`` — the same copy with the segments in the kernel arguments (no table to keep).
``AdamSet``  — one launch of the fused Adam/AdamW update over a list of segments.
``adam_step`` — the same update over one contiguous range (zs_adam_step_ex; no table to keep).

Both upload their segment table once; ``run(stream)`` only enqueues a kernel on ``stream``.
They raise ``ZeroAmdError`` on any failure; there is no CPU path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from ._lib import AdamHParams, AdamSeg

_PU64 = ctypes.POINTER(ctypes.c_uint64)
_PI64 = ctypes.POINTER(ctypes.c_int64)


def stream_handle(stream) -> int:
    """uintptr_t for a torch.cuda.Stream (or an int handle)."""
    return int(stream) if isinstance(stream, int) else int(stream.cuda_stream)


# Segment tables built from tensors are checked against those tensors' storage before anything is
# launched when this is on (``ZERO_AMD_CHECK_EXTENTS=1``; tests/conftest.py sets it): the raw-pointer
# entry points cannot check, and one segment past its buffer faults the device and fails every
# later call in the process (the r04 session that lost a whole suite to one bad table).
CHECK_EXTENTS = os.environ.get("ZERO_AMD_CHECK_EXTENTS", "0") not in ("", "0")


def check_extents_enabled() -> bool:
    return CHECK_EXTENTS


def check_extents(ptrs, nbytes, tensors, what: str = "segment") -> None:
    """Raise ``ValueError`` unless every segment [ptrs[i], ptrs[i] + nbytes[i]) with nbytes > 0 and
    ptrs != 0 (0 = zero fill) lies inside the storage of one of ``tensors`` (None entries ignored)."""
    ptrs = np.asarray(ptrs, dtype=np.uint64).reshape(-1)
    nb = np.asarray(nbytes, dtype=np.int64).reshape(-1)
    if ptrs.shape != nb.shape:
        raise ValueError(f"zero_amd: {what}: {ptrs.size} pointers for {nb.size} lengths")
    if (nb < 0).any():
        raise ValueError(f"zero_amd: {what}: negative length")
    live = (nb > 0) & (ptrs != 0)
    if not live.any():
        return
    spans = sorted({(int(t.untyped_storage().data_ptr()), int(t.untyped_storage().nbytes()))
                    for t in tensors if t is not None})
    if not spans:
        raise ValueError(f"zero_amd: {what}: no tensors to check the segments against")
    lo = np.array([s for s, _ in spans], np.uint64)
    hi = lo + np.array([n for _, n in spans], np.uint64)
    p, n = ptrs[live], nb[live].astype(np.uint64)
    k = np.searchsorted(lo, p, side="right") - 1
    ok = (k >= 0) & (p + n <= hi[np.maximum(k, 0)])
    if not ok.all():
        j = int(np.nonzero(~ok)[0][0])
        raise ValueError(f"zero_amd: {what} {int(np.nonzero(live)[0][j])}: [{int(p[j]):#x}, +{int(n[j])}) "
                         "is outside every buffer it may touch (the copy was not launched)")


def _check_bounds(src, dst, nb, bounds):
    if bounds is not None and CHECK_EXTENTS:
        src_t, dst_t = bounds
        check_extents(src, nb, src_t, "source segment")
        check_extents(dst, nb, dst_t, "destination segment")


class CopySet:
    """Copy ``nbytes[i]`` bytes from ``src[i]`` to ``dst[i]`` (src 0 = zero fill).  ``bounds``:
    (source tensors, destination tensors) the segments must lie in, checked when
    ``CHECK_EXTENTS`` is on."""

    def __init__(self, src, dst, nbytes, bounds=None):
        src = np.ascontiguousarray(np.asarray(src, dtype=np.uint64))
        dst = np.ascontiguousarray(np.asarray(dst, dtype=np.uint64))
        nb = np.ascontiguousarray(np.asarray(nbytes, dtype=np.int64))
        assert src.shape == dst.shape == nb.shape
        _check_bounds(src, dst, nb, bounds)
        self.nbytes = int(nb.sum()) if nb.size else 0
        self.nseg = int(nb.size)
        h = ctypes.c_void_p()
        _lib.call("zs_copyset_create", src.ctypes.data_as(_PU64), dst.ctypes.data_as(_PU64),
                  nb.ctypes.data_as(_PI64), int(nb.size), ctypes.byref(h))
        self._h = h

    def run(self, stream) -> None:
        _lib.call("zs_copyset_run", self._h, stream_handle(stream))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            try:
                _lib.lib.zs_copyset_destroy(h)
            except Exception:  # interpreter teardown
                pass
            self._h = None


def copy_direct(src, dst, nbytes, stream, bounds=None) -> None:
    """Copy ``nbytes[i]`` bytes from ``src[i]`` to ``dst[i]`` (src 0 = zero fill) with the segments
    in the kernel arguments (zs_copy_direct): nothing uploaded, so for pointers that change on
    every call (backward's fresh gradients).  ``bounds`` as for ``CopySet``."""
    src = np.ascontiguousarray(np.asarray(src, dtype=np.uint64))
    dst = np.ascontiguousarray(np.asarray(dst, dtype=np.uint64))
    nb = np.ascontiguousarray(np.asarray(nbytes, dtype=np.int64))
    assert src.shape == dst.shape == nb.shape
    _check_bounds(src, dst, nb, bounds)
    if nb.size:
        _lib.call("zs_copy_direct", int(nb.size), src.ctypes.data, dst.ctypes.data, nb.ctypes.data,
                  stream_handle(stream))


def adam_hparams(lr, beta1, beta2, eps, weight_decay, step, *, decoupled=False, amsgrad=False,
                 maximize=False, grad_div=1.0, carry_mul=0.0) -> AdamHParams:
    hp = AdamHParams()
    _lib.call("zs_adam_hparams_init", float(lr), float(beta1), float(beta2), float(eps),
              float(weight_decay), int(bool(decoupled)), int(bool(amsgrad)), int(bool(maximize)),
              int(step), float(grad_div), float(carry_mul), ctypes.byref(hp))
    return hp


class AdamSet:
    """Fused Adam over segments; ``segs`` is an (n, 9) int64/uint64 array in zs_adam_seg order:
    g, master, master_out, p_out, m, v, vmax, carry, n."""

    FIELDS = ("g", "master", "master_out", "p_out", "m", "v", "vmax", "carry", "n")

    def __init__(self, segs: np.ndarray, g_dtype: int, p_dtype: int = _lib.ZS_BF16):
        segs = np.ascontiguousarray(np.asarray(segs, dtype=np.uint64).reshape(-1, 9))
        arr = (AdamSeg * max(len(segs), 1))()
        ctypes.memmove(arr, segs.ctypes.data, segs.nbytes)
        h = ctypes.c_void_p()
        _lib.call("zs_adamset_create", arr, len(segs), int(g_dtype), int(p_dtype), ctypes.byref(h))
        self._h = h
        self.nseg = len(segs)
        self._g = np.ascontiguousarray(segs[:, 0])  # the gradients bound now, per input row
        self._stats()

    def _stats(self):
        e, b = ctypes.c_int64(), ctypes.c_int64()
        _lib.call("zs_adamset_stats", self._h, ctypes.byref(e), ctypes.byref(b))
        self.elems, self.bytes = e.value, b.value

    def set_grads(self, g: np.ndarray, stream) -> None:
        """Re-point row i's gradient to ``g[i]`` (0 = none) in stream order (zs_adamset_set_grads:
        a patch kernel on ``stream`` when any pointer changed, nothing otherwise)."""
        g = np.ascontiguousarray(np.asarray(g, dtype=np.uint64))
        assert g.shape == (self.nseg,)
        if np.array_equal(g, self._g):
            return
        _lib.call("zs_adamset_set_grads", self._h, self.nseg, g.ctypes.data, stream_handle(stream))
        self._g = g
        self._stats()

    def run(self, hp: AdamHParams, stream) -> None:
        _lib.call("zs_adamset_run", self._h, ctypes.byref(hp), stream_handle(stream))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            try:
                _lib.lib.zs_adamset_destroy(h)
            except Exception:  # interpreter teardown
                pass
            self._h = None


def adam_step(p, g, m, v, *, step, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
              decoupled=False, grad_div=1.0, p_bf16=None, carry=None, carry_mul=0.0,
              stream=None) -> None:
    """One Adam/AdamW step over the contiguous fp32 tensors ``p`` / ``m`` / ``v`` (in place) with
    gradient sum ``g`` (fp32 or bf16, or None = zero) divided by ``grad_div``; optional bf16 copy
    of the result into ``p_bf16`` and ZeRO-1 carry.  Enqueued on ``stream`` (default: torch's
    current stream on p's device)."""
    import torch

    n = p.numel()
    for name, t in (("p", p), ("m", m), ("v", v), ("carry", carry)):
        if t is not None:
            assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n, name
    if g is not None:
        assert g.dtype in (torch.float32, torch.bfloat16) and g.is_contiguous() and g.numel() == n
    if p_bf16 is not None:
        assert p_bf16.dtype == torch.bfloat16 and p_bf16.is_contiguous() and p_bf16.numel() == n
    g_dtype = _lib.ZS_BF16 if g is not None and g.dtype == torch.bfloat16 else _lib.ZS_F32
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    st = torch.cuda.current_stream(p.device) if stream is None else stream
    _lib.call("zs_adam_step_ex", ptr(p), ptr(p_bf16), ptr(g), g_dtype, ptr(m), ptr(v), n, float(lr),
              float(beta1), float(beta2), float(eps), float(weight_decay), int(bool(decoupled)),
              int(step), float(grad_div), ptr(carry), float(carry_mul), stream_handle(st))


def convert(src, dst, stream=None) -> None:
    """dst[:] = src converted fp32 -> bf16 (round to nearest even) or bf16 -> fp32 (zs_convert);
    contiguous tensors of equal element count, enqueued on ``stream``."""
    import torch

    from .comm import zs_dtype

    assert src.numel() == dst.numel() and src.is_contiguous() and dst.is_contiguous()
    st = torch.cuda.current_stream(src.device) if stream is None else stream
    _lib.call("zs_convert", src.data_ptr(), zs_dtype(src.dtype), dst.data_ptr(), zs_dtype(dst.dtype),
              src.numel(), stream_handle(st))
