"""Python view of the native layout planner (``zs_plan_*``, csrc/zs_plan.cpp).

The planner restates the reference's ownership rule (zero1.py:55-62 for the index ranges,
zero1.py:95-100 for the broadcast owner) and derives, per rank, the *stream* of pieces whose
optimizer state that rank owns, and per bucket the segments that pack / unpack move.  It is pure
host code, so it is exercised by the CPU test-suite against the reference's ownership fixtures.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import ZS_BUCKETS_PADDED, ZS_BUCKETS_RAGGED, ZS_LAYOUT_F, ZS_LAYOUT_R, ZS_LAYOUT_Z

LAYOUTS = {"reference": ZS_LAYOUT_R, "R": ZS_LAYOUT_R, "chunk": ZS_LAYOUT_Z, "Z": ZS_LAYOUT_Z,
           "flat": ZS_LAYOUT_F, "F": ZS_LAYOUT_F}
BUCKET_MODES = {"ragged": ZS_BUCKETS_RAGGED, "padded": ZS_BUCKETS_PADDED}


def _i64p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


@dataclass(frozen=True)
class Pieces:
    param: np.ndarray       # parameter index
    param_off: np.ndarray   # element offset inside the flattened parameter
    stream_off: np.ndarray  # element offset inside the rank's optimizer-shard stream
    length: np.ndarray


@dataclass(frozen=True)
class Segments:
    param: np.ndarray
    rank: np.ndarray
    param_off: np.ndarray
    buf_off: np.ndarray     # element offset inside the bucket buffer (rank-major windows)
    length: np.ndarray


@dataclass(frozen=True)
class Bucket:
    arena_off: int          # element offset of the bucket inside the arena
    elems: int              # bucket buffer length (elements)
    even: bool              # equal windows at r*len → reduce-scatter / all-gather
    win_off: np.ndarray     # per rank: window offset inside the bucket
    win_len: np.ndarray     # per rank: window length (0 = nothing)
    win_stream: np.ndarray  # per rank: stream offset of the window's first element


class Plan:
    """Ownership + bucket layout for ``n`` parameters over ``ws`` ranks (seen from ``rank``)."""

    def __init__(self, numels, ws: int, rank: int, layout="reference", dim0=None,
                 align_elems: int = 64, window_elems: int = 0, buckets: str = "ragged"):
        self.layout = LAYOUTS[layout] if isinstance(layout, str) else int(layout)
        numels = np.ascontiguousarray(np.asarray(numels, dtype=np.int64))
        self.numels = numels
        d0 = None
        if dim0 is not None:
            d0 = np.ascontiguousarray(np.asarray(dim0, dtype=np.int64))
            assert d0.shape == numels.shape
        h = ctypes.c_void_p()
        _lib.call("zs_plan_create_ex", len(numels), _i64p(numels) if len(numels) else None,
                  _i64p(d0) if d0 is not None else None, int(ws), int(rank), self.layout,
                  int(align_elems), int(window_elems), BUCKET_MODES[buckets], ctypes.byref(h))
        self._h = h
        info = np.zeros(10, np.int64)
        _lib.call("zs_plan_info", self._h, _i64p(info))
        (self.n, self.ws, self.rank, _, self.window, self.num_buckets, self.max_stream_len,
         self.arena_elems, self.num_even, _) = (int(x) for x in info)
        self.bucket_mode = buckets

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None:
            try:
                _lib.lib.zs_plan_destroy(h)
            except Exception:  # interpreter teardown
                pass
            self._h = None

    # --- ownership (reference formulas) -----------------------------------------------------
    def owner_range(self, rank: int | None = None) -> tuple[int, int]:
        s, e = ctypes.c_int64(), ctypes.c_int64()
        _lib.call("zs_plan_owner_range", self._h, self.rank if rank is None else rank,
                  ctypes.byref(s), ctypes.byref(e))
        return s.value, e.value

    def owner_of(self, i: int) -> int:
        o = ctypes.c_int()
        _lib.call("zs_plan_owner_of", self._h, int(i), ctypes.byref(o))
        return o.value

    # --- streams / buckets ------------------------------------------------------------------
    def stream_len(self, rank: int | None = None) -> int:
        n = ctypes.c_int64()
        _lib.call("zs_plan_stream_len", self._h, self.rank if rank is None else rank, ctypes.byref(n))
        return n.value

    def pieces(self, rank: int | None = None) -> Pieces:
        r = self.rank if rank is None else rank
        n = ctypes.c_int64()
        _lib.call("zs_plan_num_pieces", self._h, r, ctypes.byref(n))
        arrs = [np.zeros(n.value, np.int64) for _ in range(4)]
        if n.value:
            _lib.call("zs_plan_pieces", self._h, r, *(_i64p(a) for a in arrs))
        return Pieces(*arrs)

    def segments(self, bucket: int) -> Segments:
        n = ctypes.c_int64()
        _lib.call("zs_plan_num_segments", self._h, int(bucket), ctypes.byref(n))
        arrs = [np.zeros(n.value, np.int64) for _ in range(5)]
        if n.value:
            _lib.call("zs_plan_segments", self._h, int(bucket), *(_i64p(a) for a in arrs))
        return Segments(*arrs)

    def bucket(self, k: int) -> Bucket:
        ao, el, ev = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
        arrs = [np.zeros(self.ws, np.int64) for _ in range(3)]
        _lib.call("zs_plan_bucket", self._h, int(k), ctypes.byref(ao), ctypes.byref(el),
                  ctypes.byref(ev), *(_i64p(a) for a in arrs))
        return Bucket(ao.value, el.value, bool(ev.value), *arrs)

    # --- bucket copies straight from the plan (zs_pack / zs_unpack) -------------------------
    def bucket_bytes(self, k: int, dtype: int) -> int:
        b = ctypes.c_int64()
        _lib.call("zs_plan_bucket_bytes", self._h, int(k), int(dtype), ctypes.byref(b))
        return b.value

    def pack(self, k: int, grad_ptrs, bucket_ptr: int, dtype: int, stream: int) -> None:
        """Copy every segment of bucket ``k`` from the per-parameter grads (device pointers
        indexed by parameter; 0 = zeros) into the bucket buffer at ``bucket_ptr``."""
        ptrs = np.ascontiguousarray(np.asarray(grad_ptrs, dtype=np.uint64))
        assert ptrs.shape == (self.n,)
        _lib.call("zs_pack", self._h, int(k), ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                  int(bucket_ptr), int(dtype), int(stream))

    def unpack(self, k: int, bucket_ptr: int, param_ptrs, dtype: int, stream: int) -> None:
        """Scatter every segment of bucket ``k`` back into the parameters."""
        ptrs = np.ascontiguousarray(np.asarray(param_ptrs, dtype=np.uint64))
        assert ptrs.shape == (self.n,)
        _lib.call("zs_unpack", self._h, int(k), int(bucket_ptr),
                  ptrs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), int(dtype), int(stream))
