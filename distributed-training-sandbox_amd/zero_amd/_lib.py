"""ctypes binding of ``libzero_amd.so`` (the C ABI declared in ``include/zero_amd.h``).

``torch`` is imported first so the library's ``libamdhip64.so.7`` / ``librccl.so.1`` NEEDED entries
resolve (by SONAME) to the copies torch already loaded: one HIP runtime and one RCCL per process.
There is no fallback: if the library is missing or fails to load, importing this module raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)
from torch.profiler import record_function

LIB_PATH = Path(os.environ.get("ZERO_AMD_LIB", Path(__file__).resolve().parent / "libzero_amd.so"))

ZS_OK, ZS_ERR_INVALID, ZS_ERR_HIP, ZS_ERR_RCCL, ZS_ERR_NOMEM = 0, 1, 2, 3, 4
ZS_F32, ZS_BF16, ZS_U8, ZS_BF16_SPLIT = 0, 1, 2, 3
ZS_LAYOUT_R, ZS_LAYOUT_Z, ZS_LAYOUT_F = 0, 1, 2
ZS_BUCKETS_RAGGED, ZS_BUCKETS_PADDED = 0, 1
ZS_SYNC_EVENT, ZS_SYNC_FLAG = 0, 1
ABI_VERSION = 13
ZS_UNIQUE_ID_BYTES = 128

# Every symbol include/zero_amd.h declares (tests check the library exports all of them).
EXPORTED = (
    "zs_abi_version", "zs_last_error", "zs_range_push", "zs_range_pop",
    "zs_plan_create", "zs_plan_create_ex", "zs_plan_destroy", "zs_plan_info", "zs_plan_owner_range", "zs_plan_owner_of",
    "zs_plan_stream_len", "zs_plan_num_pieces", "zs_plan_pieces", "zs_plan_bucket",
    "zs_plan_num_segments", "zs_plan_segments", "zs_plan_num_buckets", "zs_plan_bucket_bytes",
    "zs_pack", "zs_unpack",
    "zs_copyset_create", "zs_copyset_run", "zs_copyset_destroy", "zs_copy_direct", "zs_scale",
    "zs_convert", "zs_fp8_quantize_rows", "zs_fp8_dequantize_rows", "zs_fp8_quantize_rowset",
    "zs_fp8_dequantize_gathered",
    "zs_adam_hparams_init", "zs_adamset_create", "zs_adamset_run", "zs_adamset_set_grads", "zs_adamset_destroy",
    "zs_adamset_stats", "zs_adam_step", "zs_adam_step_ex",
    "zs_comm_unique_id", "zs_comm_init", "zs_comm_destroy", "zs_reduce_scatter", "zs_all_gather",
    "zs_all_reduce", "zs_reduce", "zs_broadcast", "zs_reduce_group", "zs_broadcast_group", "zs_all_gather_group", "zs_reduce_scatter_group",
    "zs_all_gather_group_ordered", "zs_reduce_scatter_group_ordered", "zs_stream_wait_event",
    "zs_sync_create", "zs_sync_destroy", "zs_sync_record", "zs_sync_wait", "zs_sync_set_epoch", "zs_sync_query",
    "zs_all_gather_group_synced", "zs_reduce_scatter_group_synced",
    "zs_group_start", "zs_group_end", "zs_rccl_version",
    "zs_device_alloc", "zs_device_alloc_chunked", "zs_device_free", "zs_tune",
)


class ZeroAmdError(RuntimeError):
    """A zs_* call returned a non-zero status."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed with status {code}: {msg}")
        self.code = code


class AdamSeg(ctypes.Structure):
    _fields_ = [("g", ctypes.c_uint64), ("master", ctypes.c_uint64),
                ("master_out", ctypes.c_uint64), ("p_out", ctypes.c_uint64),
                ("m", ctypes.c_uint64), ("v", ctypes.c_uint64), ("vmax", ctypes.c_uint64),
                ("carry", ctypes.c_uint64), ("n", ctypes.c_int64)]


class AdamHParams(ctypes.Structure):
    _fields_ = [("one_minus_beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("one_minus_beta2", ctypes.c_float), ("neg_step_size", ctypes.c_float),
                ("bc2_sqrt", ctypes.c_float), ("eps", ctypes.c_float),
                ("weight_decay", ctypes.c_float), ("decay_mul", ctypes.c_float),
                ("grad_div", ctypes.c_float), ("carry_mul", ctypes.c_float),
                ("amsgrad", ctypes.c_int32), ("maximize", ctypes.c_int32)]


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_PI64 = ctypes.POINTER(ctypes.c_int64)
_PU64 = ctypes.POINTER(ctypes.c_uint64)
_U = ctypes.c_uint64  # uintptr_t stream

_SIGS = {
    "zs_abi_version": ([], ctypes.c_int),
    "zs_last_error": ([], ctypes.c_char_p),
    "zs_range_push": ([ctypes.c_char_p], ctypes.c_int),
    "zs_range_pop": ([], ctypes.c_int),
    "zs_plan_create": ([_I64, _PI64, _PI64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I64,
                        ctypes.POINTER(_P)], ctypes.c_int),
    "zs_plan_create_ex": ([_I64, _PI64, _PI64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I64, _I64,
                           ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "zs_plan_destroy": ([_P], ctypes.c_int),
    "zs_plan_info": ([_P, _PI64], ctypes.c_int),
    "zs_plan_owner_range": ([_P, ctypes.c_int, _PI64, _PI64], ctypes.c_int),
    "zs_plan_owner_of": ([_P, _I64, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "zs_plan_stream_len": ([_P, ctypes.c_int, _PI64], ctypes.c_int),
    "zs_plan_num_pieces": ([_P, ctypes.c_int, _PI64], ctypes.c_int),
    "zs_plan_pieces": ([_P, ctypes.c_int, _PI64, _PI64, _PI64, _PI64], ctypes.c_int),
    "zs_plan_bucket": ([_P, _I64, _PI64, _PI64, ctypes.POINTER(ctypes.c_int), _PI64, _PI64, _PI64],
                       ctypes.c_int),
    "zs_plan_num_segments": ([_P, _I64, _PI64], ctypes.c_int),
    "zs_plan_segments": ([_P, _I64, _PI64, _PI64, _PI64, _PI64, _PI64], ctypes.c_int),
    "zs_plan_num_buckets": ([_P, _PI64], ctypes.c_int),
    "zs_plan_bucket_bytes": ([_P, _I64, ctypes.c_int, _PI64], ctypes.c_int),
    "zs_pack": ([_P, _I64, _PU64, _P, ctypes.c_int, _U], ctypes.c_int),
    "zs_unpack": ([_P, _I64, _P, _PU64, ctypes.c_int, _U], ctypes.c_int),
    "zs_copyset_create": ([_PU64, _PU64, _PI64, _I64, ctypes.POINTER(_P)], ctypes.c_int),
    "zs_copyset_run": ([_P, _U], ctypes.c_int),
    "zs_copy_direct": ([_I64, _P, _P, _P, _U], ctypes.c_int),
    "zs_copyset_destroy": ([_P], ctypes.c_int),
    "zs_scale": ([_P, _I64, ctypes.c_int, ctypes.c_double, _U], ctypes.c_int),
    "zs_convert": ([_P, ctypes.c_int, _P, ctypes.c_int, _I64, _U], ctypes.c_int),
    "zs_fp8_quantize_rows": ([_P, ctypes.c_int, _P, _P, _I64, _I64, _U], ctypes.c_int),
    "zs_fp8_dequantize_rows": ([_P, _P, _P, ctypes.c_int, _I64, _I64, _U], ctypes.c_int),
    "zs_fp8_quantize_rowset": ([_I64, _P, _P, _P, _P, _P, _P, ctypes.c_int, _U], ctypes.c_int),
    "zs_fp8_dequantize_gathered": ([_I64, _P, _P, ctypes.c_int, _I64, _I64, _P, _P, _P, _P, _P,
                                    ctypes.c_int, _U], ctypes.c_int),
    "zs_adam_hparams_init": ([ctypes.c_double] * 5 + [ctypes.c_int] * 3 +
                             [_I64, ctypes.c_double, ctypes.c_double, ctypes.POINTER(AdamHParams)],
                             ctypes.c_int),
    "zs_adamset_create": ([ctypes.POINTER(AdamSeg), _I64, ctypes.c_int, ctypes.c_int,
                           ctypes.POINTER(_P)], ctypes.c_int),
    "zs_adamset_run": ([_P, ctypes.POINTER(AdamHParams), _U], ctypes.c_int),
    "zs_adamset_set_grads": ([_P, _I64, _P, _U], ctypes.c_int),
    "zs_adamset_destroy": ([_P], ctypes.c_int),
    "zs_adamset_stats": ([_P, _PI64, _PI64], ctypes.c_int),
    "zs_adam_step": ([_P, _P, _P, ctypes.c_int, _P, _P, _I64] + [ctypes.c_float] * 5 +
                     [ctypes.c_int, _I64, ctypes.c_float, _P, ctypes.c_float, _U], ctypes.c_int),
    "zs_adam_step_ex": ([_P, _P, _P, ctypes.c_int, _P, _P, _I64] + [ctypes.c_double] * 5 +
                        [ctypes.c_int, _I64, ctypes.c_double, _P, ctypes.c_double, _U], ctypes.c_int),
    "zs_comm_unique_id": ([_P], ctypes.c_int),
    "zs_comm_init": ([_P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "zs_comm_destroy": ([_P], ctypes.c_int),
    "zs_reduce_scatter": ([_P, _P, _P, _I64, ctypes.c_int, _U], ctypes.c_int),
    "zs_all_gather": ([_P, _P, _P, _I64, ctypes.c_int, _U], ctypes.c_int),
    "zs_all_reduce": ([_P, _P, _P, _I64, ctypes.c_int, _U], ctypes.c_int),
    "zs_reduce": ([_P, _P, _P, _I64, ctypes.c_int, ctypes.c_int, _U], ctypes.c_int),
    "zs_broadcast": ([_P, _P, _P, _I64, ctypes.c_int, ctypes.c_int, _U], ctypes.c_int),
    "zs_reduce_group": ([_P, _I64, _PU64, _PU64, _PI64, ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                         _U], ctypes.c_int),
    "zs_broadcast_group": ([_P, _I64, _PU64, _PI64, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, _U],
                           ctypes.c_int),
    "zs_all_gather_group": ([_P, _I64, _PU64, _PU64, _PI64, ctypes.c_int, _U], ctypes.c_int),
    "zs_reduce_scatter_group": ([_P, _I64, _PU64, _PU64, _PI64, ctypes.c_int, _U], ctypes.c_int),
    "zs_all_gather_group_ordered": ([_P, _I64, _PU64, _PU64, _PI64, ctypes.c_int, _U, ctypes.c_uint64,
                                     _U, ctypes.c_uint64], ctypes.c_int),
    "zs_reduce_scatter_group_ordered": ([_P, _I64, _PU64, _PU64, _PI64, ctypes.c_int, _U,
                                         ctypes.c_uint64, _U, ctypes.c_uint64], ctypes.c_int),
    "zs_stream_wait_event": ([_U, ctypes.c_uint64], ctypes.c_int),
    "zs_sync_create": ([ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "zs_sync_destroy": ([_P], ctypes.c_int),
    "zs_sync_record": ([_P, _U], ctypes.c_int),
    "zs_sync_wait": ([_P, _U], ctypes.c_int),
    "zs_sync_set_epoch": ([_P, ctypes.c_uint64], ctypes.c_int),
    "zs_sync_query": ([_P, _PU64, _PU64], ctypes.c_int),
    "zs_all_gather_group_synced": ([_P, _I64, _PU64, _PU64, _PI64, ctypes.c_int, _U, _P, _U, _P],
                                   ctypes.c_int),
    "zs_reduce_scatter_group_synced": ([_P, _I64, _PU64, _PU64, _PI64, ctypes.c_int, _U, _P, _U, _P],
                                       ctypes.c_int),
    "zs_group_start": ([], ctypes.c_int),
    "zs_group_end": ([], ctypes.c_int),
    "zs_rccl_version": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "zs_device_alloc": ([_I64, ctypes.POINTER(_P)], ctypes.c_int),
    "zs_device_free": ([_P], ctypes.c_int),
    "zs_device_alloc_chunked": ([_I64, _I64, ctypes.POINTER(_P)], ctypes.c_int),
    "zs_tune": ([ctypes.c_char_p, _I64, _PI64], ctypes.c_int),
}


def _load():
    if not LIB_PATH.exists():
        raise ImportError(
            f"zero_amd: native library {LIB_PATH} not found; build it with "
            f"`make -C distributed-training-sandbox_amd` (or __graft_entry__.build())")
    lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.zs_abi_version() != ABI_VERSION:
        raise ImportError(f"zero_amd: ABI version {lib.zs_abi_version()} != {ABI_VERSION} in "
                          f"{LIB_PATH} (rebuild: make -C distributed-training-sandbox_amd)")
    return lib


lib = _load()


def check(rc: int, fn: str = "zs_*") -> None:
    if rc != ZS_OK:
        raise ZeroAmdError(fn, rc, lib.zs_last_error().decode(errors="replace"))


def call(name: str, *args) -> None:
    check(getattr(lib, name)(*args), name)


@contextlib.contextmanager
def phase_range(name: str):
    """A phase of step(): a torch.profiler range (the reference's record_function names,
    zero1.py:80-91) and a roctx range of the same name for rocprofv3 --marker-trace."""
    check(lib.zs_range_push(name.encode()), "zs_range_push")
    try:
        with record_function(name):
            yield
    finally:
        check(lib.zs_range_pop(), "zs_range_pop")


def i64_array(values):
    arr = (ctypes.c_int64 * len(values))(*values)
    return arr
