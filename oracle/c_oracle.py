"""TEST INFRASTRUCTURE — ctypes wrapper of oracle/_build/libadam_oracle.so (adam_oracle.c).

Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "libadam_oracle.so"


class OracleHParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in (
        "one_minus_beta1", "beta2", "one_minus_beta2", "neg_step_size", "bc2_sqrt", "eps",
        "weight_decay", "decay_mul", "grad_div", "carry_mul")] + [
        ("amsgrad", ctypes.c_int32), ("maximize", ctypes.c_int32)]


_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = ctypes.CDLL(str(LIB))
        _lib.oracle_hparams_init.argtypes = [ctypes.c_double] * 5 + [ctypes.c_int] * 3 + [
            ctypes.c_int64, ctypes.c_double, ctypes.c_double, ctypes.POINTER(OracleHParams)]
        P = ctypes.c_void_p
        _lib.oracle_adam_f32.argtypes = [P, P, P, P, P, P, ctypes.c_int64, ctypes.POINTER(OracleHParams)]
        _lib.oracle_adam_bf16.argtypes = [P, P, P, P, P, P, P, ctypes.c_int64,
                                          ctypes.POINTER(OracleHParams)]
        _lib.oracle_adam_bf16_split.argtypes = [P, P, P, P, P, P, P, ctypes.c_int64,
                                                ctypes.POINTER(OracleHParams)]
        _lib.oracle_split_master.argtypes = [P, P, P, ctypes.c_int64]
        _lib.oracle_join_master.argtypes = [P, P, P, ctypes.c_int64]
        _lib.oracle_num_threads.restype = ctypes.c_int
    return _lib


def hparams(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1, *,
            decoupled=False, amsgrad=False, maximize=False, grad_div=1.0, carry_mul=0.0):
    hp = OracleHParams()
    lib().oracle_hparams_init(lr, beta1, beta2, eps, weight_decay, int(decoupled), int(amsgrad),
                              int(maximize), int(step), float(grad_div), float(carry_mul),
                              ctypes.byref(hp))
    return hp


def _p(a):
    return None if a is None else a.ctypes.data


def adam_f32(p, g, m, v, hp, vmax=None, carry=None):
    """In-place fp32 update of contiguous float32 numpy arrays."""
    for a in (p, g, m, v, vmax, carry):
        assert a is None or (a.dtype == np.float32 and a.flags.c_contiguous)
    lib().oracle_adam_f32(_p(p), _p(g), _p(m), _p(v), _p(vmax), _p(carry), p.size, ctypes.byref(hp))


def adam_bf16(master, p_bits, g_bits, m, v, hp, vmax=None, carry=None):
    """In-place update: bf16 grads (uint16 bits), fp32 master/m/v, bf16 params out (uint16)."""
    lib().oracle_adam_bf16(_p(master), _p(p_bits), _p(g_bits), _p(m), _p(v), _p(vmax), _p(carry),
                           master.size, ctypes.byref(hp))


def adam_bf16_split(hi, lo, g_bits, m, v, hp, vmax=None, carry=None):
    """In-place update with a split master: bf16 params ``hi`` (uint16) + int16 residuals ``lo``
    (uint16 bits), bf16 grads, fp32 m/v (include/zero_amd.h ZS_BF16_SPLIT)."""
    for a in (hi, lo, g_bits):
        assert a is None or (a.dtype == np.uint16 and a.flags.c_contiguous)
    lib().oracle_adam_bf16_split(_p(hi), _p(lo), _p(g_bits), _p(m), _p(v), _p(vmax), _p(carry),
                                 hi.size, ctypes.byref(hp))


def split_master(master):
    """fp32 master → (hi, lo) uint16 arrays of the split encoding."""
    master = np.ascontiguousarray(master, np.float32)
    hi, lo = np.zeros(master.size, np.uint16), np.zeros(master.size, np.uint16)
    lib().oracle_split_master(_p(master), _p(hi), _p(lo), master.size)
    return hi, lo


def join_master(hi, lo):
    hi, lo = np.ascontiguousarray(hi, np.uint16), np.ascontiguousarray(lo, np.uint16)
    out = np.zeros(hi.size, np.float32)
    lib().oracle_join_master(_p(hi), _p(lo), _p(out), hi.size)
    return out


def num_threads() -> int:
    return lib().oracle_num_threads()
