"""The C-ABI library loads and exports exactly what include/zero_amd.h declares (no GPU needed)."""
import ctypes
import math
import re

import numpy as np

import pytest

from conftest import REPO


def _declared():
    text = (REPO / "include" / "zero_amd.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(zs_\w+)\s*\(", text, re.M)))


def test_header_and_library_agree():
    from zero_amd import _lib

    declared = _declared()
    assert declared, "no declarations parsed"
    assert sorted(_lib.EXPORTED) == declared
    raw = ctypes.CDLL(str(_lib.LIB_PATH))
    for name in declared:
        assert hasattr(raw, name), name


def test_library_is_gfx950_code_object():
    from zero_amd import _lib

    data = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in data
    assert b"adam_segments_kernel" in data and b"copy_segments_kernel" in data


def test_abi_version_and_error_text():
    from zero_amd import _lib

    assert _lib.lib.zs_abi_version() == _lib.ABI_VERSION == 13
    h = ctypes.c_void_p()
    rc = _lib.lib.zs_plan_create_ex(0, None, None, 0, 0, 0, 64, 0, 0, ctypes.byref(h))
    assert rc == _lib.ZS_ERR_INVALID
    assert b"ws must be >= 1" in _lib.lib.zs_last_error()


def test_hparams_match_torch_scalars():
    """zs_adam_hparams_init derives the scalars as adam.py:508-537 does (python doubles)."""
    import numpy as np
    from zero_amd.kernels import adam_hparams

    for step, (b1, b2) in [(s, (0.9, 0.999)) for s in (1, 2, 10, 1000, 10**5, 10**7)] + \
            [(s, (0.8, 0.95)) for s in (1, 3, 77, 5000)]:
        lr, eps = 1e-3, 1e-8
        hp = adam_hparams(lr, b1, b2, eps, 0.0, step, grad_div=4.0, carry_mul=3.0)
        # torch keeps `step` in a float32 tensor (adam.py:160-185) and reads it back as a Python
        # float; exact for every step below 2**24, which the int64 step here matches
        assert float(np.float32(step)) == step
        assert hp.neg_step_size == np.float32(-(lr / (1 - b1 ** step)))
        assert hp.bc2_sqrt == np.float32((1 - b2 ** step) ** 0.5)
        assert hp.one_minus_beta1 == np.float32(1 - b1)
        assert hp.one_minus_beta2 == np.float32(1 - b2)
        assert hp.grad_div == 4.0 and hp.carry_mul == 3.0 and hp.decay_mul == 1.0
    hp = adam_hparams(1e-3, 0.9, 0.999, 1e-8, 1e-2, 1, decoupled=True)
    assert hp.weight_decay == 0.0 and hp.decay_mul == np.float32(1 - 1e-3 * 1e-2)
    hp = adam_hparams(1e-3, 0.9, 0.999, 1e-8, 1e-2, 1)
    assert math.isclose(hp.weight_decay, 1e-2, rel_tol=1e-7) and hp.decay_mul == 1.0


def test_invalid_step_rejected():
    from zero_amd._lib import ZeroAmdError
    from zero_amd.kernels import adam_hparams

    with pytest.raises(ZeroAmdError):
        adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, 0)


def test_new_entry_points_validate_arguments():
    """ABI v2 entry points reject bad arguments with ZS_ERR_INVALID and a message, without a GPU."""
    from zero_amd import _lib

    lib = _lib.lib
    h = ctypes.c_void_p()
    numels = (ctypes.c_int64 * 2)(4, 4)
    assert lib.zs_plan_create_ex(2, numels, None, 2, 0, 0, 64, 0, 7, ctypes.byref(h)) == _lib.ZS_ERR_INVALID
    assert b"bucket_mode" in lib.zs_last_error()
    assert lib.zs_scale(None, 16, 9, 2.0, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_scale(None, 16, _lib.ZS_F32, 0.0, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_scale(None, 0, _lib.ZS_F32, 2.0, 0) == _lib.ZS_OK  # empty: nothing to launch
    assert lib.zs_fp8_quantize_rows(None, 9, None, None, 1, 8, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_fp8_dequantize_rows(None, None, None, _lib.ZS_BF16, 1, 8, 0) == _lib.ZS_ERR_INVALID
    assert b"NULL" in lib.zs_last_error()
    assert lib.zs_fp8_quantize_rows(None, _lib.ZS_BF16, None, None, 0, 8, 0) == _lib.ZS_OK
    # the gather group's set forms: argument checks before any launch
    assert lib.zs_fp8_quantize_rowset(0, None, None, None, None, None, None, _lib.ZS_BF16, 0) == _lib.ZS_OK
    assert lib.zs_fp8_quantize_rowset(1, None, None, None, None, None, None, _lib.ZS_BF16, 0) \
        == _lib.ZS_ERR_INVALID
    assert lib.zs_fp8_quantize_rowset(1, None, None, None, None, None, None, 9, 0) == _lib.ZS_ERR_INVALID
    ptr = np.array([4096], np.uint64)
    for rows, cs, row_len in ((3, 2, 64), (1, 1, 12), (1, 1, 0)):  # rows > cs; row_len % 8; empty rows
        tabs = [np.array([v], np.int64) for v in (rows, cs, row_len)]
        assert lib.zs_fp8_quantize_rowset(1, ptr.ctypes.data, ptr.ctypes.data, ptr.ctypes.data,
                                          *(t.ctypes.data for t in tabs), _lib.ZS_BF16, 0) \
            == _lib.ZS_ERR_INVALID
    assert b"zs_fp8_quantize_rowset" in lib.zs_last_error()
    assert lib.zs_fp8_dequantize_gathered(0, None, None, 1, 0, 0, None, None, None, None, None,
                                          _lib.ZS_BF16, 0) == _lib.ZS_OK
    assert lib.zs_fp8_dequantize_gathered(1, None, None, 2, 8, 1, None, None, None, None, None,
                                          _lib.ZS_BF16, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_fp8_dequantize_gathered(1, None, None, 0, 8, 1, None, None, None, None, None,
                                          _lib.ZS_BF16, 0) == _lib.ZS_ERR_INVALID  # ws 0
    assert lib.zs_fp8_dequantize_gathered(1, None, None, 2, 8, 1, None, None, None, None, None,
                                          _lib.ZS_U8, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_reduce(None, None, None, 4, _lib.ZS_F32, 0, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_broadcast(None, None, None, 4, _lib.ZS_F32, 0, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_reduce_group(None, 0, None, None, None, None, _lib.ZS_F32, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_broadcast_group(None, 0, None, None, None, _lib.ZS_F32, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_all_gather_group(None, 0, None, None, None, _lib.ZS_F32, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_reduce_scatter_group(None, 0, None, None, None, _lib.ZS_F32, 0) == _lib.ZS_ERR_INVALID
    # the ordered forms: a group needs a communicator; n == 0 without events is a no-op
    assert lib.zs_all_gather_group_ordered(None, 1, None, None, None, _lib.ZS_BF16, 0, 0, 0, 0) \
        == _lib.ZS_ERR_INVALID
    assert lib.zs_reduce_scatter_group_ordered(None, 1, None, None, None, _lib.ZS_BF16, 0, 0, 0, 0) \
        == _lib.ZS_ERR_INVALID
    assert lib.zs_all_gather_group_ordered(None, 0, None, None, None, _lib.ZS_BF16, 0, 0, 0, 0) == _lib.ZS_OK
    assert b"NULL communicator" in lib.zs_last_error()
    assert lib.zs_stream_wait_event(0, 0) == _lib.ZS_ERR_INVALID
    assert b"NULL event" in lib.zs_last_error()
    from zero_amd.plan import Plan

    plan = Plan([100, 300, 5], 2, 0, window_elems=64)
    ao, el, ev = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
    arr = (ctypes.c_int64 * 2)()
    assert lib.zs_plan_bucket(plan._h, plan.num_buckets, ctypes.byref(ao), ctypes.byref(el),
                              ctypes.byref(ev), arr, arr, arr) == _lib.ZS_ERR_INVALID


def test_phase_ranges_nest_and_validate():
    """roctx phase ranges (zero1.py:80-91 names) push/pop on the host without a GPU; a NULL name
    is rejected with a message instead of reaching roctx."""
    from zero_amd import _lib

    with _lib.phase_range("all_reduce_gradients"):
        with _lib.phase_range("optimizer_step"):
            pass
    assert _lib.lib.zs_range_push(None) == _lib.ZS_ERR_INVALID
    assert b"name is NULL" in _lib.lib.zs_last_error()
    with pytest.raises(RuntimeError):
        with _lib.phase_range("broadcast_parameters"):
            raise RuntimeError("propagates; the range is still popped")


def test_contract_entry_points_validate_without_gpu():
    """SURVEY.md §8(b)'s single-call forms (zs_plan_num_buckets / zs_plan_bucket_bytes / zs_pack /
    zs_unpack / zs_adam_step) answer or reject before touching the device."""
    from zero_amd import _lib
    from zero_amd.plan import Plan

    lib = _lib.lib
    plan = Plan([100, 300, 5], 2, 0, window_elems=64)
    n = ctypes.c_int64()
    assert lib.zs_plan_num_buckets(plan._h, ctypes.byref(n)) == _lib.ZS_OK
    assert n.value == plan.num_buckets > 0
    for k in range(plan.num_buckets):
        assert plan.bucket_bytes(k, _lib.ZS_F32) == 4 * plan.bucket(k).elems
        assert plan.bucket_bytes(k, _lib.ZS_BF16) == 2 * plan.bucket(k).elems
    b = ctypes.c_int64()
    assert lib.zs_plan_bucket_bytes(plan._h, plan.num_buckets, _lib.ZS_F32, ctypes.byref(b)) == _lib.ZS_ERR_INVALID
    assert lib.zs_plan_bucket_bytes(plan._h, 0, _lib.ZS_U8, ctypes.byref(b)) == _lib.ZS_ERR_INVALID
    ptrs = (ctypes.c_uint64 * 3)(0, 0, 0)
    assert lib.zs_pack(None, 0, ptrs, 4096, _lib.ZS_F32, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_pack(plan._h, plan.num_buckets, ptrs, 4096, _lib.ZS_F32, 0) == _lib.ZS_ERR_INVALID
    assert b"out of range" in lib.zs_last_error()
    assert lib.zs_pack(plan._h, 0, ptrs, 4096, _lib.ZS_U8, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_pack(plan._h, 0, ptrs, None, _lib.ZS_F32, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_unpack(plan._h, 0, 4096, ptrs, _lib.ZS_F32, 0) == _lib.ZS_ERR_INVALID
    assert b"param_ptrs" in lib.zs_last_error()  # unpack has nowhere to put a NULL param
    for fn, f in ((lib.zs_adam_step_ex, ctypes.c_double), (lib.zs_adam_step, ctypes.c_float)):
        args = lambda n_, gd, step: (None, None, None, gd, None, None, n_, f(1e-3), f(0.9), f(0.999),  # noqa: E731
                                     f(1e-8), f(0.0), 0, step, f(1.0), None, f(0.0), 0)
        assert fn(*args(-1, _lib.ZS_F32, 1)) == _lib.ZS_ERR_INVALID
        assert fn(*args(8, _lib.ZS_U8, 1)) == _lib.ZS_ERR_INVALID
        assert fn(*args(8, _lib.ZS_F32, 1)) == _lib.ZS_ERR_INVALID
        assert b"non-NULL" in lib.zs_last_error()
        assert fn(*args(0, _lib.ZS_F32, 0)) == _lib.ZS_ERR_INVALID  # step must be >= 1
        assert fn(*args(0, _lib.ZS_BF16, 1)) == _lib.ZS_OK  # empty: nothing to launch
    bad = (None, None, None, _lib.ZS_F32, None, None, 0) + tuple(ctypes.c_float(x) for x in
                                                                 (1e-3, 0.9, 0.999, 1e-8, 0.0))
    assert lib.zs_adam_step(*bad, 0, 1, ctypes.c_float(0.0), None, ctypes.c_float(0.0), 0) == _lib.ZS_ERR_INVALID
    assert b"grad_scale" in lib.zs_last_error()


def test_literal_plan_create_is_the_general_form():
    """SURVEY.md §8(b)'s zs_plan_create(…, bucket_bytes, out) = zs_plan_create_ex with 64-element
    alignment, ragged buckets and window = bucket_bytes / (4·ws) elements (64-aligned): the same
    ownership, pieces and buckets."""
    from zero_amd import _lib
    from zero_amd.plan import Plan

    lib = _lib.lib
    numels = [4096, 64, 300, 7, 100000, 5, 12288, 1]
    arr = (ctypes.c_int64 * len(numels))(*numels)
    for ws in (1, 2, 3, 8):
        for rank in range(ws):
            for bucket_bytes in (0, 4096, 1 << 16, 1 << 20):
                h = ctypes.c_void_p()
                assert lib.zs_plan_create(len(numels), arr, None, ws, rank, 0, bucket_bytes,
                                          ctypes.byref(h)) == _lib.ZS_OK
                win = 0 if (bucket_bytes == 0 or ws == 1) else max(64, bucket_bytes // (4 * ws) // 64 * 64)
                want = Plan(numels, ws, rank, "reference", align_elems=64, window_elems=win)
                info = (ctypes.c_int64 * 10)()
                assert lib.zs_plan_info(h, info) == _lib.ZS_OK
                winfo = (ctypes.c_int64 * 10)()
                assert lib.zs_plan_info(want._h, winfo) == _lib.ZS_OK
                assert list(info) == list(winfo), (ws, rank, bucket_bytes)
                for r in range(ws):
                    s, e = ctypes.c_int64(), ctypes.c_int64()
                    assert lib.zs_plan_owner_range(h, r, ctypes.byref(s), ctypes.byref(e)) == 0
                    assert (s.value, e.value) == tuple(want.owner_range(r))
                lib.zs_plan_destroy(h)


def test_literal_adam_step_divisor_is_the_world_size():
    """zs_adam_step's grad_scale = float(1/ws) gives back the divisor ws (the integer nearest to
    1/grad_scale, which float(1/ws)'s 2^-24 relative rounding keeps within 1e-6·ws) for every ws
    checked here (1..4096 and the powers of two below 2^24), so the update divides as zero1.py:84
    does — while float(1/float(1/ws)) alone is not ws for ws = 7, 13, 14, ..."""
    import numpy as np

    for ws in list(range(1, 4097)) + [2 ** k for k in range(13, 24)]:
        r = 1.0 / float(np.float32(1.0 / ws))
        k = round(r)
        assert k == ws and abs(r - k) <= 1e-6 * k, ws  # the rule in zs_kernels.hip zs_adam_step


def test_plain_c_client(tmp_path):
    """A C99 program built with gcc against include/zero_amd.h links libzero_amd.so and drives the
    host-side entry points (ownership, buckets, segments, error codes) — the C ABI needs no Python
    or torch in the caller."""
    import shutil
    import subprocess

    from zero_amd import _lib

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = tmp_path / "abi_host"
    libdir = _lib.LIB_PATH.parent
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", str(REPO / "include"),
                    str(REPO / "tests" / "c" / "abi_host.c"), "-L", str(libdir), "-lzero_amd",
                    f"-Wl,-rpath,{libdir}", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("c-abi ok")


def test_device_alloc_validates_without_gpu():
    """ABI v10's zs_device_alloc / zs_device_free (the placement probe's private allocations):
    bad arguments are rejected before the runtime is touched; freeing NULL is a no-op."""
    from zero_amd import _lib

    lib = _lib.lib
    out = ctypes.c_void_p(123)
    assert lib.zs_device_alloc(0, ctypes.byref(out)) == _lib.ZS_ERR_INVALID
    assert b"bytes must be > 0" in lib.zs_last_error()
    assert lib.zs_device_alloc(-5, ctypes.byref(out)) == _lib.ZS_ERR_INVALID
    assert lib.zs_device_alloc(64, None) == _lib.ZS_ERR_INVALID
    assert lib.zs_device_free(None) == _lib.ZS_OK


def test_tune_knobs_validate_and_restore():
    """zs_tune (diagnostic A/B knobs): known keys take their documented ranges and report the old
    value; unknown keys and out-of-range values are rejected; nothing touches the GPU."""
    from zero_amd import _lib

    lib = _lib.lib
    prev = ctypes.c_int64(99)
    for key, good, bad, default in ((b"dq_unroll", 8, 5, 4), (b"dq_nt_store", 0, 2, 1),
                                    (b"dq_wg_per_cu", 8, 129, 0), (b"scale_nt", 1, 2, -1),
                                    (b"convert_nt", 0, -2, -1), (b"copy_nt", 1, 3, -1),
                                    (b"adam_wg_per_cu", 64, 1025, 0), (b"sync_host_flags", 0, 2, 1),
                                    (b"sync_write_kernel", 0, 2, 1), (b"sync_write_fence", 0, 2, 1),
                                    (b"sync_wait_kernel", 0, 2, 1)):
        assert lib.zs_tune(key, good, ctypes.byref(prev)) == _lib.ZS_OK
        assert prev.value == default
        assert lib.zs_tune(key, bad, None) == _lib.ZS_ERR_INVALID
        assert b"out of range" in lib.zs_last_error()
        assert lib.zs_tune(key, default, ctypes.byref(prev)) == _lib.ZS_OK
        assert prev.value == good
    assert lib.zs_tune(b"no_such_knob", 1, None) == _lib.ZS_ERR_INVALID
    assert b"unknown key" in lib.zs_last_error()
    assert lib.zs_tune(None, 1, None) == _lib.ZS_ERR_INVALID


def test_copy_direct_validates_without_gpu():
    """ABI v11's zs_copy_direct: argument checks before any launch; n == 0 and all-empty segments
    launch nothing."""
    from zero_amd import _lib

    lib = _lib.lib
    z = np.zeros(3, np.uint64)
    assert lib.zs_copy_direct(-1, None, None, None, 0) == _lib.ZS_ERR_INVALID
    assert lib.zs_copy_direct(0, None, None, None, 0) == _lib.ZS_OK
    assert lib.zs_copy_direct(3, None, None, None, 0) == _lib.ZS_ERR_INVALID
    nb = np.array([0, 0, 0], np.int64)
    assert lib.zs_copy_direct(3, z.ctypes.data, z.ctypes.data, nb.ctypes.data, 0) == _lib.ZS_OK
    nb = np.array([0, -4, 0], np.int64)
    assert lib.zs_copy_direct(3, z.ctypes.data, z.ctypes.data, nb.ctypes.data, 0) == _lib.ZS_ERR_INVALID
    nb = np.array([8, 0, 0], np.int64)
    assert lib.zs_copy_direct(3, z.ctypes.data, z.ctypes.data, nb.ctypes.data, 0) == _lib.ZS_ERR_INVALID
    assert b"dst[0] is NULL" in lib.zs_last_error()


def test_table_wrappers_refuse_out_of_range_segments_without_gpu():
    """the wrappers that build copy tables from tensors check every segment against
    the tensors' storage first (CHECK_EXTENTS, on in tests): a segment past its buffer raises a
    Python exception and nothing reaches the raw-pointer entry points (CPU tensors here: the check
    runs before any HIP call)."""
    import pytest
    import torch

    from zero_amd import kernels

    assert kernels.check_extents_enabled()  # tests/conftest.py turns it on
    src = torch.zeros(1000, dtype=torch.uint8)
    dst = torch.zeros(4 << 20, dtype=torch.uint8)
    ok = ([src.data_ptr()], [dst.data_ptr() + 100], [1000])
    kernels.check_extents(ok[0], ok[2], [src], "src")
    kernels.check_extents(ok[1], ok[2], [dst], "dst")
    # r04s's fault: segments packed past a 4 MiB destination
    over = ([src.data_ptr()], [dst.data_ptr() + (4 << 20) - 10], [1000])
    with pytest.raises(ValueError, match="outside every buffer"):
        kernels.copy_direct(*over, 0, bounds=([src], [dst]))
    with pytest.raises(ValueError, match="outside every buffer"):
        kernels.CopySet(*over, bounds=([src], [dst]))
    # a source read past its tensor, a pointer before every buffer, a negative length
    with pytest.raises(ValueError):
        kernels.check_extents([src.data_ptr() + 1], [1000], [src])
    with pytest.raises(ValueError):
        kernels.check_extents([src.data_ptr() - 16], [8], [src, dst])
    with pytest.raises(ValueError, match="negative"):
        kernels.check_extents([src.data_ptr()], [-1], [src])
    # zero fill (src 0) and empty segments are not checked; a view's storage counts
    kernels.check_extents([0, src.data_ptr() + 999], [64, 0], [src])
    kernels.check_extents([dst.data_ptr() + 5000], [64], [dst[4096:8192]])


def test_adamset_set_grads_validates_without_gpu():
    """ABI v12's zs_adamset_set_grads: a NULL set, a count other than the set's, a NULL table are
    refused before anything is launched."""
    from zero_amd import _lib

    lib = _lib.lib
    g = np.zeros(2, np.uint64)
    assert lib.zs_adamset_set_grads(None, 2, g.ctypes.data, 0) == _lib.ZS_ERR_INVALID
    assert b"NULL set" in lib.zs_last_error()
