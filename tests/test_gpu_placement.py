"""Placement probe side effects (engine.probed_zeros): the candidates are
device allocations of their own (zs_device_alloc), so building an optimizer never releases the
CALLER's cached blocks (no torch.cuda.empty_cache() inside the constructor), the kept buffer is a
placed allocation counted by placed_bytes(), and it is returned to the device with its tensors."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _segments():
    return {s["address"] for s in torch.cuda.memory_snapshot()}


@pytest.fixture
def pg1():
    import torch.distributed as dist

    from _zero_run import init_pg
    from conftest import free_port

    init_pg(0, 1, free_port())
    yield
    dist.destroy_process_group()


def test_probe_keeps_callers_cached_block(gpu, pg1):
    from zero_amd import engine, zero2
    from zero_amd.shapes import mlp_shapes

    dev = gpu
    torch.cuda.synchronize()
    params = [torch.nn.Parameter(torch.zeros(s, device=dev)) for s in mlp_shapes(12800)]  # C3, fp32
    blk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)  # the caller's own 1 GiB block ...
    addr = blk.data_ptr()
    del blk  # ... now cached by torch, not in use
    assert addr in _segments()
    before = engine.placed_bytes()
    opt = zero2.ShardedOptimizer(torch.optim.Adam(params, lr=1e-3), sync=True)
    for p in params:
        p.grad = torch.full_like(p, 1e-3)
    opt.step()  # builds the engine: state (7.9 GB fp32) placed by the probe
    torch.cuda.synchronize()
    assert addr in _segments(), "the caller's cached 1 GiB block was released by the probe"
    pl = opt.engine.placement
    assert pl.get("allocator", "").startswith("zs_device_alloc") and pl["tries"] >= 1, pl
    assert 0 <= pl["chosen"] < pl["tries"] == len(pl["gbs"]) and pl["unprobed_gbs"] == pl["gbs"][0]
    held = engine.placed_bytes() - before
    assert held >= 2 * sum(p.numel() for p in params) * 4, held  # exp_avg + exp_avg_sq at least
    # the state is outside torch's allocator: none of its storages is a torch segment
    st = opt.engine.state
    assert st.untyped_storage().data_ptr() not in _segments()
    # Adam's first step on a constant grad: every parameter moved by -lr (bias-corrected)
    assert torch.allclose(params[0][:2, :4], torch.full((2, 4), -1e-3, device=dev), rtol=1e-4)
    free0 = torch.cuda.mem_get_info(dev)[0]
    # the parameters are views of the flat arena and their grads views of the grad arena (and
    # their hooks reach the engine): everything goes when the model and the optimizer go
    del opt, st, params, p
    import gc

    gc.collect()
    torch.cuda.synchronize()
    assert engine.placed_bytes() == before  # placed buffers went back with their tensors
    assert torch.cuda.mem_get_info(dev)[0] > free0 + held // 2


def test_zero3_update_state_freed_with_optimizer(gpu, pg1):
    """ZeRO-3 update mode: the placed Adam state (here 2 x 8192^2 fp32 chunks: 1 GiB of m / v)
    goes back to the device when the model and the optimizer are dropped — the reducer's
    post-accumulate hooks hold it weakly (zero_amd/_hooks.py)."""
    import gc

    from zero_amd import engine, zero3

    before = engine.placed_bytes()
    model = torch.nn.Sequential(torch.nn.Linear(8192, 8192, bias=False),
                                torch.nn.Linear(8192, 8192, bias=False)).to(gpu)
    opt = zero3.ShardedOptimizer(torch.optim.Adam(model.parameters(), lr=1e-3), update=True)
    zero3.register_zero3_hooks(model, opt.param_managers)
    assert engine.placed_bytes() - before >= 2 * 2 * 8192 * 8192 * 4
    x = torch.randn(4, 8192, device=gpu)
    model(x).sum().backward()
    opt.step()
    torch.cuda.synchronize()
    del opt, model, x
    gc.collect()
    torch.cuda.synchronize()
    assert engine.placed_bytes() == before


def test_probe_falls_back_to_chunked_route(gpu, monkeypatch):
    """when no plain allocation reaches the acceptance rate, the probe tries 1-GiB
    physical chunks mapped side by side (zs_device_alloc_chunked) and keeps the fastest of every
    candidate; a chunked buffer works as any other (zero-filled, written and read back through
    torch) and goes back to the device with its tensor."""
    import gc

    from zero_amd import engine

    monkeypatch.setattr(engine, "PROBE_CHUNKED_TRIES", 2)
    before = engine.placed_bytes()
    n = (5 << 30) // 4 + 7  # 5 GiB + a bit of fp32: the chunked candidates round up to 6 GiB
    buf, info = engine.probed_zeros(n, torch.float32, gpu, tries=2, accept_gbs=1e9)  # never accepted
    assert info["routes"] == ["hipMalloc", "hipMalloc", "chunked", "chunked"], info
    assert info["tries"] == 4 and len(info["gbs"]) == 4 and min(info["gbs"]) > 1000.0, info
    assert info["route"] == info["routes"][info["chosen"]]
    assert info["gbs"][info["chosen"]] == max(info["gbs"])
    assert buf.numel() == n and int(torch.count_nonzero(buf)) == 0
    buf[-3:] = torch.tensor([1.0, 2.0, 3.0], device=gpu)
    buf[:5] = 4.0
    assert buf[-3:].tolist() == [1.0, 2.0, 3.0] and float(buf[:5].sum()) == 20.0
    assert engine.placed_bytes() - before in (6 << 30, n * 4)  # only the kept buffer is held
    del buf
    gc.collect()
    torch.cuda.synchronize()
    assert engine.placed_bytes() == before


def test_chunked_allocation_refuses_a_bad_chunk_size(gpu):
    import ctypes

    from zero_amd import _lib

    p = ctypes.c_void_p()
    rc = _lib.lib.zs_device_alloc_chunked(1 << 20, 12345, ctypes.byref(p))
    assert rc == _lib.ZS_ERR_INVALID and not p.value
