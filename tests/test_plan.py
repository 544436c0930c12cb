"""Layout planner (zs_plan_*, host-only C++) against the reference's ownership fixtures and the
structural invariants every pack / reduce-scatter / all-gather / unpack relies on."""
import numpy as np
import pytest

from zero_amd.plan import Plan
from oracle import zero_oracle as zo


def test_ownership_matches_reference(golden):
    """zero1.py:55-62 ranges and zero1.py:95-100 owners, bit-exact, n<=400, ws<=64."""
    z = golden("ownership.npz")
    for n in z["ns"]:
        for ws in z["wss"]:
            n, ws = int(n), int(ws)
            start, end, owner = z[f"n{n}_ws{ws}_start"], z[f"n{n}_ws{ws}_end"], z[f"n{n}_ws{ws}_owner"]
            plan = Plan(np.ones(n, np.int64), ws, 0)
            for r in range(ws):
                s, e = plan.owner_range(r)
                if end[r] > start[r]:
                    assert (s, e) == (start[r], end[r]), (n, ws, r)
                else:
                    assert s == e, (n, ws, r)
            got = [plan.owner_of(i) for i in range(n)]
            assert got == owner.tolist(), (n, ws)


def test_oracle_ownership_matches_reference(golden):
    z = golden("ownership.npz")
    for n in (1, 2, 7, 12, 13, 64, 291, 326, 400):
        for ws in z["wss"]:
            ws = int(ws)
            own = z[f"n{n}_ws{ws}_owner"]
            assert [zo.owner_of(n, ws, i) for i in range(n)] == own.tolist()
            for r in range(ws):
                s, e = zo.owner_range(n, ws, r)
                if z[f"n{n}_ws{ws}_end"][r] > z[f"n{n}_ws{ws}_start"][r]:
                    assert (s, e) == (z[f"n{n}_ws{ws}_start"][r], z[f"n{n}_ws{ws}_end"][r])


def _coverage(plan, numels):
    """Every element of every param appears in exactly one rank's pieces and exactly once in the
    buckets; bucket offsets are in range and disjoint; piece starts are aligned."""
    ws = plan.ws
    cover = [np.zeros(n, np.int32) for n in numels]
    for r in range(ws):
        pc = plan.pieces(r)
        L = plan.stream_len(r)
        used = np.zeros(L, np.int8)
        for i, po, so, ln in zip(pc.param, pc.param_off, pc.stream_off, pc.length):
            assert so % 64 == 0
            assert so + ln <= L
            cover[i][po:po + ln] += 1
            assert used[so:so + ln].sum() == 0
            used[so:so + ln] = 1
    for c in cover:
        assert (c == 1).all()
    seen = [np.zeros(n, np.int32) for n in numels]
    arena_used = np.zeros(max(plan.arena_elems, 1), np.int8)
    stream_seen = [np.zeros(plan.stream_len(r), np.int32) for r in range(ws)]
    for k in range(plan.num_buckets):
        b = plan.bucket(k)
        assert b.arena_off % 64 == 0 and b.arena_off + b.elems <= plan.arena_elems
        assert arena_used[b.arena_off:b.arena_off + b.elems].sum() == 0
        arena_used[b.arena_off:b.arena_off + b.elems] = 1
        assert b.even == (k < plan.num_even)
        if b.even:  # one equal-count reduce-scatter / all-gather: window r at r*len
            w = int(b.win_len[0])
            assert (b.win_len == w).all() and (b.win_off == np.arange(ws) * w).all()
            assert b.elems == ws * w and w <= plan.window
        for r in range(ws):
            assert b.win_off[r] % 64 == 0 and b.win_off[r] + b.win_len[r] <= b.elems
            lo, n = int(b.win_stream[r]), int(b.win_len[r])
            hi = min(lo + n, plan.stream_len(r))
            if hi > lo:
                stream_seen[r][lo:hi] += 1
        s = plan.segments(k)
        used = np.zeros(b.elems, np.int8)
        for i, r, po, bo, ln in zip(s.param, s.rank, s.param_off, s.buf_off, s.length):
            assert b.win_off[r] <= bo and bo + ln <= b.win_off[r] + b.win_len[r]
            assert used[bo:bo + ln].sum() == 0
            used[bo:bo + ln] = 1
            seen[i][po:po + ln] += 1
            # the element's stream position is the same through the piece and through the window
            pc = plan.pieces(r)
            j = np.nonzero((pc.param == i) & (pc.param_off <= po) & (po < pc.param_off + pc.length))[0]
            assert len(j) == 1
            assert pc.stream_off[j[0]] + (po - pc.param_off[j[0]]) == b.win_stream[r] + (bo - b.win_off[r])
    for c in seen:
        assert (c == 1).all()
    for r in range(ws):  # every stream position lies in exactly one window
        assert (stream_seen[r] == 1).all()


@pytest.mark.parametrize("buckets", ["ragged", "padded"])
@pytest.mark.parametrize("layout", ["reference", "chunk", "flat"])
@pytest.mark.parametrize("ws", [1, 2, 3, 4, 8])
def test_layout_invariants(layout, ws, buckets):
    rng = np.random.default_rng(ws)
    shapes = [(int(rng.integers(1, 40)), int(rng.integers(1, 9))) for _ in range(23)]
    shapes += [(16, 16), (16,), (1,), (0,), (5, 3)]
    numels = [int(np.prod(s)) for s in shapes]
    dim0 = [s[0] for s in shapes]
    for window in (0, 64, 128, 1000):
        plan = Plan(numels, ws, 0, layout, dim0=dim0, window_elems=window, buckets=buckets)
        _coverage(plan, numels)
        if buckets == "padded" or layout == "flat":
            assert plan.num_even == plan.num_buckets
        if window:
            assert plan.window % 64 == 0


@pytest.mark.parametrize("ws", [1, 2, 3, 4, 8])
def test_chunk_layout_matches_torch_chunk(ws):
    """Layout Z pieces are torch.chunk(ws, dim=0)[rank] (zero3.py:107-108), incl. uneven d0."""
    import torch

    shapes = [(16, 4), (10000 // 625, 3), (7, 2), (3,), (2, 5), (1, 1)]
    numels = [int(np.prod(s)) for s in shapes]
    plan = Plan(numels, ws, 0, "chunk", dim0=[s[0] for s in shapes])
    for r in range(ws):
        pc = plan.pieces(r)
        for i, s in enumerate(shapes):
            t = torch.arange(numels[i]).reshape(s)
            chunks = t.chunk(ws, dim=0)
            j = np.nonzero(pc.param == i)[0]
            assert len(j) == 1
            po, ln = int(pc.param_off[j[0]]), int(pc.length[j[0]])
            want = chunks[r].reshape(-1) if r < len(chunks) else torch.zeros(0, dtype=t.dtype)
            assert torch.equal(t.reshape(-1)[po:po + ln], want)


def test_flat_layout_balanced():
    numels = [4096 * 4096, 4096] * 6
    for ws in (2, 4, 8):
        plan = Plan(numels, ws, 0, "flat")
        lens = [plan.stream_len(r) for r in range(ws)]
        assert len(set(lens)) == 1
        assert lens[0] * ws - sum(numels) < 64 * ws + 64 * len(numels)


def test_reference_layout_padding_smollm3():
    """Layout R pads to the largest owner (SmolLM3-3B at ws=8 ≈ 1.52×)."""
    from zero_amd.shapes import smollm3_3b_shapes

    numels = [int(np.prod(s)) for s in smollm3_3b_shapes()]
    assert sum(numels) == 3_075_098_624 and len(numels) == 326
    plan = Plan(numels, 8, 0, "reference")
    ratio = plan.max_stream_len * 8 / sum(numels)
    assert 1.4 < ratio < 1.6


def _bus_elems(plan):
    """Elements one rank's links carry for the reduce phase: ring RS moves (ws-1)/ws of an even
    bucket, a reduce moves its whole message."""
    tot = 0.0
    for k in range(plan.num_buckets):
        b = plan.bucket(k)
        tot += b.elems * (plan.ws - 1) / plan.ws if b.even else int(b.win_len.sum())
    return tot


@pytest.mark.parametrize("ws,max_ratio", [(2, 1.0), (4, 0.85), (8, 0.70)])
def test_ragged_buckets_cut_smollm3_traffic(ws, max_ratio):
    """Ragged tails (grouped reduce per owner) instead of zero-padding every window to the longest
    stream: SmolLM3-3B Layout R moves ~1/3 fewer bytes at ws=8 (SURVEY.md §7 padding figures)."""
    from zero_amd.shapes import smollm3_3b_shapes

    numels = [int(np.prod(s)) for s in smollm3_3b_shapes()]
    W = (256 << 20) // (ws * 2)
    rag = Plan(numels, ws, 0, "reference", window_elems=W, buckets="ragged")
    pad = Plan(numels, ws, 0, "reference", window_elems=W, buckets="padded")
    assert rag.arena_elems < pad.arena_elems or ws == 2
    r = _bus_elems(rag) / _bus_elems(pad)
    assert r <= max_ratio + 1e-9, r
    # no bucket buffer exceeds the requested bucket size
    assert max(rag.bucket(k).elems for k in range(rag.num_buckets)) <= ws * W


def test_invalid_arguments_raise():
    from zero_amd._lib import ZeroAmdError

    with pytest.raises(ZeroAmdError):
        Plan([4, 4], 0, 0)
    with pytest.raises(ZeroAmdError):
        Plan([4, 4], 2, 2)
    with pytest.raises(ZeroAmdError):
        Plan([6, 4], 2, 0, "chunk", dim0=[4, 4])  # 6 % 4 != 0
    plan = Plan([4, 4], 2, 0)
    with pytest.raises(ZeroAmdError):
        plan.segments(5)
    with pytest.raises(ZeroAmdError):
        plan.bucket(5)
    with pytest.raises(ZeroAmdError):
        plan.owner_of(2)


def test_empty_and_tiny():
    plan = Plan([], 4, 1)
    assert plan.num_buckets == 0 and plan.stream_len() == 0
    plan = Plan([3], 4, 3)  # ws > n: ranks 1..3 own nothing
    assert plan.owner_range(3) == (1, 1) and plan.stream_len(3) == 0
    assert plan.owner_of(0) == 0


def test_grad_bucket_grouping():
    """overlap.plan_grad_buckets: reverse order, size cap, no key mixing, aligned disjoint slots."""
    from zero_amd.overlap import plan_grad_buckets

    rng = np.random.default_rng(0)
    numels = [int(x) for x in rng.integers(1, 5000, 40)] + [100000]
    keys = sorted(int(k) for k in rng.integers(0, 4, len(numels)))
    groups, bkeys, slot, bucket_of, boff, blen = plan_grad_buckets(numels, keys, 4 * 8192, 4)
    flat = [i for g in groups for i in g]
    assert flat == list(range(len(numels)))[::-1]
    for k, g in enumerate(groups):
        assert len({keys[i] for i in g}) == 1 and bkeys[k] == keys[g[0]]
        assert blen[k] <= 8192 or len(g) == 1
        for i in g:
            assert bucket_of[i] == k and slot[i] % 64 == 0
            assert boff[k] <= slot[i] and slot[i] + numels[i] <= boff[k] + blen[k]
    ends = sorted((slot[i], slot[i] + numels[i]) for i in range(len(numels)))
    assert all(a[1] <= b[0] for a, b in zip(ends, ends[1:]))
    with pytest.raises(ValueError):
        plan_grad_buckets([1, 2], [0, 0], 64, 4, order=[0, 0])


def test_smollm3_shapes_match_transformers_model():
    """shapes.smollm3_3b_shapes (the bench's synthetic set) is exactly the parameter list of
    transformers' SmolLM3-3B (built on the meta device: no memory)."""
    import torch
    from zero_amd.shapes import smollm3_3b_shapes
    from zero_amd.training_utils import smollm3 as sm
    from transformers import SmolLM3ForCausalLM

    with torch.device("meta"):
        model = SmolLM3ForCausalLM(sm.smollm3_config())
    got = [tuple(p.shape) for p in model.parameters()]
    assert got == [tuple(s) for s in smollm3_3b_shapes()]
    assert sm.model_flops_per_token(model.config, 8192) > 6 * 3.0e9


def test_arena_auto_owner_shares_and_validation():
    """arena="auto"'s sample windows follow the reference's index ranges (zero1.py:55-62): bytes per
    owner, empty owners included; an unknown arena is rejected before anything is built."""
    import types

    import pytest
    import torch

    from zero_amd import _sharded

    ps = [torch.zeros(n) for n in (5, 7, 11)]
    opt = types.SimpleNamespace(world_size=4, params=ps)
    assert _sharded._owner_bytes(opt) == [20, 28, 44, 0]
    opt = types.SimpleNamespace(world_size=2, params=ps + [torch.zeros(3, dtype=torch.bfloat16)])
    assert _sharded._owner_bytes(opt) == [48, 50]
    with pytest.raises(ValueError, match="arena must be"):
        _sharded.ShardedOptimizerBase(torch.optim.Adam([torch.nn.Parameter(torch.zeros(4))]),
                                      arena="fastest")
