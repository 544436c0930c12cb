"""Sync objects (include/zero_amd.h zs_sync, ABI v12): the engines' cross-stream ordering as a HIP
event or as a stream memory operation on a device flag word.  Both kinds must order
a consumer stream after a producer stream exactly like hipStreamWaitEvent, including when the
producer is far behind the host (the flag wait is then enqueued) and when it has finished (the
host sees the word and enqueues nothing), and a flag created while the legacy null stream is busy
must order as any other (its slab is zeroed by the host before any word is handed out)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SLEEP_CYCLES = 50_000_000  # ~20 ms of a spinning kernel: the producer is far behind the host


FLAG_METHODS = {  # zs_tune knobs: (sync_write_kernel, sync_write_fence, sync_wait_kernel)
    "store_kernel+wait_kernel": (1, 1, 1),      # the defaults (round 6)
    "store_kernel+wait_value": (1, 1, 0),
    "write_value+wait_value": (0, 1, 0),        # round 5: hipStreamWriteValue64 / WaitValue64
    "relaxed_store+wait_kernel": (1, 0, 1),
}


@pytest.fixture(params=list(FLAG_METHODS))
def flag_record(request):
    """How a flag sync's record writes its word and its wait waits: the library's one-wave store
    kernel (a system-scope release, or relaxed) or hipStreamWriteValue64, and its s_sleep polling
    wave or hipStreamWaitValue64 — every combination must order alike."""
    from zero_amd import _lib

    w, f, k = FLAG_METHODS[request.param]
    _lib.call("zs_tune", b"sync_write_kernel", w, None)
    _lib.call("zs_tune", b"sync_write_fence", f, None)
    _lib.call("zs_tune", b"sync_wait_kernel", k, None)
    yield request.param
    for key in (b"sync_write_kernel", b"sync_write_fence", b"sync_wait_kernel"):
        _lib.call("zs_tune", key, 1, None)


@pytest.mark.parametrize("kind", ["flag", "event"])
def test_sync_orders_consumer_after_producer(gpu, kind, flag_record):
    from zero_amd.comm import StreamEvent

    prod, cons = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    src = torch.zeros(1 << 20, device=gpu)
    dst = torch.full((1 << 20,), -1.0, device=gpu)
    ev = StreamEvent(kind)
    for it in range(1, 4):
        with torch.cuda.stream(prod):
            torch.cuda._sleep(SLEEP_CYCLES)  # the host runs far ahead of the producer
            src.fill_(float(it))
        ev.record(prod)
        ev.wait(cons)
        with torch.cuda.stream(cons):
            dst.copy_(src)  # must see this iteration's fill
        cons.synchronize()
        assert bool((dst == float(it)).all()), (kind, it)
    torch.cuda.synchronize()


def test_flag_created_while_null_stream_is_busy(gpu):
    """A new flag sync (possibly a new slab) while the legacy null stream holds queued work, then a
    record on a non-blocking stream and a wait on another: must complete (pytest's timeout catches
    a wait whose epoch was overwritten by a late zero fill)."""
    from zero_amd.comm import StreamEvent

    torch.cuda._sleep(SLEEP_CYCLES)  # on the null (default) stream
    prod, cons = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    evs = [StreamEvent("flag") for _ in range(5000)]  # more than one slab of 4096 words
    x = torch.zeros(16, device=gpu)
    for k, ev in enumerate(evs[-3:]):
        with torch.cuda.stream(prod):
            x.add_(1.0)
        ev.record(prod)
        ev.wait(cons)
        with torch.cuda.stream(cons):
            y = x.clone()
        cons.synchronize()
        assert float(y[0]) == k + 1
    torch.cuda.synchronize()


def test_unrecorded_sync_waits_for_nothing(gpu):
    from zero_amd.comm import StreamEvent

    s = torch.cuda.Stream(gpu)
    for kind in ("flag", "event"):
        StreamEvent(kind).wait(s)
    s.synchronize()


@pytest.mark.parametrize("kind", ["flag", "event"])
def test_wait_after_producer_finished(gpu, kind, flag_record):
    """The producer's record has executed before the wait is asked for: the flag wait is then
    skipped on the host (the word already holds the epoch) and the consumer still sees the data."""
    from zero_amd.comm import StreamEvent

    prod, cons = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    src = torch.zeros(1 << 16, device=gpu)
    dst = torch.full((1 << 16,), -1.0, device=gpu)
    ev = StreamEvent(kind)
    for it in range(1, 4):
        with torch.cuda.stream(prod):
            src.fill_(float(it))
        ev.record(prod)
        prod.synchronize()
        ev.wait(cons)
        with torch.cuda.stream(cons):
            dst.copy_(src)
        cons.synchronize()
        assert bool((dst == float(it)).all()), (kind, it)


@pytest.mark.parametrize("busy", [True, False])
def test_synced_prologue_orders_after_stream(gpu, busy, flag_record):
    """zs_all_gather_group_synced with no collective (n = 0): `stream` runs after everything
    enqueued on after_stream, busy or already idle, and `done` orders a third stream after
    `stream`."""
    from zero_amd import _lib
    from zero_amd.comm import Sync

    after, side, cons = (torch.cuda.Stream(gpu) for _ in range(3))
    ready, done = Sync(_lib.ZS_SYNC_FLAG), Sync(_lib.ZS_SYNC_FLAG)
    src = torch.zeros(1 << 16, device=gpu)
    mid = torch.full((1 << 16,), -1.0, device=gpu)
    dst = torch.full((1 << 16,), -1.0, device=gpu)
    for it in range(1, 4):
        with torch.cuda.stream(after):
            if busy:
                torch.cuda._sleep(SLEEP_CYCLES // 4)
            src.fill_(float(it))
        if not busy:
            after.synchronize()
        rc = _lib.lib.zs_all_gather_group_synced(None, 0, None, None, None, _lib.ZS_F32,
                                                  after.cuda_stream, ready.h, side.cuda_stream,
                                                  done.h)
        assert rc == 0
        with torch.cuda.stream(side):
            mid.copy_(src)
        done.record(side.cuda_stream)
        done.wait(cons.cuda_stream)
        with torch.cuda.stream(cons):
            dst.copy_(mid)
        cons.synchronize()
        assert bool((dst == float(it)).all()), (busy, it)
    torch.cuda.synchronize()


@pytest.mark.parametrize("kind", ["flag", "event"])
def test_device_flag_words_order_streams(gpu, kind, flag_record):
    """The fallback flag words in device memory (zs_tune("sync_host_flags", 0): every wait
    enqueued, none skipped on the host) order streams as the pinned host words do."""
    from zero_amd import _lib
    from zero_amd.comm import StreamEvent

    _lib.call("zs_tune", b"sync_host_flags", 0, None)
    try:
        evs = [StreamEvent(kind) for _ in range(3)]
    finally:
        _lib.call("zs_tune", b"sync_host_flags", 1, None)
    prod, cons = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    src = torch.zeros(1 << 16, device=gpu)
    dst = torch.full((1 << 16,), -1.0, device=gpu)
    for it, ev in enumerate(evs, 1):
        for behind in (True, False):
            with torch.cuda.stream(prod):
                if behind:
                    torch.cuda._sleep(SLEEP_CYCLES // 4)
                src.fill_(float(it))
            ev.record(prod)
            if not behind:
                prod.synchronize()
            ev.wait(cons)
            with torch.cuda.stream(cons):
                dst.copy_(src)
            cons.synchronize()
            assert bool((dst == float(it)).all()), (kind, it, behind)


def _flag_syncs(host_words: bool, n: int):
    from zero_amd import _lib
    from zero_amd.comm import Sync

    _lib.call("zs_tune", b"sync_host_flags", int(host_words), None)
    try:
        return [Sync(_lib.ZS_SYNC_FLAG) for _ in range(n)]
    finally:
        _lib.call("zs_tune", b"sync_host_flags", 1, None)


@pytest.mark.parametrize("host_words", [True, False], ids=["host_word", "device_word"])
def test_flag_epochs_cross_2_pow_32(gpu, host_words, flag_record):
    """a flag sync seeded at epoch 2^32 - 3 orders a slow producer before its
    consumer on every record across 2^32 (ABI v13: 64-bit words; v12's 32-bit epoch wrapped there,
    the GPU's unsigned >= was then satisfied by the stale pre-wrap word and the host skipped the
    first wait).  Both word locations: pinned host (satisfied waits skipped on the host) and device
    memory (every wait enqueued)."""
    (sy,) = _flag_syncs(host_words, 1)
    start = (1 << 32) - 3
    sy.set_epoch(start)
    assert sy.query() == (start, start)
    prod, cons = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    src = torch.zeros(1 << 20, device=gpu)
    dst = torch.full((1 << 20,), -1.0, device=gpu)
    for it in range(1, 8):  # epochs 2^32 - 2 ... 2^32 + 4
        with torch.cuda.stream(prod):
            torch.cuda._sleep(SLEEP_CYCLES // 2)  # the host runs far ahead of the producer
            src.fill_(float(it))
        sy.record(prod.cuda_stream)
        sy.wait(cons.cuda_stream)
        with torch.cuda.stream(cons):
            dst.copy_(src)
        cons.synchronize()
        assert bool((dst == float(it)).all()), (host_words, it)
    torch.cuda.synchronize()
    assert sy.query() == (start + 7, start + 7)
    assert sy.query()[0] > (1 << 32)


@pytest.mark.parametrize("host_words", [True, False], ids=["host_word", "device_word"])
def test_flag_record_from_two_streams_keeps_epochs_in_order(gpu, host_words, flag_record):
    """a record from a second stream while the first stream's record is still pending.
    The second write waits for the first, so the word ends at the latest epoch (v12 let the slow
    first write land last and move the word back, so a later wait for the latest epoch could never
    be satisfied), and a consumer of the second record sees the first producer's work too."""
    (sy,) = _flag_syncs(host_words, 1)
    a, b, cons = (torch.cuda.Stream(gpu) for _ in range(3))
    src = torch.zeros(1 << 20, device=gpu)
    dst = torch.full((1 << 20,), -1.0, device=gpu)
    for it in range(1, 4):
        with torch.cuda.stream(a):
            torch.cuda._sleep(SLEEP_CYCLES)  # a's record executes long after b's
            src.fill_(float(it))
        sy.record(a.cuda_stream)
        sy.record(b.cuda_stream)
        sy.wait(cons.cuda_stream)
        with torch.cuda.stream(cons):
            dst.copy_(src)
        cons.synchronize()
        assert bool((dst == float(it)).all()), (host_words, it)
        torch.cuda.synchronize()
        epoch, word = sy.query()
        assert epoch == 2 * it and word == epoch, (epoch, word)


def test_set_epoch_refusals(gpu):
    from zero_amd import _lib
    from zero_amd.comm import Sync

    (sy,) = _flag_syncs(True, 1)
    sy.set_epoch(10)
    with pytest.raises(_lib.ZeroAmdError):
        sy.set_epoch(9)  # epochs only grow
    ev = Sync(_lib.ZS_SYNC_EVENT)
    with pytest.raises(_lib.ZeroAmdError):
        ev.set_epoch(5)
    assert ev.query() == (0, 0)
