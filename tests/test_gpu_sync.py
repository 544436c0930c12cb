"""Sync objects (include/zero_amd.h zs_sync, ABI v12): the engines' cross-stream ordering as a HIP
event or as a stream memory operation on a device flag word.  Both kinds must order
a consumer stream after a producer stream exactly like hipStreamWaitEvent, including when the
producer is far behind the host, and a flag created while the legacy null stream is busy must not
be zeroed behind a record (its slab is zero-filled to completion before any word is handed out)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SLEEP_CYCLES = 50_000_000  # ~20 ms of a spinning kernel: the producer is far behind the host


@pytest.mark.parametrize("kind", ["flag", "event"])
def test_sync_orders_consumer_after_producer(gpu, kind):
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
