import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "distributed-training-sandbox_amd"
GOLDEN = REPO / "tests" / "golden"
for p in (str(REPO), str(PKG), str(REPO / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
# The multi-rank GPU tests put up to 8 ranks (+ this process) on the box's one GPU.  At HIP's
# default of 4 hardware queues per process that is more queues than the device schedules at once;
# an over-subscribed 8-rank run stalled with half the ranks inside a backward pass while the
# others waited in a collective.  Two queues per process keep 9 processes within the limit (in a
# queue shared by two streams, a wait is always behind the record it waits for, in host order).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "2")


def free_port() -> int:
    """A free TCP port BELOW the ephemeral range (32768+), so no outgoing connection (gloo's own
    pair sockets included) can grab it between this check and the rendezvous bind."""
    import random
    import socket

    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free port in 20000-32000")


def pytest_runtest_logreport(report):
    """ZS_FAIL_LOG=<file>: append each failure's report as it happens (a GPU run that is killed
    later still leaves the reasons of the failures before it)."""
    path = os.environ.get("ZS_FAIL_LOG")
    if path and report.failed:
        with open(path, "a") as f:
            f.write(f"==== {report.nodeid} ({report.when})\n{report.longreprtext[-6000:]}\n")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = np.load(GOLDEN / name)
        return cache[name]

    return load


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _release_communicators():
    """Destroy every RCCL communicator a test leaves behind (RcclComm closes itself when
    collected; optimizer / runtime reference cycles keep it alive until a collection).  A live
    communicator in this process stalled the 8-rank single-GPU tests spawned after it."""
    yield
    import gc

    gc.collect()
