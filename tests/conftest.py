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
# every segment table the Python side builds from tensors is checked against their storage before
# launch (zero_amd/kernels.py CHECK_EXTENTS): an out-of-range segment raises instead of faulting
os.environ.setdefault("ZERO_AMD_CHECK_EXTENTS", "1")
# This process (single-process kernel tests, rank 0 of the multi-rank ones) runs at the box's
# default number of HIP hardware queues; only the ranks spawned beside it are given two
# (tests/_zero_run.py CHILD_ENV), so up to 8 processes on the one GPU stay within the queues the
# device schedules at once.


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
