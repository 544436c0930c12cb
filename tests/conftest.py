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
