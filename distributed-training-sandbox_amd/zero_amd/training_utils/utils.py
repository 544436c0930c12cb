"""Process-group helpers used by the ShardedOptimizer drop-ins.

Mirrors ``get`` / ``set_seed`` of the reference's zero/training_utils/utils.py:24-79 (the HF model
and dataset loaders there are not on the ZeRO path and are not provided).
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch
import torch.distributed as dist


def set_seed(seed: int = 42) -> None:
    """utils.py:24-38: seed python, numpy, torch CPU and every GPU."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


class _CacheMesh:
    """utils.py:41-52: ``get`` optionally bound to a registered DeviceMesh."""

    def __init__(self, func):
        self.func = func
        self._mesh = None

    def __call__(self, what, dm=None):
        return self.func(what, self._mesh if dm is None else dm)

    def register_mesh(self, mesh):
        self._mesh = mesh
        return self


@_CacheMesh
def get(what: str, dm=None):
    """utils.py:55-79: 'ws' | 'pg' | 'rank' | 'grank' | 'lrank'."""
    pg = dm.get_group() if dm is not None else None
    if what == "ws":
        return dist.get_world_size(pg)
    if what == "pg":
        return pg
    if what in ("rank", "grank"):
        return dist.get_rank(pg)
    if what == "lrank":
        return dm.get_local_rank() if dm is not None else int(os.environ.get("LOCAL_RANK", 0))
    raise ValueError(f"Invalid string: {what}")
