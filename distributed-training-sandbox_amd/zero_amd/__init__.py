"""zero_amd — MI355X-native ZeRO sharded-optimizer step (drop-in for the sandbox's zero/zeroN.py).

Modules mirror the reference: ``zero_amd.zero1`` / ``zero2`` / ``zero3`` each export
``ShardedOptimizer``; ``zero3`` also ``Zero3ParamManager`` and ``register_zero3_hooks``;
``zero_amd.training_utils`` exports ``get``, ``set_seed`` and ``print_memory_stats``.
Importing the package loads ``libzero_amd.so``; it raises if the library is missing.
"""
from . import _lib  # noqa: F401  (fail loudly at import if the native library is absent)

__all__ = ["zero1", "zero2", "zero3", "training_utils"]
