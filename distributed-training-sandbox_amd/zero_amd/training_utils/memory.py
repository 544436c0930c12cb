"""Per-rank memory report for the ZeRO harness (what zero/training_utils/memory.py:37-50 prints).

One pass over the model and the optimizer state builds a ``MemoryReport``; ``print_memory_stats``
renders it in the reference's five-line format so the harness output reads the same.  Sizes are
logical (numel × element size, in MiB) — the quantity the reference reports — and, separately,
physical: the distinct storages behind those tensors.  The two differ for the drop-ins on purpose:
``optimizer.optimizer.state[p]`` holds *views* of one flat fp32 shard buffer, and ZeRO-3 parameters
are views of one flat chunk arena, so the physical column shows what is really resident.
"Total allocated" / "Max allocated" are torch's allocator figures, as the reference prints them.
The placed buffers of 1 GiB or more (optimizer state, parameter / gradient arenas:
``engine.probed_zeros``) are device allocations of their own outside torch's cache, so torch's two
figures alone under-report the drop-in's residency against the reference's (whose whole state
lives in torch's allocator).  When anything is placed, two more lines follow: the placed bytes
(held now, and the device's high-water mark with the placement probe's candidates), and the
combined figures comparable to the reference's — "Total incl. placed" (torch's allocated + placed,
both now) and "Max incl. placed", an upper bound: the sum of the two peaks, which need not
coincide in time.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

_MIB = float(1 << 20)


def _walk(tensors):
    """(logical MiB, physical MiB) of an iterable of tensors / None; storages counted once."""
    logical, seen, physical = 0, set(), 0
    for t in tensors:
        if not torch.is_tensor(t):
            continue
        logical += t.numel() * t.element_size()
        st = t.untyped_storage()
        key = (st.data_ptr(), t.device)
        if key not in seen:
            seen.add(key)
            physical += st.nbytes()
    return logical / _MIB, physical / _MIB


def _state_tensors(optimizer):
    inner = getattr(optimizer, "optimizer", optimizer)  # a ShardedOptimizer wraps torch's
    for per_param in inner.state.values():
        yield from per_param.values()


@dataclass(frozen=True)
class MemoryReport:
    params_mb: float
    grads_mb: float
    optimizer_mb: float
    params_physical_mb: float
    grads_physical_mb: float
    optimizer_physical_mb: float
    allocated_mb: float
    max_allocated_mb: float
    placed_mb: float = 0.0
    placed_peak_mb: float = 0.0

    def lines(self, prefix: str, rank: int):
        out = [f"\nGPU {rank} - {prefix}:",
               f"  Model parameters: {self.params_mb:.2f} MB",
               f"  Gradients: {self.grads_mb:.2f} MB",
               f"  Optimizer states: {self.optimizer_mb:.2f} MB",
               f"  Total allocated: {self.allocated_mb:.2f} MB",
               f"  Max allocated: {self.max_allocated_mb:.2f} MB"]
        if self.placed_peak_mb:
            out.append(f"  Placed outside torch's allocator: {self.placed_mb:.2f} MB "
                       f"(peak {self.placed_peak_mb:.2f} MB incl. placement-probe candidates)")
            out.append(f"  Total incl. placed: {self.total_mb:.2f} MB "
                       f"(max <= {self.max_total_mb:.2f} MB, the sum of the two peaks)")
        return out + ["-" * 40]

    @property
    def total_mb(self) -> float:
        """torch's allocated + the placed buffers: the residency the reference's "Total
        allocated" counts (its state is all in torch's allocator)."""
        return self.allocated_mb + self.placed_mb

    @property
    def max_total_mb(self) -> float:
        """An upper bound of the combined peak (the two peaks need not coincide)."""
        return self.max_allocated_mb + self.placed_peak_mb


def memory_report(model, optimizer, device) -> MemoryReport:
    params = list(model.parameters())
    p_l, p_p = _walk(params)
    g_l, g_p = _walk(p.grad for p in params)
    o_l, o_p = _walk(_state_tensors(optimizer))
    on_gpu = torch.cuda.is_available() and torch.device(device).type == "cuda"
    from ..engine import placed_bytes, placed_peak_bytes

    placed = placed_bytes(device) / _MIB if on_gpu else 0.0
    placed_peak = placed_peak_bytes(device) / _MIB if on_gpu else 0.0
    alloc = torch.cuda.memory_allocated(device) / _MIB if on_gpu else 0.0
    peak = torch.cuda.max_memory_allocated(device) / _MIB if on_gpu else 0.0
    return MemoryReport(p_l, g_l, o_l, p_p, g_p, o_p, alloc, peak, placed, placed_peak)


def print_memory_stats(prefix: str, model, optimizer, rank, device):
    """memory.py:37-50's report (same lines), computed by ``memory_report``."""
    print("\n".join(memory_report(model, optimizer, device).lines(prefix, rank)))
