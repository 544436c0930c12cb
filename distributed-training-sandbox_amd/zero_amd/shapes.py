"""Synthetic parameter sets of BASELINE.json's configs.

C1-C3: the reference harness MLP, 6 × nn.Linear(D, D) (zero1.py:237-249) → 12 tensors.
C4: SmolLM3-3B (transformers.SmolLM3Config defaults: hidden 2048, intermediate 11008, 36 layers,
    16 heads / 4 KV heads of 128, vocab 128256, tied embeddings) → 326 tensors, 3,075,098,624 params.
C5: Llama-3.1-8B (hidden 4096, intermediate 14336, 32 layers, 32 / 8 heads, vocab 128256,
    untied lm_head) → 291 tensors, 8,030,261,248 params.
Order follows HF ``named_parameters()`` (embed, per layer q,k,v,o,gate,up,down, two norms, final
norm, lm_head).
"""
from __future__ import annotations


def mlp_shapes(D: int, layers: int = 6):
    out = []
    for _ in range(layers):
        out += [(D, D), (D,)]
    return out


def _decoder(vocab, hidden, inter, layers, kv_dim, tied):
    out = [(vocab, hidden)]
    for _ in range(layers):
        out += [(hidden, hidden), (kv_dim, hidden), (kv_dim, hidden), (hidden, hidden),
                (inter, hidden), (inter, hidden), (hidden, inter), (hidden,), (hidden,)]
    out.append((hidden,))
    if not tied:
        out.append((vocab, hidden))
    return out


def smollm3_3b_shapes():
    return _decoder(128256, 2048, 11008, 36, 4 * 128, tied=True)


def llama31_8b_shapes():
    return _decoder(128256, 4096, 14336, 32, 8 * 128, tied=False)


def decoder_shapes(config: str, layers: int):
    """C4 / C5 with ``layers`` decoder layers (test-size copies of the sets)."""
    if config == "C4":
        return _decoder(128256, 2048, 11008, layers, 4 * 128, tied=True)
    if config == "C5":
        return _decoder(128256, 4096, 14336, layers, 8 * 128, tied=False)
    raise ValueError(f"{config} is not a decoder parameter set")


CONFIGS = {
    "C1": ("reference MLP 6xLinear(10000,10000)", lambda: mlp_shapes(10000)),
    "C2": ("MLP 6xLinear(4096,4096)", lambda: mlp_shapes(4096)),
    "C3": ("MLP 6xLinear(12800,12800)", lambda: mlp_shapes(12800)),
    "C4": ("SmolLM3-3B", smollm3_3b_shapes),
    "C5": ("Llama-3.1-8B", llama31_8b_shapes),
}
