"""SmolLM3 training step on the MI355X ZeRO optimizer.

The reference's FSDP2 script (fsdp/train_fsdp.py:56-170) builds SmolLM3-3B from its config in bf16,
shards it with ``fully_shard`` and steps ``torch.optim.AdamW(lr=1e-5)``, quoting 1849 tok/s
(ZeRO-3-like) / 3000 tok/s (ZeRO-2-like) on two A100-80GB (train_fsdp.py:85-86).  Here the same
model (``transformers`` SmolLM3, random init — no checkpoint download) trains with
``zero_amd.zero2.ShardedOptimizer(AdamW)`` in backward-overlapped mode: grads accumulate into
per-owner buckets whose RCCL reduces start during backward, the fused HIP AdamW (bf16 params,
fp32 master / exp_avg / exp_avg_sq) updates each rank's shard, and the updated bf16 params are
broadcast back.  The forward / backward GEMMs and attention are the caller's (PyTorch-ROCm).
"""
from __future__ import annotations

import torch


def smollm3_config(layers: int | None = None, hidden: int | None = None,
                   intermediate: int | None = None, heads: int | None = None,
                   kv_heads: int | None = None, vocab: int | None = None):
    """SmolLM3-3B (transformers.SmolLM3Config defaults) or a shrunken copy for tests."""
    from transformers import SmolLM3Config

    kw = dict(use_cache=False)
    for k, v in (("num_hidden_layers", layers), ("hidden_size", hidden),
                 ("intermediate_size", intermediate), ("num_attention_heads", heads),
                 ("num_key_value_heads", kv_heads), ("vocab_size", vocab)):
        if v is not None:
            kw[k] = v
    if vocab is not None:  # the default special-token ids point past a small vocabulary
        kw.update(pad_token_id=None, bos_token_id=None, eos_token_id=None)
    cfg = SmolLM3Config(**kw)
    if layers is not None and getattr(cfg, "no_rope_layers", None) is not None:
        cfg.no_rope_layers = list(cfg.no_rope_layers)[:layers]
    return cfg


def build_model(cfg, device, dtype=torch.bfloat16, seed: int = 42):
    """train_fsdp.py:62-65 (``from_config``, bf16), seeded as train_fsdp.py:56."""
    from transformers import SmolLM3ForCausalLM

    torch.manual_seed(seed)
    with torch.device(device):  # initialise on the GPU (3B params: seconds, not a CPU minute)
        model = SmolLM3ForCausalLM(cfg)
    model = model.to(dtype=dtype)
    model.train()
    return model


def model_flops_per_token(cfg, seq_len: int) -> float:
    """The reference's accounting, fsdp/utils.py:94-115 (embeddings and norms ignored)."""
    head_dim = cfg.hidden_size // cfg.num_attention_heads
    mlp = 18 * cfg.hidden_size * cfg.intermediate_size
    attn = 12 * head_dim * (cfg.num_attention_heads + cfg.num_key_value_heads)
    attn_dot = 12 * cfg.num_attention_heads * head_dim * seq_len
    return float((mlp + attn + attn_dot) * cfg.num_hidden_layers)


def train_step(model, optimizer, input_ids):
    """train_fsdp.py:140-160: forward (causal-LM loss on the inputs), backward, step, zero_grad."""
    loss = model(input_ids=input_ids, labels=input_ids).loss
    loss.backward()
    optimizer.step()
    optimizer.zero_grad()
    return loss
