"""A module tree over a synthetic parameter set, so the ZeRO-3 hooks can drive it.

BASELINE.json configs[4] (and configs[3] for ZeRO-3) are *parameter sets* — SmolLM3-3B / Llama-3.1-8B
shapes with synthetic gradients — not models.  To run them through the
reference's ZeRO-3 machinery (zero3.py:56-77: gather in the forward / backward pre-hooks, release
in the post-hooks, reduce the gradients) each decoder layer's tensors become one ``nn.Module``
whose forward is a custom autograd function: forward passes a tiny activation through, backward
hands every parameter its gradient from a *gradient source* (by default fixed synthetic tensors
resident in HBM, returned as fresh aliases — ``detach()``: a new tensor on the same storage — so
autograd's AccumulateGrad adopts them without a copy).
The gathered weights are not multiplied with anything: an iteration is exactly ZeRO-3's
communication and update — all-gather per layer in forward, again in backward, reduce-scatter of
the gradients, fused Adam on the chunks.
"""
from __future__ import annotations

import torch
from torch import nn


def decoder_layer_groups(n_params: int, per_layer: int = 9, n_layers: int | None = None):
    """Parameter-index groups of a shapes._decoder set: [embed], one group per decoder layer
    (q, k, v, o, gate, up, down, 2 norms), then the tail (final norm [+ untied lm_head])."""
    if n_layers is None:
        n_layers = (n_params - 2) // per_layer
    groups = [[0]]
    for layer in range(n_layers):
        groups.append(list(range(1 + layer * per_layer, 1 + (layer + 1) * per_layer)))
    groups.append(list(range(1 + n_layers * per_layer, n_params)))
    assert sum(len(g) for g in groups) == n_params
    return groups


class _PassThrough(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, layer, *params):
        ctx.layer = layer
        return x.view_as(x)  # an alias: no kernel launch, just an autograd node per layer

    @staticmethod
    def backward(ctx, gx):
        return (gx, None, *ctx.layer.grads())


class ParamLayer(nn.Module):
    def __init__(self, params):
        super().__init__()
        self.n = len(params)
        for k, p in enumerate(params):  # direct parameters: the hooks gather recurse=False
            self.register_parameter(f"p{k}", p)
        self.grad_source = None  # callable -> list of full-shape tensors, one per parameter

    def grads(self):
        return self.grad_source()

    def forward(self, x):
        # the registered parameters p0 … p{n-1} in order (the dict itself: no per-name lookups)
        return _PassThrough.apply(x, self, *self._parameters.values())


class ParamSetModel(nn.Module):
    """``groups`` of ``params`` as a sequence of ParamLayer modules (parameter order kept)."""

    def __init__(self, params, groups):
        super().__init__()
        self.layers = nn.ModuleList(ParamLayer([params[i] for i in g]) for g in groups)
        self.groups = [list(g) for g in groups]

    def set_grad_source(self, grads):
        """Every backward hands parameter i the tensor grads[i] (as a fresh alias, no copy: the
        alias is referenced only by autograd, so AccumulateGrad adopts it instead of cloning)."""
        for layer, g in zip(self.layers, self.groups):
            srcs = [grads[i] for i in g]
            layer.grad_source = lambda srcs=srcs: [t.detach() for t in srcs]

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x
