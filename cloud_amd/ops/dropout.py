"""Dropout (K8) and the host side of the stateless dropout RNG.

Every dropping kernel (LayerNorm in/out dropout, attention-probability dropout,
standalone dropout) derives its keep-mask from ``hash(seed, element_index)``
(``csrc/include/ca_rng.h``), so the backward regenerates the mask from the
seed saved on the autograd context instead of storing it.  Seeds come from a
per-process counter started from ``torch.initial_seed()`` (reproducible under
``torch.manual_seed``) -- no device synchronisation, capturable.
"""
from __future__ import annotations

import torch

from . import _ext, raw

_state = {"base": None, "ctr": 0}


def manual_seed(seed: int):
    _state["base"] = int(seed) & 0x7FFFFFFFFFFFFFFF
    _state["ctr"] = 0


def next_seed() -> int:
    if _state["base"] is None:
        _state["base"] = int(torch.initial_seed()) & 0x7FFFFFFFFFFFFFFF
    _state["ctr"] += 1
    return (_state["base"] * 0x9E3779B1 + _state["ctr"] * 0x632BE5AB) & 0x7FFFFFFFFFFFFFFF


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        ctx.p, ctx.seed = p, seed
        return raw.dropout(x.contiguous(), p, seed)

    @staticmethod
    def backward(ctx, dy):
        return raw.dropout(dy.contiguous(), ctx.p, ctx.seed), None, None


def dropout(x, p=0.5, training=True):
    """Inverted dropout; HIP kernel for bf16 CUDA tensors, torch otherwise."""
    if not training or p <= 0.0:
        return x
    if x.dtype == torch.bfloat16 and x.numel() % 8 == 0 and _ext.use_native(x):
        return _DropoutFn.apply(x, float(p), next_seed())
    return torch.nn.functional.dropout(x, p, training=True)
