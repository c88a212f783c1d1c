"""Keras-named activations (``tf.keras.activations``) on torch tensors."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def linear(x):
    return x


def relu(x):
    return torch.relu(x)


def elu(x):
    return F.elu(x)


def selu(x):
    return F.selu(x)


def gelu(x):
    return F.gelu(x)


def tanh(x):
    return torch.tanh(x)


def sigmoid(x):
    return torch.sigmoid(x)


def softmax(x):
    return torch.softmax(x.float(), dim=-1).to(x.dtype) if x.dtype != torch.float32 else torch.softmax(x, dim=-1)


def softplus(x):
    return F.softplus(x)


def swish(x):
    return F.silu(x)


_ALL = {"linear": linear, None: linear, "relu": relu, "elu": elu, "selu": selu, "gelu": gelu, "tanh": tanh,
        "sigmoid": sigmoid, "softmax": softmax, "softplus": softplus, "swish": swish, "silu": swish}


def get(identifier):
    if callable(identifier):
        return identifier
    try:
        return _ALL[identifier]
    except KeyError as e:
        raise ValueError(f"Unknown activation: {identifier!r}") from e


def serialize(fn):
    for k, v in _ALL.items():
        if v is fn and k is not None:
            return k
    return getattr(fn, "__name__", "linear")
