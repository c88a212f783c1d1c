"""Keras initializer names -> in-place torch initialisers on [out, ..., in] weights."""
from __future__ import annotations

import math

import torch


def _fans(t):
    if t.ndim < 2:
        return t.numel(), t.numel()
    out = t.shape[0]
    inn = t.numel() // out
    recept = t[0].numel() // t.shape[-1] if t.ndim > 2 else 1
    fan_in = inn
    fan_out = out * recept
    return fan_in, fan_out


def zeros(t):
    return torch.nn.init.zeros_(t)


def ones(t):
    return torch.nn.init.ones_(t)


def glorot_uniform(t):
    fi, fo = _fans(t)
    lim = math.sqrt(6.0 / (fi + fo))
    return torch.nn.init.uniform_(t, -lim, lim)


def glorot_normal(t):
    fi, fo = _fans(t)
    return torch.nn.init.normal_(t, 0.0, math.sqrt(2.0 / (fi + fo)))


def he_normal(t):
    fi, _ = _fans(t)
    return torch.nn.init.normal_(t, 0.0, math.sqrt(2.0 / fi))


def he_uniform(t):
    fi, _ = _fans(t)
    lim = math.sqrt(6.0 / fi)
    return torch.nn.init.uniform_(t, -lim, lim)


def random_normal(t, std=0.05):
    return torch.nn.init.normal_(t, 0.0, std)


def random_uniform(t, lim=0.05):
    return torch.nn.init.uniform_(t, -lim, lim)


_ALL = {"zeros": zeros, "ones": ones, "glorot_uniform": glorot_uniform, "glorot_normal": glorot_normal,
        "he_normal": he_normal, "he_uniform": he_uniform, "random_normal": random_normal,
        "random_uniform": random_uniform}


def get(identifier):
    if callable(identifier):
        return identifier
    try:
        return _ALL[identifier]
    except KeyError as e:
        raise ValueError(f"Unknown initializer {identifier!r}") from e
