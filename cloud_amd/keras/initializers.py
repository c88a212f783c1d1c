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


class Initializer:
    """Keras initializer object: called on the weight tensor in cloud_amd's layout
    (dense ``[out, in]``, conv ``[out, kh, kw, in]``)."""

    def __call__(self, t):  # pragma: no cover - abstract
        raise NotImplementedError


class Constant(Initializer):
    """``Constant(value)``: a scalar fills; an array is taken in Keras's layout
    (dense ``[in, out]``, conv ``[kh, kw, in, out]``) or in cloud_amd's, whichever matches."""

    def __init__(self, value=0.0):
        self.value = value

    def __call__(self, t):
        import numpy as np

        v = np.asarray(self.value, dtype=np.float32)
        with torch.no_grad():
            if v.ndim == 0 or v.size == 1:
                return t.fill_(float(v.reshape(-1)[0]))
            if tuple(v.shape) == tuple(t.shape):
                src = v
            elif v.ndim == 2 and tuple(v.T.shape) == tuple(t.shape):
                src = v.T
            elif v.ndim == 4 and tuple(np.transpose(v, (3, 0, 1, 2)).shape) == tuple(t.shape):
                src = np.transpose(v, (3, 0, 1, 2))
            else:
                src = np.broadcast_to(v, tuple(t.shape))
            return t.copy_(torch.from_numpy(np.ascontiguousarray(src)).to(t.dtype))


class _Named(Initializer):
    fn = None

    def __init__(self, *args, **kwargs):
        self.args, self.kwargs = args, kwargs

    def __call__(self, t):
        return type(self).fn(t, *self.args, **self.kwargs)


class Zeros(_Named):
    fn = staticmethod(zeros)


class Ones(_Named):
    fn = staticmethod(ones)


class GlorotUniform(_Named):
    fn = staticmethod(glorot_uniform)


class GlorotNormal(_Named):
    fn = staticmethod(glorot_normal)


class HeNormal(_Named):
    fn = staticmethod(he_normal)


class HeUniform(_Named):
    fn = staticmethod(he_uniform)


class RandomNormal(Initializer):
    def __init__(self, mean=0.0, stddev=0.05, seed=None):
        self.mean, self.stddev = mean, stddev

    def __call__(self, t):
        return torch.nn.init.normal_(t, self.mean, self.stddev)


class RandomUniform(Initializer):
    def __init__(self, minval=-0.05, maxval=0.05, seed=None):
        self.minval, self.maxval = minval, maxval

    def __call__(self, t):
        return torch.nn.init.uniform_(t, self.minval, self.maxval)


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
