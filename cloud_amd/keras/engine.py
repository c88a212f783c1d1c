"""Keras-style layer engine on PyTorch modules.

``Layer`` is an ``nn.Module`` that builds its weights lazily from the first
input shape (Keras semantics) and can be called either on real tensors or on
symbolic :class:`KerasTensor` placeholders (functional API).  Layout is
channels-last (NHWC), which is also the native layout of the MI355X kernels.

Mixed precision (``mixed_precision.set_global_policy("mixed_bfloat16")``):
matrix weights are created in bf16 (the optimizer's flat arena keeps their
fp32 master copy), normalisation parameters stay fp32, and the model's final
outputs are returned as fp32 -- the ``mixed_bfloat16`` policy of Keras.
"""
from __future__ import annotations

import itertools
import os

import numpy as np
import torch
import torch.nn as nn

_uid = itertools.count()
_name_counts: dict = {}


def _unique_name(base):
    n = _name_counts.get(base, 0)
    _name_counts[base] = n + 1
    return base if n == 0 else f"{base}_{n}"


def _snake(name):
    out = []
    for i, ch in enumerate(name):
        if ch.isupper() and i and not name[i - 1].isupper():
            out.append("_")
        out.append(ch.lower())
    return "".join(out)


def _auto_policy_name():
    """``CLOUD_AMD_PRECISION=auto`` (default): ``mixed_bfloat16`` when this process
    trains on an MI355X, else ``float32``.  Decided from the KFD device count and the
    launcher's device pin -- never by initialising HIP.  This is the MI355X analogue
    of TF's default on current GPUs, where "float32" Dense/Conv2D math already runs
    at reduced (TF32) precision on the matrix units: here the matrix work is bf16 on
    MFMA with fp32 master weights, fp32 losses and fp32 model outputs."""
    if os.environ.get("CLOUD_AMD_DEVICE") == "cpu":
        return "float32"
    try:
        from ..core.topology import visible_gpu_count

        return "mixed_bfloat16" if visible_gpu_count() > 0 else "float32"
    except Exception:  # pragma: no cover
        return "float32"


class Policy:
    def __init__(self, name="float32"):
        if name == "auto":
            name = _auto_policy_name()
        if name not in ("float32", "mixed_bfloat16", "bfloat16"):
            raise ValueError(f"Unsupported dtype policy {name!r}")
        self.name = name

    @property
    def compute_dtype(self):
        return torch.float32 if self.name == "float32" else torch.bfloat16

    @property
    def variable_dtype(self):
        return torch.bfloat16 if self.name == "bfloat16" else torch.float32

    def __repr__(self):
        return f"<Policy {self.name}>"


_POLICY = None


def global_policy():
    global _POLICY
    if _POLICY is None:  # resolved on first use (after the launcher has pinned the device)
        _POLICY = Policy(os.environ.get("CLOUD_AMD_PRECISION", "auto"))
    return _POLICY


def set_global_policy(policy):
    global _POLICY
    _POLICY = policy if isinstance(policy, Policy) else Policy(policy)


class KerasTensor:
    """Symbolic tensor of the functional API: shape (with None batch) + producing node."""

    def __init__(self, shape, layer=None, inputs=(), name=None, dtype="float32"):
        self.shape = tuple(shape)
        self.layer = layer
        self.inputs = tuple(inputs)
        self.name = name or f"kt_{next(_uid)}"
        self.dtype = dtype
        self.id = next(_uid)

    def __repr__(self):
        return f"<KerasTensor shape={self.shape} from={getattr(self.layer, 'name', None)}>"


def _shape_of(x):
    if isinstance(x, KerasTensor):
        return x.shape
    if isinstance(x, (list, tuple)):
        return [_shape_of(t) for t in x]
    return (None,) + tuple(x.shape[1:])


class Layer(nn.Module):
    """Base Keras layer: lazy ``build``, ``call``, config round-trip, numpy weights."""

    def __init__(self, name=None, trainable=True, dtype=None, input_shape=None, batch_input_shape=None, **kwargs):
        super().__init__()
        self.name = name or _unique_name(_snake(type(self).__name__))
        self._trainable = trainable
        self.built = False
        self._dtype_policy = Policy(dtype) if isinstance(dtype, str) and dtype in (
            "float32", "mixed_bfloat16", "bfloat16") else global_policy()
        if batch_input_shape is not None:
            input_shape = tuple(batch_input_shape[1:])
        self._input_shape_arg = tuple(input_shape) if input_shape is not None else None
        self.input_spec = None
        self._build_shape = None

    # -- properties ------------------------------------------------------------
    @property
    def compute_dtype(self):
        return self._dtype_policy.compute_dtype

    @property
    def trainable(self):
        return self._trainable

    @trainable.setter
    def trainable(self, v):
        self._trainable = bool(v)
        for p in self.parameters():
            p.requires_grad_(self._trainable)

    @property
    def weights(self):
        return list(self.parameters())

    @property
    def trainable_weights(self):
        return [p for p in self.parameters() if p.requires_grad]

    trainable_variables = trainable_weights

    @property
    def non_trainable_weights(self):
        return [p for p in self.parameters() if not p.requires_grad] + list(self.buffers())

    # -- building ----------------------------------------------------------------
    def build(self, input_shape):
        self.built = True

    def _maybe_build(self, input_shape, device=None):
        if not self.built:
            self._build_shape = input_shape
            self.build(input_shape)
            self.built = True
            if device is not None:
                self.to(device)
            if not self._trainable:
                for p in self.parameters():
                    p.requires_grad_(False)

    def add_weight(self, name, shape, initializer="zeros", dtype=None, trainable=True):
        from . import initializers

        t = torch.empty(tuple(shape), dtype=torch.float32)
        initializers.get(initializer)(t)
        p = nn.Parameter(t.to(dtype or torch.float32), requires_grad=trainable)
        self.register_parameter(name, p)
        return p

    def compute_output_shape(self, input_shape):
        """Symbolic shape inference by running the layer on a zero batch of 1 (CPU)."""
        def mk(s):
            return torch.zeros((1,) + tuple(d if d is not None else 1 for d in s[1:]))

        with torch.no_grad():
            x = [mk(s) for s in input_shape] if isinstance(input_shape, list) else mk(input_shape)
            self._maybe_build(input_shape)
            was = self.training
            self.eval()
            try:
                y = self.call(x)
            finally:
                self.train(was)
        if isinstance(y, (list, tuple)):
            return [(None,) + tuple(t.shape[1:]) for t in y]
        return (None,) + tuple(y.shape[1:])

    # -- calling -----------------------------------------------------------------
    def call(self, inputs, training=None):  # pragma: no cover - abstract
        return inputs

    def _eager_device(self):
        for p in self.parameters():
            return p.device
        from ..parallel.strategy import get_strategy

        return get_strategy().device or torch.device("cpu")

    def _convert_inputs(self, inputs):
        """numpy / python inputs -> tensors on the model's (or strategy's) device, floats as float32."""
        def conv(a):
            if isinstance(a, (np.ndarray, np.generic)):
                t = torch.as_tensor(np.asarray(a))
                if t.is_floating_point():
                    t = t.float()
                return t.to(self._eager_device())
            return a

        if isinstance(inputs, (list, tuple)):
            return type(inputs)(conv(a) for a in inputs)
        return conv(inputs)

    def __call__(self, inputs, *args, **kwargs):
        inputs = self._convert_inputs(inputs)
        symbolic = isinstance(inputs, KerasTensor) or (
            isinstance(inputs, (list, tuple)) and inputs and all(isinstance(t, KerasTensor) for t in inputs))
        if symbolic:
            ins = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
            shape = self.compute_output_shape(_shape_of(inputs))
            if isinstance(shape, list):
                return [KerasTensor(s, self, ins) for s in shape]
            return KerasTensor(shape, self, ins)
        dev = None
        first = inputs[0] if isinstance(inputs, (list, tuple)) else inputs
        if isinstance(first, torch.Tensor):
            dev = first.device
        self._maybe_build(_shape_of(inputs), dev)
        return super().__call__(inputs, *args, **kwargs)

    def forward(self, inputs, training=None, **kwargs):
        return self.call(inputs, training=self.training if training is None else training, **kwargs)

    # -- config / weights -----------------------------------------------------------
    def get_config(self):
        cfg = {"name": self.name, "trainable": self._trainable}
        if self._input_shape_arg is not None:
            cfg["input_shape"] = list(self._input_shape_arg)
        return cfg

    @classmethod
    def from_config(cls, config):
        return cls(**config)

    def get_weights(self):
        return [t.detach().float().cpu().numpy() for t in itertools.chain(self.parameters(), self.buffers())]

    def set_weights(self, weights):
        tensors = list(itertools.chain(self.parameters(), self.buffers()))
        if len(weights) != len(tensors):
            raise ValueError(f"expected {len(tensors)} weight arrays, got {len(weights)}")
        with torch.no_grad():
            for t, w in zip(tensors, weights):
                t.copy_(torch.as_tensor(np.asarray(w)).to(t.dtype).reshape(t.shape))

    def count_params(self):
        return int(sum(p.numel() for p in self.parameters()))

    def extra_repr(self):
        return self.name


class InputLayer(Layer):
    def __init__(self, input_shape=None, batch_size=None, dtype=None, name=None, **kw):
        super().__init__(name=name or _unique_name("input"), input_shape=input_shape, **kw)
        self.built = True

    def call(self, inputs, training=None):
        return inputs


def Input(shape=None, batch_size=None, name=None, dtype=None):
    """Functional-API placeholder (``tf.keras.Input``)."""
    layer = InputLayer(input_shape=shape, name=name)
    kt = KerasTensor((None,) + tuple(shape), layer, (), name=layer.name)
    kt.is_input = True
    return kt
