"""TensorFlow-shaped namespace over cloud_amd: ``from cloud_amd import tf``.

The reference's workloads (``TFC/core/tests/testdata/*.py``, ``.../examples``)
are TF-2 Keras programs.  This module exposes the subset of the ``tf.*`` names
they use, mapped onto the cloud_amd runtime, so such a script ports by changing
its import line:

* ``tf.keras``                      -> :mod:`cloud_amd.keras`
* ``tf.distribute.*Strategy`` / ``ReduceOp`` / ``experimental_set_strategy``
* ``tf.data.Dataset`` / ``AUTOTUNE``
* ``tf.GradientTape``               -> torch autograd (``tape.gradient``)
* ``tf.function``                   -> identity decorator (eager PyTorch: HIP-graph
  capture of a training step measured no faster than eager on ROCm 7.2, so none is offered)
* ``tf.nn.compute_average_loss``, ``tf.config.list_physical_devices``

This is an API-name layer for user scripts, not a numerics or device shim:
everything underneath is the MI355X path.
"""
from __future__ import annotations

import types

import torch

from . import keras  # noqa: F401
from .keras.data import AUTOTUNE as _AUTOTUNE
from .keras.data import Dataset as _Dataset
from .keras.losses import compute_average_loss as _cal
from .parallel import strategy as _st
from .version import __version__  # noqa: F401


class GradientTape:
    """``with tf.GradientTape() as tape: ...; tape.gradient(loss, vars)`` on autograd."""

    def __init__(self, persistent=False, watch_accessed_variables=True):
        self.persistent = persistent

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def watch(self, tensor):
        if isinstance(tensor, torch.Tensor) and not tensor.requires_grad:
            tensor.requires_grad_(True)

    def gradient(self, target, sources):
        single = isinstance(sources, torch.Tensor)
        srcs = [sources] if single else list(sources)
        grads = torch.autograd.grad(target, srcs, allow_unused=True, retain_graph=self.persistent)
        out = [g if g is not None else torch.zeros_like(s) for g, s in zip(grads, srcs)]
        return out[0] if single else out


def function(fn=None, **_kw):
    """``@tf.function``: runs eagerly (identity)."""
    if fn is None:
        return lambda f: f
    return fn


distribute = types.SimpleNamespace(
    OneDeviceStrategy=_st.OneDeviceStrategy,
    MirroredStrategy=_st.MirroredStrategy,
    MultiWorkerMirroredStrategy=_st.MultiWorkerMirroredStrategy,
    ReduceOp=_st.ReduceOp,
    experimental_set_strategy=_st.experimental_set_strategy,
    get_strategy=_st.get_strategy,
    has_strategy=_st.has_strategy,
    experimental=types.SimpleNamespace(MultiWorkerMirroredStrategy=_st.MultiWorkerMirroredStrategy,
                                       TPUStrategy=_st.TPUStrategy),
    cluster_resolver=types.SimpleNamespace(TFConfigClusterResolver=_st.ClusterResolver.from_env),
)

data = types.SimpleNamespace(Dataset=_Dataset, AUTOTUNE=_AUTOTUNE,
                             experimental=types.SimpleNamespace(AUTOTUNE=_AUTOTUNE))

nn = types.SimpleNamespace(compute_average_loss=_cal)


def _list_physical_devices(device_type=None):
    devs = []
    if device_type in (None, "CPU"):
        devs.append(types.SimpleNamespace(name="/physical_device:CPU:0", device_type="CPU"))
    if device_type in (None, "GPU") and torch.cuda.is_available():
        devs += [types.SimpleNamespace(name=f"/physical_device:GPU:{i}", device_type="GPU")
                 for i in range(torch.cuda.device_count())]
    return devs


config = types.SimpleNamespace(list_physical_devices=_list_physical_devices,
                               experimental=types.SimpleNamespace(list_physical_devices=_list_physical_devices))


def constant(value, dtype=None):
    return torch.as_tensor(value, dtype=dtype)


float32, int32, int64, bfloat16 = torch.float32, torch.int32, torch.int64, torch.bfloat16
