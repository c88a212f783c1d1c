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

from . import config as _ca_config
from . import keras  # noqa: F401
from .keras.data import AUTOTUNE as _AUTOTUNE
from .keras.data import Dataset as _Dataset
from .keras.losses import compute_average_loss as _cal
from .parallel import strategy as _st
from .version import __version__  # noqa: F401


class GradientTape:
    """``with tf.GradientTape() as tape: ...; tape.gradient(loss, vars)`` on autograd.

    Variables that live in a fused optimizer's flat arenas (after the first
    ``optimizer.apply_gradients``) take the runtime's training-step path:

    * the native Dense / Conv2D backward writes their weight gradients straight into the
      arena (``ops/dense.py``), so ``gradient()`` first zeroes the owning optimizer's
      gradient arena and then runs ``backward(inputs=sources)``, which accumulates every
      other gradient into the same arena slices;
    * under a multi-replica strategy, ``CLOUD_AMD_TAPE_REDUCE`` picks the semantics:
      ``overlap`` (default) -- the optimizer's bucketed all-reduce
      (:class:`cloud_amd.parallel.ddp.GradAllReducer`) launches each bucket from the backward
      hooks as its gradients complete (overlapped with the rest of backward) and is joined
      before ``gradient()`` returns: the returned gradients are the cross-replica SUM, as
      Horovod's ``DistributedGradientTape`` returns them, and ``apply_gradients`` does not
      reduce them again.  A non-linear transform between ``gradient()`` and
      ``apply_gradients`` (``clip_by_global_norm``) then sees the global sum.  ``replica`` --
      TF ``MirroredStrategy`` semantics: per-replica gradients, summed in
      ``apply_gradients`` (no overlap with backward);
    * the returned tensors are views of the arena (``v.grad``): no copy, and
      ``apply_gradients`` recognises them.  They are valid until the next ``gradient()``
      over the same variables; ``tf.identity``-style copies (``g.clone()``) keep them.  A
      ``persistent=True`` tape returns copies (a second ``gradient()`` overwrites the arena).

    Other sources (plain tensors, variables before the optimizer's first step) get
    ``torch.autograd.grad`` results (zeros for unconnected sources).  Reference pattern:
    ``TFC/core/tests/testdata/mnist_example_using_ctl.py:124-129``.
    """

    def __init__(self, persistent=False, watch_accessed_variables=True):
        self.persistent = persistent

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def watch(self, tensor):
        if isinstance(tensor, torch.Tensor) and not tensor.requires_grad:
            tensor.requires_grad_(True)

    @staticmethod
    def _owners(srcs):
        owners = {}
        for s in srcs:
            ref = getattr(s, "_ca_opt", None) if getattr(s, "_ca_arena", False) else None
            opt = ref() if ref is not None else None
            if opt is not None:
                owners[id(opt)] = opt
        return list(owners.values())

    def gradient(self, target, sources, output_gradients=None):
        single = isinstance(sources, torch.Tensor)
        srcs = [sources] if single else list(sources)
        owners = self._owners(srcs)
        for opt in owners:
            opt.zero_grad()  # the arena slots are accumulated into in place
        for opt in owners:
            opt._ca_tape_fresh = True  # apply_gradients: these slots were written this step
        reducers = [o.reducer for o in owners if getattr(o, "reducer", None) is not None and o.reducer.world > 1]
        overlap = _ca_config.get("CLOUD_AMD_TAPE_REDUCE") == "overlap"
        if owners and all(getattr(s, "_ca_arena", False) and s.grad is not None for s in srcs):
            if overlap:
                target.backward(gradient=output_gradients, inputs=srcs, retain_graph=self.persistent)
                for r in reducers:
                    r.finish()  # buckets launched during backward; the compute stream joins them
                    r.tape_reduced = True
            else:  # per-replica gradients (TF semantics): apply_gradients reduces them
                self._backward_unreduced(reducers, lambda: target.backward(
                    gradient=output_gradients, inputs=srcs, retain_graph=self.persistent))
            out = [s.grad for s in srcs]
            if self.persistent:
                # a persistent tape may be asked again: the next gradient() re-zeroes and
                # overwrites the arena, so the caller keeps copies, not views
                out = [g.clone() for g in out]
            return out[0] if single else out
        # mixed / non-arena sources: no bucket may launch while autograd.grad runs (the copies
        # apply_gradients makes would race a reduction already in flight); the optimizer
        # reduces the whole arena in apply_gradients instead
        box = []
        self._backward_unreduced(reducers, lambda: box.append(torch.autograd.grad(
            target, srcs, grad_outputs=output_gradients, allow_unused=True, retain_graph=self.persistent)))
        grads = box[0]
        out = []
        for g, s in zip(grads, srcs):
            if g is None and getattr(s, "_ca_arena", False) and s.grad is not None:
                g = s.grad  # written in place by a native backward (autograd saw no gradient)
            out.append(g if g is not None else torch.zeros_like(s))
        return out[0] if single else out


def _backward_unreduced_impl(reducers, fn):
    """Run ``fn`` (a backward) with the reducers' bucket launches off; they are reset after,
    so ``apply_gradients`` all-reduces the whole arena."""
    prev = [(r, r._sync_enabled) for r in reducers]
    for r, _ in prev:
        r._sync_enabled = False
    try:
        fn()
    finally:
        for r, was in prev:
            r._sync_enabled = was
            r.reset()
            r.tape_reduced = False


GradientTape._backward_unreduced = staticmethod(_backward_unreduced_impl)


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
