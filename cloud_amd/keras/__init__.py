"""Keras-compatible high-level API on cloud_amd (``tf.keras`` names).

The reference's workloads are Keras programs (``TFC/core/tests/testdata``);
this package gives them a native MI355X runtime: ``layers``, ``Sequential`` /
``Model`` (functional + subclassed), ``compile``/``fit``/``evaluate``/``predict``
under the distribution strategies, ``optimizers`` (fused HIP kernels),
``losses``, ``metrics``, ``callbacks``, ``datasets``, ``applications`` and
save / load.  Layout is channels-last (NHWC).
"""
from . import activations, applications, callbacks, datasets, initializers, layers, losses, metrics, optimizers  # noqa
from . import regularizers  # noqa: F401
from .data import AUTOTUNE, Dataset  # noqa: F401
from .engine import Input, Layer, Policy, global_policy, set_global_policy  # noqa: F401
from .models import Model, Sequential, clone_model, load_model  # noqa: F401


class mixed_precision:  # namespace parity: tf.keras.mixed_precision
    Policy = Policy
    set_global_policy = staticmethod(set_global_policy)
    global_policy = staticmethod(global_policy)


class utils:
    @staticmethod
    def to_categorical(y, num_classes=None):
        import numpy as np

        y = np.asarray(y, dtype=np.int64).reshape(-1)
        n = num_classes or int(y.max()) + 1
        out = np.zeros((len(y), n), dtype=np.float32)
        out[np.arange(len(y)), y] = 1.0
        return out
