"""Weight regularizers (``tf.keras.regularizers``): L1, L2, L1L2.

A layer built with ``kernel_regularizer=`` / ``bias_regularizer=`` reports
``regularization_loss()``; ``Model.train_step`` adds the sum over layers to the
training loss (the reference's cloud_fit model uses ``l2(0.01)``,
``TFC/experimental/cloud_fit/tests/unit/client_test.py:72-84``).  Penalties are
computed in fp32 on the (possibly bf16) weights.
"""
from __future__ import annotations


class Regularizer:
    def __call__(self, w):  # pragma: no cover - abstract
        raise NotImplementedError

    def get_config(self):
        return {}


class L1L2(Regularizer):
    def __init__(self, l1=0.0, l2=0.0):
        self.l1, self.l2 = float(l1), float(l2)

    def __call__(self, w):
        w = w.float()
        out = 0.0
        if self.l1:
            out = out + self.l1 * w.abs().sum()
        if self.l2:
            out = out + self.l2 * (w * w).sum()
        return out

    def get_config(self):
        return {"l1": self.l1, "l2": self.l2}


class L1(L1L2):
    def __init__(self, l1=0.01):
        super().__init__(l1=l1)


class L2(L1L2):
    def __init__(self, l2=0.01):
        super().__init__(l2=l2)


def l1(l1=0.01):  # noqa: E741 - Keras name
    return L1(l1)


def l2(l2=0.01):
    return L2(l2)


def l1_l2(l1=0.01, l2=0.01):  # noqa: E741
    return L1L2(l1, l2)


_NAMES = {"l1": L1, "l2": L2, "l1_l2": L1L2}


def get(identifier):
    if identifier is None or isinstance(identifier, Regularizer):
        return identifier
    if callable(identifier):
        return identifier
    if isinstance(identifier, str) and identifier in _NAMES:
        return _NAMES[identifier]()
    if isinstance(identifier, dict):
        return L1L2(**identifier.get("config", identifier))
    raise ValueError(f"Unknown regularizer {identifier!r}")


def serialize(reg):
    if reg is None:
        return None
    return {"class_name": "L1L2", "config": reg.get_config()} if isinstance(reg, Regularizer) else None
