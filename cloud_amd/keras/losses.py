"""Keras losses (``tf.keras.losses``) with the distributed-averaging convention.

``SparseCategoricalCrossentropy(from_logits=True)`` runs the fused HIP
softmax-xent kernel (loss + dlogits in one pass) on MI355X.  When the model's
last layer is a softmax and ``from_logits=False`` (the reference's MNIST
models, ``mnist_example_using_fit.py:61-66``), ``Model.fit`` feeds the
pre-softmax logits to the same fused kernel -- mathematically identical,
numerically better.

Reductions follow Keras: ``SUM_OVER_BATCH_SIZE`` (default, ``AUTO``), ``SUM``,
``NONE``; :func:`compute_average_loss` is ``tf.nn.compute_average_loss``
(per-example losses summed and divided by the GLOBAL batch size, used by the
reference custom training loop ``mnist_example_using_ctl.py:93-101``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import ops


class Reduction:
    AUTO = "auto"
    NONE = "none"
    SUM = "sum"
    SUM_OVER_BATCH_SIZE = "sum_over_batch_size"


def _reduce(per, reduction):
    if reduction == Reduction.NONE:
        return per
    if reduction == Reduction.SUM:
        return per.sum()
    return per.mean()


class Loss:
    name = "loss"

    def __init__(self, reduction=Reduction.AUTO, name=None):
        self.reduction = reduction
        if name:
            self.name = name

    def __call__(self, y_true, y_pred, sample_weight=None):
        if not isinstance(y_true, torch.Tensor):
            y_true = torch.as_tensor(y_true).to(y_pred.device)
        per = self.per_example(y_true, y_pred)
        if sample_weight is not None:
            per = per * torch.as_tensor(sample_weight, device=per.device, dtype=per.dtype)
        return _reduce(per, self.reduction)

    def get_config(self):
        return {"reduction": self.reduction, "name": self.name}


class SparseCategoricalCrossentropy(Loss):
    name = "sparse_categorical_crossentropy"

    def __init__(self, from_logits=False, reduction=Reduction.AUTO, name=None, label_smoothing=0.0):
        super().__init__(reduction, name)
        self.from_logits = from_logits
        self.label_smoothing = label_smoothing

    def per_example(self, y_true, y_pred):
        y = y_true.reshape(-1).long()
        if self.from_logits:
            return F.cross_entropy(y_pred.float(), y, reduction="none", label_smoothing=self.label_smoothing)
        p = y_pred.float().clamp_min(1e-7)
        return F.nll_loss(torch.log(p / p.sum(-1, keepdim=True)), y, reduction="none")

    def fused_logits_loss(self, logits, y_true, acc=None, acc_weight=1.0):
        """(mean loss, correct flags) via the fused softmax-xent kernel; ``acc`` (device fp32
        [3]) accumulates [loss sum, correct count, rows] for the metrics inside the kernel."""
        return ops.softmax_cross_entropy(logits, y_true.reshape(-1), label_smoothing=self.label_smoothing, acc=acc,
                                         acc_weight=acc_weight)


class CategoricalCrossentropy(Loss):
    name = "categorical_crossentropy"

    def __init__(self, from_logits=False, reduction=Reduction.AUTO, name=None, label_smoothing=0.0):
        super().__init__(reduction, name)
        self.from_logits, self.label_smoothing = from_logits, label_smoothing

    def per_example(self, y_true, y_pred):
        t = y_true.float()
        if self.label_smoothing:
            t = t * (1 - self.label_smoothing) + self.label_smoothing / t.shape[-1]
        if self.from_logits:
            return -(t * torch.log_softmax(y_pred.float(), -1)).sum(-1)
        p = y_pred.float().clamp_min(1e-7)
        return -(t * torch.log(p / p.sum(-1, keepdim=True))).sum(-1)


class BinaryCrossentropy(Loss):
    name = "binary_crossentropy"

    def __init__(self, from_logits=False, reduction=Reduction.AUTO, name=None):
        super().__init__(reduction, name)
        self.from_logits = from_logits

    def per_example(self, y_true, y_pred):
        t = y_true.float().reshape(y_pred.shape)
        if self.from_logits:
            per = F.binary_cross_entropy_with_logits(y_pred.float(), t, reduction="none")
        else:
            per = F.binary_cross_entropy(y_pred.float().clamp(1e-7, 1 - 1e-7), t, reduction="none")
        return per.reshape(per.shape[0], -1).mean(-1)


class MeanSquaredError(Loss):
    name = "mean_squared_error"

    def per_example(self, y_true, y_pred):
        d = (y_pred.float() - y_true.float().reshape(y_pred.shape)) ** 2
        return d.reshape(d.shape[0], -1).mean(-1)


class MeanAbsoluteError(Loss):
    name = "mean_absolute_error"

    def per_example(self, y_true, y_pred):
        d = (y_pred.float() - y_true.float().reshape(y_pred.shape)).abs()
        return d.reshape(d.shape[0], -1).mean(-1)


_ALIASES = {
    "sparse_categorical_crossentropy": SparseCategoricalCrossentropy,
    "categorical_crossentropy": CategoricalCrossentropy,
    "binary_crossentropy": BinaryCrossentropy,
    "mse": MeanSquaredError, "mean_squared_error": MeanSquaredError,
    "mae": MeanAbsoluteError, "mean_absolute_error": MeanAbsoluteError,
}


def get(identifier):
    if isinstance(identifier, Loss) or (callable(identifier) and not isinstance(identifier, str)):
        return identifier
    try:
        return _ALIASES[identifier]()
    except KeyError as e:
        raise ValueError(f"Unknown loss {identifier!r}") from e


def compute_average_loss(per_example_loss, global_batch_size=None, sample_weight=None):
    """``tf.nn.compute_average_loss``: sum(per-example) / global batch size."""
    per = per_example_loss
    if sample_weight is not None:
        per = per * sample_weight
    if global_batch_size is None:
        from ..parallel.strategy import get_strategy

        global_batch_size = per.shape[0] * get_strategy().num_replicas_in_sync
    return per.sum() / float(global_batch_size)


sparse_categorical_crossentropy = SparseCategoricalCrossentropy().per_example
