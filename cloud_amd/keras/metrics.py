"""Keras metrics (``tf.keras.metrics``): stateful ``update_state`` / ``result`` /
``reset_state`` objects whose state is a (total, count) pair, so replicas can
all-reduce it once per epoch/log interval (C3 in SURVEY.md) instead of every step."""
from __future__ import annotations

import torch


def _tensorize(args):
    """numpy / python arguments -> tensors on the device of the tensor arguments."""
    dev = next((a.device for a in args if isinstance(a, torch.Tensor)), None)
    out = []
    for a in args:
        if a is not None and not isinstance(a, torch.Tensor):
            a = torch.as_tensor(a)
            if dev is not None:
                a = a.to(dev)
        out.append(a)
    return out


class Metric:
    name = "metric"

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        fn = cls.__dict__.get("update_state")
        if fn is not None and not getattr(fn, "_tensorized", False):
            def update_state(self, *args, sample_weight=None, _fn=fn):
                return _fn(self, *_tensorize(args), sample_weight=sample_weight)

            update_state._tensorized = True
            cls.update_state = update_state

    def __init__(self, name=None, dtype=None):
        if name:
            self.name = name
        self.reset_state()

    def reset_state(self):
        self.total = 0.0
        self.count = 0.0

    reset_states = reset_state

    def _acc(self, values, weight=None):
        v = values.detach().float()
        if weight is not None:
            w = torch.as_tensor(weight, dtype=torch.float32, device=v.device).reshape(-1)
            self.total += float((v.reshape(-1) * w).sum())
            self.count += float(w.sum())
        else:
            self.total += float(v.sum())
            self.count += float(v.numel())

    def result(self):
        return self.total / self.count if self.count else 0.0

    def state(self):
        return [self.total, self.count]

    def set_state(self, s):
        self.total, self.count = float(s[0]), float(s[1])

    def __call__(self, *a, **k):
        self.update_state(*a, **k)
        return self.result()


class Mean(Metric):
    name = "mean"

    def update_state(self, values, sample_weight=None):
        if not isinstance(values, torch.Tensor):
            values = torch.as_tensor(values, dtype=torch.float32)
        self._acc(values.reshape(-1), sample_weight)


class Sum(Metric):
    name = "sum"

    def update_state(self, values, sample_weight=None):
        v = torch.as_tensor(values, dtype=torch.float32)
        self.total += float(v.sum())
        self.count = 1.0

    def result(self):
        return self.total


class SparseCategoricalAccuracy(Metric):
    name = "sparse_categorical_accuracy"

    def update_state(self, y_true, y_pred, sample_weight=None):
        pred = y_pred.argmax(-1).reshape(-1)
        self._acc((pred == y_true.reshape(-1).to(pred.device).long()).float(), sample_weight)


class CategoricalAccuracy(Metric):
    name = "categorical_accuracy"

    def update_state(self, y_true, y_pred, sample_weight=None):
        self._acc((y_pred.argmax(-1) == y_true.argmax(-1)).float().reshape(-1), sample_weight)


class BinaryAccuracy(Metric):
    name = "binary_accuracy"

    def __init__(self, name=None, threshold=0.5):
        self.threshold = threshold
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        p = (y_pred.float() > self.threshold).float().reshape(y_true.shape)
        self._acc((p == y_true.float()).float().reshape(-1), sample_weight)


class Accuracy(Metric):
    name = "accuracy"

    def update_state(self, y_true, y_pred, sample_weight=None):
        self._acc((y_pred.reshape(-1) == y_true.reshape(-1)).float(), sample_weight)


class MeanSquaredError(Metric):
    name = "mean_squared_error"

    def update_state(self, y_true, y_pred, sample_weight=None):
        d = (y_pred.float() - y_true.float().reshape(y_pred.shape)) ** 2
        self._acc(d.reshape(d.shape[0], -1).mean(-1), sample_weight)


class MeanAbsoluteError(Metric):
    name = "mean_absolute_error"

    def update_state(self, y_true, y_pred, sample_weight=None):
        d = (y_pred.float() - y_true.float().reshape(y_pred.shape)).abs()
        self._acc(d.reshape(d.shape[0], -1).mean(-1), sample_weight)


def get(identifier, loss=None):
    """Resolve a metric name the way Keras does (``"accuracy"`` depends on the loss)."""
    if isinstance(identifier, Metric):
        return identifier
    name = str(identifier).lower()
    if name in ("accuracy", "acc"):
        lname = getattr(loss, "name", str(loss))
        if "sparse" in lname:
            m = SparseCategoricalAccuracy()
        elif "binary" in lname:
            m = BinaryAccuracy()
        else:
            m = CategoricalAccuracy()
        m.name = identifier
        return m
    table = {"sparse_categorical_accuracy": SparseCategoricalAccuracy,
             "categorical_accuracy": CategoricalAccuracy, "binary_accuracy": BinaryAccuracy,
             "mse": MeanSquaredError, "mean_squared_error": MeanSquaredError,
             "mae": MeanAbsoluteError, "mean_absolute_error": MeanAbsoluteError}
    if name not in table:
        raise ValueError(f"Unknown metric {identifier!r}")
    m = table[name]()
    m.name = identifier
    return m
