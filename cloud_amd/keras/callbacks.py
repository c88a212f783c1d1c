"""Keras callbacks (``tf.keras.callbacks``) used by the reference workloads:
ModelCheckpoint / EarlyStopping / LearningRateScheduler / TensorBoard
(``call_run_within_script_with_keras_fit.py:93-101``, ``mnist_example_using_fit.py:74-95``,
``save_and_load.py:89-125``).  Saving callbacks write from the chief (rank 0)
only, like TF's chief-only checkpointing under MultiWorkerMirroredStrategy.
TensorBoard writes scalar summaries as JSONL (no TensorFlow in this stack).
"""
from __future__ import annotations

import csv
import json
import math
import os
import time

import numpy as np


def _is_chief():
    from ..parallel.strategy import get_strategy

    try:
        return get_strategy().is_chief
    except Exception:  # pragma: no cover
        return True


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None): ...
    def on_train_end(self, logs=None): ...
    def on_epoch_begin(self, epoch, logs=None): ...
    def on_epoch_end(self, epoch, logs=None): ...
    def on_train_batch_begin(self, batch, logs=None): ...
    def on_train_batch_end(self, batch, logs=None): ...
    def on_test_begin(self, logs=None): ...
    def on_test_end(self, logs=None): ...
    def on_test_batch_begin(self, batch, logs=None): ...
    def on_test_batch_end(self, batch, logs=None): ...
    def on_predict_begin(self, logs=None): ...
    def on_predict_end(self, logs=None): ...


class CallbackList:
    def __init__(self, callbacks=None, model=None, params=None):
        self.callbacks = list(callbacks or [])
        for c in self.callbacks:
            c.set_model(model)
            c.set_params(params or {})

    def _call(self, name, *a):
        for c in self.callbacks:
            getattr(c, name)(*a)

    def __getattr__(self, name):
        if name.startswith("on_"):
            return lambda *a: self._call(name, *a)
        raise AttributeError(name)


class History(Callback):
    def on_train_begin(self, logs=None):
        self.epoch = []
        self.history = {}

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class LambdaCallback(Callback):
    def __init__(self, on_epoch_begin=None, on_epoch_end=None, on_batch_begin=None, on_batch_end=None,
                 on_train_begin=None, on_train_end=None):
        super().__init__()
        if on_epoch_begin: self.on_epoch_begin = on_epoch_begin  # noqa: E701
        if on_epoch_end: self.on_epoch_end = on_epoch_end  # noqa: E701
        if on_batch_begin: self.on_train_batch_begin = on_batch_begin  # noqa: E701
        if on_batch_end: self.on_train_batch_end = on_batch_end  # noqa: E701
        if on_train_begin: self.on_train_begin = on_train_begin  # noqa: E701
        if on_train_end: self.on_train_end = on_train_end  # noqa: E701


class LearningRateScheduler(Callback):
    def __init__(self, schedule, verbose=0):
        super().__init__()
        self.schedule, self.verbose = schedule, verbose

    def on_epoch_begin(self, epoch, logs=None):
        opt = self.model.optimizer
        try:
            lr = self.schedule(epoch, float(opt.lr))
        except TypeError:
            lr = self.schedule(epoch)
        opt.lr = float(lr)
        if self.verbose:
            print(f"\nEpoch {epoch + 1}: LearningRateScheduler setting learning rate to {lr}.")

    def on_epoch_end(self, epoch, logs=None):
        if logs is not None:
            logs["lr"] = float(self.model.optimizer.lr)


class _Monitor(Callback):
    def __init__(self, monitor="val_loss", mode="auto", min_delta=0.0):
        super().__init__()
        self.monitor, self.min_delta = monitor, abs(min_delta)
        if mode == "auto":
            mode = "max" if ("acc" in monitor or monitor.startswith("fmeasure")) else "min"
        self.mode = mode
        self.best = -math.inf if mode == "max" else math.inf

    def _improved(self, cur):
        if self.mode == "max":
            return cur > self.best + self.min_delta
        return cur < self.best - self.min_delta


class EarlyStopping(_Monitor):
    def __init__(self, monitor="val_loss", min_delta=0, patience=0, verbose=0, mode="auto", baseline=None,
                 restore_best_weights=False):
        super().__init__(monitor, mode, min_delta)
        self.patience, self.verbose, self.restore = patience, verbose, restore_best_weights
        self.wait = 0
        self.stopped_epoch = 0
        self.best_weights = None

    def on_train_begin(self, logs=None):
        self.wait = 0
        self.best = -math.inf if self.mode == "max" else math.inf

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        if self._improved(cur):
            self.best, self.wait = cur, 0
            if self.restore:
                self.best_weights = self.model.get_weights()
        else:
            self.wait += 1
            if self.wait >= self.patience:
                self.stopped_epoch = epoch
                self.model.stop_training = True
                if self.restore and self.best_weights is not None:
                    self.model.set_weights(self.best_weights)

    def on_train_end(self, logs=None):
        if self.stopped_epoch and self.verbose:
            print(f"Epoch {self.stopped_epoch + 1}: early stopping")


class ModelCheckpoint(_Monitor):
    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False, save_weights_only=False,
                 mode="auto", save_freq="epoch"):
        super().__init__(monitor, mode)
        self.filepath, self.verbose = str(filepath), verbose
        self.save_best_only, self.save_weights_only = save_best_only, save_weights_only

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        if self.save_best_only:
            cur = logs.get(self.monitor)
            if cur is None or not self._improved(cur):
                return
            self.best = cur
        path = self.filepath.format(epoch=epoch + 1, **logs)
        # collective: every replica calls, the chief writes, all wait (saving.chief_only)
        if self.save_weights_only:
            self.model.save_weights(path)
        else:
            self.model.save(path)
        if self.verbose and _is_chief():
            print(f"\nEpoch {epoch + 1}: saving model to {path}")


class TensorBoard(Callback):
    """Scalar summaries to ``<log_dir>/{train,validation}/scalars.jsonl`` (chief only)."""

    def __init__(self, log_dir="logs", histogram_freq=0, write_graph=True, update_freq="epoch", **kw):
        super().__init__()
        self.log_dir = str(log_dir)

    def on_epoch_end(self, epoch, logs=None):
        if not _is_chief():
            return
        for split in ("train", "validation"):
            vals = {k[4:] if split == "validation" else k: v for k, v in (logs or {}).items()
                    if (k.startswith("val_") if split == "validation" else not k.startswith("val_"))}
            if not vals:
                continue
            d = os.path.join(self.log_dir, split)
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, "scalars.jsonl"), "a") as f:
                f.write(json.dumps({"epoch": epoch, "wall_time": time.time(), **vals}) + "\n")


class CSVLogger(Callback):
    def __init__(self, filename, separator=",", append=False):
        super().__init__()
        self.filename, self.sep, self.append = filename, separator, append
        self._keys = None

    def on_epoch_end(self, epoch, logs=None):
        if not _is_chief():
            return
        logs = logs or {}
        new = self._keys is None
        if new:
            self._keys = sorted(logs)
        mode = "a" if (self.append or not new) else "w"
        with open(self.filename, mode, newline="") as f:
            w = csv.writer(f, delimiter=self.sep)
            if new and mode == "w":
                w.writerow(["epoch"] + self._keys)
            w.writerow([epoch] + [logs.get(k) for k in self._keys])


class TerminateOnNaN(Callback):
    def on_train_batch_end(self, batch, logs=None):
        loss = (logs or {}).get("loss")
        if loss is not None and (np.isnan(loss) or np.isinf(loss)):
            print(f"Batch {batch}: Invalid loss, terminating training")
            self.model.stop_training = True


class ProgbarLogger(Callback):
    def __init__(self, count_mode="steps"):
        super().__init__()

    def on_epoch_begin(self, epoch, logs=None):
        self._t0 = time.time()
        if self.params.get("verbose") and _is_chief():
            print(f"Epoch {epoch + 1}/{self.params.get('epochs', '?')}", flush=True)

    def on_epoch_end(self, epoch, logs=None):
        if self.params.get("verbose") and _is_chief():
            dt = time.time() - self._t0
            steps = self.params.get("steps") or "?"
            metrics = " - ".join(f"{k}: {v:.4f}" for k, v in (logs or {}).items() if isinstance(v, (int, float)))
            print(f"{steps}/{steps} - {dt:.1f}s - {metrics}", flush=True)
