"""Trials, objectives and metric tracking (KerasTuner ``Trial`` / ``Objective``)."""
from __future__ import annotations

import json
import os


class TrialStatus:
    RUNNING = "RUNNING"
    IDLE = "IDLE"
    INVALID = "INVALID"
    STOPPED = "STOPPED"
    COMPLETED = "COMPLETED"


class Objective:
    def __init__(self, name, direction):
        if direction not in ("min", "max"):
            raise ValueError("direction must be 'min' or 'max'")
        self.name, self.direction = name, direction

    def __eq__(self, other):
        return isinstance(other, Objective) and (self.name, self.direction) == (other.name, other.direction)

    def __repr__(self):
        return f"Objective(name={self.name!r}, direction={self.direction!r})"


def infer_metric_direction(metric):
    """KerasTuner convention: accuracy-like -> max, loss/error-like -> min."""
    name = metric[4:] if metric.startswith("val_") else metric
    if name in ("loss", "mse", "mae", "mape", "msle", "logcosh") or any(
            s in name for s in ("loss", "error", "crossentropy", "hinge")):
        return "min"
    if any(s in name for s in ("acc", "auc", "precision", "recall", "f1", "iou")):
        return "max"
    return "min"


class MetricHistory:
    def __init__(self, direction="min"):
        self.direction = direction
        self.history = []  # (step, value)

    def update(self, value, step=0):
        self.history.append((int(step), float(value)))

    def best(self):
        if not self.history:
            return None
        vals = [v for _, v in self.history]
        return max(vals) if self.direction == "max" else min(vals)


class Trial:
    def __init__(self, hyperparameters, trial_id=None, status=TrialStatus.RUNNING):
        self.hyperparameters = hyperparameters
        self.trial_id = trial_id
        self.status = status
        self.score = None
        self.best_step = None
        self.metrics = {}

    def update_metric(self, name, value, step=0, direction="min"):
        self.metrics.setdefault(name, MetricHistory(direction)).update(value, step)

    def get_state(self):
        hp = self.hyperparameters
        return {"trial_id": self.trial_id, "status": self.status, "score": self.score, "best_step": self.best_step,
                "hyperparameters": hp.get_config() if hasattr(hp, "get_config") else hp,
                "metrics": {k: {"direction": m.direction, "history": m.history} for k, m in self.metrics.items()}}

    def save(self, path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(self.get_state(), f, indent=2, default=str)
        os.replace(tmp, path)

    def summary(self):
        hp = self.hyperparameters
        lines = [f"Trial {self.trial_id} summary", "Hyperparameters:"]
        for k, v in (hp.values or {}).items() if hasattr(hp, "values") else []:
            lines.append(f"{k}: {v}")
        lines.append(f"Score: {self.score}")
        return "\n".join(lines)
