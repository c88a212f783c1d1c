"""Hyper-parameter search space (KerasTuner ``HyperParameters`` API, written from
scratch -- keras-tuner is not part of this stack).

``hp.Choice / Int / Float / Boolean / Fixed`` both *declare* a parameter in the
space and *return* its current value (the trial's value, or the default), so
a model-building function ``build_model(hp)`` reads exactly like KerasTuner
code (reference ``tuner/tests/integration/tuner_integration_test.py:45-80``).
"""
from __future__ import annotations

import math
import random

import numpy as np


class HyperParameter:
    def __init__(self, name, default=None):
        self.name = name
        self.default = default

    def get_config(self):
        return {"name": self.name, "default": self.default}

    @classmethod
    def from_config(cls, cfg):
        return cls(**cfg)


class Choice(HyperParameter):
    def __init__(self, name, values, ordered=None, default=None):
        values = list(values)
        if not values:
            raise ValueError("Choice needs at least one value")
        super().__init__(name, values[0] if default is None else default)
        self.values = values
        self.ordered = ordered

    def random_sample(self, rng):
        return self.values[rng.randrange(len(self.values))]

    def grid(self):
        return list(self.values)

    def get_config(self):
        c = super().get_config()
        c.update(values=self.values, ordered=self.ordered)
        return c

    def __repr__(self):
        return f"Choice(name={self.name!r}, values={self.values}, default={self.default!r})"


def _sample_scaled(rng, lo, hi, sampling):
    u = rng.random()
    if sampling == "log":
        return math.exp(math.log(lo) + u * (math.log(hi) - math.log(lo)))
    if sampling == "reverse_log":
        return hi + lo - math.exp(math.log(lo) + u * (math.log(hi) - math.log(lo)))
    return lo + u * (hi - lo)


class Int(HyperParameter):
    def __init__(self, name, min_value, max_value, step=1, sampling=None, default=None):
        super().__init__(name, int(min_value) if default is None else default)
        self.min_value, self.max_value = int(min_value), int(max_value)
        self.step = step
        self.sampling = sampling

    def random_sample(self, rng):
        if self.step and self.step != 1:
            vals = self.grid()
            return vals[rng.randrange(len(vals))]
        v = _sample_scaled(rng, self.min_value, self.max_value + 1 - 1e-9, self.sampling)
        return int(min(self.max_value, max(self.min_value, math.floor(v))))

    def grid(self):
        return list(range(self.min_value, self.max_value + 1, self.step or 1))

    def get_config(self):
        c = super().get_config()
        c.update(min_value=self.min_value, max_value=self.max_value, step=self.step, sampling=self.sampling)
        return c

    def __repr__(self):
        return (f"Int(name={self.name!r}, min_value={self.min_value}, max_value={self.max_value}, "
                f"step={self.step}, sampling={self.sampling}, default={self.default})")


class Float(HyperParameter):
    def __init__(self, name, min_value, max_value, step=None, sampling=None, default=None):
        super().__init__(name, float(min_value) if default is None else default)
        self.min_value, self.max_value = float(min_value), float(max_value)
        self.step = step
        self.sampling = sampling

    def random_sample(self, rng):
        if self.step:
            vals = self.grid()
            return vals[rng.randrange(len(vals))]
        return float(_sample_scaled(rng, self.min_value, self.max_value, self.sampling))

    def grid(self, n=10):
        if self.step:
            out, v = [], self.min_value
            while v <= self.max_value + 1e-12:
                out.append(v)
                v += self.step
            return out
        if self.sampling == "log":
            return list(np.exp(np.linspace(math.log(self.min_value), math.log(self.max_value), n)))
        return list(np.linspace(self.min_value, self.max_value, n))

    def get_config(self):
        c = super().get_config()
        c.update(min_value=self.min_value, max_value=self.max_value, step=self.step, sampling=self.sampling)
        return c

    def __repr__(self):
        return (f"Float(name={self.name!r}, min_value={self.min_value}, max_value={self.max_value}, "
                f"step={self.step}, sampling={self.sampling}, default={self.default})")


class Boolean(HyperParameter):
    def __init__(self, name, default=False):
        super().__init__(name, bool(default))

    def random_sample(self, rng):
        return rng.random() < 0.5

    def grid(self):
        return [True, False]

    def __repr__(self):
        return f"Boolean(name={self.name!r}, default={self.default})"


class Fixed(HyperParameter):
    def __init__(self, name, value):
        super().__init__(name, value)
        self.value = value

    def random_sample(self, rng):
        return self.value

    def grid(self):
        return [self.value]

    def get_config(self):
        return {"name": self.name, "value": self.value}

    def __repr__(self):
        return f"Fixed(name={self.name!r}, value={self.value!r})"


_CLASSES = {c.__name__: c for c in (Choice, Int, Float, Boolean, Fixed)}


class HyperParameters:
    def __init__(self):
        self.space = []
        self.values = {}
        self._names = {}

    def _register(self, hp):
        if hp.name in self._names:
            return self._names[hp.name]
        self.space.append(hp)
        self._names[hp.name] = hp
        self.values.setdefault(hp.name, hp.default)
        return hp

    def _value(self, hp):
        hp = self._register(hp)
        if self.values is None:
            return hp.default
        return self.values.get(hp.name, hp.default)

    def Choice(self, name, values, ordered=None, default=None, **kw):
        return self._value(Choice(name, values, ordered, default))

    def Int(self, name, min_value, max_value, step=1, sampling=None, default=None, **kw):
        return self._value(Int(name, min_value, max_value, step, sampling, default))

    def Float(self, name, min_value, max_value, step=None, sampling=None, default=None, **kw):
        return self._value(Float(name, min_value, max_value, step, sampling, default))

    def Boolean(self, name, default=False, **kw):
        return self._value(Boolean(name, default))

    def Fixed(self, name, value, **kw):
        return self._value(Fixed(name, value))

    def get(self, name):
        if name in (self.values or {}):
            return self.values[name]
        if name in self._names:
            return self._names[name].default
        raise KeyError(f"{name} does not exist")

    def __getitem__(self, name):
        return self.get(name)

    def __contains__(self, name):
        return name in self._names

    def copy(self):
        return HyperParameters.from_config(self.get_config())

    def get_config(self):
        return {"space": [{"class_name": type(h).__name__, "config": h.get_config()} for h in self.space],
                "values": dict(self.values or {})}

    @classmethod
    def from_config(cls, cfg):
        hps = cls()
        for s in cfg["space"]:
            hps._register(_CLASSES[s["class_name"]].from_config(s["config"]))
        hps.values = dict(cfg.get("values") or {})
        return hps

    def random_values(self, seed=None):
        rng = random.Random(seed)
        return {h.name: h.random_sample(rng) for h in self.space}
