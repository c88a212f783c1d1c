"""Hyper-parameter tuning: KerasTuner-compatible API on a local study service.

``CloudTuner`` / ``CloudOracle`` keep the reference signatures
(``TFC/tuner/tuner.py``); the Vizier backend is :mod:`.study_service` and
:mod:`.scheduler` runs many tuners concurrently on the node's MI355X GPUs.
"""
from .hyperparameters import HyperParameters  # noqa: F401
from .trial import Objective, Trial, TrialStatus  # noqa: F401
from .tuner import (BayesianOptimization, CloudOracle, CloudTuner, GridSearch, Oracle, RandomSearch,  # noqa: F401
                    Tuner)
