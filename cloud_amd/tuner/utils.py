"""``study_config`` <-> HyperParameters / Objective converters.

Same study_config schema and conversion rules as reference
``TFC/tuner/utils.py:47-399`` so existing study configs port unchanged,
including its documented quirks: an ``Int`` with ``step != 1`` becomes a
DISCRETE parameter over ``range(min, max, step)`` (max excluded), a stepped
``Float`` becomes DISCRETE by accumulation (max excluded), ``Boolean`` becomes
CATEGORICAL ``["True", "False"]``, ``Fixed`` becomes a one-value CATEGORICAL
(str/bool) or DISCRETE (number, as float).
"""
from __future__ import annotations

from . import hyperparameters as hp_module
from .trial import Objective, infer_metric_direction

DISCRETE, CATEGORICAL, DOUBLE, INTEGER = "DISCRETE", "CATEGORICAL", "DOUBLE", "INTEGER"
SCALE_UNSPECIFIED = "SCALE_TYPE_UNSPECIFIED"
LINEAR, LOG, REVERSE_LOG = "UNIT_LINEAR_SCALE", "UNIT_LOG_SCALE", "UNIT_REVERSE_LOG_SCALE"
GOAL_UNSPECIFIED, MAXIMIZE, MINIMIZE = "GOAL_TYPE_UNSPECIFIED", "MAXIMIZE", "MINIMIZE"

_SAMPLING_TO_SCALE = {"linear": LINEAR, "log": LOG, "reverse_log": REVERSE_LOG}
_SCALE_TO_SAMPLING = {v: k for k, v in _SAMPLING_TO_SCALE.items()}


def make_study_config(objective, hyperparams):
    return {
        "algorithm": "ALGORITHM_UNSPECIFIED",
        "automatedStoppingConfig": {"decayCurveStoppingConfig": {"useElapsedTime": True}},
        "metrics": [{"metric": o.name, "goal": format_goal(o.direction)} for o in format_objective(objective)],
        "parameters": _convert_hyperparams_to_optimizer_params(hyperparams),
    }


def convert_study_config_to_objective(study_config):
    metrics = study_config.get("metrics")
    if not metrics:
        raise ValueError('"metrics" not found in study_config {}'.format(study_config))
    if not isinstance(metrics, list):
        raise ValueError('study_config["metrics"] should be a list of {"metric": ...}')
    if not metrics[0].get("metric"):
        raise ValueError('"metric" not found in study_config["metrics"][0]')
    return [format_objective(m["metric"], format_goal(m["goal"]))[0] for m in metrics]


def _is_parameter_valid(param):
    if not param.get("parameter"):
        raise ValueError('"parameter" (name) is not specified.')
    t = param.get("type")
    if not t:
        raise ValueError("Parameter {} type is not specified.".format(param))
    spec_key = {DISCRETE: "discrete_value_spec", CATEGORICAL: "categorical_value_spec",
                DOUBLE: "double_value_spec", INTEGER: "integer_value_spec"}.get(t)
    if spec_key is None:
        raise ValueError("Unknown parameter type: {}.".format(t))
    spec = param.get(spec_key)
    if not spec:
        raise ValueError("Parameter {} is missing {}.".format(param, spec_key))
    if t in (DISCRETE, CATEGORICAL):
        if not isinstance(spec.get("values"), list):
            raise ValueError('Parameter spec {} is missing "values".'.format(spec))
    else:
        kind = float if t == DOUBLE else int
        if not (isinstance(spec.get("min_value"), kind) and isinstance(spec.get("max_value"), kind)):
            raise ValueError('Parameter spec {} requires both "min_value" and "max_value".'.format(spec))


def convert_study_config_to_hps(study_config):
    params = study_config.get("parameters")
    if not params:
        raise ValueError("Parameters are not found in the study_config: ", study_config)
    if not isinstance(params, list):
        raise ValueError("Parameters should be a list of parameter with at least 1 parameter, found ", params)
    hps = hp_module.HyperParameters()
    for p in params:
        _is_parameter_valid(p)
        name, t = p["parameter"], p["type"]
        sampling = _format_sampling(p.get("scale_type")) if p.get("scale_type") not in (None, SCALE_UNSPECIFIED) \
            else None
        if t == DISCRETE:
            hps.Choice(name, p["discrete_value_spec"]["values"])
        elif t == CATEGORICAL:
            hps.Choice(name, p["categorical_value_spec"]["values"])
        elif t == DOUBLE:
            s = p["double_value_spec"]
            hps.Float(name, min_value=s["min_value"], max_value=s["max_value"], sampling=sampling)
        else:
            s = p["integer_value_spec"]
            hps.Int(name, min_value=s["min_value"], max_value=s["max_value"], sampling=sampling)
    return hps


def _convert_hyperparams_to_optimizer_params(hyperparams):
    out = []
    for hp in hyperparams.space:
        p = {"parameter": hp.name}
        if isinstance(hp, hp_module.Choice):
            if isinstance(hp.values[0], str):
                p["type"], p["categorical_value_spec"] = CATEGORICAL, {"values": hp.values}
            else:
                p["type"], p["discrete_value_spec"] = DISCRETE, {"values": hp.values}
        elif isinstance(hp, hp_module.Int):
            if hp.step is not None and hp.step != 1:
                p["type"] = DISCRETE
                p["discrete_value_spec"] = {"values": list(range(hp.min_value, hp.max_value, hp.step))}
            else:
                p["type"] = INTEGER
                p["integer_value_spec"] = {"min_value": hp.min_value, "max_value": hp.max_value}
                if hp.sampling is not None:
                    p.update(_get_scale_type(hp.sampling))
        elif isinstance(hp, hp_module.Float):
            if hp.step is not None:
                vals, v = [], hp.min_value
                while v < hp.max_value:
                    vals.append(v)
                    v += hp.step
                p["type"], p["discrete_value_spec"] = DISCRETE, {"values": vals}
            else:
                p["type"] = DOUBLE
                p["double_value_spec"] = {"min_value": hp.min_value, "max_value": hp.max_value}
                if hp.sampling is not None:
                    p.update(_get_scale_type(hp.sampling))
        elif isinstance(hp, hp_module.Boolean):
            p["type"], p["categorical_value_spec"] = CATEGORICAL, {"values": ["True", "False"]}
        elif isinstance(hp, hp_module.Fixed):
            if isinstance(hp.value, (str, bool)):
                p["type"], p["categorical_value_spec"] = CATEGORICAL, {"values": [str(hp.value)]}
            else:
                p["type"], p["discrete_value_spec"] = DISCRETE, {"values": [float(hp.value)]}
        else:
            raise ValueError("`HyperParameter` type not recognized: {}".format(hp))
        out.append(p)
    return out


def format_objective(objective, direction=None):
    if isinstance(objective, Objective):
        return [objective]
    if isinstance(objective, str):
        return [Objective(objective, direction or infer_metric_direction(objective))]
    if isinstance(objective, list) and objective:
        if isinstance(objective[0], Objective):
            return objective
        if isinstance(objective[0], str):
            return [Objective(m, infer_metric_direction(m)) for m in objective]
    raise TypeError("Objective should be either string or Objective, found {}".format(objective))


def format_goal(metric_direction):
    return {"max": MAXIMIZE, "min": MINIMIZE, MAXIMIZE: "max", MINIMIZE: "min"}.get(metric_direction,
                                                                                   GOAL_UNSPECIFIED)


def _get_scale_type(sampling):
    return {"scale_type": _SAMPLING_TO_SCALE.get(sampling, SCALE_UNSPECIFIED)}


def _format_sampling(scale_type):
    return _SCALE_TO_SAMPLING.get(scale_type)


def get_trial_id(optimizer_trial):
    return optimizer_trial["name"].split("/")[-1]


def convert_optimizer_trial_to_hps(hps, optimizer_trial):
    hps = hp_module.HyperParameters.from_config(hps.get_config())
    hps.values = {}
    for p in optimizer_trial["parameters"]:
        if "floatValue" in p:
            hps.values[p["parameter"]] = float(p["floatValue"])
        if "intValue" in p:
            hps.values[p["parameter"]] = int(p["intValue"])
        if "stringValue" in p:
            hps.values[p["parameter"]] = str(p["stringValue"])
    return hps
