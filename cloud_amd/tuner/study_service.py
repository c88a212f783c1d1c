"""Local study service: the on-node replacement for the Cloud AI Platform
Optimizer (Vizier) that reference ``CloudOracle`` talks to over REST.

Data model = the Optimizer REST schema (reference
``TFC/tuner/api/ml_public_google_rest_v1.json``): a *Study* holds a
``studyConfig`` (metrics, parameters, algorithm, automatedStoppingConfig) and
*Trials* in states REQUESTED / ACTIVE / STOPPING / COMPLETED with parameters,
measurements, ``finalMeasurement``, ``clientId`` and ``trialInfeasible``.

Semantics kept from the service:

* ``suggest`` is idempotent per ``client_id`` while that client's trial is
  still ACTIVE (a restarted tuner gets the same trial back);
* at most 1000 trials per study, and an exhausted grid, raise
  :class:`TooManyTrials` (the service's HTTP 429; the oracle then stops);
* ``create_study`` on an existing id raises :class:`StudyExists` (HTTP 409);
  ``get``/``delete`` of an unknown study raise :class:`StudyNotFound` (404);
* automated early stopping (median / decay-curve rule) through
  ``check_early_stopping_state``.

Many tuner processes (one per MI355X) share a study: every mutation runs
under an exclusive ``flock`` on the study directory and state is written
atomically (tmp + rename), so concurrent suggest / complete calls are safe.
Algorithms: RANDOM_SEARCH, GRID_SEARCH, and GAUSSIAN_PROCESS_BANDIT (also the
ALGORITHM_UNSPECIFIED default): a numpy GP with expected improvement.
"""
from __future__ import annotations

import contextlib
import fcntl
import itertools
import json
import math
import os
import random
import time

import numpy as np

MAX_TRIALS = 1000


def _curve(t, metric, use_elapsed):
    """(x, y) points of a trial's measurements: x = stepCount or elapsed seconds."""
    pts = []
    for m in t.get("measurements", []):
        vals = [m2["value"] for m2 in m.get("metrics", []) if m2.get("metric") == metric]
        if not vals:
            continue
        x = float((m.get("elapsedTime") or {}).get("seconds", 0)) if use_elapsed else float(m.get("stepCount", 0))
        pts.append((x, float(vals[0])))
    return pts


def _final_value(t, metric):
    fm = t.get("finalMeasurement") or {}
    vals = [m["value"] for m in fm.get("metrics", []) if m.get("metric") == metric]
    return float(vals[0]) if vals else None


def fit_decay_curve(xs, ys):
    """Least-squares fit of a saturating learning curve ``y = a + b * x**(-c)``
    (power-law decay toward an asymptote ``a``) over a small grid of exponents ``c``
    (linear in a, b for fixed c).  Returns (predict(x), residual std)."""
    x = np.maximum(np.asarray(xs, dtype=np.float64), 1e-9)
    y = np.asarray(ys, dtype=np.float64)
    best = None
    for c in (0.25, 0.5, 0.75, 1.0, 1.5, 2.0):
        A = np.stack([np.ones_like(x), x ** (-c)], 1)
        coef, *_ = np.linalg.lstsq(A, y, rcond=None)
        sse = float(((A @ coef - y) ** 2).sum())
        if best is None or sse < best[0]:
            best = (sse, c, coef)
    sse, c, (a, b) = best
    sigma = math.sqrt(sse / max(len(x) - 2, 1))
    return (lambda q: float(a + b * max(float(q), 1e-9) ** (-c))), sigma


def decay_curve_should_stop(trial, done, metric, maximize, use_elapsed=False, min_points=3, z=1.0):
    """Stop if the trial's extrapolated final objective, moved ``z`` residual standard
    deviations in the favourable direction, is still worse than the best completed
    trial.  Needs ``min_points`` measurements at distinct x and >= 1 completed trial;
    the horizon is the median final x of the completed trials (never below the
    trial's own last x)."""
    pts = _curve(trial, metric, use_elapsed)
    finals = [(t, _final_value(t, metric)) for t in done]
    finals = [(t, v) for t, v in finals if v is not None]
    if len({x for x, _ in pts}) < min_points or not finals:
        return False
    horizons = [max((x for x, _ in _curve(t, metric, use_elapsed)), default=0.0) for t, _ in finals]
    horizon = max(float(np.median(horizons)), max(x for x, _ in pts))
    predict, sigma = fit_decay_curve([x for x, _ in pts], [y for _, y in pts])
    pred = predict(horizon)
    best = max(v for _, v in finals) if maximize else min(v for _, v in finals)
    optimistic = pred + z * sigma if maximize else pred - z * sigma
    return bool(optimistic < best if maximize else optimistic > best)


def median_should_stop(trial, done, metric, maximize, use_elapsed=False, min_completed=3):
    """Median rule: best value so far worse than the median of the completed trials'
    best values up to the same x."""
    mine_pts = _curve(trial, metric, use_elapsed)
    if not mine_pts:
        return False
    upto = mine_pts[-1][0]

    def best_upto(pts):
        vals = [y for x, y in pts if x <= upto]
        if not vals:
            return None
        return max(vals) if maximize else min(vals)

    others = [best_upto(_curve(t, metric, use_elapsed)) for t in done]
    others = [v for v in others if v is not None]
    mine = best_upto(mine_pts)
    if len(others) < min_completed or mine is None:
        return False
    med = float(np.median(others))
    return bool(mine < med if maximize else mine > med)


class StudyExists(Exception):
    pass


class StudyNotFound(Exception):
    pass


class TooManyTrials(Exception):
    pass


def default_root():
    return os.path.abspath(os.environ.get("CLOUD_AMD_STUDY_DIR", os.path.expanduser("~/.cloud_amd/studies")))


def _ts():
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


class StudyService:
    def __init__(self, root=None):
        self.root = os.path.abspath(root or default_root())
        os.makedirs(self.root, exist_ok=True)

    # -- storage ------------------------------------------------------------------
    @staticmethod
    def study_id_of(name):
        return name.rstrip("/").split("/studies/")[-1].split("/")[0]

    def _dir(self, study_id):
        return os.path.join(self.root, study_id)

    @contextlib.contextmanager
    def _locked(self, study_id):
        d = self._dir(study_id)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, ".lock"), "a+") as lf:
            fcntl.flock(lf, fcntl.LOCK_EX)
            try:
                yield
            finally:
                fcntl.flock(lf, fcntl.LOCK_UN)

    def _read(self, study_id):
        p = os.path.join(self._dir(study_id), "study.json")
        if not os.path.exists(p):
            raise StudyNotFound(study_id)
        with open(p) as f:
            return json.load(f)

    def _write(self, study_id, data):
        p = os.path.join(self._dir(study_id), "study.json")
        tmp = p + f".tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(data, f, indent=1)
        os.replace(tmp, p)

    # -- studies --------------------------------------------------------------------
    def create_study(self, parent, study_id, study_config):
        with self._locked(study_id):
            if os.path.exists(os.path.join(self._dir(study_id), "study.json")):
                raise StudyExists(study_id)
            study = {"name": f"{parent}/studies/{study_id}", "studyConfig": study_config, "state": "ACTIVE",
                     "createTime": _ts()}
            self._write(study_id, {"study": study, "trials": [], "next_id": 1})
            return dict(study)

    def get_study(self, name):
        return self._read(self.study_id_of(name))["study"]

    def list_studies(self, parent=None):
        out = []
        for d in sorted(os.listdir(self.root)):
            p = os.path.join(self.root, d, "study.json")
            if os.path.exists(p):
                with open(p) as f:
                    s = json.load(f)["study"]
                if parent is None or s["name"].startswith(parent):
                    out.append(s)
        return out

    def delete_study(self, name):
        sid = self.study_id_of(name)
        with self._locked(sid):
            p = os.path.join(self._dir(sid), "study.json")
            if not os.path.exists(p):
                raise StudyNotFound(sid)
            os.remove(p)

    # -- trials ---------------------------------------------------------------------
    def list_trials(self, study_name):
        return self._read(self.study_id_of(study_name))["trials"]

    def get_trial(self, trial_name):
        sid = self.study_id_of(trial_name)
        for t in self._read(sid)["trials"]:
            if t["name"] == trial_name:
                return t
        raise KeyError(trial_name)

    def _mutate_trial(self, trial_name, fn):
        sid = self.study_id_of(trial_name)
        with self._locked(sid):
            data = self._read(sid)
            for t in data["trials"]:
                if t["name"] == trial_name:
                    fn(t, data)
                    self._write(sid, data)
                    return dict(t)
        raise KeyError(trial_name)

    def suggest(self, study_name, client_id, count=1, max_trials=None):
        """New (or this client's still pending) trials.  ``max_trials`` is checked under
        the study lock, so N concurrent tuner processes never create more trials than the
        cap between their own ``list_trials`` check and the suggestion."""
        sid = self.study_id_of(study_name)
        with self._locked(sid):
            data = self._read(sid)
            study = data["study"]
            if study.get("state") != "ACTIVE":
                return {"studyState": study.get("state", "INACTIVE")}
            mine = [t for t in data["trials"] if t.get("clientId") == client_id and t["state"] in ("ACTIVE",
                                                                                                  "REQUESTED")]
            if mine:
                return {"trials": mine[:count], "studyState": "ACTIVE"}
            if max_trials and len(data["trials"]) >= max_trials:
                return {"studyState": "ACTIVE"}  # the oracle's cap: no trial, search ends
            if len(data["trials"]) >= MAX_TRIALS:
                raise TooManyTrials(f"study {sid} reached {MAX_TRIALS} trials")
            out = []
            for _ in range(count):
                params = self._next_params(study["studyConfig"], data["trials"])
                if params is None:
                    if out:
                        break
                    raise TooManyTrials(f"search space of study {sid} is exhausted")
                tid = data["next_id"]
                data["next_id"] += 1
                trial = {"name": f"{study['name']}/trials/{tid}", "state": "ACTIVE", "parameters": params,
                         "clientId": client_id, "measurements": [], "startTime": _ts(),
                         "startTs": time.time()}
                dev = os.environ.get("CLOUD_AMD_TRIAL_DEVICE")  # set by TrialScheduler per worker
                if dev:
                    trial["device"] = dev
                data["trials"].append(trial)
                out.append(trial)
            self._write(sid, data)
            return {"trials": out, "studyState": "ACTIVE"}

    def add_measurement(self, trial_name, measurement):
        def fn(t, _):
            t.setdefault("measurements", []).append(measurement)

        return self._mutate_trial(trial_name, fn)

    def stop_trial(self, trial_name):
        def fn(t, _):
            if t["state"] != "COMPLETED":
                t["state"] = "STOPPING"

        return self._mutate_trial(trial_name, fn)

    def complete_trial(self, trial_name, trial_infeasible=False, infeasible_reason=None, final_measurement=None):
        def fn(t, _):
            t["state"] = "COMPLETED"
            t["endTime"] = _ts()
            t["endTs"] = time.time()
            if trial_infeasible:
                t["trialInfeasible"] = True
                t["infeasibleReason"] = infeasible_reason
            fm = final_measurement or (t["measurements"][-1] if t.get("measurements") else None)
            if fm is not None:
                t["finalMeasurement"] = fm

        return self._mutate_trial(trial_name, fn)

    def delete_trial(self, trial_name):
        sid = self.study_id_of(trial_name)
        with self._locked(sid):
            data = self._read(sid)
            data["trials"] = [t for t in data["trials"] if t["name"] != trial_name]
            self._write(sid, data)

    # -- early stopping ---------------------------------------------------------------
    def check_early_stopping_state(self, trial_name):
        """Automated early stopping (``checkEarlyStoppingState``) by the study's
        ``automatedStoppingConfig``:

        * ``decayCurveStoppingConfig`` (what reference ``tuner/utils.py:66-68`` emits):
          extrapolate this trial's learning curve to the completed trials' typical
          final step (or elapsed time with ``useElapsedTime``) and stop when even an
          optimistic prediction is worse than the best completed trial;
        * ``medianAutomatedStoppingConfig``: stop when the trial's best value so far is
          worse than the median of the completed trials' best values up to the same
          step (``useElapsedTime`` likewise switches the axis)."""
        sid = self.study_id_of(trial_name)
        data = self._read(sid)
        cfg = data["study"]["studyConfig"]
        asc = cfg.get("automatedStoppingConfig") or {}
        if not asc:
            return {"shouldStop": False}
        metric = cfg["metrics"][0]["metric"]
        maximize = cfg["metrics"][0].get("goal") == "MAXIMIZE"
        trial = next((t for t in data["trials"] if t["name"] == trial_name), None)
        if trial is None or not trial.get("measurements"):
            return {"shouldStop": False}
        done = [t for t in data["trials"]
                if t["state"] == "COMPLETED" and not t.get("trialInfeasible") and t["name"] != trial_name]
        if "decayCurveStoppingConfig" in asc:
            rule = asc["decayCurveStoppingConfig"] or {}
            return {"shouldStop": decay_curve_should_stop(trial, done, metric, maximize,
                                                          bool(rule.get("useElapsedTime")))}
        rule = asc.get("medianAutomatedStoppingConfig") or {}
        return {"shouldStop": median_should_stop(trial, done, metric, maximize, bool(rule.get("useElapsedTime")))}

    # -- suggestion algorithms -------------------------------------------------------
    def _next_params(self, cfg, trials):
        algo = cfg.get("algorithm", "ALGORITHM_UNSPECIFIED")
        specs = cfg["parameters"]
        seen = {json.dumps(t["parameters"], sort_keys=True) for t in trials}
        if algo == "GRID_SEARCH":
            for combo in itertools.product(*[_grid(p) for p in specs]):
                params = [_pv(p, v) for p, v in zip(specs, combo)]
                if json.dumps(params, sort_keys=True) not in seen:
                    return params
            return None
        rng = random.Random(len(trials) * 7919 + 17)
        done = [t for t in trials if t["state"] == "COMPLETED" and t.get("finalMeasurement")
                and not t.get("trialInfeasible")]
        if algo in ("ALGORITHM_UNSPECIFIED", "GAUSSIAN_PROCESS_BANDIT") and len(done) >= max(3, 2 * len(specs)):
            return self._gp_suggest(cfg, specs, done, rng, seen)
        for _ in range(200):
            params = [_pv(p, _sample(p, rng)) for p in specs]
            if json.dumps(params, sort_keys=True) not in seen:
                return params
        return None if _finite(specs) else [_pv(p, _sample(p, rng)) for p in specs]

    def _gp_suggest(self, cfg, specs, done, rng, seen):
        metric = cfg["metrics"][0]["metric"]
        sign = 1.0 if cfg["metrics"][0].get("goal") == "MAXIMIZE" else -1.0
        X, y = [], []
        for t in done:
            vals = {p["parameter"]: _pval(p) for p in t["parameters"]}
            fm = {m["metric"]: m["value"] for m in t["finalMeasurement"].get("metrics", [])}
            if metric not in fm:
                continue
            X.append([_encode(s, vals.get(s["parameter"])) for s in specs])
            y.append(sign * float(fm[metric]))
        if len(X) < 2:
            return [_pv(p, _sample(p, rng)) for p in specs]
        X, y = np.asarray(X), np.asarray(y)
        mu, sd = y.mean(), y.std() + 1e-9
        yn = (y - mu) / sd
        ls, noise = 0.3, 1e-3

        def k(a, b):
            d = ((a[:, None, :] - b[None, :, :]) ** 2).sum(-1)
            return np.exp(-0.5 * d / ls ** 2)

        K = k(X, X) + noise * np.eye(len(X))
        L = np.linalg.cholesky(K)
        alpha = np.linalg.solve(L.T, np.linalg.solve(L, yn))
        cands, raw = [], []
        for _ in range(512):
            vals = [_sample(p, rng) for p in specs]
            params = [_pv(p, v) for p, v in zip(specs, vals)]
            if json.dumps(params, sort_keys=True) in seen:
                continue
            raw.append(params)
            cands.append([_encode(s, v) for s, v in zip(specs, vals)])
        if not cands:
            return None
        C = np.asarray(cands)
        Ks = k(C, X)
        m = Ks @ alpha
        v = np.clip(1.0 - (np.linalg.solve(L, Ks.T) ** 2).sum(0), 1e-12, None)
        s = np.sqrt(v)
        best = yn.max()
        z = (m - best) / s
        cdf = 0.5 * (1 + np.vectorize(math.erf)(z / math.sqrt(2)))
        pdf = np.exp(-0.5 * z ** 2) / math.sqrt(2 * math.pi)
        ei = (m - best) * cdf + s * pdf
        return raw[int(np.argmax(ei))]


def _finite(specs):
    return all(p["type"] in ("DISCRETE", "CATEGORICAL", "INTEGER") for p in specs)


def _grid(p):
    t = p["type"]
    if t == "DISCRETE":
        return list(p["discrete_value_spec"]["values"])
    if t == "CATEGORICAL":
        return list(p["categorical_value_spec"]["values"])
    if t == "INTEGER":
        s = p["integer_value_spec"]
        return list(range(s["min_value"], s["max_value"] + 1))
    s = p["double_value_spec"]
    if p.get("scale_type") == "UNIT_LOG_SCALE":
        return list(np.exp(np.linspace(math.log(s["min_value"]), math.log(s["max_value"]), 10)))
    return list(np.linspace(s["min_value"], s["max_value"], 10))


def _sample(p, rng):
    t = p["type"]
    if t in ("DISCRETE", "CATEGORICAL"):
        vals = _grid(p)
        return vals[rng.randrange(len(vals))]
    if t == "INTEGER":
        s = p["integer_value_spec"]
        if p.get("scale_type") == "UNIT_LOG_SCALE" and s["min_value"] > 0:
            return int(round(math.exp(rng.uniform(math.log(s["min_value"]), math.log(s["max_value"])))))
        return rng.randint(s["min_value"], s["max_value"])
    s = p["double_value_spec"]
    if p.get("scale_type") == "UNIT_LOG_SCALE" and s["min_value"] > 0:
        return math.exp(rng.uniform(math.log(s["min_value"]), math.log(s["max_value"])))
    return rng.uniform(s["min_value"], s["max_value"])


def _pv(p, v):
    """Parameter value entry in the Optimizer wire format."""
    t = p["type"]
    if t == "CATEGORICAL":
        return {"parameter": p["parameter"], "stringValue": str(v)}
    if t == "INTEGER":
        return {"parameter": p["parameter"], "intValue": str(int(v))}
    return {"parameter": p["parameter"], "floatValue": float(v)}


def _pval(entry):
    if "stringValue" in entry:
        return entry["stringValue"]
    if "intValue" in entry:
        return int(entry["intValue"])
    return float(entry["floatValue"])


def _encode(spec, v):
    """Map a parameter value into [0, 1] for the GP."""
    t = spec["type"]
    if t in ("DISCRETE", "CATEGORICAL"):
        vals = [str(x) for x in _grid(spec)]
        return vals.index(str(v)) / max(len(vals) - 1, 1) if str(v) in vals else 0.5
    s = spec["integer_value_spec"] if t == "INTEGER" else spec["double_value_spec"]
    lo, hi = float(s["min_value"]), float(s["max_value"])
    v = float(v)
    if spec.get("scale_type") == "UNIT_LOG_SCALE" and lo > 0:
        return (math.log(v) - math.log(lo)) / max(math.log(hi) - math.log(lo), 1e-12)
    return (v - lo) / max(hi - lo, 1e-12)
