"""Tuner: study_config converters (reference tuner/tests/unit/utils_test.py
golden values), oracle lifecycle (tuner_test.py), local study service
semantics (optimizer_client_test.py) and a real multi-process search."""
import json
import time
import os
import threading

import numpy as np
import pytest

from cloud_amd.parallel import strategy as S
from cloud_amd.tuner import CloudOracle, CloudTuner, HyperParameters, RandomSearch, GridSearch, Objective
from cloud_amd.tuner import optimizer_client, utils
from cloud_amd.tuner.scheduler import TrialScheduler
from cloud_amd.tuner.study_service import StudyExists, StudyService, TooManyTrials
from cloud_amd.tuner.trial import TrialStatus

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(autouse=True)
def _cpu():
    S.experimental_set_strategy(S.OneDeviceStrategy("/cpu:0"))
    yield
    S.experimental_set_strategy(None)


def _cfg(params, metric="accuracy"):
    return {"algorithm": "ALGORITHM_UNSPECIFIED", "metrics": [{"goal": "MAXIMIZE", "metric": metric}],
            "parameters": params}


def test_hps_to_study_config_golden():
    hps = HyperParameters()
    hps.Int("units", 32, 128, step=32)
    assert utils._convert_hyperparams_to_optimizer_params(hps) == [
        {"parameter": "units", "type": "DISCRETE", "discrete_value_spec": {"values": [32, 64, 96]}}]
    hps = HyperParameters()
    hps.Float("learning_rate", 1e-4, 1e-1, sampling="log")
    assert utils._convert_hyperparams_to_optimizer_params(hps) == [
        {"parameter": "learning_rate", "type": "DOUBLE", "double_value_spec": {"min_value": 1e-4, "max_value": 0.1},
         "scale_type": "UNIT_LOG_SCALE"}]
    hps = HyperParameters()
    hps.Choice("model_type", ["LINEAR", "WIDE_AND_DEEP"])
    hps.Boolean("has_beta")
    hps.Fixed("beta", 1)
    hps.Fixed("name", "x")
    out = utils._convert_hyperparams_to_optimizer_params(hps)
    assert out[0]["categorical_value_spec"] == {"values": ["LINEAR", "WIDE_AND_DEEP"]}
    assert out[1]["categorical_value_spec"] == {"values": ["True", "False"]}
    assert out[2] == {"parameter": "beta", "type": "DISCRETE", "discrete_value_spec": {"values": [1.0]}}
    assert out[3]["categorical_value_spec"] == {"values": ["x"]}
    hps = HyperParameters()
    hps.Float("f", 0.0, 0.3, step=0.1)
    assert np.allclose(utils._convert_hyperparams_to_optimizer_params(hps)[0]["discrete_value_spec"]["values"],
                       [0.0, 0.1, 0.2])


def test_study_config_to_hps_and_objective():
    cfg = _cfg([{"parameter": "units", "type": "INTEGER", "integer_value_spec": {"min_value": 1, "max_value": 4}},
                {"parameter": "lr", "type": "DOUBLE", "double_value_spec": {"min_value": 1e-4, "max_value": 0.1},
                 "scale_type": "UNIT_LOG_SCALE"}])
    hps = utils.convert_study_config_to_hps(cfg)
    assert [type(h).__name__ for h in hps.space] == ["Int", "Float"] and hps.space[1].sampling == "log"
    assert utils.convert_study_config_to_objective(cfg) == [Objective("accuracy", "max")]
    with pytest.raises(ValueError, match="metrics"):
        utils.convert_study_config_to_objective({"parameters": []})
    with pytest.raises(ValueError, match="min_value"):
        utils.convert_study_config_to_hps(_cfg([{"parameter": "x", "type": "DOUBLE",
                                                 "double_value_spec": {"min_value": 1, "max_value": 2}}]))
    assert utils.format_goal("max") == "MAXIMIZE" and utils.format_goal("MINIMIZE") == "min"
    assert utils.format_objective("val_loss") == [Objective("val_loss", "min")]
    t = {"name": "projects/p/locations/r/studies/s/trials/7", "parameters": [
        {"parameter": "units", "intValue": "3"}, {"parameter": "lr", "floatValue": 0.01}]}
    assert utils.get_trial_id(t) == "7"
    assert utils.convert_optimizer_trial_to_hps(hps, t).values == {"units": 3, "lr": 0.01}


def _hps():
    hps = HyperParameters()
    hps.Int("units", 8, 32, step=8)
    hps.Choice("act", ["relu", "tanh"])
    return hps


def test_oracle_init_rules(tmp_path):
    with pytest.raises(ValueError, match="either study_config"):
        CloudOracle(objective="acc", hyperparameters=_hps(), study_config=_cfg([]), study_dir=str(tmp_path))
    with pytest.raises(ValueError, match="must be set"):
        CloudOracle(objective="acc", study_dir=str(tmp_path))
    o = CloudOracle("proj", "reg", objective="acc", hyperparameters=_hps(), max_trials=3, study_id="abc",
                    study_dir=str(tmp_path))
    assert o.study_id == "CloudTuner_study_abc"
    assert o.study_config["parameters"][0]["discrete_value_spec"]["values"] == [8, 16, 24]


def test_oracle_lifecycle(tmp_path):
    o = CloudOracle("proj", "reg", objective="acc", hyperparameters=_hps(), max_trials=3, study_id="life",
                    study_dir=str(tmp_path))
    t1 = o.create_trial("tuner0")
    assert t1.status == TrialStatus.RUNNING and t1.trial_id == "1"
    assert o.create_trial("tuner0").trial_id == "1"  # idempotent per client while ACTIVE
    o.update_trial("1", {"acc": 0.5}, step=1)
    o.end_trial("1")
    assert o.trials["1"].score == 0.5
    with pytest.raises(ValueError, match="not found"):
        o.end_trial("1")
    t2 = o.create_trial("tuner0")
    with pytest.raises(ValueError, match="Unexpected status"):
        o.end_trial(t2.trial_id, "RUNNING")
    t2 = o.create_trial("tuner0")  # still ACTIVE in the study: same trial comes back
    assert t2.trial_id == "2"
    o.update_trial(t2.trial_id, {"acc": 0.9}, step=1)
    o.end_trial(t2.trial_id, TrialStatus.COMPLETED)
    t3 = o.create_trial("tuner1")
    o.end_trial(t3.trial_id, TrialStatus.INVALID)
    assert o.create_trial("tuner0").status == TrialStatus.STOPPED  # max_trials reached
    best = o.get_best_trials(2)
    assert [b.score for b in best] == [0.9, 0.5]


def test_service_semantics(tmp_path):
    svc = StudyService(str(tmp_path))
    cfg = _cfg([{"parameter": "c", "type": "CATEGORICAL", "categorical_value_spec": {"values": ["a", "b"]}}])
    cfg["algorithm"] = "GRID_SEARCH"
    svc.create_study("projects/p/locations/r", "s1", cfg)
    with pytest.raises(StudyExists):
        svc.create_study("projects/p/locations/r", "s1", cfg)
    c = optimizer_client.create_or_load_study("p", "r", "s1", cfg, root=str(tmp_path))  # 409 -> load
    a = c.get_suggestions("t0")["trials"][0]
    c.complete_trial(a["name"].split("/")[-1], False)
    b = c.get_suggestions("t0")["trials"][0]
    assert {a["parameters"][0]["stringValue"], b["parameters"][0]["stringValue"]} == {"a", "b"}
    c.complete_trial("2", False)
    assert c.get_suggestions("t0") == {}  # grid exhausted == HTTP 429
    assert len(c.list_trials()) == 2 and c.list_studies()[0]["name"].endswith("/studies/s1")
    c.delete_study()
    with pytest.raises(ValueError, match="not found"):
        c.delete_study()


def test_service_concurrent_suggest_is_safe(tmp_path):
    svc = StudyService(str(tmp_path))
    cfg = _cfg([{"parameter": "x", "type": "DOUBLE", "double_value_spec": {"min_value": 0.0, "max_value": 1.0}}])
    svc.create_study("projects/p/locations/r", "c", cfg)
    got = []

    def worker(i):
        for _ in range(5):
            r = svc.suggest("projects/p/locations/r/studies/c", f"t{i}")
            tid = r["trials"][0]["name"]
            svc.complete_trial(tid)
            got.append(tid)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    assert len(got) == 20 and len(set(got)) == 20


def _stop_study(tmp_path, rule):
    svc = StudyService(str(tmp_path))
    cfg = _cfg([{"parameter": "x", "type": "DOUBLE", "double_value_spec": {"min_value": 0.0, "max_value": 1.0}}])
    cfg["automatedStoppingConfig"] = rule
    svc.create_study("projects/p/locations/r", "e", cfg)
    return svc, "projects/p/locations/r/studies/e"


def _trial_with_curve(svc, name, curve, complete):
    # a fresh client per trial: suggest() hands a client its still-ACTIVE trial back
    t = svc.suggest(name, "client%d" % len(svc.list_trials(name)))["trials"][0]["name"]
    for step, acc in curve:
        svc.add_measurement(t, {"stepCount": step, "elapsedTime": {"seconds": 10 * step},
                                "metrics": [{"metric": "accuracy", "value": acc}]})
    if complete:
        svc.complete_trial(t)
    return t


def test_early_stopping_median_rule(tmp_path):
    svc, name = _stop_study(tmp_path, {"medianAutomatedStoppingConfig": {"useElapsedTime": False}})
    for _ in range(3):
        _trial_with_curve(svc, name, [(1, 0.9)], True)
    t = _trial_with_curve(svc, name, [(1, 0.1)], False)
    assert svc.check_early_stopping_state(t)["shouldStop"]
    t2 = _trial_with_curve(svc, name, [(1, 0.95)], False)
    assert not svc.check_early_stopping_state(t2)["shouldStop"]


def test_decay_curve_rule_extrapolates_the_learning_curve(tmp_path):
    """The oracle's default config (decayCurveStoppingConfig): a curve that is still
    low but rising fast toward a good asymptote keeps running; one that has flattened
    below the best completed trial stops -- even though at the last measured step both
    are below every completed trial (where a median rule would stop both)."""
    from cloud_amd.tuner.study_service import fit_decay_curve

    pred, sigma = fit_decay_curve([1, 2, 4, 8], [0.9 - 0.8 / x ** 0.5 for x in (1, 2, 4, 8)])
    assert abs(pred(100) - (0.9 - 0.08)) < 1e-6 and sigma < 1e-9
    for use_elapsed in (False, True):
        svc, name = _stop_study(tmp_path / str(use_elapsed), {"decayCurveStoppingConfig":
                                                                  {"useElapsedTime": use_elapsed}})
        steps = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32)
        _trial_with_curve(svc, name, [(s, 0.85 - 0.5 / s) for s in steps], True)   # best final ~0.83
        _trial_with_curve(svc, name, [(s, 0.80 - 0.5 / s) for s in steps], True)
        rising = _trial_with_curve(svc, name, [(s, 1.0 - 0.8 / s ** 0.5) for s in (1, 2, 3, 4)], False)
        flat = _trial_with_curve(svc, name, [(s, 0.52 - 0.02 / s) for s in (1, 2, 3, 4)], False)
        assert not svc.check_early_stopping_state(rising)["shouldStop"]   # -> ~0.86 at step 32
        assert svc.check_early_stopping_state(flat)["shouldStop"]
        few = _trial_with_curve(svc, name, [(1, 0.1), (2, 0.11)], False)  # too few points to judge
        assert not svc.check_early_stopping_state(few)["shouldStop"]


def test_trial_cap_1000(tmp_path, monkeypatch):
    from cloud_amd.tuner import study_service

    monkeypatch.setattr(study_service, "MAX_TRIALS", 2)
    svc = StudyService(str(tmp_path))
    cfg = _cfg([{"parameter": "x", "type": "DOUBLE", "double_value_spec": {"min_value": 0.0, "max_value": 1.0}}])
    svc.create_study("projects/p/locations/r", "cap", cfg)
    name = "projects/p/locations/r/studies/cap"
    for _ in range(2):
        svc.complete_trial(svc.suggest(name, "t")["trials"][0]["name"])
    with pytest.raises(TooManyTrials):
        svc.suggest(name, "t")


def _build(hp):
    from cloud_amd import keras

    m = keras.Sequential([keras.layers.Dense(hp.Int("units", 8, 32, step=8), activation=hp.Choice("act", ["relu",
                                                                                                     "tanh"]),
                                             input_shape=(20,)), keras.layers.Dense(2, activation="softmax")])
    m.compile(optimizer="adam", loss="sparse_categorical_crossentropy", metrics=["acc"])
    return m


def test_cloud_tuner_search_and_summaries(tmp_path, capsys):
    rng = np.random.default_rng(0)
    x = rng.normal(size=(256, 20)).astype("float32")
    y = (x[:, 0] > 0).astype("int64")
    tuner = CloudTuner(_build, project_id="p", region="r", objective="acc", hyperparameters=_hps(), max_trials=3,
                       study_id="search", study_dir=str(tmp_path / "studies"), directory=str(tmp_path / "res"))
    tuner.search_space_summary()
    tuner.search(x, y, epochs=2, batch_size=32, validation_data=(x, y))
    tuner.results_summary()
    out = capsys.readouterr().out
    import re

    assert re.search(r"Search space summary(?=.*units \(Int\))(?=.*act \(Choice\))", out, re.DOTALL)
    assert re.search(r"Results summary.*Trial .* summary.*Hyperparameters.*", out, re.DOTALL)
    best = tuner.get_best_models(1)[0]
    assert best.predict(x[:4]).shape == (4, 2)
    assert len(tuner.get_best_hyperparameters(2)) == 2
    assert os.path.exists(tmp_path / "res" / "untitled_project" / "trial_1" / "trial.json")


def test_random_and_grid_search(tmp_path):
    rng = np.random.default_rng(1)
    x = rng.normal(size=(64, 20)).astype("float32")
    y = (x[:, 0] > 0).astype("int64")
    g = GridSearch(_build, objective="acc", max_trials=10, study_dir=str(tmp_path), directory=str(tmp_path / "g"))
    g.search(x, y, epochs=1, batch_size=32)
    trials = g.oracle.service.list_trials()
    assert len(trials) == 6  # 3 units x 2 activations, then exhausted
    r = RandomSearch(_build, objective="acc", max_trials=2, study_dir=str(tmp_path), directory=str(tmp_path / "r"))
    r.search(x, y, epochs=1, batch_size=32)
    assert len(r.oracle.service.list_trials()) == 2


def test_failed_trial_is_infeasible(tmp_path, monkeypatch):
    monkeypatch.setenv("CLOUD_AMD_FAULT", "0:0:raise")
    rng = np.random.default_rng(2)
    x = rng.normal(size=(64, 20)).astype("float32")
    y = (x[:, 0] > 0).astype("int64")
    tuner = CloudTuner(_build, objective="acc", hyperparameters=_hps(), max_trials=2, study_id="fail",
                       study_dir=str(tmp_path), directory=str(tmp_path / "res"))
    tuner.search(x, y, epochs=1, batch_size=32)
    trials = tuner.oracle.service.list_trials()
    assert all(t.get("trialInfeasible") for t in trials)


def test_distributed_tuning_four_workers(tmp_path):
    env = {"STUDY_ID": "dist", "STUDY_DIR": str(tmp_path), "PYTHONPATH": os.path.join(HERE, "data")}
    import sys

    sys.path.insert(0, os.path.join(HERE, "data"))
    sched = TrialScheduler("tuner_worker:run", n_gpus=0, workers=4, env=env)
    res = sched.run(timeout=600)
    assert res["exit_codes"] == [0, 0, 0, 0]
    with open(tmp_path / "CloudTuner_study_dist" / "study.json") as f:
        trials = json.load(f)["trials"]
    assert len(trials) == 6 and all(t["state"] == "COMPLETED" for t in trials)
    assert len({t["clientId"] for t in trials}) >= 2


def test_scheduler_packs_from_measured_footprint(tmp_path):
    """Default (measured) packing: a probe worker reports its trial's peak HBM and the
    scheduler adds workers until the GPU holds trials_per_gpu(peak * headroom)."""
    import sys

    sys.path.insert(0, os.path.join(HERE, "data"))
    env = {"STUDY_ID": "packed", "STUDY_DIR": str(tmp_path), "PYTHONPATH": os.path.join(HERE, "data"),
           "FAKE_FOOTPRINT_GB": "1.0"}
    sched = TrialScheduler("tuner_worker:run", n_gpus=0, env=env, hbm_gb=4.0, max_workers=8,
                           state_dir=str(tmp_path / "sched"), timeline=True)
    assert sched.packing_from_footprint(1.0) == 2          # 4 GB * 0.9 // (1.0 * 1.25)
    assert sched.packing_from_footprint(0.05) == 57
    res = sched.run(timeout=600)
    assert res["footprint_gb"] == 1.0 and res["trials_per_gpu"] == 2 and res["workers"] == 2
    assert res["exit_codes"] == [0, 0]
    with open(tmp_path / "CloudTuner_study_packed" / "study.json") as f:
        trials = json.load(f)["trials"]
    assert len(trials) == 6 and all(t["state"] == "COMPLETED" for t in trials)
    assert all(t["startTs"] <= t["endTs"] for t in trials)
    # per-worker phase marks: the probe, then 7 gated standbys (1 released, 6 dismissed)
    tl = res["timeline"]
    assert tl["tuner0"]["entered"] <= tl["tuner0"]["exited"] and "imported" not in tl["tuner0"]
    standby = [tl[f"tuner{i}"] for i in range(1, 8)]
    assert sum("released" in m for m in standby) == 1 and sum("dismissed" in m for m in standby) == 6
    assert all(m["imported"] <= m.get("released", m.get("dismissed")) for m in standby)


def test_scheduler_places_trials_round_robin_over_eight_gpus(tmp_path):
    """BASELINE config 4 (one trial per MI355X and packing within each GPU's HBM) on an
    8-GPU placement rehearsed on CPU: one probe worker per GPU, packing from the measured
    footprint, round-robin device assignment, and each trial's device in the study."""
    import sys

    sys.path.insert(0, os.path.join(HERE, "data"))
    env = {"STUDY_ID": "eight", "STUDY_DIR": str(tmp_path), "PYTHONPATH": os.path.join(HERE, "data"),
           "FAKE_FOOTPRINT_GB": "1.0", "MAX_TRIALS": "16", "CLOUD_AMD_SCHED_FAKE_DEVICES": "1",
           "OMP_NUM_THREADS": "1"}
    sched = TrialScheduler("tuner_worker:run", n_gpus=8, env=env, hbm_gb=4.0, max_workers=16,
                           state_dir=str(tmp_path / "sched"), timeline=True)
    # probe wave = one worker per GPU; standbys capped by max_workers - GPUs
    assert sched.devices() == ["cuda:%d" % i for i in range(8)]
    assert sched.standby_count() == 8
    res = sched.run(timeout=900)
    assert res["footprint_gb"] == 1.0 and res["trials_per_gpu"] == 2   # 4 GB * 0.9 // 1.25
    assert res["workers"] == 16 and res["exit_codes"] == [0] * 16
    assert sched.devices() == ["cuda:%d" % (i % 8) for i in range(16)]
    tl = res["timeline"]
    probes = [tl["tuner%d" % i] for i in range(8)]
    assert all("imported" not in m for m in probes)          # probes run at once, ungated
    assert sum("released" in tl["tuner%d" % i] for i in range(8, 16)) == 8
    with open(tmp_path / "CloudTuner_study_eight" / "study.json") as f:
        trials = json.load(f)["trials"]
    assert len(trials) == 16 and all(t["state"] == "COMPLETED" for t in trials)
    for t in trials:  # trial -> device record follows the worker's round-robin slot
        i = int(t["clientId"][len("tuner"):])
        assert t["device"] == "cuda:%d" % (i % 8), t
    assert len({t["device"] for t in trials}) >= 2


def test_standby_gate_gives_up_without_scheduler(tmp_path):
    from cloud_amd.tuner.scheduler import _await_gate

    gate = str(tmp_path / "gate.json")
    t0 = time.time()
    assert _await_gate(gate, parent=-1, deadline_s=30) is False        # parent gone
    assert _await_gate(gate, deadline_s=0.2) is False                  # deadline
    assert _await_gate(str(tmp_path / "gone" / "g.json"), deadline_s=30) is False  # state dir removed
    assert time.time() - t0 < 5
    TrialScheduler._open_gate(gate, True)
    assert _await_gate(gate) is True


def test_tuner_reports_footprint_after_first_trial(tmp_path, monkeypatch):
    from cloud_amd.utils import hbm

    out = tmp_path / "fp.json"
    monkeypatch.setenv("CLOUD_AMD_FOOTPRINT_FILE", str(out))
    monkeypatch.setattr(hbm, "trial_footprint_gb", lambda device=None: 3.5)
    rng = np.random.default_rng(2)
    x = rng.normal(size=(64, 20)).astype("float32")
    y = (x[:, 0] > 0).astype("int64")
    tuner = CloudTuner(_build, objective="acc", hyperparameters=_hps(), max_trials=2, study_id="fp",
                       study_dir=str(tmp_path), directory=str(tmp_path / "res"))
    tuner.search(x, y, epochs=1, batch_size=32)
    assert json.load(open(out))["peak_gb"] == 3.5


def test_reported_footprint_includes_validation_arrays(tmp_path, monkeypatch):
    """The probe reports after batch 0 of its first trial, before evaluate() uploads the
    validation set at epoch end: the validation bytes are added to the measured peak."""
    from cloud_amd.utils import hbm

    out = tmp_path / "fp.json"
    monkeypatch.setenv("CLOUD_AMD_FOOTPRINT_FILE", str(out))
    monkeypatch.setattr(hbm, "trial_footprint_gb", lambda device=None: 1.0)
    rng = np.random.default_rng(3)
    x = rng.normal(size=(64, 20)).astype("float32")
    y = (x[:, 0] > 0).astype("int64")
    xv = rng.normal(size=(4096, 1024)).astype("float32")  # 16 MiB
    yv = np.zeros(4096, dtype="int64")
    tuner = CloudTuner(_build, objective="acc", hyperparameters=_hps(), max_trials=1, study_id="fpv",
                       study_dir=str(tmp_path), directory=str(tmp_path / "res"))
    assert abs(hbm.array_gb((xv, yv)) - (xv.nbytes + yv.nbytes) / 2 ** 30) < 1e-12
    tuner._val_gb = 0.0
    monkeypatch.setattr(tuner, "run_trial", lambda trial, *a, **k: None)
    tuner.search(x, y, epochs=1, batch_size=32, validation_data=(xv, yv))
    got = json.load(open(out))["peak_gb"]
    assert abs(got - (1.0 + (xv.nbytes + yv.nbytes) / 2 ** 30)) < 1e-9


def test_worker_pool_reused_across_studies(tmp_path):
    """Warm pool: the workers import once, then run two studies back to back (the second
    starts its trials with no interpreter start / import on its critical path)."""
    import sys

    from cloud_amd.tuner.scheduler import WorkerPool

    sys.path.insert(0, os.path.join(HERE, "data"))
    pool = WorkerPool(3, preload=["tuner_worker"], env={"PYTHONPATH": os.path.join(HERE, "data"),
                                                        "OMP_NUM_THREADS": "1"})
    try:
        warm_s = pool.wait_ready()
        assert warm_s > 0
        pids = [p.pid for p in pool._procs]
        walls = []
        for sid in ("pool_a", "pool_b"):
            env = {"STUDY_ID": sid, "STUDY_DIR": str(tmp_path), "MAX_TRIALS": "6"}
            sched = TrialScheduler("tuner_worker:run", n_gpus=0, workers=3, env=env, pool=pool, timeline=True)
            res = sched.run(timeout=600)
            assert res["pool"] and res["exit_codes"] == [0, 0, 0], res
            walls.append(res["wall_s"])
            with open(tmp_path / ("CloudTuner_study_" + sid) / "study.json") as f:
                trials = json.load(f)["trials"]
            assert len(trials) == 6 and all(t["state"] == "COMPLETED" for t in trials)
            assert all("imported" not in m for m in res["timeline"].values())  # no per-study import
        assert [p.pid for p in pool._procs] == pids and all(p.is_alive() for p in pool._procs)
        # measured packing on a pool: one probe, then the packing wave on idle warm workers
        env = {"STUDY_ID": "pool_c", "STUDY_DIR": str(tmp_path), "MAX_TRIALS": "6", "FAKE_FOOTPRINT_GB": "1.0"}
        sched = TrialScheduler("tuner_worker:run", n_gpus=0, env=env, pool=pool, hbm_gb=4.0, max_workers=3)
        res = sched.run(timeout=600)
        assert res["footprint_gb"] == 1.0 and res["workers"] == 2 and res["exit_codes"] == [0, 0]
    finally:
        pool.close()
    assert all(not p.is_alive() for p in pool._procs)
