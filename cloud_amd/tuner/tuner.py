"""``CloudOracle`` / ``CloudTuner`` on the local study service.

API parity with reference ``TFC/tuner/tuner.py:32-376`` (itself a KerasTuner
``Oracle`` / ``Tuner``): same constructor arguments (``project_id`` and
``region`` are kept as study-name components; there is no cloud project), the
same ``study_config`` XOR (``objective`` + ``hyperparameters``) rule, the same
trial lifecycle (create -> update per epoch with early-stop polling -> end
COMPLETED / INVALID(infeasible)), ``get_best_trials`` ordering, and the
``CloudTuner_study_<id>`` naming that lets many tuner processes (one per
MI355X, distinct ``tuner_id``) share a study.

The KerasTuner base classes are re-implemented here (keras-tuner is not in
this stack): ``Tuner.search / results_summary / search_space_summary /
get_best_models / get_best_hyperparameters``, trial directories under
``<directory>/<project_name>/trial_<id>/``, oracle state in ``oracle.json``.
``RandomSearch`` / ``GridSearch`` / ``BayesianOptimization`` are the same
machinery with a fixed study algorithm.
"""
from __future__ import annotations

import datetime
import json
import logging
import os
import time
import traceback

from .. import monitoring
from . import hyperparameters as hp_module
from . import optimizer_client, utils
from .trial import Objective, Trial, TrialStatus

log = logging.getLogger("cloud_amd.tuner")


class Oracle:
    """KerasTuner-style oracle base: owns trials and their persistence."""

    def __init__(self, objective=None, hyperparameters=None, max_trials=None, allow_new_entries=True,
                 tune_new_entries=True):
        self.objective = utils.format_objective(objective) if objective is not None else None
        self.hyperparameters = hyperparameters or hp_module.HyperParameters()
        self.max_trials = max_trials
        self.allow_new_entries, self.tune_new_entries = allow_new_entries, tune_new_entries
        self.trials = {}
        self.ongoing_trials = {}
        self._dir = None

    def _set_project_dir(self, directory, project_name):
        self._dir = os.path.join(directory, project_name)
        os.makedirs(self._dir, exist_ok=True)

    def _get_trial_dir(self, trial_id):
        return os.path.join(self._dir or ".", f"trial_{trial_id}")

    def _save_trial(self, trial):
        if self._dir is not None and trial.trial_id is not None:
            trial.save(os.path.join(self._get_trial_dir(trial.trial_id), "trial.json"))

    def save(self):
        if self._dir is None:
            return
        state = {"ongoing_trials": {k: t.trial_id for k, t in self.ongoing_trials.items()},
                 "trial_ids": sorted(self.trials), "hyperparameters": self.hyperparameters.get_config()}
        tmp = os.path.join(self._dir, "oracle.json.tmp")
        with open(tmp, "w") as f:
            json.dump(state, f, indent=2, default=str)
        os.replace(tmp, os.path.join(self._dir, "oracle.json"))

    def get_space(self):
        return self.hyperparameters.copy()


class CloudOracle(Oracle):
    def __init__(self, project_id="local", region="local", objective=None, hyperparameters=None, study_config=None,
                 max_trials=None, study_id=None, study_dir=None, algorithm=None):
        if study_config:
            if objective or hyperparameters:
                raise ValueError('Please configure either study_config or "objective, and hyperparameters".')
            objective = utils.convert_study_config_to_objective(study_config)
            hyperparameters = utils.convert_study_config_to_hps(study_config)
            self.study_config = study_config
        else:
            if not (objective and hyperparameters):
                raise ValueError("If study_config is not set, objective and hyperparameters must be set.")
            self.study_config = utils.make_study_config(objective, hyperparameters)
        if algorithm:
            self.study_config["algorithm"] = algorithm
        super().__init__(objective=objective, hyperparameters=hyperparameters, max_trials=max_trials,
                         allow_new_entries=False, tune_new_entries=False)
        if not project_id:
            raise ValueError('"project_id" is not found.')
        if not region:
            raise ValueError('"region" is not found.')
        self.project_id, self.region = project_id, region
        self.objective = utils.format_objective(objective)
        self.hyperparameters = hyperparameters
        self.max_trials = max_trials
        if study_id:
            self.study_id = "CloudTuner_study_{}".format(study_id)
        else:
            self.study_id = "CloudTuner_study_{}".format(datetime.datetime.now().strftime("%Y%m%d_%H%M%S"))
        self.service = optimizer_client.create_or_load_study(self.project_id, self.region, self.study_id,
                                                             self.study_config, root=study_dir)
        self._start_time = None

    def create_trial(self, tuner_id):
        trial_list = self.service.list_trials()
        stopping = [t for t in trial_list if t["state"] == "STOPPING"]
        if (self.max_trials and len(trial_list) >= self.max_trials) or stopping:
            hps = self.hyperparameters.copy()
            hps.values = None
            return Trial(hyperparameters=hps, trial_id="n", status=TrialStatus.STOPPED)
        suggestions = self.service.get_suggestions(tuner_id, max_trials=self.max_trials)
        if "trials" not in suggestions:
            return Trial(hyperparameters={}, status=TrialStatus.STOPPED)
        opt_trial = suggestions["trials"][0]
        trial_id = utils.get_trial_id(opt_trial)
        trial = Trial(hyperparameters=utils.convert_optimizer_trial_to_hps(self.hyperparameters.copy(), opt_trial),
                      trial_id=trial_id, status=TrialStatus.RUNNING)
        log.info("Hyperparameters requested by tuner (%s): %s ", tuner_id, trial.hyperparameters.values)
        self._start_time = time.time()
        monitoring.inc(monitoring.TRIALS, 1, event="created", tuner=str(tuner_id))
        self.trials[trial_id] = trial
        self.ongoing_trials[tuner_id] = trial
        self._save_trial(trial)
        self.save()
        return trial

    def update_trial(self, trial_id, metrics, step=0):
        elapsed = time.time() - (self._start_time or time.time())
        if elapsed < 0 or step < 0:
            raise ValueError("Both elapsed_secs and step must be non-negative.")
        if elapsed == 0 and step == 0:
            raise ValueError("At least one of {elapsed_secs, step} must be positive")
        metric_list = []
        for ob in self.objective:
            if ob.name not in metrics:
                log.info('Objective "%s" is not found in metrics.', ob.name)
                continue
            metric_list.append({"metric": ob.name, "value": float(metrics.get(ob.name))})
        self.service.report_intermediate_objective_value(step, elapsed, metric_list, trial_id)
        trial = self.trials[trial_id]
        for k, v in metrics.items():
            if isinstance(v, (int, float)):
                trial.update_metric(k, v, step, next((o.direction for o in self.objective if o.name == k), "min"))
        log.info("UpdateTrial: polls the stop decision.")
        if self.service.should_trial_stop(trial_id):
            trial.status = TrialStatus.STOPPED
            monitoring.inc(monitoring.TRIALS, 1, event="early_stopped")
        return trial.status

    def end_trial(self, trial_id, status="COMPLETED"):
        trial = None
        for tuner_id, t in list(self.ongoing_trials.items()):
            if t.trial_id == trial_id:
                log.info("End trial requested by tuner (%s)", tuner_id)
                trial = self.ongoing_trials.pop(tuner_id)
                break
        if not trial:
            raise ValueError("Ongoing trial with id: {} not found.".format(trial_id))
        trial.status = status
        if status == TrialStatus.COMPLETED:
            infeasible, reason = False, None
        elif status == TrialStatus.INVALID:
            infeasible, reason = True, status
        else:
            raise ValueError('Unexpected status passed. Expected "COMPLETED" or "INVALID", found {}'.format(status))
        opt_trial = self.service.complete_trial(trial_id, infeasible, reason)
        monitoring.inc(monitoring.TRIALS, 1, event=str(status).lower())
        if status == TrialStatus.COMPLETED and opt_trial.get("finalMeasurement"):
            fm = opt_trial["finalMeasurement"]
            trial.best_step = fm.get("stepCount", 1)
            trial.score = fm["metrics"][0]["value"] if fm.get("metrics") else None
        self._save_trial(trial)
        self.save()

    def get_best_trials(self, num_trials=1):
        if len(self.objective) > 1:
            raise ValueError("Getting the best trials for multi-objective optimization is not supported. ")
        maximizing = utils.format_goal(self.objective[0].direction) == "MAXIMIZE"
        done = [t for t in self.service.list_trials() if t["state"] == "COMPLETED" and not t.get("trialInfeasible")
                and t.get("finalMeasurement", {}).get("metrics")]
        done.sort(key=lambda t: t["finalMeasurement"]["metrics"][0]["value"], reverse=maximizing)
        out = []
        for ot in done[:num_trials]:
            fm = ot["finalMeasurement"]
            t = Trial(hyperparameters=utils.convert_optimizer_trial_to_hps(self.hyperparameters.copy(), ot),
                      trial_id=utils.get_trial_id(ot), status=TrialStatus.COMPLETED)
            t.best_step = fm.get("stepCount", 1)
            t.score = fm["metrics"][0]["value"]
            out.append(t)
        return out


class _TunerCallback:
    """Reports epoch logs to the oracle; stops fit when the oracle says so."""

    def __init__(self, tuner, trial):
        from ..keras.callbacks import Callback

        class CB(Callback):
            def on_train_batch_end(cb, batch, logs=None):
                # the scheduler's probe worker: report the measured footprint after the
                # first optimizer step of the first trial (the training step is the trial's
                # memory peak; the scheduler adds its headroom), so the packing wave starts
                # a whole trial earlier than after the trial ends
                if tuner._early_report_pending and batch == 0:
                    from ..utils import hbm

                    tuner._early_report_pending = False
                    if hbm.report_footprint(extra_gb=tuner._val_gb) is not None:
                        tuner._reported = True

            def on_epoch_end(cb, epoch, logs=None):
                status = tuner.oracle.update_trial(trial.trial_id, dict(logs or {}), step=epoch + 1)
                if status == TrialStatus.STOPPED:
                    cb.model.stop_training = True
                tuner._maybe_checkpoint(trial, cb.model, logs or {}, epoch)

        self.cb = CB()


class Tuner:
    """KerasTuner-style search loop over an oracle."""

    def __init__(self, oracle, hypermodel, directory=None, project_name=None, executions_per_trial=1,
                 tuner_id=None, overwrite=False, max_model_size=None, optimizer=None, loss=None, metrics=None,
                 **kwargs):
        self.oracle = oracle
        self.hypermodel = hypermodel if callable(hypermodel) else hypermodel.build
        self.directory = directory or os.environ.get("CLOUD_AMD_TUNER_DIR", "tuner_results")
        self.project_name = project_name or "untitled_project"
        self.executions_per_trial = executions_per_trial
        self.tuner_id = tuner_id or os.environ.get("KERASTUNER_TUNER_ID") or os.environ.get("CLOUD_AMD_TUNER_ID") \
            or "tuner0"
        self.oracle._set_project_dir(self.directory, self.project_name)
        self._best_scores = {}

    @property
    def project_dir(self):
        return os.path.join(self.directory, self.project_name)

    def search_space_summary(self, extended=False):
        print("Search space summary")
        hps = self.oracle.get_space()
        print(f"Default search space size: {len(hps.space)}")
        for hp in hps.space:
            print(f"{hp.name} ({type(hp).__name__})")
            cfg = hp.get_config()
            cfg.pop("name", None)
            print(cfg)

    def results_summary(self, num_trials=10):
        print("Results summary")
        print(f"Results in {self.project_dir}")
        print(f"Showing {num_trials} best trials")
        for o in self.oracle.objective:
            print(f"Objective(name='{o.name}', direction='{o.direction}')")
        for t in self.oracle.get_best_trials(num_trials):
            print()
            print(f"Trial {t.trial_id} summary")
            print("Hyperparameters:")
            for k, v in (t.hyperparameters.values or {}).items():
                print(f"{k}: {v}")
            print(f"Score: {t.score}")

    def _build(self, hp):
        from ..utils import hbm

        model = self.hypermodel(hp)
        hbm.note_model(model)
        return model

    def run_trial(self, trial, *fit_args, **fit_kwargs):
        cb = _TunerCallback(self, trial).cb
        callbacks = list(fit_kwargs.pop("callbacks", []) or []) + [cb]
        hist = None
        for _ in range(self.executions_per_trial):
            model = self._build(trial.hyperparameters)
            hist = model.fit(*fit_args, callbacks=callbacks, verbose=fit_kwargs.pop("verbose", 0), **fit_kwargs)
        return hist

    def _maybe_checkpoint(self, trial, model, logs, epoch):
        ob = self.oracle.objective[0]
        v = logs.get(ob.name)
        if v is None:
            return
        best = self._best_scores.get(trial.trial_id)
        better = best is None or (v > best if ob.direction == "max" else v < best)
        if better:
            self._best_scores[trial.trial_id] = v
            d = self.oracle._get_trial_dir(trial.trial_id)
            os.makedirs(d, exist_ok=True)
            from ..parallel.strategy import get_strategy

            if get_strategy().is_chief:
                model.save_weights(os.path.join(d, "checkpoint.pt"))

    def search(self, *fit_args, **fit_kwargs):
        from ..utils import faults  # noqa: F401  (fault injection reaches trials through fit)
        from ..utils import hbm

        from .. import config

        self._reported = False
        # measured after batch 0 of the first trial, before evaluate() uploads the
        # validation set to the device: its bytes are added to the reported peak
        self._val_gb = hbm.array_gb(fit_kwargs.get("validation_data"))
        # CLOUD_AMD_TUNER_EARLY_FOOTPRINT: report after the first step (default) or the first trial
        self._early_report_pending = bool(os.environ.get("CLOUD_AMD_FOOTPRINT_FILE")) and bool(
            config.get("CLOUD_AMD_TUNER_EARLY_FOOTPRINT"))
        while True:
            trial = self.oracle.create_trial(self.tuner_id)
            if trial.status == TrialStatus.STOPPED:
                log.info("Oracle triggered exit")
                break
            try:
                self.run_trial(trial, *fit_args, **dict(fit_kwargs))
            except Exception as e:  # a failing trial is infeasible, the search continues
                log.warning("trial %s failed: %s\n%s", trial.trial_id, e, traceback.format_exc())
                self.oracle.end_trial(trial.trial_id, TrialStatus.INVALID)
                continue
            self.oracle.end_trial(trial.trial_id, TrialStatus.COMPLETED)
            if not self._reported:  # the scheduler packs more workers per GPU from this measurement
                hbm.report_footprint(extra_gb=self._val_gb)
                self._reported = True
                self._early_report_pending = False

    def get_best_hyperparameters(self, num_trials=1):
        return [t.hyperparameters for t in self.oracle.get_best_trials(num_trials)]

    def get_best_models(self, num_models=1):
        models = []
        for t in self.oracle.get_best_trials(num_models):
            m = self.hypermodel(t.hyperparameters)
            ck = os.path.join(self.oracle._get_trial_dir(t.trial_id), "checkpoint.pt")
            if os.path.exists(ck):
                m.load_weights(ck)
            models.append(m)
        return models


class CloudTuner(Tuner):
    def __init__(self, hypermodel, project_id="local", region="local", objective=None, hyperparameters=None,
                 study_config=None, max_trials=None, study_id=None, study_dir=None, **kwargs):
        oracle = CloudOracle(project_id=project_id, region=region, objective=objective,
                             hyperparameters=hyperparameters, study_config=study_config, max_trials=max_trials,
                             study_id=study_id, study_dir=study_dir)
        super().__init__(oracle=oracle, hypermodel=hypermodel, **kwargs)


def _local_tuner(algorithm):
    class _T(Tuner):
        def __init__(self, hypermodel, objective, max_trials, hyperparameters=None, study_id=None, study_dir=None,
                     **kwargs):
            hps = hyperparameters
            if hps is None:  # declare the space by building once with defaults (KerasTuner style)
                hps = hp_module.HyperParameters()
                hypermodel(hps)
            oracle = CloudOracle(objective=objective, hyperparameters=hps, max_trials=max_trials,
                                 study_id=study_id or f"{algorithm.lower()}_{int(time.time() * 1e3)}",
                                 study_dir=study_dir, algorithm=algorithm)
            super().__init__(oracle=oracle, hypermodel=hypermodel, **kwargs)

    _T.__name__ = algorithm.title().replace("_", "")
    return _T


RandomSearch = _local_tuner("RANDOM_SEARCH")
GridSearch = _local_tuner("GRID_SEARCH")
BayesianOptimization = _local_tuner("GAUSSIAN_PROCESS_BANDIT")
__all__ = ["CloudOracle", "CloudTuner", "Oracle", "Tuner", "RandomSearch", "GridSearch", "BayesianOptimization",
           "Objective"]
