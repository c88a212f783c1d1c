"""Optimizer client with the reference's method surface
(``TFC/tuner/optimizer_client.py:35-443``) on the local study service.

The REST round trips, long-running-operation polling and HTTP error codes of
the reference become direct calls; the *semantics* are kept: 429 (trial cap /
exhausted space) -> ``get_suggestions`` returns ``{}``; an INACTIVE study with
no trials -> :class:`SuggestionInactiveError`; 404 on delete -> ValueError;
create-or-load tolerates concurrent creators (409 -> load, retried
``NUM_TRIES_FOR_STUDIES`` times one second apart).
"""
from __future__ import annotations

import time

from . import constants
from .study_service import StudyExists, StudyNotFound, StudyService, TooManyTrials


class SuggestionInactiveError(Exception):
    """Indicates that GetSuggestion was called on an inactive study."""


class _OptimizerClient:
    def __init__(self, service, project_id, region, study_id):
        self.service = service
        self.project_id, self.region, self.study_id = project_id, region, study_id

    def get_suggestions(self, client_id, max_trials=None):
        try:
            resp = self.service.suggest(self._make_study_name(), client_id,
                                        count=constants.SUGGESTION_COUNT_PER_REQUEST, max_trials=max_trials)
        except TooManyTrials:
            return {}
        if "trials" not in resp:
            if resp.get("studyState") == "INACTIVE":
                raise SuggestionInactiveError("The study is stopped due to an internal error.")
            return {}
        return resp

    def report_intermediate_objective_value(self, step, elapsed_secs, metric_list, trial_id):
        measurement = {"stepCount": step, "elapsedTime": {"seconds": int(elapsed_secs)}, "metrics": metric_list}
        self.service.add_measurement(self._make_trial_name(trial_id), measurement)

    def should_trial_stop(self, trial_id):
        name = self._make_trial_name(trial_id)
        resp = self.service.check_early_stopping_state(name)
        if resp.get("shouldStop"):
            self.service.stop_trial(name)
            return True
        return False

    def complete_trial(self, trial_id, trial_infeasible, infeasibility_reason=None):
        return self.service.complete_trial(self._make_trial_name(trial_id), trial_infeasible, infeasibility_reason)

    def list_trials(self):
        return self.service.list_trials(self._make_study_name())

    def list_studies(self):
        return self.service.list_studies(self._make_parent_name())

    def delete_study(self, study_name=None):
        name = study_name or self._make_study_name()
        try:
            self.service.delete_study(name)
        except StudyNotFound as e:
            raise ValueError(f"DeleteStudy failed. Study not found: {name}.") from e

    def _make_parent_name(self):
        return f"projects/{self.project_id}/locations/{self.region}"

    def _make_study_name(self):
        return f"{self._make_parent_name()}/studies/{self.study_id}"

    def _make_trial_name(self, trial_id):
        return f"{self._make_study_name()}/trials/{trial_id}"


def create_or_load_study(project_id, region, study_id, study_config, service=None, root=None):
    service = service or StudyService(root)
    parent = f"projects/{project_id}/locations/{region}"
    try:
        service.create_study(parent, study_id, study_config)
    except StudyExists:
        for i in range(constants.NUM_TRIES_FOR_STUDIES):
            try:
                service.get_study(f"{parent}/studies/{study_id}")
                break
            except StudyNotFound:
                if i == constants.NUM_TRIES_FOR_STUDIES - 1:
                    raise
                time.sleep(1)
    return _OptimizerClient(service, project_id, region, study_id)
