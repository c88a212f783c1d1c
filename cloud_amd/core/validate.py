"""Fail-fast argument checking for ``run()``.

Same checks and error-message prefixes as reference ``TFC/core/validate.py:23-218``
(tests match on the prefixes), with the GCP SKU / TPU-TF-version checks
replaced by local-node capability checks: an MI355X job must fit the GPUs of
the node, and TPU workers have no analogue here.
"""
from __future__ import annotations

import os

from . import machine_config, topology


def validate(entry_point, requirements_txt, distribution_strategy, chief_config, worker_config, worker_count,
             region, entry_point_args, stream_logs, docker_image_bucket_name, called_from_notebook,
             job_labels=None, docker_base_image=None, check_node=False):
    _validate_files(entry_point, requirements_txt)
    _validate_distribution_strategy(distribution_strategy)
    _validate_cluster_config(chief_config, worker_count, worker_config, docker_base_image)
    topology.validate_job_labels(job_labels or {})
    _validate_other_args(region, entry_point_args, stream_logs, docker_image_bucket_name, called_from_notebook)
    if check_node:
        validate_node_capacity(chief_config, worker_config, worker_count)


def _validate_files(entry_point, requirements_txt):
    cwd = os.getcwd()
    if entry_point is not None and not os.path.isfile(os.path.join(cwd, entry_point)):
        raise ValueError("Invalid `entry_point`. Expected a relative path in the current directory tree. "
                         "Received: {}".format(entry_point))
    if requirements_txt is not None and not os.path.isfile(os.path.join(cwd, requirements_txt)):
        raise ValueError("Invalid `requirements_txt`. Expected a relative path in the current directory tree. "
                         "Received: {}".format(requirements_txt))
    if entry_point is not None and not (entry_point.endswith("py") or entry_point.endswith("ipynb")):
        raise ValueError("Invalid `entry_point`. Expected a python file or an iPython notebook. "
                         "Received: {}".format(entry_point))


def _validate_distribution_strategy(distribution_strategy):
    if distribution_strategy not in ("auto", None):
        raise ValueError('Invalid `distribution_strategy` input. Expected "auto" or None. '
                         "Received {}.".format(distribution_strategy))


def _validate_cluster_config(chief_config, worker_count, worker_config, docker_base_image=None):
    if not isinstance(chief_config, machine_config.MachineConfig):
        raise ValueError('Invalid `chief_config` input. Expected "auto" or `MachineConfig` instance. '
                         "Received {}.".format(chief_config))
    if worker_count < 0:
        raise ValueError("Invalid `worker_count` input. Expected a postive integer value. "
                         "Received {}.".format(worker_count))
    if worker_count > 0 and not isinstance(worker_config, machine_config.MachineConfig):
        raise ValueError('Invalid `worker_config` input. Expected "auto" or `MachineConfig` instance. '
                         "Received {}.".format(worker_config))
    if machine_config.is_tpu_config(chief_config):
        raise ValueError("Invalid `chief_config` input. `chief_config` cannot be a TPU config. "
                         "Received {}.".format(chief_config))
    if machine_config.is_tpu_config(worker_config) and worker_count > 0:
        if worker_count != 1:
            raise ValueError("Invalid `worker_count` input. Expected worker_count=1 for TPU `worker_config`. "
                             "Received {}.".format(worker_count))
        raise NotImplementedError("TPU workers are not supported on MI355X nodes; use an MI355X "
                                  "`worker_config` (e.g. COMMON_MACHINE_CONFIGS['MI355X_8X']).")


def _validate_other_args(region, args, stream_logs, docker_image_bucket_name, called_from_notebook):
    if not isinstance(region, str):
        raise ValueError("Invalid `region` input. Expected None or a string value. Received {}.".format(region))
    if args is not None and not isinstance(args, list):
        raise ValueError("Invalid `entry_point_args` input. Expected None or a list. Received {}.".format(args))
    if not isinstance(stream_logs, bool):
        raise ValueError("Invalid `stream_logs` input. Expected a boolean. Received {}.".format(stream_logs))
    # The reference required a GCS bucket for notebook builds (validate.py:209-218);
    # staging is local here, so a bucket name is accepted but never required.


def cluster_gpu_count(chief_config, worker_config, worker_count):
    n = chief_config.accelerator_count if chief_config.is_gpu else 0
    if worker_count > 0 and worker_config is not None and worker_config.is_gpu:
        n += worker_count * worker_config.accelerator_count
    return n


def cpu_rehearsal():
    """``CLOUD_AMD_DEVICE=cpu`` exported by the caller: a GPU-shaped job (same machine
    configs, same strategy auto-selection) whose ranks train on the CPU over gloo -- the
    multi-rank launch path rehearsed on a host without GPUs."""
    return os.environ.get("CLOUD_AMD_DEVICE") == "cpu"


def validate_node_capacity(chief_config, worker_config, worker_count, available=None):
    """All ranks of a single-node job must map onto distinct local GPUs."""
    need = cluster_gpu_count(chief_config, worker_config, worker_count)
    if need == 0 or cpu_rehearsal():
        return
    have = topology.visible_gpu_count() if available is None else available
    if need > have:
        raise ValueError("Invalid cluster config: the job needs {} GPUs (chief + {} worker(s)) but this node "
                         "exposes {}.".format(need, worker_count, have))
