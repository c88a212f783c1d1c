"""Client side of ``cloud_fit`` (reference ``experimental/cloud_fit/client.py``).

Serialises a compiled model, its ``fit`` arguments (datasets / arrays,
validation data, callbacks -- cloudpickled) into ``remote_dir`` using the
reference's layout::

    <remote_dir>/training_assets/   fit kwargs, x, validation data, callbacks
    <remote_dir>/model/             the compiled input model (cloud_amd saved model)
    <remote_dir>/output/            the trained model, written by the chief

and launches ``python -m cloud_amd.experimental.cloud_fit.remote --remote_dir
<dir> --distribution_strategy <name>`` as a local multi-process job (one rank
per MI355X, or CPU ranks on a GPU-less node).  Returns the job id as soon as the job
is submitted (its supervisor runs it to completion on its own).
"""
from __future__ import annotations

import datetime
import logging
import os
import shutil
import tempfile

from ...core import launcher, machine_config, stage, topology
from . import utils

log = logging.getLogger("cloud_amd.cloud_fit")
DEFAULT_DISTRIBUTION_STRATEGY = utils.MULTI_WORKER_MIRRORED_STRATEGY_NAME
ASSET_FILES = ("fit_kwargs.pkl", "x.pkl", "validation_data.pkl", "callbacks.pkl")


def cloud_fit(model, remote_dir, region=None, project_id=None, image_uri=None,
              distribution_strategy=DEFAULT_DISTRIBUTION_STRATEGY, job_spec=None, job_id=None, wait=False,
              **fit_kwargs):
    """Serialise ``model`` and the ``fit`` arguments into ``remote_dir`` and submit the
    training job; returns the job id right after submission, as the reference does
    (``client.py:227-286``).  The job runs under its detached supervisor:
    ``python -m cloud_amd.jobs describe|stream-logs|cancel <job_id>`` follows it, and
    ``cloud_amd.core.launcher.Job.attach(job_id).wait()`` blocks on it.  ``wait=True``
    blocks here and raises ``RuntimeError`` if the job fails."""
    if distribution_strategy not in utils.SUPPORTED_DISTRIBUTION_STRATEGIES:
        raise ValueError("{} is not supported. Supported Strategies are {}".format(
            distribution_strategy, list(utils.SUPPORTED_DISTRIBUTION_STRATEGIES.keys())))
    args = ["--remote_dir", remote_dir, "--distribution_strategy", distribution_strategy]
    if job_spec:
        job_spec["trainingInput"]["args"] = args
    else:
        job_spec = _default_job_spec(region=region, image_uri=image_uri, entry_point_args=args,
                                     distribution_strategy=distribution_strategy)
    _serialize_assets(remote_dir, model, **fit_kwargs)
    job_spec["trainingInput"]["useChiefInTfConfig"] = "True"
    if job_id:
        job_spec["jobId"] = job_id
    return _submit_job(job_spec, wait=wait)


def _serialize_assets(remote_dir, model, **fit_kwargs):
    import cloudpickle

    if "x" in fit_kwargs and hasattr(fit_kwargs["x"], "__next__"):
        raise NotImplementedError("Generators are not supported; pass arrays or a cloud_amd Dataset.")
    assets = os.path.join(remote_dir, "training_assets")
    os.makedirs(assets, exist_ok=True)
    kw = dict(fit_kwargs)
    parts = {"x.pkl": {k: kw.pop(k) for k in ("x", "y") if k in kw},
             "validation_data.pkl": kw.pop("validation_data", None),
             "callbacks.pkl": kw.pop("callbacks", None)}
    parts["fit_kwargs.pkl"] = kw
    by_value = _user_modules(parts["callbacks.pkl"])
    for m in by_value:
        cloudpickle.register_pickle_by_value(m)
    try:
        for name, obj in parts.items():
            with open(os.path.join(assets, name), "wb") as f:
                cloudpickle.dump(obj, f)
    finally:
        for m in by_value:
            cloudpickle.unregister_pickle_by_value(m)
    model.save(os.path.join(remote_dir, "model"))


def _user_modules(callbacks):
    """Modules of user-defined callback classes that the job may not be able to
    import (scripts, test modules): pickled by value so they travel with the job."""
    import sys

    mods = []
    for cb in callbacks or []:
        name = type(cb).__module__
        mod = sys.modules.get(name)
        f = getattr(mod, "__file__", "") or ""
        if mod is None or name == "__main__" or name.startswith("cloud_amd") or "-packages" in f:
            continue
        if mod not in mods:
            mods.append(mod)
    return mods


def _default_job_spec(region=None, image_uri=None, entry_point_args=None,
                      distribution_strategy=DEFAULT_DISTRIBUTION_STRATEGY):
    n = topology.visible_gpu_count()
    cpu = machine_config.COMMON_MACHINE_CONFIGS["CPU"]
    one = machine_config.COMMON_MACHINE_CONFIGS["MI355X_1X"]
    if distribution_strategy == utils.MIRRORED_STRATEGY_NAME:
        chief = machine_config.MachineConfig(cpu_cores=16, memory=256, accelerator_type="MI355X",
                                             accelerator_count=max(1, min(n, 8))) if n else cpu
        workers, wcfg = 0, None
    else:  # reference default: 1 master + 1 worker
        chief = one if n >= 2 else cpu
        workers, wcfg = 1, (one if n >= 2 else cpu)
    return {"jobId": "cloud_fit_{}".format(datetime.datetime.now().strftime("%Y%m%d%H%M%S")),
            "trainingInput": {"chief_config": chief, "worker_count": workers, "worker_config": wcfg,
                              "region": region or topology.get_region(), "args": entry_point_args or []}}


def _submit_job(job_spec, wait=False):
    ti = job_spec["trainingInput"]
    job_id = job_spec["jobId"]
    tmp = tempfile.mkdtemp(prefix="cloud_fit_")
    entry = os.path.join(tmp, "cloud_fit_entry.py")
    with open(entry, "w") as f:
        f.write("from cloud_amd.experimental.cloud_fit import remote\nremote.main()\n")
    try:
        job_dir, target = stage.stage_job(job_id, entry, None, entry_point_args=ti["args"])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    try:
        job = launcher.deploy_job(job_id, job_dir, target, ti["chief_config"], ti["worker_count"],
                                  ti["worker_config"], ti["args"], False, wait=wait)
    except Exception as e:
        raise RuntimeError("Submitting job to the local launcher failed.") from e
    log.info("Job submitted: %s (logs: %s)", job_id, os.path.join(job_dir, "logs"))
    if wait and job.returncode not in (0, None):
        raise RuntimeError(f"cloud_fit job {job_id} failed with exit code {job.returncode}")
    return job_id
