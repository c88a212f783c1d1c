"""``run()`` / ``remote()``: take a training script from a local debug run to a
distributed run on the MI355X GPUs of this node.

Signature and semantics follow reference ``TFC/core/run.py:31-246``:
no-op when already remote, unknown kwargs rejected, ``"auto"`` machine
configs, validation, wrapper generation with strategy auto-selection,
staging (the Docker-build analogue), launch (the AI-Platform-submit analogue)
and ``sys.exit(0)`` afterwards when called from a script so the local copy
never trains.  Additional keyword-only controls (all optional):

* ``wait``: block until the job finishes (default: ``stream_logs``);
* ``jobs_dir``: where job directories go (default ``$CLOUD_AMD_JOBS_DIR`` or ``./jobs``);
* ``profile``: wrap rank 0 in ``rocprofv3 --kernel-trace --stats``;
* ``exit``: set False to return the :class:`~cloud_amd.core.launcher.Job`
  instead of exiting (library use, tests, notebooks).

Fixes relative to the reference: ``entry_point=None`` with
``distribution_strategy=None`` no longer raises AttributeError; a CPU chief
gets a CPU OneDevice strategy.
"""
from __future__ import annotations

import os
import sys
import time

from . import launcher, machine_config, preprocess, stage, topology, validate


def remote():
    """True inside a launched job (or a torchrun-launched rank)."""
    return bool(os.environ.get("TF_KERAS_RUNNING_REMOTELY") or os.environ.get("CLOUD_AMD_RUNNING_REMOTELY")
                or os.environ.get("TORCHELASTIC_RUN_ID"))


def run(entry_point=None, requirements_txt=None, distribution_strategy="auto", docker_base_image=None,
        chief_config="auto", worker_config="auto", worker_count=0, entry_point_args=None, stream_logs=False,
        docker_image_bucket_name=None, job_labels=None, *, wait=None, jobs_dir=None, profile=False, exit=None,
        **kwargs):
    if remote():
        return None
    t_run = time.time()
    if kwargs:
        raise TypeError("Unknown keyword arguments: %s" % (kwargs.keys(),))
    job_labels = dict(job_labels or {})
    if chief_config == "auto":
        chief_config = machine_config.COMMON_MACHINE_CONFIGS["MI355X_1X"]
    if worker_config == "auto":
        worker_config = machine_config.COMMON_MACHINE_CONFIGS["MI355X_1X"]
    if not isinstance(worker_count, int):
        worker_count = int(worker_count)
    region = topology.get_region()
    called_from_notebook = _called_from_notebook()

    validate.validate(entry_point, requirements_txt, distribution_strategy, chief_config, worker_config,
                      worker_count, region, entry_point_args, stream_logs, docker_image_bucket_name,
                      called_from_notebook, job_labels=job_labels, docker_base_image=docker_base_image,
                      check_node=True)

    if entry_point is None and called_from_notebook:
        # run() inside a notebook with no entry point: the reference pulled the live notebook
        # from Colab (TFC/core/preprocess.py:166-167,196-212); here the notebook file the
        # kernel serves is located and converted like an .ipynb entry point
        nb = current_notebook_path()
        if nb is None:
            raise RuntimeError("run() was called from a notebook with entry_point=None, but the notebook file "
                               "could not be located (no JPY_SESSION_NAME / __session__); pass "
                               "entry_point='<notebook>.ipynb'.")
        entry_point = os.path.relpath(nb) if not os.path.relpath(nb).startswith("..") else nb
        validate.validate(entry_point, requirements_txt, distribution_strategy, chief_config, worker_config,
                          worker_count, region, entry_point_args, stream_logs, docker_image_bucket_name,
                          called_from_notebook, job_labels=job_labels, docker_base_image=docker_base_image)

    job_id = launcher.generate_job_id()
    root = os.path.abspath(jobs_dir) if jobs_dir else stage.jobs_root()
    os.makedirs(root, exist_ok=True)
    wrapper = None
    is_notebook = entry_point is not None and entry_point.endswith("ipynb")
    if distribution_strategy == "auto" or is_notebook or entry_point is None:
        wrapper = preprocess.get_preprocessed_entry_point(entry_point, chief_config, worker_config, worker_count,
                                                          distribution_strategy,
                                                          called_from_notebook=called_from_notebook)
    try:
        job_dir, target = stage.stage_job(job_id, entry_point, wrapper, requirements_txt=requirements_txt,
                                          entry_point_args=entry_point_args, root=root)
    finally:
        if wrapper is not None and os.path.exists(wrapper):
            os.remove(wrapper)

    # ranks can report run() -> first-step latency against this clock (bench.py does)
    job = launcher.deploy_job(job_id, job_dir, target, chief_config, worker_count, worker_config,
                              entry_point_args, stream_logs, job_labels=job_labels, wait=wait, profile=profile,
                              extra_env={"CLOUD_AMD_RUN_T0": repr(t_run)})
    do_exit = (not called_from_notebook) if exit is None else bool(exit)
    if do_exit:
        rc = job.wait() if (wait or stream_logs) else 0
        sys.exit(rc or 0)
    return job


def current_notebook_path(user_ns=None, environ=None):
    """Path of the notebook this kernel is running, or None.

    Two mechanisms, in order: ``JPY_SESSION_NAME`` (jupyter_server >= 2 exports the
    notebook's path into the kernel's environment) and the ``__session__`` global that
    ipykernel puts into the user namespace.  Relative paths are taken against the
    kernel's working directory; only an existing ``.ipynb`` counts."""
    environ = os.environ if environ is None else environ
    cands = [environ.get("JPY_SESSION_NAME")]
    if user_ns is None:
        try:
            import IPython

            ip = IPython.get_ipython()
            user_ns = getattr(ip, "user_ns", None) or {}
        except Exception:  # noqa: BLE001 - no IPython
            user_ns = {}
    cands.append(user_ns.get("__session__"))
    for c in cands:
        if not c or not isinstance(c, str):
            continue
        path = c if os.path.isabs(c) else os.path.abspath(c)
        if path.endswith(".ipynb") and os.path.isfile(path):
            return path
    return None


def _called_from_notebook():
    try:
        import IPython  # noqa: F401
    except ImportError:
        return False
    try:
        shell = IPython.get_ipython().__class__.__name__
        return "Shell" in shell
    except NameError:
        return False
