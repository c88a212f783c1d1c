"""cloud_amd -- MI355X-native local->distributed training framework.

Same public surface as TensorFlow Cloud (reference ``TFC/__init__.py:16-27``):
``run``, ``remote``, ``MachineConfig``, ``AcceleratorType``,
``COMMON_MACHINE_CONFIGS``, ``CloudTuner``, ``CloudOracle`` -- re-designed for
one process per MI355X, RCCL over xGMI and hand-written CDNA4 kernels.
Heavy submodules are imported lazily so ``import cloud_amd`` (and a ``run()``
launch) stays cheap.
"""
from .version import __version__  # noqa: F401

_LAZY = {
    "run": ("cloud_amd.core.run", "run"),
    "remote": ("cloud_amd.core.run", "remote"),
    "MachineConfig": ("cloud_amd.core.machine_config", "MachineConfig"),
    "AcceleratorType": ("cloud_amd.core.machine_config", "AcceleratorType"),
    "COMMON_MACHINE_CONFIGS": ("cloud_amd.core.machine_config", "COMMON_MACHINE_CONFIGS"),
    "CloudTuner": ("cloud_amd.tuner.tuner", "CloudTuner"),
    "CloudOracle": ("cloud_amd.tuner.tuner", "CloudOracle"),
}


def __getattr__(name):
    if name in _LAZY:
        import importlib

        mod, attr = _LAZY[name]
        val = getattr(importlib.import_module(mod), attr)
        globals()[name] = val
        return val
    raise AttributeError(f"module 'cloud_amd' has no attribute {name!r}")


__all__ = ["__version__", *_LAZY]


def _autostart_monitoring():
    """The analogue of the reference's ``REGISTER_TF_METRICS_EXPORTER``
    (``src/cpp/monitoring/stackdriver_exporter.cc:128``): in a launched rank with
    ``CLOUD_AMD_MONITORING_EXPORTER_ENABLED`` set, importing the package starts the
    native periodic exporter -- no user code needed."""
    import os

    if os.environ.get("CLOUD_AMD_MONITORING_EXPORTER_ENABLED", "").lower() not in ("1", "true", "yes", "on"):
        return
    if not (os.environ.get("CLOUD_AMD_RUNNING_REMOTELY") or os.environ.get("TORCHELASTIC_RUN_ID")):
        return  # only ranks export; the launching process does not
    try:
        from . import monitoring

        monitoring.autostart()
    except Exception as e:  # noqa: BLE001 - metrics must never break a job
        import sys

        print("[cloud_amd] monitoring exporter not started: %s" % e, file=sys.stderr)


_autostart_monitoring()
