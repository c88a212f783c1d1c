"""Metrics + periodic exporter (Python face of the native ``cloud_amd._monitoring``).

Parity target: the reference's C++ Stackdriver exporter (``src/cpp/monitoring``)
-- the registry, the 10 s background exporter, the allow-list and the
histogram->distribution conversion are native C++ here too; the sink is a local
JSONL file (``<dir>/metrics.jsonl``) or a Prometheus textfile instead of
Cloud Monitoring.  Env switches (renamed from ``TF_MONITORING_STACKDRIVER_*``):
``CLOUD_AMD_MONITORING_EXPORTER_ENABLED``, ``CLOUD_AMD_MONITORING_PROJECT_ID``,
``CLOUD_AMD_MONITORING_METRICS_WHITELIST``, ``CLOUD_AMD_MONITORING_INTERVAL_S``,
``CLOUD_AMD_MONITORING_DIR``.
"""
from __future__ import annotations

import importlib
import os

STEP_TIME = "/cloud_amd/train/step_time_ms"
THROUGHPUT = "/cloud_amd/train/images_per_sec"
FIRST_STEP = "/cloud_amd/train/first_step_latency_s"
ALLREDUCE = "/cloud_amd/comm/allreduce_ms"
EXPOSED_COMM = "/cloud_amd/comm/exposed_ms"
GETNEXT = "/cloud_amd/data/getnext_duration_us"
TRIALS = "/cloud_amd/tuner/trials"
JOBS = "/cloud_amd/launcher/jobs"

_mod = None


def native():
    """The native module (built by ``python -m cloud_amd._build``)."""
    global _mod
    if _mod is None:
        _mod = importlib.import_module("cloud_amd._monitoring")
    return _mod


def available():
    try:
        native()
        return True
    except ImportError:
        return False


def _labels(labels):
    """Caller labels plus this process's ``rank`` in a multi-rank job (every rank
    exports into the same job directory)."""
    out = {str(k): str(v) for k, v in (labels or {}).items()}
    if "rank" not in out and os.environ.get("WORLD_SIZE", "1") not in ("", "1") and os.environ.get("RANK"):
        out["rank"] = os.environ["RANK"]
    return out


def inc(name, delta=1, **labels):
    if available():
        native().counter_inc(name, int(delta), _labels(labels))


def gauge(name, value, **labels):
    if available():
        native().gauge_set(name, float(value), _labels(labels))


def observe(name, value, bounds=None, **labels):
    if available():
        native().observe(name, float(value), _labels(labels), list(bounds or []))


def snapshot():
    return native().snapshot() if available() else {}


def start_exporter(directory=None, sink="jsonl", interval_s=0.0, force=False):
    """Start the background exporter (no-op unless enabled by env or ``force``)."""
    if not available():
        return False
    directory = directory or os.environ.get("CLOUD_AMD_MONITORING_DIR") or os.environ.get("CLOUD_AMD_JOB_DIR") or "."
    return native().start_exporter(os.path.abspath(directory), sink, float(interval_s), bool(force))


_AUTO = {"started": False}


def enabled():
    return os.environ.get("CLOUD_AMD_MONITORING_EXPORTER_ENABLED", "").lower() in ("1", "true", "yes", "on")


def autostart():
    """Start the exporter once per process if the env switch is on (called from the
    package import); a final export runs at interpreter exit so short jobs and the
    last interval are not lost."""
    if _AUTO["started"] or not enabled() or not available():
        return False
    sink = os.environ.get("CLOUD_AMD_MONITORING_SINK", "jsonl")
    ok = start_exporter(sink=sink)
    if ok:
        import atexit

        _AUTO["started"] = True
        atexit.register(stop_exporter)
    return ok


def export_now():
    if available():
        native().export_now()


def stop_exporter():
    if available():
        native().stop_exporter()
