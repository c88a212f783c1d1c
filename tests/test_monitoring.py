"""Native metrics library: C++ golden-test binary (reference
stackdriver_client_test.cc expectations) + the Python bindings and exporter."""
import json
import os
import subprocess
import time

import pytest

from cloud_amd import _build, monitoring


@pytest.fixture(scope="module", autouse=True)
def _built():
    _build.build_monitoring()


def test_cpp_golden_binary():
    exe = _build.build_monitoring_test()
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout


def test_distribution_math_python():
    d = monitoring.native().convert_distribution([-1.0, 1.0], [0.0])
    assert d == {"count": 2, "mean": 0.0, "sum_of_squared_deviation": 2.0, "bounds": [0.0], "bucket_counts": [1, 1]}


def test_registry_and_jsonl_exporter(tmp_path):
    m = monitoring.native()
    m.clear()
    monitoring.inc(monitoring.JOBS, 2, state="ok")
    for v in (10.0, 20.0, 30.0):
        monitoring.observe(monitoring.STEP_TIME, v)
    monitoring.gauge(monitoring.THROUGHPUT, 7500.0)
    snap = monitoring.snapshot()
    assert snap[monitoring.JOBS][0]["value"] == 2 and snap[monitoring.JOBS][0]["labels"] == {"state": "ok"}
    assert snap[monitoring.STEP_TIME][0]["value"]["count"] == 3
    assert monitoring.start_exporter(str(tmp_path), interval_s=0.02, force=True)
    time.sleep(0.3)
    monitoring.stop_exporter()
    lines = [json.loads(ln) for ln in open(tmp_path / "metrics.jsonl")]
    types = {ln["timeSeries"]["metric"]["type"] for ln in lines}
    assert "custom.cloud_amd" + monitoring.STEP_TIME in types
    desc = [json.loads(ln) for ln in open(tmp_path / "descriptors.jsonl")]
    assert len(desc) == len({d["metricDescriptor"]["type"] for d in desc})  # once per metric


def test_prometheus_sink(tmp_path):
    monitoring.native().clear()
    monitoring.observe(monitoring.STEP_TIME, 5.0, bounds=[1.0, 10.0])
    monitoring.start_exporter(str(tmp_path), sink="prometheus", interval_s=10, force=True)
    monitoring.export_now()
    monitoring.stop_exporter()
    text = open(tmp_path / "metrics.prom").read()
    assert 'le="10"' in text and "_count 1" in text


def test_exporter_disabled_by_default(tmp_path, monkeypatch):
    monkeypatch.delenv("CLOUD_AMD_MONITORING_EXPORTER_ENABLED", raising=False)
    assert monitoring.start_exporter(str(tmp_path)) is False
