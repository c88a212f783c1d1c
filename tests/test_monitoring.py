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


def test_exporter_autostarts_in_a_two_rank_run_job(tmp_path):
    """CLOUD_AMD_MONITORING_EXPORTER_ENABLED=1 on a run() job: every rank starts the
    native exporter by importing the package (the REGISTER_TF_METRICS_EXPORTER analogue)
    and the job dir's metrics.jsonl gets step-time, all-reduce and tuner-trial series."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    app = tmp_path / "app"
    app.mkdir()
    (app / "train.py").write_text(
        "import os, sys\n"
        "import numpy as np\n"
        "import cloud_amd as tfc\n"
        "from cloud_amd import keras\n"
        "cpu = tfc.COMMON_MACHINE_CONFIGS['CPU']\n"
        "tfc.run(chief_config=cpu, worker_config=cpu, worker_count=1, stream_logs=True)\n"
        "x = np.random.default_rng(0).standard_normal((256, 8)).astype('float32')\n"
        "y = (x[:, 0] > 0).astype('int64')\n"
        "m = keras.Sequential([keras.layers.Dense(16, activation='relu'), keras.layers.Dense(2, activation='softmax')])\n"
        "m.compile(optimizer='sgd', loss='sparse_categorical_crossentropy')\n"
        "m.fit(x, y, batch_size=32, epochs=2, verbose=0)\n"
        "from cloud_amd.tuner.tuner import CloudOracle\n"
        "from cloud_amd.tuner import hyperparameters as hp\n"
        "hps = hp.HyperParameters(); hps.Choice('units', [8, 16])\n"
        "o = CloudOracle('p', 'r', objective='acc', hyperparameters=hps, max_trials=2,\n"
        "                study_id='mon%s' % os.environ['RANK'], study_dir=os.path.join(os.environ['CLOUD_AMD_JOB_DIR'], 'st'))\n"
        "t = o.create_trial('t0'); o.update_trial(t.trial_id, {'acc': 0.5}, step=1); o.end_trial(t.trial_id)\n"
        "print('DONE', os.environ['RANK'], flush=True)\n")
    env = dict(os.environ, CLOUD_AMD_NUM_GPUS="0", CLOUD_AMD_JOBS_DIR=str(tmp_path / "jobs"), PYTHONPATH=root,
               CLOUD_AMD_MONITORING_EXPORTER_ENABLED="1", CLOUD_AMD_MONITORING_INTERVAL_S="0.5",
               OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "CLOUD_AMD_RUNNING_REMOTELY", "TORCHELASTIC_RUN_ID", "CLOUD_AMD_MONITORING_DIR"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "train.py"], cwd=str(app), env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    job_dir = tmp_path / "jobs" / os.listdir(tmp_path / "jobs")[0]
    lines = [json.loads(l) for l in open(job_dir / "metrics.jsonl")]  # every line is whole JSON
    assert lines
    text = open(job_dir / "metrics.jsonl").read()
    for name in ("train/step_time_ms", "comm/allreduce_ms", "comm/exposed_ms", "tuner/trials",
                 "data/getnext_duration_us"):
        assert name in text, name
    # both ranks exported, told apart by the rank label
    assert '"rank":"0"' in text.replace(" ", "") and '"rank":"1"' in text.replace(" ", "")
