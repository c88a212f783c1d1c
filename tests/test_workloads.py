"""The reference's workloads (TFC/core/tests/testdata + examples), ported to
cloud_amd, run end to end on CPU: directly, and through run() as multi-process
jobs (gloo).  Sizes shrink with CLOUD_AMD_EXAMPLE_SMALL=1."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WL = os.path.join(ROOT, "examples", "workloads")


def _env(tmp_path, **extra):
    env = dict(os.environ)
    env.update({"CLOUD_AMD_EXAMPLE_SMALL": "1", "CLOUD_AMD_NUM_GPUS": "0", "CLOUD_AMD_DEVICE": "cpu",
                "CLOUD_AMD_JOBS_DIR": str(tmp_path / "jobs"), "PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2"})
    env.update(extra)
    return env


def _run(cmd, tmp_path, cwd=None, timeout=600, **extra):
    p = subprocess.run(cmd, cwd=cwd or str(tmp_path), env=_env(tmp_path, **extra), capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p.stdout


def _job_results(tmp_path):
    out = []
    for log in sorted(glob.glob(str(tmp_path / "jobs" / "*" / "logs" / "*.log"))):
        out += [ln.strip() for ln in open(log) if ln.startswith("RESULT")]
    return out


def test_fit_workload(tmp_path):
    out = _run([sys.executable, os.path.join(WL, "mnist_example_using_fit.py")], tmp_path)
    assert "Learning rate for epoch 2 is 0.001" in out and "RESULT fit" in out


def test_mlp_no_reqs_workload(tmp_path):
    assert "RESULT mlp" in _run([sys.executable, os.path.join(WL, "mnist_example_using_fit_no_reqs.py")], tmp_path)


def test_save_and_load_workload(tmp_path):
    out = _run([sys.executable, os.path.join(WL, "save_and_load.py"), "--path", str(tmp_path / "m")], tmp_path)
    line = [ln for ln in out.splitlines() if ln.startswith("RESULT")][0]
    vals = dict(kv.split("=") for kv in line.split()[2:])
    assert float(vals["restored_acc"]) > float(vals["untrained_acc"])
    assert os.path.isdir(str(tmp_path / "m"))


def test_keras_tuner_workload(tmp_path):
    out = _run([sys.executable, os.path.join(WL, "keras_tuner_cifar_example.py"), "--path", str(tmp_path / "best"),
                "--directory", str(tmp_path / "tdir")], tmp_path)
    assert "RESULT tuner" in out and "Results summary" in out


def test_ctl_workload_two_workers_via_run(tmp_path):
    """call_run_on_script_with_keras_ctl: chief + 1 worker, the script builds its own MWMS."""
    _run([sys.executable, os.path.join(ROOT, "examples", "call_run_on_script_with_keras_ctl.py")], tmp_path,
         CLOUD_AMD_EXAMPLE_CPU="1")
    res = _job_results(tmp_path)
    assert len(res) == 2, res
    assert all("replicas=2" in r for r in res)
    losses = {r.split("loss=")[1] for r in res}
    assert len(losses) == 1, res  # strategy.reduce(SUM) gives every replica the same number


@pytest.mark.timeout(900)
def test_run_within_script_resnet50(tmp_path):
    """call_run_within_script_with_keras_fit: local epoch, then run() relaunches the same file remotely."""
    out = _run([sys.executable, os.path.join(ROOT, "examples", "call_run_within_script_with_keras_fit.py")],
               tmp_path, CLOUD_AMD_EXAMPLE_CPU="1", CLOUD_AMD_EXAMPLE_OUT=str(tmp_path / "out"), timeout=900)
    assert "Job submitted successfully." in out
    res = _job_results(tmp_path)
    assert len(res) == 2 and all("remote=True" in r for r in res), res


def test_multi_file_example_via_run(tmp_path):
    d = os.path.join(ROOT, "examples", "multi_file_example")
    out = _run([sys.executable, "scale_model.py"], tmp_path, cwd=d, CLOUD_AMD_EXAMPLE_CPU="1")
    assert "Job submitted successfully." in out
    res = _job_results(tmp_path)
    assert len(res) == 1 and "remote=True" in res[0] and "epochs=2" in res[0], res
