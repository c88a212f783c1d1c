"""The reference's single-process workloads (TFC/core/tests/testdata ports in
examples/workloads) end to end on one MI355X: the Keras fit / custom-loop / save-and-load /
KerasTuner scripts run unchanged apart from the import line, on the native kernels (the
CPU twins of these tests are in test_workloads.py).  Small sizes (CLOUD_AMD_EXAMPLE_SMALL)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WL = os.path.join(ROOT, "examples", "workloads")


def _run(args, tmp_path, timeout=110):
    env = dict(os.environ)
    env.pop("CLOUD_AMD_DEVICE", None)
    env.update({"CLOUD_AMD_EXAMPLE_SMALL": "1", "CLOUD_AMD_JOBS_DIR": str(tmp_path / "jobs"), "PYTHONPATH": ROOT})
    p = subprocess.run([sys.executable, *args], cwd=str(tmp_path), env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p.stdout


def _result(out, tag):
    lines = [ln for ln in out.splitlines() if ln.startswith("RESULT " + tag)]
    assert lines, out[-2000:]
    return lines[-1]


def test_fit_workload_gpu(tmp_path):
    out = _run([os.path.join(WL, "mnist_example_using_fit.py")], tmp_path)
    assert "Learning rate for epoch 2 is 0.001" in out
    _result(out, "fit")


def test_save_and_load_workload_gpu(tmp_path):
    out = _run([os.path.join(WL, "save_and_load.py"), "--path", str(tmp_path / "m")], tmp_path)
    vals = dict(kv.split("=") for kv in _result(out, "save_and_load").split()[2:])
    assert float(vals["restored_acc"]) > float(vals["untrained_acc"])


def test_keras_tuner_workload_gpu(tmp_path):
    out = _run([os.path.join(WL, "keras_tuner_cifar_example.py"), "--path", str(tmp_path / "best"),
                "--directory", str(tmp_path / "tdir")], tmp_path)
    assert "Results summary" in out
    _result(out, "tuner")


def test_mlp_no_reqs_workload_gpu(tmp_path):
    _result(_run([os.path.join(WL, "mnist_example_using_fit_no_reqs.py")], tmp_path), "mlp")


@pytest.mark.timeout(300)
def test_ctl_workload_two_ranks_share_the_gpu(tmp_path):
    """call_run_on_script_with_keras_ctl through run(): chief + worker (MultiWorkerMirrored),
    both ranks on this box's one GPU over gloo (CLOUD_AMD_SHARED_GPU) -- the DP data plane on
    device tensors; strategy.reduce gives both replicas the same loss."""
    import glob

    env = dict(os.environ)
    env.pop("CLOUD_AMD_DEVICE", None)
    env.update({"CLOUD_AMD_EXAMPLE_SMALL": "1", "CLOUD_AMD_JOBS_DIR": str(tmp_path / "jobs"), "PYTHONPATH": ROOT,
                "CLOUD_AMD_SHARED_GPU": "1", "CLOUD_AMD_DIST_BACKEND": "gloo", "CLOUD_AMD_NUM_GPUS": "2"})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "call_run_on_script_with_keras_ctl.py")],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    res = []
    for log in sorted(glob.glob(str(tmp_path / "jobs" / "*" / "logs" / "*.log"))):
        res += [ln.strip() for ln in open(log) if ln.startswith("RESULT")]
    assert len(res) == 2 and all("replicas=2" in r for r in res), res
    assert len({r.split("loss=")[1] for r in res}) == 1, res
