"""The example notebooks (scripts/make_notebooks.py) and the notebook / cloud-build /
model-search examples, run on CPU with small sizes: the notebook code goes through the
same converter run() uses for .ipynb entry points (magics, shell lines, comments dropped)."""
import glob
import os
import subprocess
import sys

import pytest

from cloud_amd.core import preprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = os.path.join(ROOT, "examples", "notebooks")


def _env(tmp_path, **extra):
    env = dict(os.environ)
    env.update({"CLOUD_AMD_EXAMPLE_SMALL": "1", "CLOUD_AMD_EXAMPLE_CPU": "1", "CLOUD_AMD_NUM_GPUS": "0",
                "CLOUD_AMD_DEVICE": "cpu", "CLOUD_AMD_JOBS_DIR": str(tmp_path / "jobs"), "PYTHONPATH": ROOT,
                "CLOUD_AMD_REPO": ROOT, "OMP_NUM_THREADS": "2", "CLOUD_AMD_EXAMPLE_OUT": str(tmp_path / "out")})
    env.update(extra)
    return env


def _run_notebook(path, tmp_path, timeout=600):
    code = "".join(preprocess.notebook_code_lines(path))
    script = os.path.join(os.path.dirname(path), "_nb_%s.py" % os.getpid())
    with open(script, "w") as f:
        f.write(code)
    try:
        p = subprocess.run([sys.executable, script], cwd=os.path.dirname(path), env=_env(tmp_path),
                           capture_output=True, text=True, timeout=timeout)
    finally:
        os.remove(script)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p.stdout


def _job_results(tmp_path):
    out = []
    for log in sorted(glob.glob(str(tmp_path / "jobs" / "*" / "logs" / "*.log"))):
        out += [ln.strip() for ln in open(log) if ln.startswith("RESULT")]
    return out


def test_all_notebooks_convert_and_compile():
    paths = glob.glob(os.path.join(NB, "*.ipynb")) + [os.path.join(ROOT, "examples", "workloads",
                                                                   "mnist_example_using_fit.ipynb")]
    assert len(paths) == 5
    for p in paths:
        code = "".join(preprocess.notebook_code_lines(p))
        compile(code, p, "exec")
        assert "%time" not in code and "!echo" not in code


def test_notebook_entry_point_via_run(tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "call_run_on_notebook_with_keras_fit.py")],
                       cwd=str(tmp_path), env=_env(tmp_path), capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    res = _job_results(tmp_path)
    assert len(res) == 1 and "RESULT notebook_fit" in res[0], res


def test_run_within_notebook(tmp_path):
    out = _run_notebook(os.path.join(NB, "call_run_within_nb.ipynb"), tmp_path)
    assert "Job submitted successfully." in out
    res = _job_results(tmp_path)
    assert len(res) == 2 and all("remote=True" in r for r in res), res


def test_cloud_tuner_notebook(tmp_path):
    out = _run_notebook(os.path.join(NB, "cloud_tuner.ipynb"), tmp_path)
    assert "Results summary" in out and "RESULT tuner_nb" in out


def test_cloud_fit_notebook(tmp_path):
    out = _run_notebook(os.path.join(NB, "cloud_fit.ipynb"), tmp_path)
    assert "RESULT cloud_fit_nb" in out


def test_cloud_build_example(tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "call_run_on_script_with_keras_fit_cloud_build.py"),
                        "--bucket_name", "local-bucket"], cwd=str(tmp_path), env=_env(tmp_path),
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert any("RESULT mlp" in r for r in _job_results(tmp_path))


@pytest.mark.timeout(900)
def test_automodel_example(tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "call_run_within_script_with_automodel.py"),
                        "--path", str(tmp_path / "am")], cwd=str(tmp_path), env=_env(tmp_path),
                       capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    res = _job_results(tmp_path)
    assert len(res) == 1 and "remote=True" in res[0], res
