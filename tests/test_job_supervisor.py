"""Detached job supervision and job inspection by id (VERDICT r5 missing #1-#3).

Reference behaviour: ``run()`` submits and exits (``TFC/core/run.py:232-246``); the managed
service keeps running the job, fails it as a group and answers ``describe`` /
``stream-logs`` by id (``TFC/core/deploy.py:170-211``).  Here the submitting side drops
its ``Job`` handle right after submission and every check goes through ``job.json`` and
``python -m cloud_amd.jobs``."""
import gc
import json
import os
import signal
import subprocess
import sys
import time

import pytest

from cloud_amd import jobs as jobs_cli
from cloud_amd.core import launcher, machine_config as mc, run as run_mod

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CPU = mc.COMMON_MACHINE_CONFIGS["CPU"]

SLEEPER = (
    "import os, sys, time\n"
    "print('rank', os.environ['RANK'], 'up', flush=True)\n"
    "if os.environ.get('QUICK'):\n"
    "    sys.exit(int(os.environ.get('QUICK_RC', '0')))\n"
    "time.sleep(600)\n")


@pytest.fixture
def env(tmp_path, monkeypatch):
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    monkeypatch.setenv("CLOUD_AMD_HOME", str(tmp_path / "home"))
    monkeypatch.setenv("CLOUD_AMD_JOBS_DIR", str(tmp_path / "jobs"))
    for k in ("QUICK", "QUICK_RC", "WORLD_SIZE", "RANK", "CLOUD_AMD_RUNNING_REMOTELY", "TF_KERAS_RUNNING_REMOTELY",
              "TORCHELASTIC_RUN_ID"):
        monkeypatch.delenv(k, raising=False)
    app = tmp_path / "proj"
    app.mkdir()
    (app / "train.py").write_text(SLEEPER)
    monkeypatch.chdir(app)
    return tmp_path


def _submit(workers=1, **kw):
    """Fire-and-forget submission; returns only the job id (the handle is dropped)."""
    job = run_mod.run(entry_point="train.py", chief_config=CPU, worker_config=CPU, worker_count=workers,
                      distribution_strategy=None, exit=False, wait=False, **kw)
    job_id = job.job_id
    del job
    gc.collect()
    return job_id


def _meta(job_id):
    return json.load(open(os.path.join(launcher.find_job_dir(job_id), "job.json")))


def _wait_for(pred, timeout=60.0):
    t_end = time.time() + timeout
    while time.time() < t_end:
        v = pred()
        if v:
            return v
        time.sleep(0.1)
    raise AssertionError("condition not reached in %.0f s" % timeout)


def _pid_gone(pid):
    return not launcher._pid_alive(pid)


def _cli(*args, cwd=None):
    e = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "cloud_amd.jobs"] + list(args), capture_output=True, text=True,
                          env=e, cwd=cwd, timeout=120)


def test_detached_job_fails_as_a_group_after_client_dropped_it(env):
    job_id = _submit(workers=1)
    m = _wait_for(lambda: (lambda m: m if m.get("state") == "RUNNING" and len(m.get("pids", [])) == 2 else None)(
        _meta(job_id)))
    pid0, pid1 = m["pids"]
    assert m["supervisor_pid"] not in (None, os.getpid())
    os.kill(pid1, signal.SIGKILL)  # rank 1 dies
    m = _wait_for(lambda: (lambda m: m if m.get("state") == "FAILED" else None)(_meta(job_id)), timeout=60)
    assert m["failed_rank"] == 1
    assert m["exit_codes"][1] == -signal.SIGKILL
    assert m["exit_codes"][0] == -signal.SIGTERM  # the supervisor took rank 0 down with it
    assert _pid_gone(pid0) and _pid_gone(pid1)
    _wait_for(lambda: _pid_gone(m["supervisor_pid"]), timeout=30)
    # ... and any other process can inspect it by id (from another working directory)
    r = _cli("describe", job_id, cwd=str(env))
    assert r.returncode == 1, r.stdout + r.stderr
    assert "state: FAILED" in r.stdout and "failedRank: 1" in r.stdout
    assert "exitCodes: [%d, %d]" % (-signal.SIGTERM, -signal.SIGKILL) in r.stdout
    rj = _cli("describe", job_id, "--json")
    assert json.loads(rj.stdout)["exit_codes"] == m["exit_codes"]
    lst = _cli("list")
    assert job_id in lst.stdout and "FAILED" in lst.stdout


def test_cancel_by_id(env):
    job_id = _submit(workers=0)
    m = _wait_for(lambda: (lambda m: m if m.get("state") == "RUNNING" else None)(_meta(job_id)))
    r = _cli("cancel", job_id)
    assert r.returncode == 0 and "CANCELLED" in r.stdout, r.stdout + r.stderr
    m = _meta(job_id)
    assert m["state"] == "CANCELLED" and m["exit_codes"] == [-signal.SIGTERM]
    assert _pid_gone(m["pids"][0])


def test_stream_logs_by_id_and_success(env, monkeypatch):
    monkeypatch.setenv("QUICK", "1")
    job_id = _submit(workers=1)
    r = _cli("stream-logs", job_id)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[chief-0] rank 0 up" in r.stdout and "[worker-0] rank 1 up" in r.stdout
    m = _meta(job_id)
    assert m["state"] == "SUCCEEDED" and m["exit_codes"] == [0, 0] and m["returncode"] == 0
    one = _cli("stream-logs", job_id, "--rank", "1", "--no-follow")
    assert one.stdout.strip() == "rank 1 up"
    assert _cli("describe", "no_such_job").returncode == 2


def test_supervisor_death_does_not_orphan_ranks(env):
    """SIGKILL to the supervisor itself: its ranks die with it (PR_SET_PDEATHSIG) and a
    client reports the job LOST instead of RUNNING forever."""
    job_id = _submit(workers=0)
    m = _wait_for(lambda: (lambda m: m if m.get("state") == "RUNNING" else None)(_meta(job_id)))
    os.kill(m["supervisor_pid"], signal.SIGKILL)
    _wait_for(lambda: _pid_gone(m["pids"][0]), timeout=30)
    _wait_for(lambda: _pid_gone(m["supervisor_pid"]), timeout=30)
    job = launcher.Job.attach(job_id)
    assert job.wait(30) == 1 and job.state == "LOST"


def test_run_fire_and_forget_exits_zero_and_prints_job_commands(env, monkeypatch, capsys):
    monkeypatch.setenv("QUICK", "1")
    monkeypatch.setenv("QUICK_RC", "4")
    with pytest.raises(SystemExit) as e:
        run_mod.run(entry_point="train.py", chief_config=CPU, distribution_strategy=None)
    assert e.value.code == 0  # submitted; the job's own failure is the job's state
    out = capsys.readouterr().out
    job_id = out.split("Your job ID is: ")[1].split()[0]
    assert "python -m cloud_amd.jobs describe %s" % job_id in out
    job = launcher.Job.attach(job_id)
    assert job.wait(60) == 4 and job.state == "FAILED"
    assert jobs_cli.main(["describe", job_id]) == 1
