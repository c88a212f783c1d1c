"""Wrapper generation, staging, the local launcher and run() (parity: reference
core/tests/unit/{preprocess,containerize,deploy}_test.py, with a real local
multi-process job instead of mocked cloud calls)."""
import json
import os
import shutil
import sys

import pytest

from cloud_amd.core import launcher, machine_config as mc, preprocess, run as run_mod, stage, validate

HERE = os.path.dirname(os.path.abspath(__file__))
CPU = mc.COMMON_MACHINE_CONFIGS["CPU"]


def _lines(path):
    with open(path) as f:
        return f.readlines()


@pytest.mark.parametrize("chief,workers,expect", [
    (mc.COMMON_MACHINE_CONFIGS["MI355X_1X"], 0, "strategy = _ca_strategy.OneDeviceStrategy(device='/gpu:0')\n"),
    (CPU, 0, "strategy = _ca_strategy.OneDeviceStrategy(device='/cpu:0')\n"),
    (mc.COMMON_MACHINE_CONFIGS["MI355X_4X"], 0, "strategy = _ca_strategy.MirroredStrategy()\n"),
    (mc.COMMON_MACHINE_CONFIGS["MI355X_1X"], 2, "strategy = _ca_strategy.MultiWorkerMirroredStrategy()\n"),
])
def test_wrapper_golden(tmp_path, chief, workers, expect):
    p = preprocess.get_preprocessed_entry_point("dir/train.py", chief, mc.COMMON_MACHINE_CONFIGS["MI355X_1X"],
                                                workers, "auto", output_dir=str(tmp_path))
    assert _lines(p) == preprocess.HEADER + [expect, "_ca_strategy.experimental_set_strategy(strategy)\n",
                                             "__file__ = os.path.abspath('train.py')\n",
                                             "exec(compile(open('train.py').read(), 'train.py', 'exec'))\n"]


def test_wrapper_no_strategy(tmp_path):
    p = preprocess.get_preprocessed_entry_point("train.py", CPU, CPU, 0, None, output_dir=str(tmp_path))
    assert not any("strategy" in ln and "=" in ln for ln in _lines(p)[len(preprocess.HEADER):])


def test_wrapper_notebook(tmp_path):
    nb = {"cells": [{"cell_type": "markdown", "source": ["# t"]},
                    {"cell_type": "code", "source": ["!pip install x\n", "%matplotlib inline\n", "# c\n",
                                                     "import os\n", "print('hi')"]}],
          "nbformat": 4}
    f = tmp_path / "nb.ipynb"
    f.write_text(json.dumps(nb))
    p = preprocess.get_preprocessed_entry_point(str(f), CPU, CPU, 0, "auto", output_dir=str(tmp_path))
    body = _lines(p)[len(preprocess.HEADER) + 2:]
    assert body[:2] == ["import os\n", "print('hi')\n"]
    assert not any(ln.startswith(("!", "%", "#")) for ln in body)


def test_stage_file_map_and_manifest(tmp_path):
    app = tmp_path / "proj"
    app.mkdir()
    (app / "train.py").write_text("print('x')\n")
    (app / "util.py").write_text("X = 1\n")
    (app / "req.txt").write_text("numpy\n")
    wrapper = tmp_path / "wrap.py"
    wrapper.write_text("print(1)\n")
    fmap = stage.file_path_map(str(app / "train.py"), str(wrapper), str(app / "req.txt"))
    assert fmap[str(app)] == "app" and fmap[str(wrapper)] == os.path.join("app", "wrap.py")
    jd, target = stage.stage_job("job_x", str(app / "train.py"), str(wrapper), str(app / "req.txt"),
                                 ["--epochs", "1"], root=str(tmp_path / "jobs"))
    assert os.path.exists(os.path.join(jd, "app", "util.py")) and target.endswith("wrap.py")
    man = json.load(open(os.path.join(jd, "manifest.json")))
    assert man["entrypoint"] == ["python", os.path.join("app", "wrap.py"), "--epochs", "1"]
    assert man["requirements"] == "req.txt" and man["framework"]["arch"] == "gfx950"


def test_plan_ranks_and_tf_config():
    ranks = launcher.plan_ranks(mc.COMMON_MACHINE_CONFIGS["MI355X_2X"], 1, mc.COMMON_MACHINE_CONFIGS["MI355X_1X"])
    assert [(r["role"], r["index"], r["gpu"]) for r in ranks] == [("chief", 0, 0), ("chief", 0, 1), ("worker", 0, 2)]
    cfg = launcher.tf_config_for(ranks, 2, 1000)
    assert cfg["task"] == {"type": "worker", "index": 0} and len(cfg["cluster"]["worker"]) == 1
    assert launcher.log_name(ranks[1]) == "chief-0-gpu1.log"
    assert launcher.generate_job_id().startswith("cloud_amd_train_")


def _stage_script(tmp_path):
    app = tmp_path / "proj"
    app.mkdir()
    shutil.copy(os.path.join(HERE, "data", "allreduce_script.py"), app / "train.py")
    return app


def _results(job):
    out = []
    for i in range(len(job.ranks)):
        for ln in open(job.log_path(i)):
            if ln.startswith("RESULT "):
                out.append(json.loads(ln[7:]))
    return out


def test_local_multiprocess_job(tmp_path, monkeypatch, capsys):
    app = _stage_script(tmp_path)
    monkeypatch.chdir(app)
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    job = run_mod.run(entry_point="train.py", chief_config=CPU, worker_config=CPU, worker_count=2,
                      entry_point_args=["--flag"], jobs_dir=str(tmp_path / "jobs"), exit=False, wait=True,
                      job_labels={"test": "launch"})
    assert job.wait(120) == 0
    out = capsys.readouterr().out
    assert "Job submitted successfully." in out and "Your job ID is: " in out
    res = _results(job)
    assert len(res) == 3
    assert all(r["sum"] == 6.0 and r["replicas"] == 3 for r in res)
    assert {r["strategy"] for r in res} == {"MultiWorkerMirroredStrategy"}
    assert sorted(r["tf_config"]["task"]["type"] for r in res) == ["chief", "worker", "worker"]
    assert all(r["remote"] == "1" and r["argv"] == ["--flag"] for r in res)
    meta = json.load(open(os.path.join(job.job_dir, "job.json")))
    assert meta["state"] == "SUCCEEDED" and meta["exit_codes"] == [0, 0, 0] and meta["labels"] == {"test": "launch"}


def test_watchdog_marks_failure(tmp_path, monkeypatch):
    app = _stage_script(tmp_path)
    monkeypatch.chdir(app)
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    monkeypatch.setenv("FAIL_RANK", "1")
    job = run_mod.run(entry_point="train.py", chief_config=CPU, worker_config=CPU, worker_count=1,
                      jobs_dir=str(tmp_path / "jobs"), exit=False, wait=True)
    assert job.wait(120) == 3
    meta = json.load(open(os.path.join(job.job_dir, "job.json")))
    assert meta["state"] == "FAILED" and 3 in meta["exit_codes"]


def test_run_remote_noop_and_kwargs(monkeypatch):
    monkeypatch.setenv("TF_KERAS_RUNNING_REMOTELY", "1")
    assert run_mod.remote() and run_mod.run(entry_point="whatever.py") is None
    monkeypatch.delenv("TF_KERAS_RUNNING_REMOTELY")
    monkeypatch.delenv("TORCHELASTIC_RUN_ID", raising=False)
    monkeypatch.delenv("CLOUD_AMD_RUNNING_REMOTELY", raising=False)
    assert not run_mod.remote()
    with pytest.raises(TypeError, match="Unknown keyword"):
        run_mod.run(entry_point="x.py", bogus=1)


def test_run_exits_when_called_from_script(tmp_path, monkeypatch):
    app = _stage_script(tmp_path)
    monkeypatch.chdir(app)
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    with pytest.raises(SystemExit) as e:
        run_mod.run(entry_point="train.py", chief_config=CPU, jobs_dir=str(tmp_path / "jobs"), stream_logs=True)
    assert e.value.code == 0


def test_debug_sync_mode_serialises_rank_launches(tmp_path, monkeypatch):
    """CLOUD_AMD_DEBUG_SYNC=1 reaches every rank with HIP's blocking-launch switches set
    (fault localisation); the native launch check reads the same variable."""
    app = tmp_path / "app"
    app.mkdir()
    (app / "probe.py").write_text(
        "import json, os\n"
        "keys = ['CLOUD_AMD_DEBUG_SYNC', 'HIP_LAUNCH_BLOCKING', 'AMD_SERIALIZE_KERNEL']\n"
        "json.dump({k: os.environ.get(k) for k in keys},\n"
        "          open(os.path.join(os.environ['CLOUD_AMD_JOB_DIR'], 'env.json'), 'w'))\n")
    job_dir = tmp_path / "job"
    (job_dir / "logs").mkdir(parents=True)
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    monkeypatch.setenv("CLOUD_AMD_DEBUG_SYNC", "1")
    monkeypatch.delenv("HIP_LAUNCH_BLOCKING", raising=False)
    monkeypatch.delenv("AMD_SERIALIZE_KERNEL", raising=False)
    job = launcher.launch("dbg", str(job_dir), str(app / "probe.py"), CPU, 0, None)
    assert job.wait(60) == 0
    env = json.load(open(job_dir / "env.json"))
    assert env == {"CLOUD_AMD_DEBUG_SYNC": "1", "HIP_LAUNCH_BLOCKING": "1", "AMD_SERIALIZE_KERNEL": "3"}
    hdr = open(os.path.join(HERE, "..", "csrc", "include", "ca_common.h")).read()
    assert 'getenv("CLOUD_AMD_DEBUG_SYNC")' in hdr and "hipDeviceSynchronize" in hdr


def test_launcher_never_touches_hip_and_sets_rccl_env(tmp_path, monkeypatch):
    """A 2-GPU job is sized from KFD sysfs (a fake tree here) with every torch.cuda entry
    point booby-trapped in the launcher process; both ranks get the xGMI RCCL defaults."""
    import torch

    from test_core_config import _fake_kfd

    def boom(*a, **k):
        raise AssertionError("launcher initialised HIP")

    for name in ("device_count", "is_available", "init", "_lazy_init", "current_device", "set_device"):
        monkeypatch.setattr(torch.cuda, name, boom)
    kfd = tmp_path / "kfd"
    _fake_kfd(str(kfd), n_gpus=2)
    for v in ("CLOUD_AMD_NUM_GPUS", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
              "NCCL_MIN_NCHANNELS", "HSA_NO_SCRATCH_RECLAIM", "CLOUD_AMD_RCCL_CHANNELS", "CLOUD_AMD_RCCL_ENV"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("CLOUD_AMD_KFD_ROOT", str(kfd))
    app = tmp_path / "app"
    app.mkdir()
    (app / "probe.py").write_text(
        "import json, os\n"
        "keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'NCCL_MIN_NCHANNELS', 'HSA_NO_SCRATCH_RECLAIM']\n"
        "json.dump({k: os.environ.get(k) for k in keys},\n"
        "          open(os.path.join(os.environ['CLOUD_AMD_JOB_DIR'], 'env%s.json' % os.environ['RANK']), 'w'))\n")
    job_dir = tmp_path / "job"
    (job_dir / "logs").mkdir(parents=True)
    validate.validate_node_capacity(mc.COMMON_MACHINE_CONFIGS["MI355X_2X"], None, 0)
    with pytest.raises(ValueError, match="needs 4 GPUs"):
        validate.validate_node_capacity(mc.COMMON_MACHINE_CONFIGS["MI355X_4X"], None, 0)
    job = launcher.launch("kfd", str(job_dir), str(app / "probe.py"),
                          mc.COMMON_MACHINE_CONFIGS["MI355X_2X"], 0, None)
    assert job.wait(60) == 0
    for r in range(2):
        env = json.load(open(job_dir / ("env%d.json" % r)))
        assert env == {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": "2", "NCCL_MIN_NCHANNELS": "1",
                       "HSA_NO_SCRATCH_RECLAIM": "1"}
    meta = json.load(open(job_dir / "job.json"))
    assert meta["node"]["source"] == "kfd" and meta["node"]["gpus"] == 2
    assert meta["comm_env"]["NCCL_MIN_NCHANNELS"] == "1"


# ---- launcher fidelity -------------------------------------------

def test_stream_logs_all_ranks_prefixed_and_failure_tail(tmp_path, monkeypatch, capsys):
    """stream_logs=True tails EVERY rank (reference deploy.py:187-211 streams the job), each
    line tagged with its role; a failing rank 1 is named with the tail of its log."""
    app = _stage_script(tmp_path)
    monkeypatch.chdir(app)
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    monkeypatch.setenv("FAIL_RANK", "1")
    job = run_mod.run(entry_point="train.py", chief_config=CPU, worker_config=CPU, worker_count=2,
                      jobs_dir=str(tmp_path / "jobs"), exit=False, wait=True, stream_logs=True)
    assert job.wait(120) == 3
    cap = capsys.readouterr()
    out_lines = cap.out.splitlines()
    for tag in ("[chief-0] RESULT ", "[worker-0] RESULT ", "[worker-1] RESULT "):
        assert any(ln.startswith(tag) for ln in out_lines), cap.out
    assert job.meta["failed_rank"] == 1
    assert "rank 1 (worker-0) exited with code 3" in cap.err
    tail_lines = [ln for ln in cap.err.splitlines() if ln.startswith("    ")]
    assert any("RESULT" in ln for ln in tail_lines) and len(tail_lines) <= 50


def test_stream_single_rank_unprefixed(tmp_path, monkeypatch, capsys):
    app = _stage_script(tmp_path)
    monkeypatch.chdir(app)
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    job = run_mod.run(entry_point="train.py", chief_config=CPU, jobs_dir=str(tmp_path / "jobs"), exit=False,
                      wait=True, stream_logs=True)
    assert job.wait(120) == 0
    out = capsys.readouterr().out
    assert any(ln.startswith("RESULT ") for ln in out.splitlines()), out


def test_launcher_process_never_imports_torch(tmp_path):
    """run() -> stage -> deploy in the launching process must not import torch (a cold
    import costs ~2 s of run() -> first-step latency); the ranks import it themselves."""
    import subprocess

    app = _stage_script(tmp_path)
    code = (
        "import sys, os\n"
        "import cloud_amd as tfc\n"
        "job = tfc.run(entry_point='train.py', chief_config=tfc.COMMON_MACHINE_CONFIGS['CPU'],\n"
        "              jobs_dir=%r, exit=False, wait=True)\n"
        "assert job.returncode == 0, job.meta\n"
        "print('TORCH_IMPORTED', 'torch' in sys.modules)\n" % str(tmp_path / "jobs"))
    env = dict(os.environ, CLOUD_AMD_NUM_GPUS="0", PYTHONPATH=os.path.dirname(HERE))
    for k in ("WORLD_SIZE", "RANK", "CLOUD_AMD_RUNNING_REMOTELY", "TF_KERAS_RUNNING_REMOTELY", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", code], cwd=str(app), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "TORCH_IMPORTED False" in r.stdout, r.stdout


def test_stage_links_code_copies_data_and_honours_cloudamdignore(tmp_path):
    proj = tmp_path / "proj"
    (proj / "build").mkdir(parents=True)
    (proj / "profiles").mkdir()
    (proj / "pkg").mkdir()
    (proj / "train.py").write_text("print('hi')\n")
    (proj / "pkg" / "mod.py").write_text("x = 1\n")
    (proj / "pkg" / "obj.o").write_text("object")
    (proj / "build" / "big.o").write_text("object")
    (proj / "profiles" / "p.txt").write_text("x")
    (proj / "data.csv").write_text("1,2\n")
    cwd = os.getcwd()
    os.chdir(proj)
    try:
        # no .cloudamdignore: a user package called build/ or profiles/ ships
        job_dir, _ = stage.stage_job("j0", "train.py", None, root=str(tmp_path / "jobs"))
        app0 = os.path.join(job_dir, "app")
        assert os.path.isfile(os.path.join(app0, "build", "big.o"))
        assert os.path.isfile(os.path.join(app0, "profiles", "p.txt"))
        (proj / ".cloudamdignore").write_text("# project excludes\nbuild/\nprofiles\n*.o\n")
        job_dir, target = stage.stage_job("j1", "train.py", None, root=str(tmp_path / "jobs"))
    finally:
        os.chdir(cwd)
    app = os.path.join(job_dir, "app")
    assert os.path.isfile(os.path.join(app, "pkg", "mod.py"))
    assert not os.path.exists(os.path.join(app, "build"))
    assert not os.path.exists(os.path.join(app, "profiles"))
    assert not os.path.exists(os.path.join(app, "pkg", "obj.o"))
    # code is hard-linked (same inode), data is copied (its own inode)
    assert os.stat(os.path.join(app, "pkg", "mod.py")).st_ino == os.stat(proj / "pkg" / "mod.py").st_ino
    assert os.stat(os.path.join(app, "data.csv")).st_ino != os.stat(proj / "data.csv").st_ino
    man = json.load(open(os.path.join(job_dir, "manifest.json")))
    assert man["framework"]["torch"] and "hip" in man["framework"]


def test_job_writing_a_staged_file_leaves_the_source_tree_unchanged(tmp_path):
    """A rank that rewrites / appends to a file it finds in its cwd (a checkpoint, a CSV log)
    changes the job's copy only -- and two jobs staged from one directory stay apart."""
    proj = tmp_path / "proj"
    proj.mkdir()
    (proj / "train.py").write_text("print('hi')\n")
    (proj / "model.h5").write_bytes(b"ORIGINAL")
    (proj / "log.csv").write_text("epoch,loss\n")
    cwd = os.getcwd()
    os.chdir(proj)
    try:
        jd1, _ = stage.stage_job("w1", "train.py", None, root=str(tmp_path / "jobs"))
        jd2, _ = stage.stage_job("w2", "train.py", None, root=str(tmp_path / "jobs"))
    finally:
        os.chdir(cwd)
    for jd, tag in ((jd1, b"JOB1"), (jd2, b"JOB2")):
        with open(os.path.join(jd, "app", "model.h5"), "wb") as f:  # truncating rewrite
            f.write(tag)
        with open(os.path.join(jd, "app", "log.csv"), "a") as f:
            f.write("0,1.0\n")
    assert (proj / "model.h5").read_bytes() == b"ORIGINAL"
    assert (proj / "log.csv").read_text() == "epoch,loss\n"
    assert open(os.path.join(jd1, "app", "model.h5"), "rb").read() == b"JOB1"
    assert open(os.path.join(jd2, "app", "model.h5"), "rb").read() == b"JOB2"


def _write_nb(path):
    nb = {"cells": [{"cell_type": "code", "source": ["import json\n", "print('NB_RAN', 6 * 7)\n"]},
                    {"cell_type": "markdown", "source": ["text"]}],
          "metadata": {}, "nbformat": 4, "nbformat_minor": 4}
    path.write_text(json.dumps(nb))


@pytest.mark.parametrize("mechanism", ["JPY_SESSION_NAME", "__session__"])
def test_run_in_notebook_without_entry_point(tmp_path, monkeypatch, mechanism, capsys):
    """run(entry_point=None) inside a notebook kernel locates the notebook file (reference
    preprocess.py:166-167,196-212 fetched the live Colab notebook) and runs its cells."""
    proj = tmp_path / "nbproj"
    proj.mkdir()
    nb = proj / "analysis.ipynb"
    _write_nb(nb)
    monkeypatch.chdir(proj)
    monkeypatch.setenv("CLOUD_AMD_NUM_GPUS", "0")
    monkeypatch.delenv("JPY_SESSION_NAME", raising=False)
    monkeypatch.setattr(run_mod, "_called_from_notebook", lambda: True)
    if mechanism == "JPY_SESSION_NAME":
        monkeypatch.setenv("JPY_SESSION_NAME", str(nb))
    else:
        fake_ns = {"__session__": "analysis.ipynb"}

        class _IP:
            user_ns = fake_ns

        import types

        fake_ipython = types.SimpleNamespace(get_ipython=lambda: _IP())
        monkeypatch.setitem(sys.modules, "IPython", fake_ipython)
    job = run_mod.run(entry_point=None, chief_config=CPU, jobs_dir=str(tmp_path / "jobs"), exit=False, wait=True)
    assert job.wait(120) == 0
    log = open(job.log_path(0)).read()
    assert "NB_RAN 42" in log, log


def test_run_in_notebook_not_found_is_clear_error(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.delenv("JPY_SESSION_NAME", raising=False)
    monkeypatch.setattr(run_mod, "_called_from_notebook", lambda: True)
    monkeypatch.setattr(run_mod, "current_notebook_path", lambda *a, **k: None)
    with pytest.raises(RuntimeError, match="could not be located"):
        run_mod.run(entry_point=None, chief_config=CPU, jobs_dir=str(tmp_path / "jobs"), exit=False)
