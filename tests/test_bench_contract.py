"""bench.py launch contract: by default the headline bench stages
and spawns its ranks through cloud_amd.run(); the world size a rank sees must equal
--gpus; a node with too few GPUs is a hard error."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--model", "tiny", "--device", "cpu", "--batch", "4", "--image-size", "32", "--classes", "10",
        "--steps", "2", "--warmup", "1"]


def _env(tmp_path, **kw):
    env = dict(os.environ, CLOUD_AMD_JOBS_DIR=str(tmp_path / "jobs"), OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "CLOUD_AMD_RUNNING_REMOTELY", "TORCHELASTIC_RUN_ID",
              "TF_KERAS_RUNNING_REMOTELY"):
        env.pop(k, None)
    env.update(kw)
    return env


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_two_ranks_via_run_cpu(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + TINY,
                       env=_env(tmp_path), capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout[-3000:]
    j = lines[0]
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2"
    assert j["launched_via"] == "cloud_amd.run()"
    assert j["run_to_first_step_s"] is not None and j["run_to_first_step_s"] > 0
    ph = j["startup_phases_rank0"]  # run() -> first step split at the wrapper and the script body
    assert set(ph) == {"launch_s", "rank_setup_s", "first_step_s"} and all(v >= 0 for v in ph.values())
    assert abs(sum(ph.values()) - j["run_to_first_step_s"]) < 0.5
    assert j["comm"]["buckets"] >= 1 and j["comm"]["allreduce_ms"] > 0
    assert j["backend"] == "gloo" and j["config"]["global_batch"] == 8
    probe = j["comm"]["comm_probe"]  # both transports measured on the same buffers
    assert set(probe) == {"torch", "bench_transport"} and probe["torch"]["16"]["busbw_gbs"] > 0  # CPU: no RCCL
    assert probe["bench_transport"] == "torch"
    # overlap budget: per-bucket readiness needs device events -> none on CPU ranks
    assert "overlap_budget" in j and j["overlap_budget"] is None
    assert j["comm"]["sliced_optimizer"] is False  # gloo is not stream-ordered
    ss = j["step_stats_rank0"]
    assert ss["host_launch_ms"]["min"] <= ss["host_launch_ms"]["median"] <= ss["host_launch_ms"]["max"]
    assert ss["host_before"]["n_affinity"] >= 1 and isinstance(j["warnings"], list)
    # per-step host evidence for slow-step diagnosis: GC pauses, page faults, allocator segments
    assert len(ss["probe_steps"]) == 2 and len(ss["host_launch_ms_steps"]) == 2
    assert {"gc_ms", "gc_gen", "minflt", "majflt", "dev_alloc"} <= set(ss["probe_steps"][0])
    assert j["gc_frozen_objects"] > 0  # runtime.gc_control.freeze() ran after warmup
    # N > 1: the DP-engine A/B after the timed region: 12 cells of <= 5
    # timed steps -- per-bucket optimizer x bucket size x transport -- each with ms/step and
    # the exposed communication; the headline value is the default configuration's
    ab = j["dp_ab"]
    cells = ab["cells"]
    assert len(cells) == 12 and ab["steps_per_cell"] == 5
    assert {(c["transport"], c["bucket_mb"], c["sliced"]) for c in cells} == {
        (t, b, sl) for t in ("torch", "rccl") for b in (16.0, 32.0, 64.0) for sl in (False, True)}
    for c in cells:
        assert "error" not in c, c
        assert c["ms_per_step"] > 0 and c["exposed_comm_ms"] >= 0 and c["steps"] == 5 and c["buckets"] >= 1
        assert c["sliced_active"] is False  # gloo is not stream-ordered: the cell reports it ran whole-arena
    assert ab["best"] in cells
    job = os.listdir(tmp_path / "jobs")
    assert len(job) == 1
    meta = json.load(open(tmp_path / "jobs" / job[0] / "job.json"))
    assert meta["world_size"] == 2 and meta["state"] == "SUCCEEDED"


def test_bench_too_many_gpus_fails(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=_env(tmp_path, CLOUD_AMD_NUM_GPUS="1"), capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert r.returncode != 0
    assert "needs 2 GPUs" in r.stderr and not _json_lines(r.stdout)


def test_bench_world_mismatch_is_an_error(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--via-run", "0"] + TINY,
                       env=_env(tmp_path, WORLD_SIZE="1", RANK="0"), capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert r.returncode == 3, r.stderr[-2000:]
    assert "WORLD_SIZE=1" in r.stderr and not _json_lines(r.stdout)


def test_step_stats_names_gc_pause_of_slow_step():
    """A slow step's warning carries the probe row of that step (here: a 3 s GC pause)."""
    sys.path.insert(0, ROOT)
    from cloud_amd.utils import benchlaunch

    dev = [70.0] * 5 + [3100.0] + [70.0] * 4
    host = [60.0] * 5 + [3300.0] + [60.0] * 4
    probe = [{"gc_ms": 0.0, "gc_gen": -1, "minflt": 10, "majflt": 0, "dev_alloc": 0, "dev_free": 0,
              "alloc_retry": 0} for _ in dev]
    probe[5].update(gc_ms=3050.0, gc_gen=2, majflt=812)
    st = benchlaunch.step_stats(dev, host, {"ctx_involuntary": 1}, {"ctx_involuntary": 2}, probe=probe)
    assert len(st["warnings"]) == 2 and "slow steps [5]" in st["warnings"][0]
    assert "'gc_ms': 3050.0" in st["warnings"][1] and "'majflt': 812" in st["warnings"][1]
    assert st["gc_ms_total"] == 3050.0


def test_gc_freeze_control(monkeypatch):
    import gc

    sys.path.insert(0, ROOT)
    from cloud_amd.runtime import gc_control

    monkeypatch.setenv("CLOUD_AMD_GC_FREEZE", "0")
    assert gc_control.freeze() == 0
    monkeypatch.setenv("CLOUD_AMD_GC_FREEZE", "1")
    try:
        assert gc_control.freeze() > 0 and gc.get_freeze_count() > 0
    finally:
        gc_control.unfreeze()
    assert gc.get_freeze_count() == 0
