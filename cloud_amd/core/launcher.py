"""On-node job launcher: one process per MI355X (replaces reference ``TFC/core/deploy.py``).

``deploy_job`` keeps the reference's contract -- generate a job id, "submit",
print the same three info lines, optionally stream logs, return the job id --
but the "cluster" is the local node:

* world size = chief GPUs + worker_count x worker GPUs (CPU machines: one
  process each, gloo);
* every rank gets ``RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
  MASTER_ADDR=127.0.0.1 / MASTER_PORT`` (torch.distributed rendezvous, RCCL
  over xGMI on GPU), ``TF_CONFIG``-shaped cluster JSON with ``chief`` /
  ``worker`` roles (``use_chief_in_tf_config`` semantics of reference
  ``deploy.py:159-161``), the remote markers, and per-rank log files
  ``logs/<role>-<index>[-gpu<k>].log``;
* a detached supervisor process (:mod:`.supervisor`) owns the ranks: if any rank exits
  non-zero the rest of the group is terminated, exit codes go to ``job.json`` and the
  job is marked FAILED -- also after the submitting process has exited (fire-and-forget
  ``run()``); ``python -m cloud_amd.jobs describe|stream-logs|cancel <id>`` attaches to
  it by id;
* ``stream_logs=True`` tails every rank's log to stdout until the job ends (reference
  ``deploy.py:187-211`` streams the whole job); with more than one rank each line is
  prefixed ``[chief-0]`` / ``[worker-1]`` / ``[chief-0-gpu3]`` (the log file's stem);
* when the job fails, the failing rank and the last 50 lines of its log are printed.

The launcher process never initialises the GPU: it sizes the job from the KFD
topology in sysfs (:mod:`cloud_amd.core.topology`) and never calls into HIP, so
forking ranks is safe on the MI355X pool.

Multi-GPU jobs also get RCCL transport defaults sized for the xGMI mesh
(:func:`rccl_env`): every variable is ``setdefault`` -- a value the user exported
wins -- and ``CLOUD_AMD_RCCL_ENV=0`` turns the whole set off.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import time
import uuid

from .. import config
from . import supervisor, topology

SUPERVISOR_PID = "supervisor.pid"
PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def generate_job_id(prefix="cloud_amd_train"):
    return "{}_{}".format(prefix, str(uuid.uuid4()).replace("-", "_"))


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def plan_ranks(chief_config, worker_count, worker_config):
    """List of dicts: one per process, with role/index/local device."""
    ranks = []
    machines = [("chief", 0, chief_config)] + [("worker", i, worker_config) for i in range(worker_count)]
    gpu = 0
    for role, idx, cfg in machines:
        n = cfg.num_processes
        for k in range(n):
            ranks.append({"role": role, "index": idx, "proc_in_machine": k,
                          "gpu": gpu if cfg.is_gpu else None})
            if cfg.is_gpu:
                gpu += 1
    for r, info in enumerate(ranks):
        info["rank"] = r
    return ranks


def tf_config_for(ranks, rank, port):
    chief = ["127.0.0.1:{}".format(port)]
    workers = sorted({r["index"] for r in ranks if r["role"] == "worker"})
    cluster = {"chief": chief}
    if workers:
        cluster["worker"] = ["127.0.0.1:{}".format(port + 1 + i) for i in workers]
    me = ranks[rank]
    return {"cluster": cluster, "task": {"type": me["role"], "index": me["index"]}}


def log_name(info):
    name = "{}-{}".format(info["role"], info["index"])
    if info["gpu"] is not None and info["proc_in_machine"] > 0:
        name += "-gpu{}".format(info["proc_in_machine"])
    return name + ".log"


def rccl_env(world, links):
    """RCCL settings for a ``world``-rank job on one MI355X node with ``links``
    point-to-point xGMI links per GPU (7 in the full 8-GPU mesh).

    * ``NCCL_MIN_NCHANNELS`` = links: at least one ring/channel per xGMI link, so a
      collective is never limited to a single ~153 GB/s link (one ring uses one link
      per direction).  RCCL may pick more channels by itself; this is a floor.
      ``CLOUD_AMD_RCCL_CHANNELS`` overrides the value.
    * ``HSA_NO_SCRATCH_RECLAIM=1``: keeps the ROCr scratch pool of the RCCL kernels
      resident instead of reclaiming it after every launch (read at HIP start-up, so
      only ranks this launcher starts get it).

    Gradient buckets are sized separately (``CLOUD_AMD_BUCKET_MB``, bench
    ``--bucket-mb``).  These values are a starting point that the driver's 8-GPU runs
    measure (bench JSON ``comm``), not a tuned optimum."""
    if world <= 1 or os.environ.get("CLOUD_AMD_RCCL_ENV", "1") == "0":
        return {}
    ch = os.environ.get("CLOUD_AMD_RCCL_CHANNELS") or str(max(links, 1))
    return {"NCCL_MIN_NCHANNELS": ch, "HSA_NO_SCRATCH_RECLAIM": "1"}


def _print_logs_info(job_id, job_dir):
    print("Job submitted successfully.")
    print("Your job ID is: ", job_id)
    print("Please access your job logs at the following URL:")
    print("file://{}".format(os.path.join(job_dir, "logs")))
    # the reference's gcloud hints (cloud_fit/client.py:277-286), for the local job service
    print("To describe the job:  python -m cloud_amd.jobs describe {}".format(job_id))
    print("To stream its logs:   python -m cloud_amd.jobs stream-logs {}".format(job_id))
    print("To cancel it:         python -m cloud_amd.jobs cancel {}".format(job_id))


class Job:
    """Client handle of a job run by its detached supervisor (:mod:`.supervisor`).

    The supervisor owns the ranks; this object only reads ``job.json`` (written
    atomically by the supervisor) and signals the supervisor.  It can be dropped at any
    time -- the job keeps running, fails as a group and records its final state -- and
    re-created from the job id with :meth:`attach` (``python -m cloud_amd.jobs``)."""

    def __init__(self, job_id, job_dir, ranks, meta, supervisor=None):
        self.job_id, self.job_dir, self.ranks = job_id, job_dir, ranks
        self._meta = meta
        self._sup = supervisor  # Popen of the supervisor when this process started it

    @classmethod
    def attach(cls, job_id, jobs_dir=None):
        """The job with this id (or job directory path)."""
        job_dir = find_job_dir(job_id, jobs_dir)
        meta = supervisor.read_json(os.path.join(job_dir, supervisor.JOB_META))
        return cls(meta["job_id"], job_dir, meta["ranks"], meta)

    # -- state ------------------------------------------------------------------------
    def refresh(self):
        try:
            self._meta = supervisor.read_json(os.path.join(self.job_dir, supervisor.JOB_META))
        except (OSError, ValueError):  # between the supervisor's write and rename: keep the last
            pass
        return self._meta

    @property
    def meta(self):
        return self.refresh()

    @property
    def state(self):
        return self.refresh().get("state")

    @property
    def returncode(self):
        m = self.refresh()
        return m.get("returncode") if m.get("state") in supervisor.TERMINAL_STATES else None

    def supervisor_pid(self):
        pid = self._meta.get("supervisor_pid")
        if pid is None and self._sup is not None:
            pid = self._sup.pid
        if pid is None:  # the launcher records it beside job.json right after the spawn
            try:
                with open(os.path.join(self.job_dir, SUPERVISOR_PID)) as f:
                    pid = int(f.read().strip())
            except (OSError, ValueError):
                pid = None
        return pid

    def supervisor_alive(self):
        if self._sup is not None:
            return self._sup.poll() is None
        pid = self.supervisor_pid()
        if pid is None:  # submitted this instant: the pid file is not written yet
            return time.time() - float(self._meta.get("start_time") or 0) < 60
        return _pid_alive(pid)

    def done(self):
        m = self.refresh()
        if m.get("state") in supervisor.TERMINAL_STATES:
            return True
        if m.get("state") in ("SUBMITTED", "RUNNING") and not self.supervisor_alive():
            # the supervisor is gone without a final word (killed): re-read once, then say so
            m = self.refresh()
            if m.get("state") not in supervisor.TERMINAL_STATES:
                m = dict(m, state="LOST", returncode=1, error="supervisor exited without recording a final state")
                supervisor.write_json_atomic(os.path.join(self.job_dir, supervisor.JOB_META), m)
                self._meta = m
            return True
        return False

    def wait(self, timeout=None):
        t_end = None if timeout is None else time.time() + timeout
        while not self.done():
            if t_end is not None and time.time() >= t_end:
                return None
            time.sleep(0.05)
        return self.returncode if self.state != "LOST" else 1

    def cancel(self, wait=True, timeout=60):
        """Ask the supervisor to stop the job (SIGTERM to every rank, SIGKILL after the
        grace period); returns the final state when ``wait``."""
        self.refresh()
        pid = self.supervisor_pid()
        if pid and not self.done():
            try:
                os.kill(pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        if wait:
            self.wait(timeout)
        return self.state

    # -- logs -------------------------------------------------------------------------
    def log_path(self, rank=0):
        return os.path.join(self.job_dir, "logs", log_name(self.ranks[rank]))

    def stream(self, ranks=None, out=None, prefix=None):
        """Tail the logs of ``ranks`` (default: every rank) to ``out`` until the job
        finishes.  ``prefix`` (default: on when more than one log is streamed) starts each
        line with ``[<role>-<index>]``; a line is only written once it is complete."""
        out = out or sys.stdout
        if ranks is None:
            ranks = list(range(len(self.ranks)))
        elif isinstance(ranks, int):
            ranks = [ranks]
        if prefix is None:
            prefix = len(ranks) > 1
        tails = []  # [rank, file or None, partial line]
        for r in ranks:
            tails.append([r, None, ""])

        def pump(final=False):
            wrote = False
            for t in tails:
                r, f, part = t
                if f is None:
                    path = self.log_path(r)
                    if not os.path.exists(path):
                        continue
                    f = t[1] = open(path, "r", errors="replace")
                chunk = f.read()
                if not chunk and not (final and part):
                    continue
                data = part + chunk
                lines = data.split("\n")
                t[2] = lines.pop()  # incomplete tail (no newline yet)
                if final and t[2]:
                    lines.append(t[2])
                    t[2] = ""
                tag = "[%s] " % log_name(self.ranks[r])[:-4] if prefix else ""
                for ln in lines:
                    out.write(tag + ln.replace("\x08", "") + "\n")
                wrote = wrote or bool(lines)
            if wrote:
                out.flush()
            return wrote

        try:
            while not self.done():
                if not pump():
                    time.sleep(0.05)
            pump(final=True)
        finally:
            for t in tails:
                if t[1] is not None:
                    t[1].close()

    def log_tail(self, rank, n=50):
        """Last ``n`` lines of one rank's log."""
        try:
            with open(self.log_path(rank), "r", errors="replace") as f:
                return f.read().splitlines()[-n:]
        except OSError:
            return []

    def failure_report(self, n=50):
        """Text naming the rank that failed first, its exit code and its last ``n`` log lines
        (None if the job did not fail)."""
        if self.returncode in (None, 0):
            return None
        r = self.meta.get("failed_rank")
        if r is None:
            codes = self.meta.get("exit_codes") or []
            r = next((i for i, c in enumerate(codes) if c not in (None, 0)), 0)
        code = (self.meta.get("exit_codes") or [None] * (r + 1))[r]
        lines = ["[cloud_amd] job %s FAILED: rank %d (%s) exited with code %s; last %d lines of %s:"
                 % (self.job_id, r, log_name(self.ranks[r])[:-4], code, n, self.log_path(r))]
        lines += ["    " + ln for ln in self.log_tail(r, n)]
        return "\n".join(lines)


def launch(job_id, job_dir, target, chief_config, worker_count, worker_config, entry_point_args=None,
           job_labels=None, extra_env=None, profile=False, python=None, kill_grace_s=15.0):
    """Hand a staged job to its supervisor, which spawns and watches every rank; returns
    the client :class:`Job` at once."""
    ranks = plan_ranks(chief_config, worker_count, worker_config)
    world = len(ranks)
    port = free_port()
    app_dir = os.path.dirname(target)
    python = python or sys.executable
    # CLOUD_AMD_DEVICE=cpu (validate.cpu_rehearsal): GPU-shaped job, CPU ranks over gloo
    rehearsal = os.environ.get("CLOUD_AMD_DEVICE") == "cpu"
    any_gpu = any(r["gpu"] is not None for r in ranks) and not rehearsal
    node = topology.describe_node()
    n_gpu_ranks = sum(1 for r in ranks if r["gpu"] is not None)
    comm_env = rccl_env(n_gpu_ranks, topology.xgmi_links_per_gpu(n_gpu_ranks)) if any_gpu else {}
    meta = {
        "job_id": job_id, "state": "RUNNING", "start_time": time.time(), "world_size": world,
        "chief_config": chief_config.to_dict(), "worker_count": worker_count,
        "worker_config": worker_config.to_dict() if worker_config is not None and worker_count > 0 else None,
        "labels": dict(job_labels or {}), "args": list(entry_point_args or []),
        "backend": "nccl(rccl)" if any_gpu else "gloo", "master_port": port, "cpu_rehearsal": rehearsal,
        "ranks": ranks, "node": node, "comm_env": {k: os.environ.get(k, v) for k, v in comm_env.items()},
    }
    # each GPU rank pinned to the cores of its GPU's NUMA node (KFD io_links + sysfs
    # cpulist; CLOUD_AMD_CPU_AFFINITY=0 leaves placement to the OS scheduler)
    cpu_sets = [None] * len(ranks)
    if any_gpu and config.get("CLOUD_AMD_CPU_AFFINITY"):
        try:
            cpu_sets = topology.rank_cpu_sets([r["gpu"] for r in ranks])
        except Exception:  # noqa: BLE001 - placement is an optimisation, never a launch failure
            cpu_sets = [None] * len(ranks)
    for info, cpus in zip(ranks, cpu_sets):
        info["cpus"] = topology.format_cpulist(cpus) if cpus else None
    spec = []
    for info, cpus in zip(ranks, cpu_sets):
        env = dict(os.environ)
        for k, v in comm_env.items():
            env.setdefault(k, v)
        env.update(extra_env or {})
        env.update({
            "RANK": str(info["rank"]), "WORLD_SIZE": str(world),
            "LOCAL_RANK": str(info["gpu"] if info["gpu"] is not None else info["rank"]),
            "LOCAL_WORLD_SIZE": str(world),
            "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
            "TF_CONFIG": json.dumps(tf_config_for(ranks, info["rank"], port)),
            "TF_KERAS_RUNNING_REMOTELY": "1", "CLOUD_AMD_RUNNING_REMOTELY": "1",
            "CLOUD_AMD_JOB_ID": job_id, "CLOUD_AMD_JOB_DIR": job_dir,
            "CLOUD_AMD_LAUNCH_TIME": str(meta["start_time"]),
            "PYTHONPATH": PKG_ROOT + os.pathsep + env.get("PYTHONPATH", ""),
            "PYTHONUNBUFFERED": "1",
        })
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if not any_gpu:
            env["CLOUD_AMD_DEVICE"] = "cpu"
        if env.get("CLOUD_AMD_DEBUG_SYNC") == "1":  # kernel-fault localisation mode
            env.setdefault("HIP_LAUNCH_BLOCKING", "1")
            env.setdefault("AMD_SERIALIZE_KERNEL", "3")
        cmd = [python, target] + list(entry_point_args or [])
        if profile and info["rank"] == 0:
            prof_dir = os.path.join(job_dir, "profile")
            cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", prof_dir, "-o", "rank0",
                   "--output-format", "csv", "--"] + cmd
        # only what differs from this process's environment goes to disk: the supervisor
        # inherits the rest
        delta = {k: v for k, v in env.items() if os.environ.get(k) != v}
        spec.append({"rank": info["rank"], "cmd": cmd, "cwd": app_dir, "env": delta,
                     "log": os.path.join(job_dir, "logs", log_name(info)), "cpus": sorted(cpus) if cpus else None})
    meta["state"] = "SUBMITTED"
    supervisor.write_json_atomic(os.path.join(job_dir, supervisor.LAUNCH_SPEC),
                                 {"ranks": spec, "kill_grace_s": kill_grace_s})
    supervisor.write_json_atomic(os.path.join(job_dir, supervisor.JOB_META), meta)
    _register(job_id, job_dir)
    sup = supervisor.start(job_dir, python=python, pkg_root=PKG_ROOT)
    with open(os.path.join(job_dir, SUPERVISOR_PID), "w") as f:
        f.write("%d\n" % sup.pid)
    job = Job(job_id, job_dir, ranks, meta, supervisor=sup)
    try:
        from .. import monitoring

        monitoring.inc(monitoring.JOBS, 1, backend=meta["backend"], world=str(world))
    except Exception:  # metrics are best-effort in the launcher
        pass
    return job


def _pid_alive(pid):
    """True while ``pid`` runs (a zombie counts as exited)."""
    if not pid:
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open("/proc/%d/stat" % pid) as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except OSError:
        return True


def index_dir():
    """Where job ids are mapped to job directories, so ``python -m cloud_amd.jobs`` finds a
    job from any working directory (``$CLOUD_AMD_HOME/jobs``, default ``~/.cloud_amd/jobs``)."""
    home = os.environ.get("CLOUD_AMD_HOME") or os.path.join(os.path.expanduser("~"), ".cloud_amd")
    return os.path.join(home, "jobs")


def _register(job_id, job_dir):
    try:
        d = index_dir()
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, job_id), "w") as f:
            f.write(os.path.abspath(job_dir) + "\n")
    except OSError:  # the index is a convenience; the job directory is the record
        pass


def find_job_dir(job_id, jobs_dir=None):
    """Directory of job ``job_id``: a path to a job directory, ``<jobs_dir>/<id>``,
    ``$CLOUD_AMD_JOBS_DIR/<id>``, ``./jobs/<id>``, then the id index."""
    from . import stage

    if os.path.isfile(os.path.join(job_id, supervisor.JOB_META)):
        return os.path.abspath(job_id)
    cands = [os.path.join(jobs_dir, job_id)] if jobs_dir else []
    cands.append(os.path.join(stage.jobs_root(), job_id))
    try:
        with open(os.path.join(index_dir(), job_id)) as f:
            cands.append(f.read().strip())
    except OSError:
        pass
    for c in cands:
        if c and os.path.isfile(os.path.join(c, supervisor.JOB_META)):
            return os.path.abspath(c)
    raise FileNotFoundError("no job %r (looked in %s)" % (job_id, ", ".join(c for c in cands if c)))


def list_jobs(jobs_dir=None):
    """Job directories known here: ``jobs_dir`` / ``$CLOUD_AMD_JOBS_DIR`` / ``./jobs`` and the index."""
    from . import stage

    seen = {}
    for root in [jobs_dir, stage.jobs_root()]:
        if root and os.path.isdir(root):
            for name in os.listdir(root):
                d = os.path.join(root, name)
                if os.path.isfile(os.path.join(d, supervisor.JOB_META)):
                    seen.setdefault(name, os.path.abspath(d))
    if os.path.isdir(index_dir()):
        for name in os.listdir(index_dir()):
            try:
                with open(os.path.join(index_dir(), name)) as f:
                    d = f.read().strip()
            except OSError:
                continue
            if os.path.isfile(os.path.join(d, supervisor.JOB_META)):
                seen.setdefault(name, d)
    return seen


def deploy_job(job_id, job_dir, target, chief_config, worker_count, worker_config, entry_point_args,
               enable_stream_logs, job_labels=None, wait=None, extra_env=None, profile=False):
    """Submit (spawn) the job, print the info lines, optionally stream/wait. Returns the Job."""
    job = launch(job_id, job_dir, target, chief_config, worker_count, worker_config, entry_point_args,
                 job_labels=job_labels, extra_env=extra_env, profile=profile)
    _print_logs_info(job_id, job_dir)
    if enable_stream_logs:
        print("Streaming job logs: ")
        job.stream()
    if wait or (wait is None and enable_stream_logs):
        job.wait()
        report = job.failure_report()
        if report:
            print(report, file=sys.stderr, flush=True)
    return job
