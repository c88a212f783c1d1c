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
* a watchdog: if any rank exits non-zero the rest of the group is terminated,
  exit codes go to ``job.json`` and the job is marked FAILED;
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
import threading
import time
import uuid

from .. import config
from . import topology

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


class Job:
    """A running local job (all rank processes + watchdog)."""

    def __init__(self, job_id, job_dir, procs, ranks, meta):
        self.job_id, self.job_dir, self.procs, self.ranks, self.meta = job_id, job_dir, procs, ranks, meta
        self._done = threading.Event()
        self.returncode = None
        self._watch = threading.Thread(target=self._watchdog, daemon=True)
        self._watch.start()

    def _write_meta(self):
        with open(os.path.join(self.job_dir, "job.json"), "w") as f:
            json.dump(self.meta, f, indent=2)

    def _watchdog(self):
        failed_at = None
        first_failure = None
        while True:
            codes = [p.poll() for p in self.procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad and failed_at is None:
                failed_at = time.time()
                # the rank that failed, before the watchdog kills the rest
                self.meta["failed_rank"], first_failure = bad[0]
                for p in self.procs:
                    if p.poll() is None:
                        try:
                            os.killpg(p.pid, signal.SIGTERM)
                        except (ProcessLookupError, PermissionError):
                            pass
            if failed_at is not None and time.time() - failed_at > 15:
                for p in self.procs:
                    if p.poll() is None:
                        try:
                            os.killpg(p.pid, signal.SIGKILL)
                        except (ProcessLookupError, PermissionError):
                            pass
            if all(c is not None for c in codes):
                break
            time.sleep(0.2)
        codes = [p.returncode for p in self.procs]
        self.meta["exit_codes"] = codes
        self.meta["end_time"] = time.time()
        self.returncode = first_failure if first_failure is not None else next((c for c in codes if c != 0), 0)
        self.meta["state"] = "SUCCEEDED" if self.returncode == 0 else "FAILED"
        self._write_meta()
        self._done.set()

    def wait(self, timeout=None):
        self._done.wait(timeout)
        return self.returncode

    def done(self):
        return self._done.is_set()

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
           job_labels=None, extra_env=None, profile=False, python=None):
    """Spawn all ranks of a staged job; returns a :class:`Job`."""
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
    procs = []
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
        logf = open(os.path.join(job_dir, "logs", log_name(info)), "w")
        p = subprocess.Popen(cmd, cwd=app_dir, env=env, stdout=logf, stderr=subprocess.STDOUT,
                             start_new_session=True)
        _pin(p.pid, cpus)
        logf.close()
        procs.append(p)
    job = Job(job_id, job_dir, procs, ranks, meta)
    job._write_meta()
    try:
        from .. import monitoring

        monitoring.inc(monitoring.JOBS, 1, backend=meta["backend"], world=str(world))
    except Exception:  # metrics are best-effort in the launcher
        pass
    return job


def _pin(pid, cpus):
    """Pin a freshly spawned rank to its CPU set from the parent (``sched_setaffinity(pid)``):
    no ``preexec_fn``, which Python documents as unsafe when the launching process has
    threads.  Popen returns after the child's exec, and the interpreter creates its worker
    threads (OpenMP, HIP) only later, at ``import torch``, so they inherit this mask."""
    if not cpus:
        return
    try:
        os.sched_setaffinity(pid, list(cpus))
    except OSError:
        pass


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
