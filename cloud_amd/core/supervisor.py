"""Detached job supervisor: owns a job's rank processes for the job's whole life.

The reference submits a job and exits (``TFC/core/run.py:232-246``: ``deploy.deploy_job``
then ``sys.exit(0)``); AI Platform then runs the job, kills it when a replica fails and
keeps its state queryable (``gcloud ai-platform jobs describe / stream-logs``,
``TFC/core/deploy.py:170-211``).  On one MI355X node that managed service is this
process:

* the launcher writes ``launch.json`` (one entry per rank: command, working directory,
  environment overrides, log file, CPU set) and starts ``python -m
  cloud_amd.core.supervisor <job_dir>`` in a session of its own, so the client may
  ``sys.exit`` right after submission;
* the supervisor spawns every rank (each in its own process group), records the pids
  in ``job.json`` and watches them: on the first non-zero exit it terminates the rest of
  the group (SIGTERM, SIGKILL after ``kill_grace_s``), then writes the exit codes, the
  failing rank and the final state (``SUCCEEDED`` / ``FAILED`` / ``CANCELLED``);
* SIGTERM / SIGINT to the supervisor (``python -m cloud_amd.jobs cancel <id>``) cancels the
  job the same way;
* every rank gets ``PR_SET_PDEATHSIG = SIGKILL``: if the supervisor itself is killed
  (SIGKILL, OOM), its ranks do not outlive it.

It never imports torch or touches HIP (forking is only safe from a process that has not
initialised the GPU), and it writes ``job.json`` atomically (temp file + rename) because
clients poll it.
"""
from __future__ import annotations

import ctypes
import json
import os
import signal
import subprocess
import sys
import time

TERMINAL_STATES = ("SUCCEEDED", "FAILED", "CANCELLED")
LAUNCH_SPEC = "launch.json"
JOB_META = "job.json"
_PR_SET_PDEATHSIG = 1


def read_json(path):
    with open(path) as f:
        return json.load(f)


def write_json_atomic(path, obj):
    tmp = "%s.tmp.%d" % (path, os.getpid())
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=2)
    os.replace(tmp, path)


def _die_with_parent():
    """preexec_fn of every rank: SIGKILL it when the supervisor dies.  The supervisor is
    single-threaded, so a preexec_fn is safe here (the client never uses one)."""
    try:
        libc = ctypes.CDLL("libc.so.6", use_errno=True)
        libc.prctl(_PR_SET_PDEATHSIG, signal.SIGKILL, 0, 0, 0)
    except OSError:
        pass
    if os.getppid() == 1:  # the supervisor died between fork and prctl
        os._exit(137)


def _signal_group(pid, sig):
    try:
        os.killpg(pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


class Supervisor:
    def __init__(self, job_dir):
        self.job_dir = os.path.abspath(job_dir)
        self.spec = read_json(os.path.join(self.job_dir, LAUNCH_SPEC))
        self.meta_path = os.path.join(self.job_dir, JOB_META)
        self.meta = read_json(self.meta_path)
        self.procs = []
        self.cancel_requested = False
        self.grace = float(self.spec.get("kill_grace_s", 15.0))

    def _on_signal(self, signum, frame):  # noqa: ARG002 - signal handler signature
        self.cancel_requested = True

    def _save(self):
        write_json_atomic(self.meta_path, self.meta)

    def spawn(self):
        for r in self.spec["ranks"]:
            env = dict(os.environ)
            env.update(r.get("env") or {})
            logf = open(r["log"], "w")
            p = subprocess.Popen(r["cmd"], cwd=r.get("cwd"), env=env, stdout=logf, stderr=subprocess.STDOUT,
                                 stdin=subprocess.DEVNULL, start_new_session=True, preexec_fn=_die_with_parent)
            logf.close()
            cpus = r.get("cpus")
            if cpus:
                try:
                    os.sched_setaffinity(p.pid, list(cpus))
                except OSError:
                    pass
            self.procs.append(p)
        self.meta.update({"state": "RUNNING", "supervisor_pid": os.getpid(),
                          "pids": [p.pid for p in self.procs], "running_time": time.time()})
        self._save()

    def watch(self, poll_s=0.1):
        stop_at = None          # when the group was told to stop (failure or cancel)
        first_failure = None
        while True:
            codes = [p.poll() for p in self.procs]
            if stop_at is None:
                bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
                if bad:
                    self.meta["failed_rank"], first_failure = bad[0]
                if bad or self.cancel_requested:
                    stop_at = time.time()
                    for p, c in zip(self.procs, codes):
                        if c is None:
                            _signal_group(p.pid, signal.SIGTERM)
                    if self.cancel_requested and not bad:
                        self.meta["cancel_time"] = stop_at
                    self.meta["stopping"] = True
                    self._save()
            elif time.time() - stop_at > self.grace:
                for p, c in zip(self.procs, codes):
                    if c is None:
                        _signal_group(p.pid, signal.SIGKILL)
            if all(c is not None for c in codes):
                break
            time.sleep(poll_s)
        codes = [p.returncode for p in self.procs]
        if first_failure is not None:
            rc = first_failure
            state = "FAILED"
        elif self.cancel_requested and "cancel_time" in self.meta:
            rc = next((c for c in codes if c != 0), 0) or -int(signal.SIGTERM)
            state = "CANCELLED"
        else:
            rc = next((c for c in codes if c != 0), 0)
            state = "SUCCEEDED" if rc == 0 else "FAILED"
        self.meta.pop("stopping", None)
        self.meta.update({"exit_codes": codes, "returncode": rc, "state": state, "end_time": time.time()})
        self._save()
        return rc

    def run(self):
        for s in (signal.SIGTERM, signal.SIGINT):
            signal.signal(s, self._on_signal)
        signal.signal(signal.SIGHUP, signal.SIG_IGN)
        try:
            self.spawn()
        except Exception as e:  # noqa: BLE001 - a rank that cannot start fails the job visibly
            for p in self.procs:
                _signal_group(p.pid, signal.SIGKILL)
            for p in self.procs:
                p.wait()
            self.meta.update({"state": "FAILED", "error": "spawn failed: %s" % e, "returncode": 1,
                              "exit_codes": [p.returncode for p in self.procs], "end_time": time.time()})
            self._save()
            return 1
        return self.watch()


def start(job_dir, python=None, pkg_root=None):
    """Start the supervisor of a staged job (``launch.json`` + ``job.json`` written) in a
    session of its own; returns the Popen handle."""
    python = python or sys.executable
    env = dict(os.environ)
    if pkg_root:
        env["PYTHONPATH"] = pkg_root + os.pathsep + env.get("PYTHONPATH", "")
    for k in ("CLOUD_AMD_RUNNING_REMOTELY", "TF_KERAS_RUNNING_REMOTELY"):
        env.pop(k, None)  # the supervisor is not a rank
    log = open(os.path.join(job_dir, "supervisor.log"), "w")  # beside job.json, not among rank logs
    try:
        return subprocess.Popen([python, "-m", "cloud_amd.core.supervisor", job_dir], env=env, stdout=log,
                                stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, start_new_session=True,
                                close_fds=True)
    finally:
        log.close()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 1:
        print("usage: python -m cloud_amd.core.supervisor <job_dir>", file=sys.stderr)
        return 2
    return Supervisor(argv[0]).run()


if __name__ == "__main__":
    rc = main()
    sys.exit(rc if 0 <= rc < 256 else 1)
