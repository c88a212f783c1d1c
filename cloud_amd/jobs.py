"""Inspect and control submitted jobs by id: ``python -m cloud_amd.jobs <command> <job_id>``.

The local counterpart of the ``gcloud ai-platform jobs describe / stream-logs / cancel``
commands the reference points its users to (``TFC/core/deploy.py:170-211``,
``TFC/experimental/cloud_fit/client.py:277-286``).  Works from any process and any
working directory: a job is found through ``--jobs-dir``, ``$CLOUD_AMD_JOBS_DIR``,
``./jobs`` or the id index the launcher keeps (``$CLOUD_AMD_HOME/jobs``).

Commands:

* ``list``                  -- every known job with its state;
* ``describe <id>``         -- state, ranks, pids, exit codes, failing rank, paths (``--json``
  prints ``job.json`` itself);
* ``stream-logs <id>``      -- tail every rank's log (``--rank N`` for one) until the job ends
  (``--no-follow``: print what is there and return);
* ``cancel <id>``           -- stop the job (SIGTERM to every rank through its supervisor,
  SIGKILL after the grace period) and wait for the final state.

Exit status of ``describe`` / ``stream-logs`` / ``cancel``: 0, or 1 when the job is FAILED /
LOST, 2 when no such job exists.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys

from .core import launcher, supervisor


def _ts(t):
    return datetime.datetime.fromtimestamp(t).strftime("%Y-%m-%d %H:%M:%S") if t else "-"


def describe(job, out=None):
    out = out or sys.stdout
    m = job.refresh()
    done = job.done()
    m = job.refresh()
    lines = [
        ("jobId", m.get("job_id")),
        ("state", m.get("state")),
        ("jobDir", job.job_dir),
        ("createTime", _ts(m.get("start_time"))),
        ("startTime", _ts(m.get("running_time"))),
        ("endTime", _ts(m.get("end_time"))),
        ("worldSize", m.get("world_size")),
        ("backend", m.get("backend")),
        ("labels", json.dumps(m.get("labels") or {})),
        ("args", json.dumps(m.get("args") or [])),
        ("supervisorPid", "%s (%s)" % (job.supervisor_pid(), "alive" if job.supervisor_alive() else "exited")),
    ]
    if done:
        lines.append(("exitCodes", json.dumps(m.get("exit_codes"))))
        lines.append(("returnCode", m.get("returncode")))
    if m.get("failed_rank") is not None:
        lines.append(("failedRank", m.get("failed_rank")))
    if m.get("error"):
        lines.append(("error", m.get("error")))
    for k, v in lines:
        out.write("%s: %s\n" % (k, v))
    out.write("ranks:\n")
    pids = m.get("pids") or [None] * len(job.ranks)
    codes = m.get("exit_codes") or [None] * len(job.ranks)
    for r, info in enumerate(job.ranks):
        out.write("- rank: %d\n  role: %s-%d\n  gpu: %s\n  pid: %s\n  exitCode: %s\n  log: %s\n"
                  % (r, info["role"], info["index"], info.get("gpu"), pids[r] if r < len(pids) else None,
                     codes[r] if r < len(codes) else None, job.log_path(r)))
    out.flush()
    return m


def _rc_for(job):
    return 1 if job.state in ("FAILED", "LOST") else 0


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m cloud_amd.jobs", description=__doc__.split("\n")[0])
    ap.add_argument("--jobs-dir", default=None, help="directory holding job directories")
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("list")
    d = sub.add_parser("describe")
    d.add_argument("job_id")
    d.add_argument("--json", action="store_true", help="print job.json")
    s = sub.add_parser("stream-logs")
    s.add_argument("job_id")
    s.add_argument("--rank", type=int, default=None)
    s.add_argument("--no-follow", action="store_true")
    c = sub.add_parser("cancel")
    c.add_argument("job_id")
    c.add_argument("--timeout", type=float, default=60.0)
    a = ap.parse_args(argv)

    if a.cmd == "list":
        for jid, d in sorted(launcher.list_jobs(a.jobs_dir).items()):
            try:
                m = supervisor.read_json(os.path.join(d, supervisor.JOB_META))
            except (OSError, ValueError):
                continue
            print("%-60s %-10s world=%-3s %s" % (jid, m.get("state"), m.get("world_size"), _ts(m.get("start_time"))))
        return 0
    try:
        job = launcher.Job.attach(a.job_id, a.jobs_dir)
    except FileNotFoundError as e:
        print(str(e), file=sys.stderr)
        return 2
    if a.cmd == "describe":
        if a.json:
            job.done()
            print(json.dumps(job.refresh(), indent=2))
        else:
            describe(job)
        return _rc_for(job)
    if a.cmd == "stream-logs":
        if a.no_follow:
            ranks = [a.rank] if a.rank is not None else range(len(job.ranks))
            for r in ranks:
                tag = "[%s] " % launcher.log_name(job.ranks[r])[:-4] if len(job.ranks) > 1 and a.rank is None else ""
                for ln in job.log_tail(r, n=10 ** 9):
                    print(tag + ln)
        else:
            job.stream(ranks=a.rank)
        job.done()
        report = job.failure_report()
        if report:
            print(report, file=sys.stderr)
        return _rc_for(job)
    if a.cmd == "cancel":
        state = job.cancel(wait=True, timeout=a.timeout)
        print("job %s: %s" % (job.job_id, state))
        return 0 if state in supervisor.TERMINAL_STATES else 1
    return 2


if __name__ == "__main__":
    sys.exit(main())
