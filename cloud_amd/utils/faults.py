"""Env-driven fault injection for failure-path tests.

``CLOUD_AMD_FAULT="rank:step:kind"`` (comma-separated list) makes the given
rank fail at the given global training step.  kinds:

* ``exit``  -- ``sys.exit(17)`` (non-zero rank exit: the launcher watchdog must
  tear down the job and record the code in job.json);
* ``raise`` -- raise RuntimeError inside the step (a tuner trial must become
  INFEASIBLE / the job must fail);
* ``hang``  -- sleep for ``CLOUD_AMD_FAULT_HANG_S`` seconds (default 3600) to
  exercise collective / watchdog timeouts.
"""
from __future__ import annotations

import os
import sys
import time


def _parse():
    spec = os.environ.get("CLOUD_AMD_FAULT", "")
    out = []
    for item in filter(None, (s.strip() for s in spec.split(","))):
        r, st, kind = item.split(":")
        out.append((int(r), int(st), kind))
    return out


def maybe_inject(step, rank=0):
    for r, st, kind in _parse():
        if r == rank and st == step:
            if kind == "exit":
                print(f"[cloud_amd.faults] injected exit at rank {rank} step {step}", flush=True)
                sys.exit(17)
            if kind == "raise":
                raise RuntimeError(f"injected fault at rank {rank} step {step}")
            if kind == "hang":
                time.sleep(float(os.environ.get("CLOUD_AMD_FAULT_HANG_S", 3600)))
