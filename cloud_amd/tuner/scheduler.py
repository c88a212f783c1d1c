"""Asynchronous trial scheduler: many tuner processes share one study.

Replaces the Vizier-side parallelism of the reference (N processes with the
same ``study_id`` and distinct ``tuner_id``, ``tuner_integration_test.py:82-116``)
with an on-node scheduler: one worker per MI355X -- or several per GPU when
the trials are small, packed by an HBM estimate into 288 GB (``trial_gb``) --
each running ``tuner.search`` against the shared local study.  Workers are
independent processes (a crashed trial is INVALID, a crashed worker does not
stop the others), results are read back from the study.

    sched = TrialScheduler("my_pkg.search:run", n_gpus=8, trial_gb=6)
    summary = sched.run()          # blocks; returns per-worker exit codes + study trials

``target`` names a function ``run(tuner_id: str, device: str) -> None`` that
builds a tuner (same study_id everywhere) and calls ``search``.
"""
from __future__ import annotations

import importlib
import json
import multiprocessing as mp
import os
import time

from ..utils import hbm


def _worker(target, tuner_id, device, env):
    os.environ.update(env)
    os.environ["CLOUD_AMD_TUNER_ID"] = tuner_id
    os.environ["KERASTUNER_TUNER_ID"] = tuner_id
    if device.startswith("cuda"):
        import torch

        torch.cuda.set_device(int(device.split(":")[1]))
        os.environ["LOCAL_RANK"] = device.split(":")[1]
    else:
        os.environ["CLOUD_AMD_DEVICE"] = "cpu"
    mod, fn = target.split(":")
    getattr(importlib.import_module(mod), fn)(tuner_id, device)


class TrialScheduler:
    def __init__(self, target, n_gpus=None, trial_gb=4.0, workers=None, max_workers=16, env=None):
        self.target = target
        if n_gpus is None:
            from ..core.topology import visible_gpu_count

            n_gpus = visible_gpu_count()
        self.n_gpus = n_gpus
        per = hbm.trials_per_gpu(trial_gb) if n_gpus else 1
        self.workers = workers or max(1, min(max_workers, (n_gpus or 1) * per))
        self.env = dict(env or {})

    def devices(self):
        if not self.n_gpus:
            return ["cpu"] * self.workers
        return [f"cuda:{i % self.n_gpus}" for i in range(self.workers)]

    def run(self, timeout=None):
        ctx = mp.get_context("spawn")
        procs = []
        t0 = time.time()
        for i, dev in enumerate(self.devices()):
            p = ctx.Process(target=_worker, args=(self.target, f"tuner{i}", dev, self.env), daemon=False)
            p.start()
            procs.append(p)
        for p in procs:
            p.join(None if timeout is None else max(0.0, timeout - (time.time() - t0)))
        codes = []
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(5)
            codes.append(p.exitcode)
        return {"workers": len(procs), "exit_codes": codes, "wall_s": time.time() - t0}


def study_report(study_dir, study_id):
    with open(os.path.join(study_dir, study_id, "study.json")) as f:
        data = json.load(f)
    return data["trials"]
