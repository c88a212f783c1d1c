"""Asynchronous trial scheduler: many tuner processes share one study.

Replaces the Vizier-side parallelism of the reference (N processes with the
same ``study_id`` and distinct ``tuner_id``, ``tuner_integration_test.py:82-116``)
with an on-node scheduler: one worker per MI355X -- or several per GPU when
the trials are small, packed by an HBM estimate into 288 GB (``trial_gb``) --
each running ``tuner.search`` against the shared local study; by default the
per-GPU packing comes from the measured HBM footprint of the first trial.  Workers are
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
import sys
import time

from ..utils import hbm


def _await_gate(gate_file, poll_s=0.01, parent=None, deadline_s=None):
    """Standby worker: wait for the scheduler's verdict (True = run, False = exit).

    A standby never outlives its scheduler: it gives up (False) when its parent process
    is gone (re-parented: ``os.getppid()`` changed), when the gate's directory was removed,
    or after ``deadline_s`` (``CLOUD_AMD_TUNER_GATE_TIMEOUT_S``)."""
    from .. import config

    parent = os.getppid() if parent is None else parent
    if deadline_s is None:
        deadline_s = config.get("CLOUD_AMD_TUNER_GATE_TIMEOUT_S")
    t_end = time.time() + deadline_s if deadline_s else None
    state_dir = os.path.dirname(gate_file)
    while True:
        if os.path.exists(gate_file):
            try:
                with open(gate_file) as fh:
                    return bool(json.load(fh)["go"])
            except (OSError, ValueError, KeyError):
                pass  # written non-atomically by an older scheduler: retry
        if os.getppid() != parent or not os.path.isdir(state_dir):
            return False
        if t_end is not None and time.time() > t_end:
            return False
        time.sleep(poll_s)


def _mark(timeline, key):
    if timeline is not None:
        timeline[key] = time.time()


def _worker(target, tuner_id, device, env, gate_file=None, timeline_file=None):
    tl = {"entered": time.time()} if timeline_file else None
    try:
        _worker_body(target, tuner_id, device, env, gate_file, tl)
    finally:
        if tl is not None:
            _mark(tl, "exited")
            tmp = timeline_file + ".tmp"
            with open(tmp, "w") as fh:
                json.dump(tl, fh)
            os.replace(tmp, timeline_file)
    from .. import config

    if config.get("CLOUD_AMD_TUNER_FAST_EXIT"):
        # every result is already in the study (written synchronously under its lock):
        # skip the interpreter / torch / HIP teardown (~0.4 s per worker on the GPU box,
        # the tail of the study's wall time); a failed worker still exits normally above
        if "torch" in sys.modules and sys.modules["torch"].cuda.is_initialized():
            sys.modules["torch"].cuda.synchronize()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


def _worker_body(target, tuner_id, device, env, gate_file, tl):
    if gate_file:
        # warm standby: pay interpreter start, `import torch`, the target module import and
        # (CLOUD_AMD_TUNER_STANDBY_HIP) the device's HIP context + the kernel library while
        # the probe wave runs; a dismissed standby gives its context back when it exits
        os.environ.update(env)
        import torch

        from .. import config

        mod_name = target.split(":")[0]
        importlib.import_module(mod_name)
        _mark(tl, "imported")
        if device.startswith("cuda") and config.get("CLOUD_AMD_TUNER_STANDBY_HIP"):
            torch.cuda.set_device(int(device.split(":")[1]))
            torch.empty(1, device=device)
            from ..ops import _ext

            _ext.load(required=False)
            _mark(tl, "device_ready")
        go = _await_gate(gate_file)
        _mark(tl, "released" if go else "dismissed")
        if not go:
            return
    os.environ.update(env)
    os.environ["CLOUD_AMD_TUNER_ID"] = tuner_id
    os.environ["KERASTUNER_TUNER_ID"] = tuner_id
    os.environ["CLOUD_AMD_TRIAL_DEVICE"] = device  # recorded on every trial this worker runs
    if device.startswith("cuda") and os.environ.get("CLOUD_AMD_SCHED_FAKE_DEVICES") != "1":
        import torch

        torch.cuda.set_device(int(device.split(":")[1]))
        os.environ["LOCAL_RANK"] = device.split(":")[1]
    else:
        # CPU node, or a placement rehearsal on a CPU host (CLOUD_AMD_SCHED_FAKE_DEVICES=1:
        # the worker keeps its assigned GPU name for the study record but computes on CPU)
        if device.startswith("cuda"):
            os.environ["LOCAL_RANK"] = device.split(":")[1]
        os.environ["CLOUD_AMD_DEVICE"] = "cpu"
    mod, fn = target.split(":")
    _mark(tl, "running")
    getattr(importlib.import_module(mod), fn)(tuner_id, device)


def _release_gpu_state():
    """Between pooled jobs: return every cached segment a job left to the driver and reset
    the peak-memory counters of every device this process touched, so the next study's
    footprint probe (``max_memory_reserved``) measures that study alone and packing by
    measured footprint never counts a previous job's pool."""
    try:
        import torch
    except Exception:  # pragma: no cover
        return
    if not (torch.cuda.is_available() and torch.cuda.is_initialized()):
        return
    import gc

    gc.collect()  # the job's tensors (a finished trial's model) become free blocks first
    for d in range(torch.cuda.device_count()):
        try:
            if torch.cuda.memory_reserved(d) == 0 and torch.cuda.max_memory_reserved(d) == 0:
                continue  # never touched: do not create a context there
            with torch.cuda.device(d):
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(d)
        except Exception as e:  # pragma: no cover - a failing device must not kill the pool
            print("[cloud_amd pool] releasing cuda:%d: %r" % (d, e), file=sys.stderr, flush=True)


def _pool_main(idx, jobs, done, preload, env):
    """A pooled tuner worker: imports once, then runs scheduler jobs until told to stop.
    Each job is (target, tuner_id, device, env, timeline_file); the job's env is applied for
    the job only."""
    os.environ.update(env or {})
    for mod in preload:
        importlib.import_module(mod)
    done.put(("ready", idx, time.time()))
    base_env = dict(os.environ)
    while True:
        job = jobs.get()
        if job is None:
            break
        target, tuner_id, device, jenv, tl_file = job
        tl = {"entered": time.time()} if tl_file else None
        code = 0
        try:
            _worker_body(target, tuner_id, device, jenv, None, tl)
        except BaseException as e:  # a failing job fails that job, the pool worker lives on
            code = 1
            print("[cloud_amd pool] %s failed: %r" % (tuner_id, e), file=sys.stderr, flush=True)
        finally:
            _release_gpu_state()
            if tl is not None:
                _mark(tl, "exited")
                tmp = tl_file + ".tmp"
                with open(tmp, "w") as fh:
                    json.dump(tl, fh)
                os.replace(tmp, tl_file)
            os.environ.clear()
            os.environ.update(base_env)
        done.put(("done", idx, code))


class WorkerPool:
    """Warm tuner workers kept across studies: ``n`` processes that paid interpreter start
    and ``import torch`` (+ ``preload`` modules) once and then run scheduler jobs back to back
    -- a study on a warm pool starts its trials immediately instead of after ~1.5 s of imports
    per worker (the reference's equivalent cost is Vizier round trips per trial).

        pool = WorkerPool(8, preload=["bench.tuner_8trials"]); pool.wait_ready()
        TrialScheduler(target, n_gpus=8, pool=pool).run()   # any number of studies
        pool.close()
    """

    def __init__(self, n, preload=(), env=None):
        ctx = mp.get_context("spawn")
        self.n = n
        self._done = ctx.Queue()
        self._jobs = [ctx.Queue() for _ in range(n)]
        self._busy = [False] * n
        self._ready = set()
        self.t_start = time.time()
        self.t_ready = None
        mods = ["torch", "cloud_amd.keras", "cloud_amd.tuner"] + list(preload)
        self._procs = [ctx.Process(target=_pool_main, args=(i, self._jobs[i], self._done, mods, dict(env or {})),
                                   daemon=True) for i in range(n)]
        for p in self._procs:
            p.start()
        self._codes = {}

    def _drain(self, block, timeout=None):
        import queue

        try:
            msg = self._done.get(block, timeout)
        except queue.Empty:
            return False
        if msg[0] == "ready":
            self._ready.add(msg[1])
        else:
            self._busy[msg[1]] = False
            self._codes[msg[1]] = msg[2]
        return True

    def wait_ready(self, timeout=600):
        t_end = time.time() + timeout
        while len(self._ready) < self.n:
            if time.time() > t_end or not all(p.is_alive() for p in self._procs):
                raise RuntimeError("worker pool did not start (%d of %d ready)" % (len(self._ready), self.n))
            self._drain(True, 0.5)
        self.t_ready = self.t_ready or time.time()
        return self.t_ready - self.t_start

    def idle(self):
        while self._drain(False):
            pass
        return [i for i in range(self.n) if not self._busy[i] and i in self._ready]

    def submit(self, i, job):
        self._busy[i] = True
        self._codes.pop(i, None)
        self._jobs[i].put(job)

    def wait(self, workers, timeout=None):
        """Exit codes of the jobs on ``workers`` once all finished (None: timed out / died)."""
        t_end = None if timeout is None else time.time() + timeout
        while any(self._busy[i] for i in workers):
            if t_end is not None and time.time() > t_end:
                break
            if not all(self._procs[i].is_alive() for i in workers if self._busy[i]):
                break
            self._drain(True, 0.2)
        return [self._codes.get(i) if not self._busy[i] else None for i in workers]

    def close(self):
        for q in self._jobs:
            q.put(None)
        for p in self._procs:
            p.join(10)
            if p.is_alive():
                p.terminate()
                p.join(5)


class TrialScheduler:
    """Run tuner workers on the node's GPUs.

    Packing (how many workers share one GPU's 288 GB):

    * ``workers=N``: exactly N workers, round-robin over the GPUs;
    * ``trial_gb=G``: ``hbm.trials_per_gpu(G)`` workers per GPU;
    * neither (default): **measured** -- a probe wave of one worker per GPU runs; the
      first worker to finish a trial reports the allocator's peak reserved HBM
      (``hbm.report_footprint``), and the scheduler then adds workers until each GPU
      holds ``trials_per_gpu(peak * headroom)`` of them.

    ``max_workers`` bounds the total (default: the CPUs this process may use, since
    every worker also needs a core for its input pipeline and launches)."""

    def __init__(self, target, n_gpus=None, trial_gb=None, workers=None, max_workers=None, env=None,
                 hbm_gb=None, headroom=1.25, state_dir=None, probe_timeout_s=None, timeline=False, pool=None):
        self.target = target
        self.pool = pool  # WorkerPool: run jobs on warm workers instead of spawning processes
        if n_gpus is None:
            from ..core.topology import hbm_gb_per_gpu, visible_gpu_count

            n_gpus = visible_gpu_count()
            hbm_gb = hbm_gb if hbm_gb is not None else (hbm_gb_per_gpu() if n_gpus else None)
        self.n_gpus = n_gpus
        self.hbm_gb = hbm_gb
        self.trial_gb = trial_gb
        self.headroom = headroom
        self.fixed_workers = workers
        try:
            cpus = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            cpus = os.cpu_count() or 1
        self.max_workers = max_workers or max(1, cpus)
        self.env = dict(env or {})
        self.state_dir = state_dir
        self.probe_timeout_s = probe_timeout_s
        self.timeline = timeline
        self._state = None
        self.footprint_gb = None
        self.per_gpu = None
        if workers:
            self.workers = workers
        elif trial_gb:
            self.per_gpu = hbm.trials_per_gpu(trial_gb, self.hbm_gb) if n_gpus else 1
            self.workers = max(1, min(self.max_workers, (n_gpus or 1) * self.per_gpu))
        else:
            self.workers = None  # decided after the probe wave

    def _slots(self):
        return max(self.n_gpus, 1)

    def standby_count(self):
        """Gated standbys started with the probe wave: bounded by ``max_workers`` and by an
        estimate of what packing can use (``CLOUD_AMD_TUNER_STANDBY_PER_GPU`` per GPU), so a
        many-core node does not start 100+ interpreters that packing then dismisses."""
        from .. import config

        per = max(0, int(config.get("CLOUD_AMD_TUNER_STANDBY_PER_GPU")))
        return max(0, min(self.max_workers - self._slots(), self._slots() * per))

    def _device(self, i):
        return f"cuda:{i % self.n_gpus}" if self.n_gpus else "cpu"

    def devices(self):
        n = self.workers or self._slots()
        return [self._device(i) for i in range(n)]

    def _spawn(self, ctx, i, footprint_file=None, gate_file=None):
        env = dict(self.env)
        if footprint_file:
            env["CLOUD_AMD_FOOTPRINT_FILE"] = footprint_file
        tl_file = os.path.join(self._state, f"timeline_tuner{i}.json") if self.timeline else None
        p = ctx.Process(target=_worker, args=(self.target, f"tuner{i}", self._device(i), env, gate_file, tl_file),
                        daemon=False)
        p.start()
        return p

    @staticmethod
    def _open_gate(path, go):
        tmp = path + ".tmp"
        with open(tmp, "w") as fh:
            json.dump({"go": bool(go)}, fh)
        os.replace(tmp, path)

    def packing_from_footprint(self, peak_gb):
        """Workers per GPU for a measured per-trial peak (GiB)."""
        hbm_gb = self.hbm_gb if self.hbm_gb is not None else hbm.HBM_GB
        return hbm.trials_per_gpu(peak_gb * self.headroom, hbm_gb)

    def _run_pool(self, timeout, t0, state):
        """run() on a WorkerPool: the probe wave, then the packing wave, on idle warm workers."""
        pool = self.pool
        pool.wait_ready()
        cap = min(self.max_workers, pool.n)
        used = []

        def start(i_slot, footprint_file=None):
            idle = [w for w in pool.idle() if w not in used]
            if not idle:
                return False
            w = idle[0]
            env = dict(self.env)
            if footprint_file:
                env["CLOUD_AMD_FOOTPRINT_FILE"] = footprint_file
            tl_file = os.path.join(state, f"timeline_tuner{i_slot}.json") if self.timeline else None
            pool.submit(w, (self.target, f"tuner{i_slot}", self._device(i_slot), env, tl_file))
            used.append(w)
            return True

        if self.workers is not None:
            for i in range(min(self.workers, cap)):
                start(i)
        else:
            files = [os.path.join(state, f"footprint_tuner{i}.json") for i in range(self._slots())]
            for i in range(min(self._slots(), cap)):
                start(i, files[i])
            limit = self.probe_timeout_s if self.probe_timeout_s is not None else timeout
            while self.footprint_gb is None:
                for f in files:
                    if os.path.exists(f):
                        with open(f) as fh:
                            self.footprint_gb = float(json.load(fh)["peak_gb"])
                        break
                if self.footprint_gb is not None or not any(pool._busy[w] for w in used):
                    break
                if limit is not None and time.time() - t0 > limit:
                    break
                pool._drain(True, 0.02)
            self.per_gpu = self.packing_from_footprint(self.footprint_gb) if self.footprint_gb else 1
            want = min(cap, self._slots() * self.per_gpu)
            if any(pool._busy[w] for w in used):
                for i in range(len(used), want):
                    if not start(i):
                        break
        self.workers = len(used)
        codes = pool.wait(used, None if timeout is None else max(0.0, timeout - (time.time() - t0)))
        return used, codes

    def run(self, timeout=None):
        import tempfile

        if self.pool is not None:
            t0 = time.time()
            state = self._state = self.state_dir or tempfile.mkdtemp(prefix="cloud_amd_sched_")
            os.makedirs(state, exist_ok=True)
            used, codes = self._run_pool(timeout, t0, state)
            out = {"workers": len(used), "exit_codes": codes, "wall_s": time.time() - t0,
                   "trials_per_gpu": self.per_gpu, "footprint_gb": self.footprint_gb, "pool": True}
            if self.timeline:
                out["timeline"] = self.read_timeline(t0)
            if self.state_dir is None:
                import shutil

                shutil.rmtree(state, ignore_errors=True)
            return out
        ctx = mp.get_context("spawn")
        t0 = time.time()
        procs = []
        state = self._state = self.state_dir or tempfile.mkdtemp(prefix="cloud_amd_sched_")
        os.makedirs(state, exist_ok=True)
        if self.workers is not None:
            procs = [self._spawn(ctx, i) for i in range(self.workers)]
        else:
            files = [os.path.join(state, f"footprint_tuner{i}.json") for i in range(self._slots())]
            procs = [self._spawn(ctx, i, files[i]) for i in range(self._slots())]
            # warm standbys for the packing wave: started now, gated until the footprint is
            # known, so their interpreter start and imports overlap the probe trial
            # (CLOUD_AMD_TUNER_STANDBY=0: spawn the packing wave only after the probe)
            from .. import config

            n_standby = self.standby_count() if config.get("CLOUD_AMD_TUNER_STANDBY") else 0
            gates = [os.path.join(state, f"gate_tuner{i}.json") for i in range(self._slots(), self._slots() + n_standby)]
            standby = [self._spawn(ctx, self._slots() + k, gate_file=g) for k, g in enumerate(gates)]
            limit = self.probe_timeout_s if self.probe_timeout_s is not None else timeout
            extra = 0
            try:
                while self.footprint_gb is None:
                    for f in files:
                        if os.path.exists(f):
                            with open(f) as fh:
                                self.footprint_gb = float(json.load(fh)["peak_gb"])
                            break
                    if self.footprint_gb is not None or all(not p.is_alive() for p in procs):
                        break
                    if limit is not None and time.time() - t0 > limit:
                        break
                    time.sleep(0.05)
                self.per_gpu = self.packing_from_footprint(self.footprint_gb) if self.footprint_gb else 1
                want = min(self.max_workers, self._slots() * self.per_gpu)
                if not any(p.is_alive() for p in procs):  # nothing left to pack into if the probe wave is done
                    want = len(procs)
                extra = max(0, want - len(procs))
            finally:
                # every gate gets a verdict, also when the probe loop raised (Ctrl-C): a
                # standby left waiting would keep multiprocessing's atexit join hanging
                for k, g in enumerate(gates):
                    self._open_gate(g, k < extra)
            procs += standby[:extra]
            for sp in standby[extra:]:
                sp.join(30)
                if sp.is_alive():
                    sp.terminate()
                    sp.join(5)
            procs += [self._spawn(ctx, i) for i in range(len(procs), want)]
            self.workers = len(procs)
        for p in procs:
            p.join(None if timeout is None else max(0.0, timeout - (time.time() - t0)))
        codes = []
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(5)
            codes.append(p.exitcode)
        out = {"workers": len(procs), "exit_codes": codes, "wall_s": time.time() - t0,
               "trials_per_gpu": self.per_gpu, "footprint_gb": self.footprint_gb}
        if self.timeline:
            out["timeline"] = self.read_timeline(t0)
        if self.state_dir is None:  # our own scratch directory (footprints, gates, timelines)
            import shutil

            shutil.rmtree(state, ignore_errors=True)
        return out

    def read_timeline(self, t0):
        """Per-worker phase marks (seconds after the scheduler started): ``entered`` (the
        spawned interpreter runs), ``imported`` / ``device_ready`` / ``released`` / ``dismissed`` (standbys),
        ``running`` (the target called), ``exited``."""
        rows = {}
        for name in sorted(os.listdir(self._state)):
            if name.startswith("timeline_") and name.endswith(".json"):
                with open(os.path.join(self._state, name)) as fh:
                    marks = json.load(fh)
                rows[name[len("timeline_"):-len(".json")]] = {k: round(v - t0, 3) for k, v in marks.items()}
        return rows


def study_report(study_dir, study_id):
    with open(os.path.join(study_dir, study_id, "study.json")) as f:
        data = json.load(f)
    return data["trials"]
