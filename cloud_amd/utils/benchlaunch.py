"""Launch contract shared by the benchmarks (``bench.py``, ``bench/bert_base_synth.py``).

* Outside a launched job, a bench stages itself and spawns ``--gpus`` ranks through
  :func:`cloud_amd.run` (the reference's ``run()`` -> multi-replica job path,
  ``TFC/core/deploy.py:98-167``); the launching process never initialises HIP.
* Inside a rank, the world size seen by ``torch.distributed`` must equal ``--gpus``:
  a mismatch is a hard error, never a silently relabelled number.
"""
from __future__ import annotations

import os
import sys


def inside_launched_rank():
    return bool(os.environ.get("CLOUD_AMD_RUNNING_REMOTELY") or os.environ.get("TORCHELASTIC_RUN_ID")
                or os.environ.get("WORLD_SIZE"))


def strip_flag(argv, flag):
    out = list(argv)
    for i, a in enumerate(out):
        if a == flag:
            return out[:i] + out[i + 2:]
        if a.startswith(flag + "="):
            return out[:i] + out[i + 1:]
    return out


def launch_via_run(script, gpus, device="auto", argv=None, tag="bench"):
    """Stage ``script`` (its directory is the app) and run it on ``gpus`` ranks via
    ``cloud_amd.run(distribution_strategy="auto")`` -- the generated wrapper installs
    MirroredStrategy (N > 1) or OneDeviceStrategy (N = 1) exactly as the reference's
    auto path does (``TFC/core/preprocess.py:137-146``) and the bench takes its DP engine
    from that strategy.  Streams every rank's log; with several ranks the streamed lines
    carry ``[chief-0]``-style prefixes, so rank 0's JSON result line is printed once more
    verbatim at the end.  Exits with the job's code."""
    import cloud_amd as tfc
    from cloud_amd.core.machine_config import AcceleratorType, MachineConfig

    argv = strip_flag(sys.argv[1:] if argv is None else argv, "--via-run")
    if device == "cpu":
        # the same GPU-shaped job (MI355X_<N>X chief: MirroredStrategy at N > 1), its ranks
        # on CPU over gloo (validate.cpu_rehearsal)
        os.environ["CLOUD_AMD_DEVICE"] = "cpu"
    chief = tfc.COMMON_MACHINE_CONFIGS.get("MI355X_%dX" % gpus) or MachineConfig(
        cpu_cores=16 * gpus, memory=256 * gpus, accelerator_type=AcceleratorType.AMD_INSTINCT_MI355X,
        accelerator_count=gpus)
    workers, wcfg = 0, "auto"
    script = os.path.abspath(script)
    os.chdir(os.path.dirname(script))
    try:
        job = tfc.run(entry_point=os.path.basename(script), distribution_strategy="auto", chief_config=chief,
                      worker_config=wcfg, worker_count=workers, entry_point_args=argv, stream_logs=True,
                      exit=False, wait=True)
    except ValueError as e:
        print("[%s] cannot launch %d rank(s) through cloud_amd.run(): %s" % (tag, gpus, e), file=sys.stderr)
        sys.exit(2)
    rc = job.returncode or 0
    if len(job.ranks) > 1:
        result = [ln for ln in job.log_tail(0, 200) if ln.startswith('{"metric"')]
        if result:
            print(result[-1], flush=True)
    if rc:
        print("[%s] job %s failed (exit codes %s); logs: %s" % (
            tag, job.job_id, job.meta.get("exit_codes"), os.path.join(job.job_dir, "logs")), file=sys.stderr)
    sys.exit(rc)


def check_world(gpus, world, tag="bench"):
    if world != gpus:
        print("[%s] error: --gpus %d but the job has WORLD_SIZE=%d ranks; refusing to report a %d-rank "
              "number as %d GPUs" % (tag, gpus, world, world, gpus), file=sys.stderr)
        sys.exit(3)


def startup_phases(t_start, t_first_done):
    """run() -> first step split into: ``launch_s`` (run() call -> the rank's wrapper runs:
    staging, launcher, interpreter start), ``rank_setup_s`` (wrapper -> the bench script
    body: strategy + torch imports), ``first_step_s`` (script body -> first step done:
    model build, HIP init, first-launch kernel loads).  None outside run()."""
    run_t0, rank_t0 = os.environ.get("CLOUD_AMD_RUN_T0"), os.environ.get("CLOUD_AMD_RANK_T0")
    if not run_t0 or not rank_t0:
        return None
    run_t0, rank_t0 = float(run_t0), float(rank_t0)
    return {"launch_s": round(rank_t0 - run_t0, 3), "rank_setup_s": round(t_start - rank_t0, 3),
            "first_step_s": round(t_first_done - t_start, 3)}


def launched_via():
    if os.environ.get("CLOUD_AMD_RUN_T0"):
        return "cloud_amd.run()"
    return "torch.distributed.run" if os.environ.get("TORCHELASTIC_RUN_ID") else "direct"


def host_state():
    """What the host looked like: 1/5/15-minute load average, this process's CPU set and
    the CPU it is on, voluntary / involuntary context switches so far."""
    st = {}
    try:
        with open("/proc/loadavg") as f:
            st["loadavg"] = [float(x) for x in f.read().split()[:3]]
    except OSError:
        st["loadavg"] = None
    try:
        cpus = sorted(os.sched_getaffinity(0))
        from ..core.topology import format_cpulist

        st["affinity"] = format_cpulist(cpus)
        st["n_affinity"] = len(cpus)
    except AttributeError:  # pragma: no cover
        st["affinity"], st["n_affinity"] = None, None
    try:
        with open("/proc/self/stat") as f:
            st["cpu"] = int(f.read().rsplit(")", 1)[1].split()[36])
    except (OSError, IndexError, ValueError):
        st["cpu"] = None
    try:
        import resource

        ru = resource.getrusage(resource.RUSAGE_SELF)
        st["ctx_voluntary"], st["ctx_involuntary"] = ru.ru_nvcsw, ru.ru_nivcsw
    except Exception:  # noqa: BLE001 - informational
        pass
    return st


class StepProbe:
    """Host-side evidence per timed step, no device synchronisation: Python garbage-collector
    pauses (``gc.callbacks``: time and generation of every collection), page faults of this
    process (``getrusage`` minor / major: a major fault is a page read back from disk or
    swap), and the PyTorch caching allocator's device allocations and frees (a new segment is
    a hipMalloc the driver must back and clear).  ``mark()`` at every step boundary."""

    def __init__(self, cuda=True):
        import gc

        self._gc = gc
        self._cuda = cuda
        self._t = None
        self._gen = -1
        self._pause = 0.0
        self.rows = []
        self._last = self._sample()
        gc.callbacks.append(self._cb)

    def _cb(self, phase, info):
        import time

        if phase == "start":
            self._t = time.perf_counter()
        elif self._t is not None:
            self._pause += (time.perf_counter() - self._t) * 1e3
            self._gen = max(self._gen, int(info.get("generation", -1)))
            self._t = None

    def _sample(self):
        import resource

        ru = resource.getrusage(resource.RUSAGE_SELF)
        allocs = frees = retries = None
        if self._cuda:
            try:
                import torch

                ms = torch.cuda.memory_stats()
                allocs, frees, retries = ms.get("num_device_alloc"), ms.get("num_device_free"), \
                    ms.get("num_alloc_retries")
            except Exception:  # noqa: BLE001 - informational
                pass
        return (ru.ru_minflt, ru.ru_majflt, allocs, frees, retries)

    def mark(self):
        cur = self._sample()
        d = [None if (a is None or b is None) else b - a for a, b in zip(self._last, cur)]
        self.rows.append({"gc_ms": round(self._pause, 3), "gc_gen": self._gen, "minflt": d[0], "majflt": d[1],
                          "dev_alloc": d[2], "dev_free": d[3], "alloc_retry": d[4]})
        self._last, self._pause, self._gen = cur, 0.0, -1

    def close(self):
        try:
            self._gc.callbacks.remove(self._cb)
        except ValueError:
            pass
        return self.rows


def _mmm(v):
    s = sorted(v)
    n = len(s)
    med = s[n // 2] if n % 2 else 0.5 * (s[n // 2 - 1] + s[n // 2])
    return {"min": round(s[0], 3), "median": round(med, 3), "max": round(s[-1], 3)}


def step_stats(device_ms, host_ms, host_before, host_after, outlier_ratio=1.5, probe=None, paced_ms=None):
    """Per-step timing of the timed region (device time between step-boundary events on
    the compute stream, host time to enqueue a step) plus the host state around it.  A
    step slower than ``outlier_ratio`` x the median adds a warning, with the evidence
    needed to name the cause: the host launch time (a starved / descheduled host makes
    host time ~ device time), involuntary context switches (another process on our
    cores), the CPU the rank ran on before and after (migration), the load average.
    ``paced_ms`` (per step: time blocked in the optimizer's run-ahead bound) splits the host
    time into the UNPACED launch time (``host_unpaced_ms``) and the pacing wait."""
    out = {"host_launch_ms": _mmm(host_ms) if host_ms else None,
           "device_ms": _mmm(device_ms) if device_ms else None,
           "host_before": host_before, "host_after": host_after, "warnings": []}
    if host_ms:
        out["host_launch_ms_steps"] = [round(v, 2) for v in host_ms]
    if host_ms and paced_ms and len(paced_ms) == len(host_ms):
        out["host_unpaced_ms"] = _mmm([max(h - p, 0.0) for h, p in zip(host_ms, paced_ms)])
        out["pacer_wait_ms_total"] = round(sum(paced_ms), 3)
    if probe:
        out["probe_steps"] = probe
        out["gc_ms_total"] = round(sum(r["gc_ms"] for r in probe), 3)
    ref = device_ms or host_ms
    if ref:
        m = out["device_ms" if device_ms else "host_launch_ms"]
        if m["median"] > 0 and m["max"] / m["median"] > outlier_ratio:
            slow = [i for i, v in enumerate(ref) if v > outlier_ratio * m["median"]]
            inv = None
            if "ctx_involuntary" in host_before and "ctx_involuntary" in host_after:
                inv = host_after["ctx_involuntary"] - host_before["ctx_involuntary"]
            out["warnings"].append(
                "slow steps %s: max/median step time %.2f > %.1f (host launch ms of those steps %s; "
                "involuntary context switches during the timed steps %s; cpu %s -> %s; loadavg %s -> %s)"
                % (slow, m["max"] / m["median"], outlier_ratio, [round(host_ms[i], 2) for i in slow if i < len(host_ms)],
                   inv, host_before.get("cpu"), host_after.get("cpu"), host_before.get("loadavg"),
                   host_after.get("loadavg")))
            if probe:
                out["warnings"].append("slow steps' host probe: %s" % [dict(step=i, **probe[i]) for i in slow
                                                                         if i < len(probe)])
    return out
