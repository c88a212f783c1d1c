"""Bounded host run-ahead for training loops.

A step's kernels are queued asynchronously, so the Python host can enqueue several steps
before the GPU finishes the first.  The tensors of every queued step stay allocated, and the
ones used on the weight-gradient side stream return to PyTorch's caching allocator only when
that stream's event completes -- so the further the host runs ahead, the more memory is in
flight and the more new segments (``hipMalloc``) the allocator requests.  Measured on MI355X
(ResNet-50 b1024, ``bench.py`` ``probe_steps``): after 5 warmup steps the timed steps 3-6 still
made 50-150 new device allocations while the host ran 5 steps ahead; on most boxes that cost
50-100 ms, on some a single step's allocations blocked the host for 3.2-4.6 s with the GPU idle
(3,800-4,800 instead of 14,500 img/s; docs/performance.md, round 4).

:class:`StepPacer` records an event at the end of every step and, before returning, waits for
the event of the step ``depth`` steps back, so at most ``depth`` steps are ever queued: memory
in flight is bounded and reaches its steady state during warmup.  With the GPU the bottleneck
(70 ms steps, ~10 ms of host launch time) the wait costs nothing.  ``CLOUD_AMD_MAX_STEPS_IN_FLIGHT``
(default 2; 0 = unbounded).

Short steps need a deeper queue: with BERT-base's 8.7-ms steps two queued steps cover only
17 ms, and one host hiccup longer than that (measured: unpaced launch time median 4.5 ms, but
spikes to 22 ms on a loaded box) drains the GPU -- 7,031 vs 7,313 seq/s on the same box
(``profiles/r6_s29``).  So the depth adapts once, early: from the GPU time between two completed
step ends the pacer sets ``depth = ceil(CLOUD_AMD_RUN_AHEAD_MS / step_ms)``, clamped to
[``CLOUD_AMD_MAX_STEPS_IN_FLIGHT``, 4] -- ResNet-50's 64-ms steps keep 2, BERT's get 3.  It is
decided during the first steps (warmup), so the allocator still reaches its steady state before
any timed step.

Since round 5 every :class:`cloud_amd.optim.FusedOptimizer` owns one and calls
:meth:`StepPacer.step_done` at the end of ``step()``: the bound is a property of the runtime,
not of the loop, so custom training loops (``tf.GradientTape`` + ``apply_gradients``),
``strategy.run`` and user scripts get it too.  ``wait_ms`` accumulates the time the host spent
blocked in the bound, so a caller can report its unpaced launch time.
"""
from __future__ import annotations

import collections

from .. import config


class StepPacer:
    MAX_ADAPTIVE_DEPTH = 4
    CALIBRATE_AT = 4  # step whose call settles the depth (steps 1-2 carry first-call costs)

    def __init__(self, device=None, depth=None, run_ahead_ms=None):
        import torch

        self._torch = torch
        self.depth = config.get("CLOUD_AMD_MAX_STEPS_IN_FLIGHT") if depth is None else int(depth)
        self.enabled = bool(self.depth) and torch.cuda.is_available() and (
            device is None or getattr(device, "type", str(device)).startswith("cuda"))
        ra = config.get("CLOUD_AMD_RUN_AHEAD_MS") if run_ahead_ms is None else float(run_ahead_ms)
        self.run_ahead_ms = float(ra or 0.0)
        self._calibrating = self.enabled and self.run_ahead_ms > 0
        self.step_ms = None  # GPU time of step CALIBRATE_AT - 1 (between two step-end events)
        self._events = collections.deque()
        self._steps = 0
        self.waits = 0
        self.wait_ms = 0.0

    def _calibrate(self):
        """Once, at step CALIBRATE_AT: wait for the previous step's end (one drain, in warmup)
        and settle the depth from that step's GPU time."""
        self._calibrating = False
        ev = self._events
        if len(ev) < 3:
            return
        import math
        import time

        t0 = time.perf_counter()
        ev[-2].synchronize()
        self.wait_ms += (time.perf_counter() - t0) * 1e3
        self.step_ms = ev[-3].elapsed_time(ev[-2])
        if self.step_ms > 0:
            want = math.ceil(self.run_ahead_ms / self.step_ms)
            self.depth = max(self.depth, min(want, self.MAX_ADAPTIVE_DEPTH))

    def step_done(self):
        """Call after enqueueing a step: records its end and blocks until at most
        ``depth`` steps are in flight."""
        if not self.enabled:
            return
        self._steps += 1
        ev = self._torch.cuda.Event(enable_timing=self._calibrating and self._steps >= self.CALIBRATE_AT - 2)
        ev.record()
        self._events.append(ev)
        if self._calibrating and self._steps >= self.CALIBRATE_AT:
            self._calibrate()
        while len(self._events) > self.depth:
            old = self._events.popleft()
            if not old.query():
                import time

                self.waits += 1
                t0 = time.perf_counter()
                old.synchronize()
                self.wait_ms += (time.perf_counter() - t0) * 1e3
