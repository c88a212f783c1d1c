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
    def __init__(self, device=None, depth=None):
        import torch

        self._torch = torch
        self.depth = config.get("CLOUD_AMD_MAX_STEPS_IN_FLIGHT") if depth is None else int(depth)
        self.enabled = bool(self.depth) and torch.cuda.is_available() and (
            device is None or getattr(device, "type", str(device)).startswith("cuda"))
        self._events = collections.deque()
        self.waits = 0
        self.wait_ms = 0.0

    def step_done(self):
        """Call after enqueueing a step: records its end and blocks until at most
        ``depth`` steps are in flight."""
        if not self.enabled:
            return
        ev = self._torch.cuda.Event()
        ev.record()
        self._events.append(ev)
        while len(self._events) > self.depth:
            old = self._events.popleft()
            if not old.query():
                import time

                self.waits += 1
                t0 = time.perf_counter()
                old.synchronize()
                self.wait_ms += (time.perf_counter() - t0) * 1e3
