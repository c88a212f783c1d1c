"""Python garbage-collector control for training loops.

A training step allocates thousands of short-lived Python objects (autograd nodes, tensor
wrappers, frames), so CPython's generational collector runs a full (generation-2) pass every
few steps, and a full pass walks every tracked object of the process -- the millions that
``import torch`` and the framework leave behind, none of which will ever be garbage.  On a
healthy host that costs tens of milliseconds once every ~10 steps, hidden behind the GPU
queue; when those pages have gone cold (a loaded, memory-pressured host) the same walk has been
seen to take seconds, leaving the GPU idle (``bench.py`` ``probe_steps``: ``gc_ms`` /
``majflt`` per step; docs/performance.md, round 4).

:func:`freeze` collects once and moves every surviving object into the permanent
generation (``gc.freeze``), so later collections only walk objects created after it: call it
after the first steps, when the model, optimizer state and compiled-kernel caches exist.
``CLOUD_AMD_GC_FREEZE=0`` turns it into a no-op.
"""
from __future__ import annotations

import gc

from .. import config


def freeze():
    """Collect, then exclude every object alive now from future collections.  Returns the
    number of objects frozen (0 when disabled)."""
    if not config.get("CLOUD_AMD_GC_FREEZE"):
        return 0
    gc.collect()
    gc.freeze()
    return gc.get_freeze_count()


def frozen_count():
    """Objects in the permanent generation now (someone -- this runtime or the caller -- froze)."""
    return gc.get_freeze_count()


def unfreeze():
    """Return the frozen objects to the collector (e.g. before tearing a model down)."""
    gc.unfreeze()
