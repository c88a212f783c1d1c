"""Fork/join of independent backward work onto a second HIP stream.

Weight-gradient GEMMs are compute bound, while the rest of a layer's backward
(BatchNorm / LayerNorm backward, dgrad epilogues, attention backward) is mostly
memory bound.  They are independent, so a layer's backward queues its weight
gradients on a per-device side stream and the two streams share the CUs:

    side = SideWork(device)
    side.run(lambda: raw.wgrad_into(dy, x, w.grad), dy, x)   # fork
    ...                                                       # main-stream work
    side.join(); notify DDP for the deferred params           # join

``run`` makes the side stream wait for everything queued so far on the main
stream (the inputs and the zeroed gradient arena), launches ``fn`` under the
side stream (its workspaces come from the side stream's allocator pool) and
marks the input tensors as used by the side stream, so the caching allocator
does not hand their memory to a main-stream tensor before the kernels that
read them have run.  ``join`` orders all later main-stream work (including
DDP's bucket events) after the side work.  Disabled (``CLOUD_AMD_WGRAD_STREAM=0``)
or on CPU, ``run`` simply calls ``fn``.
"""
from __future__ import annotations

import torch

from .. import config
from ..ops import _ext

_STREAMS = {}
_set_stream = getattr(torch._C, "_cuda_setStream", None)
_get_stream = getattr(torch._C, "_cuda_getCurrentStream", None)


class _on_stream:
    """``with torch.cuda.stream(s)`` on the raw getter / setter (the torch context builds Stream
    objects and queries the current stream twice per use -- runtime/host.py); restores the
    stream that was current on entry."""

    __slots__ = ("s", "prev")

    def __init__(self, s):
        self.s = s

    def __enter__(self):
        if _set_stream is None or _get_stream is None:  # pragma: no cover - older torch
            self.prev = torch.cuda.current_stream(self.s.device)
            torch.cuda.set_stream(self.s)
            return
        self.prev = _get_stream(self.s.device_index)
        _set_stream(stream_id=self.s.stream_id, device_index=self.s.device_index, device_type=self.s.device_type)

    def __exit__(self, *exc):
        p = self.prev
        if isinstance(p, torch.cuda.Stream):  # pragma: no cover
            torch.cuda.set_stream(p)
        else:
            _set_stream(stream_id=p[0], device_index=p[1], device_type=p[2])
        return False


def side_stream(device):
    """The per-device side stream (created once; normal priority)."""
    key = device.index if device.index is not None else torch.cuda.current_device()
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(torch.device("cuda", key))
    return st


class SideWork:
    def __init__(self, device, enabled=None):
        if enabled is None:
            enabled = config.get("CLOUD_AMD_WGRAD_STREAM")
        self.enabled = bool(enabled) and device.type == "cuda"
        self.main = torch.cuda.current_stream(device) if self.enabled else None
        self.side = side_stream(device) if self.enabled else None
        if self.enabled:
            self._ext = _ext.load(required=True)
            self._mh, self._sh = self.main.cuda_stream, self.side.cuda_stream
        self.used = False

    def run(self, fn, *tensors):
        if not self.enabled:
            return fn()
        self._ext.stream_wait(self._sh, self._mh)  # side waits for the main stream's work so far
        with _on_stream(self.side):
            r = fn()
        for t in tensors:
            if t is not None:
                t.record_stream(self.side)
        self.used = True
        return r

    def join(self):
        if self.used:
            self._ext.stream_wait(self._mh, self._sh)
            self.used = False

    def detach(self):
        """Instead of ``join``: an event marking the side work queued so far (None when
        nothing ran on the side stream) -- the caller makes the main stream wait for it
        later (``settle``), so the side stream's tail overlaps the next layer's work."""
        if not self.used:
            return None
        ev = torch.cuda.Event()
        ev.record(self.side)
        self.used = False
        return ev


# Side-stream gradients whose join (and DDP notification) is deferred across layers:
# [(event, params)], oldest first.  A backward-pass callback settles all of them, so the
# optimizer / DDP never read a gradient before the side stream has written it.
# A backward that raises (OOM inside a tuner trial, which then moves on in the same
# process) never runs its queued callback: ``begin_pass`` -- called by every forward that
# builds a graph using ``defer`` -- drops that stale state, so the next backward queues
# its own settle callback and no gradient of the failed graph is ever announced to DDP.
_PENDING = []
_CALLBACK = [False]


def begin_pass():
    """Start of a new forward/backward: discard deferred work of a backward that never
    finished.  The main stream still waits for the stale side-stream events (their
    kernels may be queued and write memory the allocator would otherwise recycle); their
    params are NOT notified (the failed step's gradients are never reduced)."""
    if _PENDING:
        for ev, _params, _notify in _PENDING:
            torch.cuda.current_stream().wait_event(ev)
        del _PENDING[:]
    _CALLBACK[0] = False


def defer(event, params, notify):
    """Queue params whose gradients the side stream finishes at ``event``; ``notify(p)``
    runs for each once the main stream has been ordered after it.  The params are marked
    ``_ca_explicit_notify``: the DP engine then ignores autograd's post-accumulate hook for
    them (it fires when the layer's backward returns, before the side stream is done)."""
    for p in params:
        p._ca_explicit_notify = True
    if event is None:
        for p in params:
            notify(p)
        return
    _PENDING.append((event, list(params), notify))
    if not _CALLBACK[0]:
        _CALLBACK[0] = True
        torch.autograd.Variable._execution_engine.queue_callback(settle_all)


def settle(keep_last=0):
    """Order the main stream after all but the newest ``keep_last`` deferred side-stream
    gradient sets and notify their params."""
    while len(_PENDING) > keep_last:
        ev, params, notify = _PENDING.pop(0)
        torch.cuda.current_stream().wait_event(ev)
        for p in params:
            notify(p)


def settle_all():
    _CALLBACK[0] = False
    settle(0)
