"""Host-side launch path of a training step (one process per GPU).

A BERT-base step issues ~280 kernel launches from Python; at ~23 us of host work per launch
the host needed 6.5-7.2 ms per 8.8-ms step (docs/performance.md, "BERT host launch path").
Measured with ``scripts/host_profile.py`` (profiles/r6_s12, r6_s14), three costs dominated
besides the launches themselves:

* autograd's per-device worker thread: ``loss.backward()`` blocks the calling thread anyway,
  but the CUDA backward runs on a device thread and every Function's Python crosses threads
  (GIL hand-offs) -- 7.2 vs 5.9 ms per step with backward on the calling thread.  With one
  process per GPU nothing runs in parallel on that thread, so :func:`configure` turns the
  engine's multithreading off (``CLOUD_AMD_AUTOGRAD_MT=1`` keeps torch's default);
* Stream objects built per launch (``torch.cuda.current_stream(d).cuda_stream``, ~4.3 us):
  ``ops._ext.stream_handle`` asks for the raw handle instead;
* ``torch.cuda.stream(...)`` contexts and ``Stream.wait_stream`` (a Python Event per call) in
  the side-stream fork of every weight-gradient GEMM: :class:`runtime.side_stream.SideWork`
  switches streams with the raw setter and orders them with a pooled native event.

The kernels, their order and their streams are unchanged, so results are bitwise those of
the previous path.
"""
from __future__ import annotations

import torch

from .. import config

_DONE = [False]


def configure():
    """Idempotent: called by every strategy and fused optimizer the framework builds."""
    if _DONE[0]:
        return
    _DONE[0] = True
    if not config.get("CLOUD_AMD_AUTOGRAD_MT"):
        torch.autograd.set_multithreading_enabled(False)
