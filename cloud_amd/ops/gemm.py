"""Dense layer / GEMM dispatch (K1).

``linear(x, w, b)`` computes ``x @ w.T + b`` for ``x: [M, K]``, ``w: [N, K]``.
The hand-written MFMA kernels register themselves here once built; until a
kernel is selected for a shape the call goes to hipBLASLt through ``torch.mm``
(the ROCm library GEMM, which is allowed for plain GEMMs).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def linear(x, w, bias=None):
    return F.linear(x, w, bias)
