"""Dense layer / 1x1-convolution GEMMs on MFMA (K1).

``linear(x, w, b)`` computes ``x @ w.T (+ b)`` for ``x: [M, K]``, ``w: [N, K]``.
On MI355X (bf16 CUDA tensors, shapes the kernel tiles) the forward, the input
gradient and the weight gradient all run on the hand-written gfx950 MFMA
kernels of ``csrc/kernels/gemm.hip``:

* forward  ``Y  = X W^T``  -- layout NT (both operands K-contiguous);
* dgrad    ``dX = dY W``   -- layout NN (W read transposed by ds_read_b64_tr_b16);
* wgrad    ``dW = dY^T X`` -- layout TN with split-K over the huge M = N*H*W
  reduction (fp32 slabs + deterministic reduce), accumulated straight into
  the parameter's gradient slice of the flat arena (no autograd add kernel).

Shapes the kernels do not tile (K % 64, N % 8) fall back to hipBLASLt through
``torch.mm`` -- still a library GEMM on MFMA, never a CPU path.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _ext

NT, NN, TN = 0, 1, 2
BK = 64


def _native_ok(M, N, K):
    return K % 8 == 0 and N % 8 == 0 and M % 8 == 0 and M > 0 and M * max(K, N) < 2 ** 31


def _gemm_mode():
    return os.environ.get("CLOUD_AMD_GEMM", "native")


def mm_nt(x, w, stats=None):
    """x [M,K] @ w[N,K]^T -> [M,N] bf16 (native)."""
    ext = _ext.load(required=True)
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    ext.gemm_bf16(NT, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), y.data_ptr(), N, M, N, K,
                  _ext.ptr(stats), 0.0, _ext.stream_handle(x.device))
    return y


def mm_nn(a, b, out=None, beta=0.0):
    """a [M,K] @ b[K,N] (+ beta*out) -> [M,N] bf16 (native; b read transposed in LDS)."""
    ext = _ext.load(required=True)
    M, K = a.shape
    N = b.shape[1]
    if K % 8 or N % 8 or b.stride(1) != 1 or a.stride(1) != 1:
        r = torch.mm(a, b)
        if out is not None:
            return out.copy_(r + beta * out) if beta else out.copy_(r)
        return r
    y = out if out is not None else torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    ext.gemm_bf16(NN, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), y.data_ptr(), N, M, N, K, 0,
                  float(beta), _ext.stream_handle(a.device))
    return y


def choose_splits(M, N, K, target_blocks=1024, min_k=512):
    tiles = ((M + 127) // 128) * ((N + (63 if N <= 64 else 127)) // (64 if N <= 64 else 128))
    s = max(1, min(K // min_k, (target_blocks + tiles - 1) // tiles))
    return s


def mm_tn_into(a, b, out, beta=0.0, splits=None):
    """out[M,N] = a^T @ b + beta*out for a [K,M], b [K,N] (both row-major): weight gradient."""
    ext = _ext.load(required=True)
    K, M = a.shape
    N = b.shape[1]
    if M % 8 or N % 8 or (M * N) % 4 or a.stride(1) != 1 or b.stride(1) != 1:
        r = torch.mm(a.t().float(), b.float())
        if beta:
            r = r + beta * out.float()
        out.copy_(r)
        return out
    splits = splits or choose_splits(M, N, K)
    splits = ext.gemm_splitk_effective(K, splits)
    ws = torch.empty(splits * M * N, dtype=torch.float32, device=a.device)
    ext.gemm_splitk(TN, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(),
                    int(out.dtype == torch.bfloat16), float(beta), M, N, K, splits, ws.data_ptr(),
                    _ext.stream_handle(a.device))
    return out


def _grad_sink(w):
    """The arena gradient slice of parameter ``w`` when it can be written in place."""
    g = getattr(w, "grad", None)
    if g is not None and getattr(w, "_ca_arena", False) and g.dtype == torch.bfloat16 and g.is_contiguous():
        return g
    return None


class _LinearFn(torch.autograd.Function):
    """y = x @ w2d^T where w2d is a 2-D view of ``param`` (passed for its .grad)."""

    @staticmethod
    def forward(ctx, x, w2d, param, stats):
        ctx.save_for_backward(x, w2d)
        ctx.param = param
        return mm_nt(x, w2d, stats=stats)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = mm_nn(dy, w) if ctx.needs_input_grad[0] else None
        dw = dparam = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            param = ctx.param
            sink = _grad_sink(param) if param is not None else None
            if sink is not None:
                mm_tn_into(dy, x, sink.view(w.shape[0], -1), beta=1.0)
                from ..parallel import ddp

                ddp.notify_grad_ready(param)
            else:
                g = torch.empty_like(w)
                mm_tn_into(dy, x, g, beta=0.0)
                if param is not None and ctx.needs_input_grad[2]:
                    dparam = g.view_as(param)
                else:
                    dw = g
        return dx, dw, dparam, None


def linear(x, w, bias=None, param=None, stats=None):
    """x @ w^T + bias; ``param`` = the leaf Parameter that ``w`` is a (reshaped) view of."""
    M, K = x.shape
    N = w.shape[0]
    if (_gemm_mode() == "native" and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and _native_ok(M, N, K) and w.is_contiguous() and _ext.use_native(x, w)):
        if param is None and w.is_leaf and w.requires_grad:
            param = w
        if param is not None:
            y = _LinearFn.apply(x.contiguous(), w.detach(), param, stats)
        else:
            y = _LinearFn.apply(x.contiguous(), w, None, stats)
        if bias is not None:
            y = y + bias
        return y
    y = F.linear(x, w, bias)
    if stats is not None:
        fill_stats_torch(y, stats)
    return y


def fill_stats_torch(y2d, stats):
    """Reference/fallback for the fused BN-statistics epilogue ([tiles][2][C], 128-row tiles;
    a buffer with fewer rows -- the persistent core's one per workgroup -- gets the column
    sums in row 0 and zeros elsewhere: consumers only ever sum the rows)."""
    M, C = y2d.shape
    tiles = stats.shape[0]
    yf = y2d.float()
    if tiles * 128 < M:
        stats.zero_()
        stats[0, 0].copy_(yf.sum(0))
        stats[0, 1].copy_((yf * yf).sum(0))
        return
    pad = tiles * 128 - M
    if pad:
        yf = torch.cat([yf, yf.new_zeros(pad, C)])
    yt = yf.view(tiles, 128, C)
    stats[:, 0].copy_(yt.sum(1))
    stats[:, 1].copy_((yt * yt).sum(1))
