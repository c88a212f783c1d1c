"""NHWC convolutions (K2) on the gfx950 implicit-GEMM MFMA kernels.

Activations are NHWC-contiguous ``[N, H, W, C]`` and weights ``[Cout, KH, KW, Cin]``
("OHWI").  On MI355X every convolution of the reference workloads runs on
``csrc/kernels/conv.hip`` (forward / dgrad / split-K wgrad; no MIOpen, hence
no per-shape kernel JIT at first use), except 1x1 stride-1 convolutions, which
are plain GEMMs on the activation memory and use ``csrc/kernels/gemm.hip``.

* the weight gradient is accumulated straight into the parameter's slice of
  the flat gradient arena (no autograd AccumulateGrad add) and the DDP engine
  is notified so the bucket can launch its all-reduce;
* the forward can also emit per-tile BatchNorm statistics partials
  (``stats=True``), consumed by :func:`cloud_amd.ops.bn_act` so the BN layer
  that follows does not re-read the convolution output for its mean/var.

CPU tensors (tests) use PyTorch's conv2d on channels-last views.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _ext, gemm


def _out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def _conv_mode():
    return os.environ.get("CLOUD_AMD_CONV", "native")


def _native_conv_ok(x, w):
    Cin = x.shape[-1]
    Cout = w.shape[0]
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and Cin % 8 == 0 and Cout % 8 == 0
            and x.is_contiguous() and x.numel() < 2 ** 31)


def choose_wgrad_splits(cout, ncols, kred, target_blocks=1024, min_k=512):
    bn = 64 if ncols <= 64 else 128
    tiles = ((cout + 127) // 128) * ((ncols + bn - 1) // bn)
    return max(1, min(max(kred // min_k, 1), (target_blocks + tiles - 1) // tiles))


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, param, stride, padding, stats):
        ext = _ext.load(required=True)
        N, H, W, Cin = x.shape
        Cout, KH, KW, _ = w.shape
        OH, OW = _out(H, KH, stride, padding), _out(W, KW, stride, padding)
        y = torch.empty((N, OH, OW, Cout), dtype=torch.bfloat16, device=x.device)
        ext.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), N, H, W, Cin, Cout, KH, KW, stride, stride,
                     padding, padding, _ext.ptr(stats), _ext.stream_handle(x.device))
        ctx.save_for_backward(x, w)
        ctx.param = param
        ctx.cfg = (stride, padding)
        return y

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load(required=True)
        x, w = ctx.saved_tensors
        stride, padding = ctx.cfg
        dy = dy.contiguous()
        N, H, W, Cin = x.shape
        Cout, KH, KW, _ = w.shape
        OH, OW = dy.shape[1], dy.shape[2]
        st = _ext.stream_handle(x.device)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            ext.conv_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), N, H, W, Cin, Cout, KH, KW, stride, stride,
                           padding, padding, 0.0, st)
        dw = dparam = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            ncols = KH * KW * Cin
            kred = N * OH * OW
            splits = choose_wgrad_splits(Cout, ncols, kred)
            splits = ext.gemm_splitk_effective(kred, splits)
            ws = torch.empty(splits * Cout * ncols, dtype=torch.float32, device=x.device)
            param = ctx.param
            sink = gemm._grad_sink(param) if param is not None else None
            if sink is not None:
                ext.conv_wgrad(dy.data_ptr(), x.data_ptr(), sink.data_ptr(), 1, 1.0, N, H, W, Cin, Cout, KH, KW,
                               stride, stride, padding, padding, splits, ws.data_ptr(), st)
                from ..parallel import ddp

                ddp.notify_grad_ready(param)
            else:
                g = torch.empty_like(w)
                ext.conv_wgrad(dy.data_ptr(), x.data_ptr(), g.data_ptr(), 1, 0.0, N, H, W, Cin, Cout, KH, KW,
                               stride, stride, padding, padding, splits, ws.data_ptr(), st)
                if param is not None:
                    dparam = g
                else:
                    dw = g
        return dx, dw, dparam, None, None, None


def stats_buffer(rows, channels, device):
    """Partials buffer for the fused BN-statistics epilogue: [ceil(rows/128)][2][C] fp32."""
    return torch.empty(((rows + 127) // 128, 2, channels), dtype=torch.float32, device=device)


def conv2d_nhwc(x, w, bias=None, stride=1, padding=0, stats=False):
    """x: [N,H,W,Cin], w: [Cout,KH,KW,Cin] -> [N,OH,OW,Cout] (NHWC contiguous).

    With ``stats=True`` returns ``(y, partials)`` where ``partials`` holds the
    per-128-row-tile channel sums / sums of squares of ``y`` (or None when the
    fused epilogue was not used).
    """
    N, H, W, Cin = x.shape
    Cout, KH, KW, Cin_w = w.shape
    assert Cin == Cin_w, f"channel mismatch {Cin} vs {Cin_w}"
    native = _conv_mode() == "native" and x.is_cuda and _native_conv_ok(x, w) and _ext.use_native(x, w)
    part = None
    if KH == 1 and KW == 1 and padding == 0 and stride == 1:
        x2 = x.reshape(N * H * W, Cin)
        if native and stats and gemm._native_ok(N * H * W, Cout, Cin):
            part = stats_buffer(N * H * W, Cout, x.device)
        y = gemm.linear(x2, w.reshape(Cout, Cin), bias, param=w, stats=part).view(N, H, W, Cout)
        return (y, part) if stats else y
    if native:
        param = w if (w.is_leaf and w.requires_grad) else None
        OH, OW = _out(H, KH, stride, padding), _out(W, KW, stride, padding)
        if stats:
            part = stats_buffer(N * OH * OW, Cout, x.device)
        y = _ConvFn.apply(x, w.detach() if param is not None else w, param, stride, padding, part)
        if bias is not None:
            y = y + bias
        return (y, part) if stats else y
    xc = x.permute(0, 3, 1, 2)          # NCHW view with channels-last strides
    wc = w.permute(0, 3, 1, 2)          # OIHW view with channels-last strides
    y = F.conv2d(xc, wc, bias, stride=stride, padding=padding)
    y = y.permute(0, 2, 3, 1)
    if not y.is_contiguous():
        y = y.contiguous()
    return (y, None) if stats else y
