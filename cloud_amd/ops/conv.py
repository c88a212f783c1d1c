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

from .. import config
from . import _ext, gemm, raw


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


def _s2d_weight(w, cx):
    """[Cout, 7, 7, Cin] -> [Cout, 4, 4, 16]: W'[o, ay, ax, (by, bx, c)] = W[o, 2ay+by, 2ax+bx, c] (zero
    where 2a+b = 7 or c >= cx)."""
    Cout = w.shape[0]
    wp = F.pad(w[..., :cx], (0, 4 - cx, 0, 1, 0, 1))          # [Cout, 8, 8, 4]
    return wp.view(Cout, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(Cout, 4, 4, 16).contiguous()


def _s2d_weight_grad(g, cx):
    """Adjoint of :func:`_s2d_weight`: [Cout, 4, 4, 16] -> [Cout, 7, 7, cx]."""
    Cout = g.shape[0]
    return g.view(Cout, 4, 4, 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(Cout, 8, 8, 4)[:, :7, :7, :cx]


class _StemS2DFn(torch.autograd.Function):
    """7x7 / stride 2 / pad 3 stem convolution as a 4x4 / stride 1 convolution over the
    space-to-depth input (K = 256 instead of 392 for the 8-channel padded input; the
    input transform replaces the per-step channel pad).  Weight gradient only (the
    network input needs none)."""

    @staticmethod
    def forward(ctx, x, w, param, stats):
        ext = _ext.load(required=True)
        N, H, W, cx = x.shape
        Cout = w.shape[0]
        OH, OW = _out(H, 7, 2, 3), _out(W, 7, 2, 3)
        Hs, Ws = OH + 3, OW + 3
        st = _ext.stream_handle(x.device)
        xs = torch.empty((N, Hs, Ws, 16), dtype=torch.bfloat16, device=x.device)
        ext.stem_s2d(x.data_ptr(), xs.data_ptr(), N, H, W, cx, Hs, Ws, 3, st)
        ws = _s2d_weight(w, cx)
        y = torch.empty((N, OH, OW, Cout), dtype=torch.bfloat16, device=x.device)
        ext.conv_fwd(xs.data_ptr(), ws.data_ptr(), y.data_ptr(), N, Hs, Ws, 16, Cout, 4, 4, 1, 1, 0, 0,
                     _ext.ptr(stats), st)
        ctx.save_for_backward(xs)
        ctx.param, ctx.cx, ctx.wshape = param, cx, w.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import raw

        (xs,) = ctx.saved_tensors
        dy = dy.contiguous()
        Cout = dy.shape[-1]
        g = torch.zeros((Cout, 4, 4, 16), dtype=torch.float32, device=dy.device)
        # the last kernel of the backward pass (nothing left to overlap it with): a wide
        # split-K grid (b1024: 869 -> 651 us at 2048 vs 512 workgroups, bench/wgrad_sweep.py)
        raw.conv_wgrad(dy, xs, g.shape, 1, 0, out=g, beta=0.0, blocks=config.get("CLOUD_AMD_STEM_WGRAD_BLOCKS"))
        gw = _s2d_weight_grad(g, ctx.cx)
        param = ctx.param
        sink = gemm._grad_sink(param) if param is not None else None
        if sink is not None:
            sink[..., :ctx.cx] += gw.to(sink.dtype)
            from ..parallel import ddp

            ddp.notify_grad_ready(param)
            return None, None, None, None
        full = torch.zeros(ctx.wshape, dtype=torch.float32, device=dy.device)
        full[..., :ctx.cx] = gw
        if param is not None:
            return None, None, full.to(param.dtype), None
        return None, full.to(torch.bfloat16), None, None


def stem_s2d_ok(x, w, stride, padding):
    """The space-to-depth stem applies: native bf16, 7x7 / 2 / pad 3, <= 4 input channels."""
    return (_conv_mode() == "native" and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and tuple(w.shape[1:3]) == (7, 7) and stride == 2 and padding == 3 and x.shape[-1] <= 4
            and x.shape[-1] <= w.shape[-1] and x.is_contiguous() and not x.requires_grad and _ext.use_native(x, w))


def stem_conv_s2d(x, w, stats=False):
    """y = conv(x, w[..., :Cx], stride 2, pad 3) for the raw (unpadded) network input x
    [N, H, W, Cx <= 4]; w: [Cout, 7, 7, Cin_w >= Cx].  ``stats`` as :func:`conv2d_nhwc`."""
    N, H, W, _ = x.shape
    Cout = w.shape[0]
    OH, OW = _out(H, 7, 2, 3), _out(W, 7, 2, 3)
    part = None
    if stats:
        # the kernel that will run decides the partial rows (one per workgroup on the
        # LDS-resident stem kernel, one per 128 output pixels on the implicit GEMM)
        rows = _ext.load(required=True).conv_stat_rows(N, OH + 3, OW + 3, 16, Cout, 4, 4, 1, 1, 0, 0)
        part = torch.empty((rows, 2, Cout), dtype=torch.float32, device=x.device)
    param = w if (w.is_leaf and w.requires_grad) else None
    y = _StemS2DFn.apply(x, w.detach() if param is not None else w, param, part)
    return (y, part) if stats else y


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
            part = raw.gemm_stats_buffer(N * H * W, Cout, Cin, x.device)
        y = gemm.linear(x2, w.reshape(Cout, Cin), bias, param=w, stats=part).view(N, H, W, Cout)
        return (y, part) if stats else y
    if native:
        param = w if (w.is_leaf and w.requires_grad) else None
        OH, OW = _out(H, KH, stride, padding), _out(W, KW, stride, padding)
        if stats:
            part = raw.conv_stats_buffer(x.shape, w, stride, padding, x.device)
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
