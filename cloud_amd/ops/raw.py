"""Autograd-free launchers for the gfx950 kernels (NHWC bf16 tensors).

These are the building blocks of both the per-op autograd Functions
(:mod:`.conv`, :mod:`.gemm`, :mod:`.batchnorm`) and the hand-scheduled
block-level forward/backward of :mod:`cloud_amd.models.fused_block`, which
chains them without autograd so that gradients can be accumulated in place
(residual gradient summed inside the dgrad GEMM epilogue, weight and BN
parameter gradients written straight into the flat gradient arena).
"""
from __future__ import annotations

import torch

from . import _ext

NT, NN, TN = 0, 1, 2


def _st(dev):
    return _ext.stream_handle(dev)


def out_hw(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def is_gemm_conv(w, stride, padding):
    return w.shape[1] == 1 and w.shape[2] == 1 and stride == 1 and padding == 0


def stats_buffer(rows, channels, device):
    return torch.empty(((rows + 127) // 128, 2, channels), dtype=torch.float32, device=device)


def wgrad_splits(m, n, kred, target_blocks=1024, min_k=512):
    bn = 64 if n <= 64 else 128
    tiles = ((m + 127) // 128) * ((n + bn - 1) // bn)
    return max(1, min(max(kred // min_k, 1), (target_blocks + tiles - 1) // tiles))


# ----------------------------------------------------------------- convolution
def conv_fwd(x, w, stride, padding, stats=None):
    """y = conv(x, w) (NHWC / OHWI, bf16); stats: optional [tiles][2][Cout] partials out."""
    ext = _ext.load(required=True)
    N, H, W, Cin = x.shape
    Cout, KH, KW, _ = w.shape
    if is_gemm_conv(w, stride, padding):
        y = torch.empty((N, H, W, Cout), dtype=torch.bfloat16, device=x.device)
        ext.gemm_bf16(NT, x.data_ptr(), Cin, w.data_ptr(), Cin, y.data_ptr(), Cout, N * H * W, Cout, Cin,
                      _ext.ptr(stats), 0.0, _st(x.device))
        return y
    OH, OW = out_hw(H, KH, stride, padding), out_hw(W, KW, stride, padding)
    y = torch.empty((N, OH, OW, Cout), dtype=torch.bfloat16, device=x.device)
    ext.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), N, H, W, Cin, Cout, KH, KW, stride, stride, padding,
                 padding, _ext.ptr(stats), _st(x.device))
    return y


def conv_dgrad(dy, w, x_shape, stride, padding, out=None, beta=0.0):
    """dx (+= beta * out) for y = conv(x, w)."""
    ext = _ext.load(required=True)
    N, H, W, Cin = x_shape
    Cout, KH, KW, _ = w.shape
    dx = out if out is not None else torch.empty(x_shape, dtype=torch.bfloat16, device=dy.device)
    if is_gemm_conv(w, stride, padding):
        ext.gemm_bf16(NN, dy.data_ptr(), Cout, w.data_ptr(), Cin, dx.data_ptr(), Cin, N * H * W, Cin, Cout, 0,
                      float(beta), _st(dy.device))
        return dx
    ext.conv_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), N, H, W, Cin, Cout, KH, KW, stride, stride, padding,
                   padding, float(beta), _st(dy.device))
    return dx


def conv_wgrad(dy, x, w_shape, stride, padding, out, beta=1.0):
    """out (bf16 or fp32, shape of w) = wgrad + beta * out, split-K over N*OH*OW."""
    ext = _ext.load(required=True)
    N, H, W, Cin = x.shape
    Cout, KH, KW, _ = w_shape
    OH, OW = dy.shape[1], dy.shape[2]
    kred = N * OH * OW
    ncols = KH * KW * Cin
    splits = ext.gemm_splitk_effective(kred, wgrad_splits(Cout, ncols, kred))
    ws = torch.empty(splits * Cout * ncols, dtype=torch.float32, device=x.device)
    obf = int(out.dtype == torch.bfloat16)
    if KH == 1 and KW == 1 and stride == 1 and padding == 0:
        ext.gemm_splitk(TN, dy.data_ptr(), Cout, x.data_ptr(), Cin, out.data_ptr(), obf, float(beta), Cout, Cin,
                        kred, splits, ws.data_ptr(), _st(x.device))
    else:
        ext.conv_wgrad(dy.data_ptr(), x.data_ptr(), out.data_ptr(), obf, float(beta), N, H, W, Cin, Cout, KH, KW,
                       stride, stride, padding, padding, splits, ws.data_ptr(), _st(x.device))
    return out


# ------------------------------------------------------------------ batchnorm
def bn_fwd(x, gamma, beta, running_mean, running_var, eps, momentum, relu, residual=None, partials=None):
    """Training BN(+res)(+ReLU).  Returns (y, stats[4C] = mean, rstd, scale, shift)."""
    ext = _ext.load(required=True)
    C = x.shape[-1]
    M = x.numel() // C
    dev = x.device
    y = torch.empty_like(x)
    stats = torch.empty(4 * C, dtype=torch.float32, device=dev)
    sp = stats.data_ptr()
    if partials is not None:
        ext.bn_fwd_partials(x.data_ptr(), _ext.ptr(residual), y.data_ptr(), M, C, partials.data_ptr(),
                            partials.shape[0], _ext.ptr(gamma), _ext.ptr(beta), float(eps), float(momentum),
                            _ext.ptr(running_mean), _ext.ptr(running_var), sp, sp + 4 * C, sp + 8 * C, int(relu),
                            _st(dev))
    else:
        ws = torch.empty(ext.bn_workspace_floats(M, C), dtype=torch.float32, device=dev)
        ext.bn_fwd(x.data_ptr(), _ext.ptr(residual), y.data_ptr(), M, C, _ext.ptr(gamma), _ext.ptr(beta),
                   float(eps), float(momentum), _ext.ptr(running_mean), _ext.ptr(running_var), sp, sp + 4 * C,
                   sp + 8 * C, ws.data_ptr(), int(relu), _st(dev))
    return y, stats


def bn_bwd(dy, y, x, gamma, stats, relu, dgamma=None, dbeta=None, want_dres=False, dx_out=None, accumulate=0):
    """BN(+res)(+ReLU) backward.  dgamma/dbeta (fp32 [C]) are written, or accumulated
    into when ``accumulate`` is set.  Returns (dx, dres-or-None)."""
    ext = _ext.load(required=True)
    C = x.shape[-1]
    M = x.numel() // C
    dev = x.device
    dx = dx_out if dx_out is not None else torch.empty_like(x)
    dres = torch.empty_like(x) if want_dres else None
    coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
    ws = torch.empty(ext.bn_workspace_floats(M, C), dtype=torch.float32, device=dev)
    sp = stats.data_ptr()
    ext.bn_bwd(dy.data_ptr(), y.data_ptr(), x.data_ptr(), M, C, _ext.ptr(gamma), sp, sp + 4 * C, dx.data_ptr(),
               _ext.ptr(dres), _ext.ptr(dgamma), _ext.ptr(dbeta), coef.data_ptr(), ws.data_ptr(),
               int(relu) | (2 if accumulate else 0), _st(dev))
    return dx, dres
