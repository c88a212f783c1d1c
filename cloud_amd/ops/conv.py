"""NHWC convolution / dense dispatch (K1/K2).

Activations are NHWC-contiguous ``[N, H, W, C]`` tensors and conv weights are
stored ``[Cout, KH, KW, Cin]`` ("OHWI"), so

* a 1x1 / stride-1 convolution IS a GEMM ``[N*H*W, Cin] x [Cin, Cout]`` on the
  activation memory as it lies (no im2col, no layout change);
* a 1x1 / stride-s convolution is a strided row gather followed by that GEMM;
* every other convolution goes to the native NHWC convolution of the ROCm stack
  through zero-copy channels-last views.

The GEMM path is routed through :mod:`cloud_amd.ops.gemm` (hand-written MFMA
kernel where it wins, hipBLASLt otherwise) so the same layer code runs the
MI355X-native path on GPU and the PyTorch reference on CPU.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import gemm


def conv2d_nhwc(x, w, bias=None, stride=1, padding=0):
    """x: [N,H,W,Cin], w: [Cout,KH,KW,Cin] -> [N,OH,OW,Cout] (NHWC contiguous)."""
    N, H, W, Cin = x.shape
    Cout, KH, KW, Cin_w = w.shape
    assert Cin == Cin_w, f"channel mismatch {Cin} vs {Cin_w}"
    if KH == 1 and KW == 1 and padding == 0:
        if stride != 1:
            x = x[:, ::stride, ::stride, :]
        N, OH, OW, _ = x.shape
        y = gemm.linear(x.reshape(N * OH * OW, Cin), w.reshape(Cout, Cin), bias, param=w)
        return y.view(N, OH, OW, Cout)
    xc = x.permute(0, 3, 1, 2)          # NCHW view with channels-last strides
    wc = w.permute(0, 3, 1, 2)          # OIHW view with channels-last strides
    y = F.conv2d(xc, wc, bias, stride=stride, padding=padding)
    y = y.permute(0, 2, 3, 1)
    if not y.is_contiguous():
        y = y.contiguous()
    return y
