"""NHWC building blocks backed by :mod:`cloud_amd.ops`.

Weights of matrix-shaped layers are stored in the compute dtype (bf16 on
MI355X) in MFMA-friendly layouts (conv: ``[Cout, KH, KW, Cin]``; dense:
``[out, in]``); normalisation parameters and biases stay fp32.  The fp32 master
copy of the matrix weights lives in the optimizer's flat arena
(:mod:`cloud_amd.optim`), not here.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops


class Conv2d(nn.Module):
    def __init__(self, cin, cout, k, stride=1, padding=0, bias=False, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.padding = cin, cout, k, stride, padding
        w = torch.empty(cout, k, k, cin, dtype=torch.float32, device=device)
        # He-normal, fan_out (ResNet convention)
        nn.init.normal_(w, 0.0, math.sqrt(2.0 / (cout * k * k)))
        self.weight = nn.Parameter(w.to(dtype))
        self.bias = nn.Parameter(torch.zeros(cout, dtype=dtype, device=device)) if bias else None

    def forward(self, x, stats=False):
        return ops.conv2d_nhwc(x, self.weight, self.bias, self.stride, self.padding, stats=stats)

    def extra_repr(self):
        return f"{self.cin}, {self.cout}, k={self.k}, s={self.stride}, p={self.padding}"


class BatchNormAct(nn.Module):
    """BatchNorm over the channel (last) dim, optional fused residual add + ReLU."""

    def __init__(self, c, relu=True, eps=1e-5, momentum=0.1, zero_init=False, device=None):
        super().__init__()
        self.c, self.relu, self.eps, self.momentum = c, relu, eps, momentum
        self.weight = nn.Parameter(torch.full((c,), 0.0 if zero_init else 1.0, device=device))
        self.bias = nn.Parameter(torch.zeros(c, device=device))
        self.register_buffer("running_mean", torch.zeros(c, device=device))
        self.register_buffer("running_var", torch.ones(c, device=device))

    def forward(self, x, residual=None, partials=None):
        if isinstance(x, tuple):  # (conv output, fused statistics partials)
            x, partials = x
        return ops.bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, residual=residual,
                          eps=self.eps, momentum=self.momentum, relu=self.relu, training=self.training,
                          partials=partials)


class Linear(nn.Module):
    def __init__(self, fin, fout, bias=True, dtype=torch.bfloat16, device=None):
        super().__init__()
        w = torch.empty(fout, fin, dtype=torch.float32, device=device)
        bound = 1.0 / math.sqrt(fin)
        nn.init.uniform_(w, -bound, bound)
        self.weight = nn.Parameter(w.to(dtype))
        self.bias = nn.Parameter(torch.zeros(fout, dtype=dtype, device=device)) if bias else None

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias)


class MaxPool2d(nn.Module):
    def __init__(self, k, stride=None, padding=0):
        super().__init__()
        self.k, self.stride, self.padding = k, stride or k, padding

    def forward(self, x):
        return ops.max_pool2d_nhwc(x, self.k, self.stride, self.padding)


class GlobalAvgPool(nn.Module):
    def forward(self, x):
        return ops.global_avg_pool_nhwc(x)
