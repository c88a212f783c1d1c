"""NHWC pooling ops (K7): MaxPool2D and global average pooling.

HIP path: ``csrc/kernels/pool.hip``.  CPU / torch-mode path: PyTorch NCHW ops on
permuted views.  Parity: Keras ``MaxPooling2D`` / ``GlobalAveragePooling2D``
(reference ``core/tests/testdata/mnist_example_using_fit.py:58``,
``core/tests/examples/call_run_within_script_with_keras_fit.py:83``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext


def _out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        ext = _ext.load(required=True)
        x = x.contiguous()
        N, H, W, C = x.shape
        OH, OW = _out(H, k, s, p), _out(W, k, s, p)
        y = torch.empty((N, OH, OW, C), dtype=x.dtype, device=x.device)
        idx = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=x.device)
        ext.maxpool_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, OH, OW, k, s, p,
                        _ext.stream_handle(x.device))
        ctx.save_for_backward(idx)
        ctx.cfg = (N, H, W, C, OH, OW, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load(required=True)
        (idx,) = ctx.saved_tensors
        N, H, W, C, OH, OW, k, s, p = ctx.cfg
        dy = dy.contiguous()
        dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
        ext.maxpool_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), N, H, W, C, OH, OW, k, s, p,
                        _ext.stream_handle(dy.device))
        return dx, None, None, None


def max_pool2d_nhwc(x, kernel_size, stride=None, padding=0):
    stride = kernel_size if stride is None else stride
    if x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and _ext.use_native(x):
        return _MaxPoolFn.apply(x, kernel_size, stride, padding)
    y = F.max_pool2d(x.permute(0, 3, 1, 2), kernel_size, stride, padding)
    return y.permute(0, 2, 3, 1).contiguous()


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ext = _ext.load(required=True)
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty((N, C), dtype=x.dtype, device=x.device)
        ext.gap_fwd(x.data_ptr(), y.data_ptr(), 1, N, H * W, C, _ext.stream_handle(x.device))
        ctx.cfg = (N, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load(required=True)
        N, H, W, C = ctx.cfg
        dy = dy.contiguous()
        dx = torch.empty((N, H, W, C), dtype=torch.bfloat16, device=dy.device)
        ext.gap_bwd(dy.data_ptr(), int(dy.dtype == torch.bfloat16), dx.data_ptr(), N, H * W, C,
                    _ext.stream_handle(dy.device))
        return dx


def global_avg_pool_nhwc(x):
    if x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and _ext.use_native(x):
        return _GapFn.apply(x)
    return x.mean(dim=(1, 2))
