"""NHWC pooling ops (K7): MaxPool2D and global average pooling.

HIP path: ``csrc/kernels/pool.hip``.  CPU / torch-mode path: PyTorch NCHW ops on
permuted views.  Parity: Keras ``MaxPooling2D`` / ``GlobalAveragePooling2D``
(reference ``core/tests/testdata/mnist_example_using_fit.py:58``,
``core/tests/examples/call_run_within_script_with_keras_fit.py:83``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import config
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


class _GmpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ext = _ext.load(required=True)
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty((N, C), dtype=x.dtype, device=x.device)
        cnt = torch.empty((N, C), dtype=torch.float32, device=x.device)
        ext.gmp_fwd(x.data_ptr(), y.data_ptr(), cnt.data_ptr(), N, H * W, C, _ext.stream_handle(x.device))
        ctx.save_for_backward(x, y, cnt)
        ctx.mark_non_differentiable(cnt)
        return y

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load(required=True)
        x, y, cnt = ctx.saved_tensors
        N, H, W, C = x.shape
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        ext.gmp_bwd(dy.data_ptr(), int(dy.dtype == torch.bfloat16), x.data_ptr(), y.data_ptr(), cnt.data_ptr(),
                    dx.data_ptr(), N, H * W, C, _ext.stream_handle(dy.device))
        return dx


def global_max_pool_nhwc(x):
    """[N, H, W, C] -> [N, C] max over H, W (Keras GlobalMaxPooling2D); ties share the
    gradient evenly, as reduce_max / amax."""
    if x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and _ext.use_native(x):
        return _GmpFn.apply(x)
    return x.amax(dim=(1, 2))


class _StemTailFn(torch.autograd.Function):
    """maxpool3x3/2/1(relu(BN(z))) for the ResNet stem in one pass each way.

    Forward: the BN statistics come from the stem convolution's epilogue partials
    (statistics-only finalize), then ``bn_relu_maxpool_s2k3`` applies BN + ReLU while
    pooling -- the 112x112x64 BN output is never written.  Backward: the max-pool
    gradient is gated by ``pooled > 0`` (the ReLU derivative at the argmax pixel) and
    reduced into the BN-backward statistics by the same kernel, so the BN backward
    runs its apply pass only."""

    @staticmethod
    def forward(ctx, z, gamma, beta, running_mean, running_var, eps, momentum, partials):
        from . import raw

        ext = _ext.load(required=True)
        N, H, W, C = z.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        stats = raw.bn_fwd_stats(z, gamma, beta, running_mean, running_var, eps, momentum, partials)
        y = torch.empty((N, OH, OW, C), dtype=torch.bfloat16, device=z.device)
        idx = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=z.device)
        ext.bn_relu_maxpool_s2k3(z.data_ptr(), stats[2 * C:].data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C,
                                 OH, OW, _ext.stream_handle(z.device))
        ctx.save_for_backward(z, stats, y, idx, gamma)
        ctx.has_beta = beta is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import raw

        ext = _ext.load(required=True)
        z, stats, y, idx, gamma = ctx.saved_tensors
        N, H, W, C = z.shape
        OH, OW = y.shape[1], y.shape[2]
        dev = z.device
        dy = dy.contiguous()
        st = _ext.stream_handle(dev)
        parts = torch.empty((ext.maxpool_bnstats_parts(N, H, W, C), 2, C), dtype=torch.float32, device=dev)
        dgamma = torch.empty(C, dtype=torch.float32, device=dev) if gamma is not None else None
        dbeta = torch.empty(C, dtype=torch.float32, device=dev) if ctx.has_beta else None
        if config.get("CLOUD_AMD_STEM_BWD_RECOMPUTE"):
            # statistics pass, then the apply pass recomputes the pooled gradient g per 2x2 block:
            # g (N x H x W x C) is never written or read back
            ext.maxpool_bwd_s2k3_bnstats(dy.data_ptr(), y.data_ptr(), idx.data_ptr(), z.data_ptr(), 0,
                                         parts.data_ptr(), N, H, W, C, OH, OW, st)
            coef = raw.bn_bwd_coef(C, N * H * W, gamma, stats, parts, dgamma=dgamma, dbeta=dbeta)
            dz = torch.empty_like(z)
            ext.maxpool_bwd_s2k3_bnapply(dy.data_ptr(), y.data_ptr(), idx.data_ptr(), z.data_ptr(), coef.data_ptr(),
                                         dz.data_ptr(), N, H, W, C, OH, OW, st)
            return dz, dgamma, dbeta, None, None, None, None, None
        g = torch.empty_like(z)
        ext.maxpool_bwd_s2k3_bnstats(dy.data_ptr(), y.data_ptr(), idx.data_ptr(), z.data_ptr(),
                                     g.data_ptr(), parts.data_ptr(), N, H, W, C, OH, OW, st)
        dz, _ = raw.bn_bwd(g, None, z, gamma, stats, False, dgamma=dgamma, dbeta=dbeta, partials=parts)
        return dz, dgamma, dbeta, None, None, None, None, None


def stem_tail_ok(z, bn, pool, partials):
    return (bn.training and bn.relu and partials is not None and z.is_cuda and z.dtype == torch.bfloat16
            and z.is_contiguous() and z.shape[-1] % 8 == 0 and 256 % (z.shape[-1] // 8) == 0
            and z.shape[0] * z.shape[1] * z.shape[2] < 2 ** 31  # the kernels' 32-bit pixel indices
            and (pool.k, pool.stride, pool.padding) == (3, 2, 1) and _ext.use_native(z))


def stem_bn_relu_maxpool(z, bn, partials):
    """The ResNet stem tail ``maxpool(bn1(z))`` of a training step, fused (see _StemTailFn)."""
    return _StemTailFn.apply(z, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, bn.momentum, partials)
