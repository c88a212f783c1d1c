"""Fused BatchNorm(+residual add)(+ReLU) for NHWC activations.

HIP path: ``csrc/kernels/bn.hip`` (stats -> finalize -> apply; backward reduce ->
finalize -> apply with the ReLU mask recomputed from the saved output and the
residual gradient emitted in the same pass).  CPU / ``CLOUD_AMD_OPS=torch``
path: plain PyTorch with identical semantics, used as the fp32 numerics
reference in tests.

Parity: Keras ``BatchNormalization`` as used by ResNet-50 in the reference
workloads (``TFC/core/tests/examples/call_run_within_script_with_keras_fit.py:80``).
"""
from __future__ import annotations

import torch

from . import _ext, raw


def _torch_bn_act(x, res, gamma, beta, running_mean, running_var, eps, momentum, relu, training):
    C = x.shape[-1]
    xf = x.float().reshape(-1, C)
    if training:
        mean = xf.mean(0)
        var = xf.var(0, unbiased=False)
        if running_mean is not None:
            with torch.no_grad():
                M = xf.shape[0]
                unb = var * (M / max(M - 1, 1))
                running_mean.mul_(1 - momentum).add_(momentum * mean)
                running_var.mul_(1 - momentum).add_(momentum * unb)
    else:
        mean, var = running_mean, running_var
    y = (xf - mean) * torch.rsqrt(var + eps)
    if gamma is not None:
        y = y * gamma
    if beta is not None:
        y = y + beta
    y = y.reshape(x.shape)
    if res is not None:
        y = y + res.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


class _BNActFn(torch.autograd.Function):
    """Autograd face of the HIP BN kernels (launchers in :mod:`.raw`); the ReLU gate of
    the backward is the 1-bit-per-channel mask the forward apply wrote."""

    @staticmethod
    def forward(ctx, x, res, gamma, beta, running_mean, running_var, eps, momentum, relu, partials):
        assert x.dtype == torch.bfloat16 and x.is_contiguous(), "bn_act expects contiguous NHWC bf16"
        C = x.shape[-1]
        if res is not None:
            assert res.shape == x.shape and res.dtype == x.dtype
            res = res.contiguous()
        if partials is not None:
            assert partials.shape[1:] == (2, C), partials.shape
        y, stats, mask = raw.bn_fwd(x, gamma, beta, running_mean, running_var, eps, momentum, relu, residual=res,
                                    partials=partials, keep_mask=True)
        ctx.save_for_backward(x, mask, gamma, stats)
        ctx.relu = relu
        ctx.has_res = res is not None
        ctx.has_beta = beta is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, gamma, stats = ctx.saved_tensors
        C = x.shape[-1]
        dev = x.device
        want_dres = ctx.has_res and ctx.needs_input_grad[1]
        dgamma = torch.empty(C, dtype=torch.float32, device=dev) if gamma is not None else None
        dbeta = torch.empty(C, dtype=torch.float32, device=dev) if ctx.has_beta else None
        dx, dres = raw.bn_bwd(dy.contiguous(), None, x, gamma, stats, ctx.relu, dgamma=dgamma, dbeta=dbeta,
                              want_dres=want_dres, mask=mask)
        return dx, dres, dgamma, dbeta, None, None, None, None, None, None


def bn_act(x, gamma, beta, running_mean, running_var, *, residual=None, eps=1e-5, momentum=0.1,
           relu=True, training=True, partials=None):
    """y = act(BN(x) [+ residual]) over the last (channel) dim of an NHWC tensor.

    ``partials``: optional [tiles][2][C] channel sum / sum-of-squares partials of
    ``x`` produced by the convolution epilogue (skips the statistics pass).
    """
    if training and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and _ext.use_native(x):
        return _BNActFn.apply(x, residual, gamma, beta, running_mean, running_var, eps, momentum, relu, partials)
    if not training and x.is_cuda and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and _ext.use_native(x):
        ext = _ext.load(required=True)
        C = x.shape[-1]
        rstd = torch.rsqrt(running_var + eps)
        scale = rstd * (gamma if gamma is not None else 1.0)
        shift = (beta if beta is not None else 0.0) - running_mean * scale
        ss = torch.cat([scale, shift]).float().contiguous()
        y = torch.empty_like(x)
        res = residual.contiguous() if residual is not None else None
        ext.bn_apply(x.contiguous().data_ptr(), _ext.ptr(res), y.data_ptr(), x.numel() // C, C, ss.data_ptr(),
                     int(relu), _ext.stream_handle(x.device))
        return y
    return _torch_bn_act(x, residual, gamma, beta, running_mean, running_var, eps, momentum, relu, training)
