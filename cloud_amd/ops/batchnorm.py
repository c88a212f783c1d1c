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

from . import _ext


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
    @staticmethod
    def forward(ctx, x, res, gamma, beta, running_mean, running_var, eps, momentum, relu, partials):
        ext = _ext.load(required=True)
        assert x.dtype == torch.bfloat16 and x.is_contiguous(), "bn_act expects contiguous NHWC bf16"
        C = x.shape[-1]
        M = x.numel() // C
        dev = x.device
        y = torch.empty_like(x)
        stats = torch.empty(4 * C, dtype=torch.float32, device=dev)  # mean, rstd, scale, shift
        if res is not None:
            assert res.shape == x.shape and res.dtype == x.dtype
            res = res.contiguous()
        if partials is not None:
            assert partials.shape[1:] == (2, C), partials.shape
            ext.bn_fwd_partials(x.data_ptr(), _ext.ptr(res), y.data_ptr(), M, C, partials.data_ptr(),
                                partials.shape[0], _ext.ptr(gamma), _ext.ptr(beta), float(eps), float(momentum),
                                _ext.ptr(running_mean), _ext.ptr(running_var), stats.data_ptr(),
                                stats.data_ptr() + 4 * C, stats.data_ptr() + 8 * C, int(relu),
                                _ext.stream_handle(dev))
        else:
            ws = torch.empty(ext.bn_workspace_floats(M, C), dtype=torch.float32, device=dev)
            ext.bn_fwd(x.data_ptr(), _ext.ptr(res), y.data_ptr(), M, C, _ext.ptr(gamma), _ext.ptr(beta),
                       float(eps), float(momentum), _ext.ptr(running_mean), _ext.ptr(running_var),
                       stats.data_ptr(), stats.data_ptr() + 4 * C, stats.data_ptr() + 8 * C, ws.data_ptr(),
                       int(relu), _ext.stream_handle(dev))
        ctx.save_for_backward(x, y, gamma, stats)
        ctx.relu = relu
        ctx.has_res = res is not None
        ctx.has_beta = beta is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load(required=True)
        x, y, gamma, stats = ctx.saved_tensors
        dy = dy.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        dev = x.device
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if (ctx.has_res and ctx.needs_input_grad[1]) else None
        dgamma = torch.empty(C, dtype=torch.float32, device=dev) if gamma is not None else None
        dbeta = torch.empty(C, dtype=torch.float32, device=dev) if ctx.has_beta else None
        coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
        ws = torch.empty(ext.bn_workspace_floats(M, C), dtype=torch.float32, device=dev)
        ext.bn_bwd(dy.data_ptr(), y.data_ptr(), x.data_ptr(), M, C, _ext.ptr(gamma), stats.data_ptr(),
                   stats.data_ptr() + 4 * C, dx.data_ptr(), _ext.ptr(dres), _ext.ptr(dgamma), _ext.ptr(dbeta),
                   coef.data_ptr(), ws.data_ptr(), int(ctx.relu), _ext.stream_handle(dev))
        if dres is None and ctx.has_res and ctx.needs_input_grad[1]:
            raise RuntimeError("residual grad requested but not produced")
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
