"""Keras ``Dense`` / ``Conv2D`` with bias and activation fused into the MFMA epilogue
(K1 / K2 of SURVEY.md, the layers of the reference workloads:
``mnist_example_using_fit.py:54-68``, ``keras_tuner_cifar_example.py:32-63``, README MLP).

* forward: ``y = act(x W^T + b)`` -- one GEMM / implicit-GEMM launch whose bf16
  epilogue adds the fp32 bias and applies the activation (``ca_gemm_ex`` /
  ``ca_conv_fwd_ex``); no separate bias-add or activation pass;
* backward: ``g = dy * act'(y)`` (one elementwise pass, from the saved output --
  or the saved pre-activation for GELU), then the native dgrad / split-K wgrad
  GEMMs and the native column-sum kernel for the bias gradient.  Gradients of
  parameters that live in an optimizer arena are written there in place and the
  data-parallel engine is notified (bucket launch during backward);
* shapes the MFMA tiles do not take directly are padded, not sent to a library:
  out-features / in-features to a multiple of 8 (the 10-way softmax heads, odd
  input widths), conv input channels to a multiple of 8 (the Cin = 1 MNIST and
  Cin = 3 CIFAR first layers).  Padding costs one small copy of the operand that
  needs it; the batch dimension is never padded (row tails are masked in-kernel).

CPU tensors (tests, CPU jobs) take the PyTorch reference path with the same math.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext, conv as _conv, gemm as _gemm

# activation codes of the GEMM epilogue (csrc/include/ca_mfma_core.h, enum Act)
ACT = {None: 0, "linear": 0, "gelu": 1, "relu": 2, "tanh": 3, "elu": 5}


def _rup8(n):
    return (n + 7) // 8 * 8


def _arena_grad(p):
    """The in-arena gradient view of parameter ``p`` (written in place), or None."""
    if p is None:
        return None
    g = getattr(p, "grad", None)
    if g is not None and getattr(p, "_ca_arena", False) and g.is_contiguous():
        return g
    return None


def _act_grad(g, y, pre, act):
    """dy * act'(.) in fp32, returned bf16 contiguous."""
    if act in (None, "linear"):
        return g.contiguous()
    gf, yf = g.float(), y.float()
    if act == "relu":
        out = torch.where(yf > 0, gf, torch.zeros_like(gf))
    elif act == "elu":
        out = torch.where(yf > 0, gf, gf * (yf + 1.0))
    elif act == "tanh":
        out = gf * (1.0 - yf * yf)
    elif act == "gelu":
        pf = pre.float()
        out = gf * (0.5 * (1.0 + torch.erf(pf * 0.7071067811865476)) + pf * 0.3989422804014327 * torch.exp(-0.5 * pf * pf))
    else:  # pragma: no cover - guarded by fusable()
        raise ValueError(act)
    return out.to(torch.bfloat16).contiguous()


def _pad2d(t, cols_out, rows_out=None):
    """Zero-pad a [rows, cols] tensor (unit column stride, any row stride; bf16 or fp32) to
    [rows_out, cols_out] in one native launch (rowops.hip pad_cols) -- F.pad is a fill plus
    a copy.  Returns ``t`` itself when there is nothing to pad."""
    rows, cols = t.shape
    rows_out = rows if rows_out is None else rows_out
    if cols == cols_out and rows == rows_out:
        return t
    if t.stride(-1) != 1:
        t = t.contiguous()
    ext = _ext.load(required=True)
    out = torch.empty((rows_out, cols_out), dtype=t.dtype, device=t.device)
    ext.pad_cols(t.data_ptr(), t.stride(0), cols, out.data_ptr(), cols_out, rows, rows_out, t.element_size(),
                 _ext.stream_handle(t.device))
    return out


def _pad2d_many(specs):
    """Several :func:`_pad2d` jobs [(t, cols_out, rows_out or None), ...] in ONE launch
    (rowops.hip pad_cols_multi); entries that need no padding are returned as-is."""
    outs, jobs = [], []
    for t, cols_out, rows_out in specs:
        rows, cols = t.shape
        rows_out = rows if rows_out is None else rows_out
        if cols == cols_out and rows == rows_out:
            outs.append(t)
            continue
        if t.stride(-1) != 1:
            t = t.contiguous()
        o = torch.empty((rows_out, cols_out), dtype=t.dtype, device=t.device)
        jobs += [t.data_ptr(), t.stride(0), cols, o.data_ptr(), cols_out, rows, rows_out, t.element_size()]
        outs.append(o)
    if jobs:
        dev = next(t for t, _, _ in specs).device
        _ext.load(required=True).pad_cols_multi(jobs, _ext.stream_handle(dev))
    return outs


def _act_grad_dev(dy, src, N, Np, act):
    """Native form of :func:`_act_grad` (rowops.hip act_grad): ``dy`` [M, N] (any row
    stride) zero-padded to Np columns and multiplied by act'(src) in one pass; ``src`` is
    the saved output (relu / elu / tanh) or pre-activation (gelu), [M, Np] contiguous."""
    ext = _ext.load(required=True)
    if dy.stride(-1) != 1:
        dy = dy.contiguous()
    M = dy.shape[0]
    out = torch.empty((M, Np), dtype=torch.bfloat16, device=dy.device)
    code = ACT[act] if act in ACT else 0
    if src is None:
        src, code = out, 0  # padding only: src is never read with act code 0 ... but must be a valid pointer
    ext.act_grad(dy.data_ptr(), dy.stride(0), N, src.data_ptr(), out.data_ptr(), M, Np, code,
                 _ext.stream_handle(dy.device))
    return out


def _bias_grad(ext, g, M, Np, N, bparam, st):
    """Column sums of g [M, Np] as the bias gradient: accumulated straight into the arena
    slot (and the DP engine notified) when there is one of the right width; otherwise
    returned as (autograd grad, db) like :func:`_deliver`."""
    ws = torch.empty(ext.colsum_workspace_floats(M, Np), dtype=torch.float32, device=g.device)
    sink = _arena_grad(bparam)
    if sink is not None and sink.dtype == torch.float32 and N == Np:
        ext.colsum(g.data_ptr(), M, Np, Np, sink.data_ptr(), 1, ws.data_ptr(), st)
        from ..parallel import ddp

        ddp.notify_grad_ready(bparam)
        return None, None
    acc = torch.empty(Np, dtype=torch.float32, device=g.device)
    ext.colsum(g.data_ptr(), M, Np, Np, acc.data_ptr(), 0, ws.data_ptr(), st)
    sl = acc[:N]
    if bparam is not None:
        return _deliver(bparam, acc, sl), None
    return None, sl


def fusable(act):
    return act in ACT


def _deliver(param, full_grad, sliced):
    """Add ``sliced`` (the parameter-shaped gradient) into the arena slot of ``param``
    and notify the DP engine; returns the autograd gradient when there is no arena."""
    sink = _arena_grad(param)
    if sink is not None:
        if (sliced.is_cuda and full_grad.dtype == torch.float32 and full_grad.is_contiguous()
                and sink.dtype in (torch.bfloat16, torch.float32) and sliced.data_ptr() == full_grad.data_ptr()):
            # the parameter-shaped block is the top-left corner of the padded gradient:
            # rows = leading dims, cols = last dim (rowops.hip slice_acc, one launch)
            cols = sliced.shape[-1]
            rows = sliced.numel() // cols
            ld = full_grad.shape[-1]
            if sliced.dim() == 1 or sliced.stride(-2) == ld:
                _ext.load(required=True).slice_acc(full_grad.data_ptr(), ld, sink.data_ptr(),
                                                    int(sink.dtype == torch.bfloat16), rows, cols,
                                                    _ext.stream_handle(sink.device))
                from ..parallel import ddp

                ddp.notify_grad_ready(param)
                return None
        sink.view_as(sliced).add_(sliced.to(sink.dtype))
        from ..parallel import ddp

        ddp.notify_grad_ready(param)
        return None
    return sliced.to(param.dtype).view_as(param)


class _DenseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, wparam, bparam):
        ext = _ext.load(required=True)
        M, K = x.shape
        N = w.shape[0]
        Kp, Np = _rup8(K), _rup8(N)
        specs = [(x, Kp, None), (w, Kp, Np)] + ([(b.float().reshape(1, N), Np, None)] if b is not None else [])
        padded = _pad2d_many(specs)  # input, weight and bias padding in one launch
        xp, wp = padded[0], padded[1]
        bp = padded[2].reshape(Np) if b is not None else None
        xp, wp = xp.contiguous(), wp.contiguous()
        st = _ext.stream_handle(x.device)
        tiles = -(-M // 128) * -(-Np // 128)
        if tiles < 32 and Kp >= 1024:
            # skinny output, long reduction (a small batch through a wide Flatten->Dense):
            # one tile would walk all of K alone -- split K over blocks into fp32 slabs,
            # reduce, then bias + activation in one elementwise pass
            splits = ext.gemm_splitk_effective(Kp, max(1, min(Kp // 512, 256 // tiles)))
            ws = torch.empty(splits * M * Np, dtype=torch.float32, device=x.device)
            if act != "gelu":
                # slabs only, then one pass: sum + bias + activation -> bf16 (gemm.hip splitk_bias_act)
                y = torch.empty((M, Np), dtype=torch.bfloat16, device=x.device)
                ext.gemm_splitk(_gemm.NT, xp.data_ptr(), Kp, wp.data_ptr(), Kp, y.data_ptr(), -1, 0.0, M, Np, Kp,
                                splits, ws.data_ptr(), st)
                ext.splitk_bias_act(ws.data_ptr(), splits, M, Np, _ext.ptr(bp), ACT[act], y.data_ptr(), st)
                pre = None
            else:
                y32 = torch.empty((M, Np), dtype=torch.float32, device=x.device)
                ext.gemm_splitk(_gemm.NT, xp.data_ptr(), Kp, wp.data_ptr(), Kp, y32.data_ptr(), 0, 0.0, M, Np, Kp,
                                splits, ws.data_ptr(), st)
                if bp is not None:
                    y32 += bp
                pre = y32.to(torch.bfloat16)
                y = _torch_act(y32, act).to(torch.bfloat16)
        else:
            y = torch.empty((M, Np), dtype=torch.bfloat16, device=x.device)
            pre = torch.empty((M, Np), dtype=torch.bfloat16, device=x.device) if act == "gelu" else None
            ext.gemm_ex(_gemm.NT, xp.data_ptr(), Kp, wp.data_ptr(), Kp, y.data_ptr(), Np, M, Np, Kp, 0, 0.0,
                        _ext.ptr(bp), ACT[act], _ext.ptr(pre), 0, Np if pre is not None else 0, st)
        ctx.save_for_backward(xp, wp, y, pre)
        ctx.act, ctx.dims = act, (M, K, N, Kp, Np)
        ctx.wparam, ctx.bparam, ctx.has_b = wparam, bparam, b is not None
        out = y if Np == N else y[:, :N]
        return out

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load(required=True)
        xp, wp, y, pre = ctx.saved_tensors
        M, K, N, Kp, Np = ctx.dims
        if ctx.act in (None, "linear") and Np == N:
            g = dy.contiguous()
        else:
            g = _act_grad_dev(dy, pre if ctx.act == "gelu" else (y if ctx.act not in (None, "linear") else None), N,
                              Np, ctx.act)
        dx = dw = db = dwp = dbp = None
        if ctx.needs_input_grad[0]:
            dxp = _gemm.mm_nn(g, wp)
            dx = dxp if Kp == K else dxp[:, :K]
        if ctx.needs_input_grad[1] or ctx.wparam is not None:
            sink = _arena_grad(ctx.wparam)
            if sink is not None and sink.dtype == torch.bfloat16 and Np == N and Kp == K:
                _gemm.mm_tn_into(g, xp, sink.view(N, K), beta=1.0)
                from ..parallel import ddp

                ddp.notify_grad_ready(ctx.wparam)
            else:
                full = torch.empty((Np, Kp), dtype=torch.float32, device=g.device)
                _gemm.mm_tn_into(g, xp, full, beta=0.0)
                sl = full[:N, :K]
                if ctx.wparam is not None:
                    dwp = _deliver(ctx.wparam, full, sl)
                else:
                    dw = sl.to(wp.dtype)
        if ctx.has_b and (ctx.needs_input_grad[2] or ctx.bparam is not None):
            dbp, db = _bias_grad(ext, g, M, Np, N, ctx.bparam, _ext.stream_handle(g.device))
        return dx, dw, db, None, dwp, dbp


def dense(x, w, b=None, act=None):
    """``act(x @ w.T + b)`` for x [..., K], w [N, K] (bf16), b [N] (fp32 or bf16).

    The native fused path runs for bf16 CUDA operands and a fusable activation; the
    returned tensor is bf16.  Otherwise PyTorch computes the same expression."""
    lead, K = x.shape[:-1], x.shape[-1]
    x2 = x.reshape(-1, K)
    if (x2.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and fusable(act)
            and _gemm._gemm_mode() == "native" and x2.shape[0] > 0 and _ext.use_native(x2, w)):
        wparam = w if (w.is_leaf and w.requires_grad) else None
        bparam = b if (b is not None and b.is_leaf and b.requires_grad) else None
        y = _DenseFn.apply(x2.contiguous(), w.detach() if wparam is not None else w,
                           None if b is None else (b.detach() if bparam is not None else b), act, wparam, bparam)
        return y.reshape(*lead, w.shape[0])
    y = F.linear(x2, w.to(x2.dtype), None if b is None else b.to(x2.dtype))
    y = _torch_act(y, act)
    return y.reshape(*lead, w.shape[0])


def _torch_act(y, act):
    if act in (None, "linear"):
        return y
    if act == "relu":
        return torch.relu(y)
    if act == "elu":
        return F.elu(y)
    if act == "tanh":
        return torch.tanh(y)
    if act == "gelu":
        return F.gelu(y)
    raise ValueError(act)


class _ConvActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, padding, act, wparam, bparam):
        ext = _ext.load(required=True)
        N, H, W, Cin = x.shape
        Cout, KH, KW, _ = w.shape
        (sh, sw), (ph, pw) = stride, padding
        Cp = _rup8(Cin)
        if Cp == Cin:
            xp, wp = x, w
        else:  # input and weight channel padding in one launch
            xp, wp = _pad2d_many([(x.reshape(-1, Cin), Cp, None), (w.reshape(-1, Cin), Cp, None)])
            xp, wp = xp.view(N, H, W, Cp), wp.view(Cout, KH, KW, Cp)
        xp, wp = xp.contiguous(), wp.contiguous()
        OH, OW = _conv._out(H, KH, sh, ph), _conv._out(W, KW, sw, pw)
        y = torch.empty((N, OH, OW, Cout), dtype=torch.bfloat16, device=x.device)
        bp = b.float().contiguous() if b is not None else None
        st = _ext.stream_handle(x.device)
        ext.conv_fwd_ex(xp.data_ptr(), wp.data_ptr(), y.data_ptr(), N, H, W, Cp, Cout, KH, KW, sh, sw, ph, pw,
                        _ext.ptr(bp), ACT[act], st)
        ctx.save_for_backward(xp, wp, y)
        ctx.cfg = (stride, padding, act, Cin, Cp)
        ctx.wparam, ctx.bparam, ctx.has_b = wparam, bparam, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        ext = _ext.load(required=True)
        xp, wp, y = ctx.saved_tensors
        (sh, sw), (ph, pw), act, Cin, Cp = ctx.cfg
        N, H, W, _ = xp.shape
        Cout, KH, KW, _ = wp.shape
        OH, OW = y.shape[1], y.shape[2]
        st = _ext.stream_handle(dy.device)
        Mo = N * OH * OW
        if act in (None, "linear"):
            g = dy.contiguous()
        else:
            g = _act_grad_dev(dy.reshape(Mo, Cout), y.reshape(Mo, Cout), Cout, Cout, act).view_as(y)
        dx = dw = db = dwp = dbp = None
        if ctx.needs_input_grad[0]:
            dxp = torch.empty_like(xp)
            ext.conv_dgrad(g.data_ptr(), wp.data_ptr(), dxp.data_ptr(), N, H, W, Cp, Cout, KH, KW, sh, sw, ph, pw,
                           0.0, st)
            dx = dxp if Cp == Cin else dxp[..., :Cin]
        if ctx.needs_input_grad[1] or ctx.wparam is not None:
            ncols, kred = KH * KW * Cp, N * OH * OW
            splits = ext.gemm_splitk_effective(kred, _conv.choose_wgrad_splits(Cout, ncols, kred))
            ws = torch.empty(splits * Cout * ncols, dtype=torch.float32, device=dy.device)
            sink = _arena_grad(ctx.wparam)
            if sink is not None and sink.dtype == torch.bfloat16 and Cp == Cin:
                ext.conv_wgrad(g.data_ptr(), xp.data_ptr(), sink.data_ptr(), 1, 1.0, N, H, W, Cp, Cout, KH, KW,
                               sh, sw, ph, pw, splits, ws.data_ptr(), st)
                from ..parallel import ddp

                ddp.notify_grad_ready(ctx.wparam)
            else:
                full = torch.empty((Cout, KH, KW, Cp), dtype=torch.float32, device=dy.device)
                ext.conv_wgrad(g.data_ptr(), xp.data_ptr(), full.data_ptr(), 0, 0.0, N, H, W, Cp, Cout, KH, KW,
                               sh, sw, ph, pw, splits, ws.data_ptr(), st)
                sl = full[..., :Cin]
                if ctx.wparam is not None:
                    dwp = _deliver(ctx.wparam, full, sl)
                else:
                    dw = sl.to(wp.dtype)
        if ctx.has_b and (ctx.needs_input_grad[2] or ctx.bparam is not None):
            dbp, db = _bias_grad(ext, g, Mo, Cout, Cout, ctx.bparam, st)
        return dx, dw, db, None, None, None, dwp, dbp


def _pair2(v):
    return (int(v), int(v)) if isinstance(v, int) else (int(v[0]), int(v[1]))


def conv2d(x, w, b=None, stride=1, padding=0, act=None):
    """``act(conv2d_nhwc(x, w) + b)``, NHWC x [N,H,W,Cin], w [Cout,KH,KW,Cin]; ``stride`` and
    ``padding`` are ints or (h, w) pairs -- rectangular kernels, strides and paddings run on
    the same implicit-GEMM kernels (their geometry carries KH / KW, sh / sw, ph / pw apart)."""
    Cout = w.shape[0]
    stride, padding = _pair2(stride), _pair2(padding)
    if (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and fusable(act) and Cout % 8 == 0
            and _conv._conv_mode() == "native" and x.shape[0] > 0 and x.numel() < 2 ** 31
            and _ext.use_native(x, w)):
        wparam = w if (w.is_leaf and w.requires_grad) else None
        bparam = b if (b is not None and b.is_leaf and b.requires_grad) else None
        return _ConvActFn.apply(x.contiguous(), w.detach() if wparam is not None else w,
                                None if b is None else (b.detach() if bparam is not None else b), stride, padding,
                                act, wparam, bparam)
    if stride[0] == stride[1] and padding[0] == padding[1]:
        y = _conv.conv2d_nhwc(x.contiguous(), w.to(x.dtype), None, stride[0], padding[0])
    else:  # rectangular geometry off the native path: the same expression in PyTorch
        y = F.conv2d(x.permute(0, 3, 1, 2), w.to(x.dtype).permute(0, 3, 1, 2), None, stride, padding)
        y = y.permute(0, 2, 3, 1).contiguous()
    if b is not None:
        y = y + b.to(y.dtype)
    return _torch_act(y, act)
