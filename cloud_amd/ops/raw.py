"""Autograd-free launchers for the gfx950 kernels (NHWC bf16 tensors).

These are the building blocks of both the per-op autograd Functions
(:mod:`.conv`, :mod:`.gemm`, :mod:`.batchnorm`) and the hand-scheduled
block-level forward/backward of :mod:`cloud_amd.models.fused_block`, which
chains them without autograd so that gradients can be accumulated in place
(residual gradient summed inside the dgrad GEMM epilogue, weight and BN
parameter gradients written straight into the flat gradient arena).
"""
from __future__ import annotations

import json
import os

import torch

from . import _ext

NT, NN, TN = 0, 1, 2

# Shape log for roofline analysis (scripts/gemm_roofline.py): with CLOUD_AMD_SHAPE_LOG=<path>,
# every GEMM / convolution launch appends one JSON line (kind, M, N, K, minimum HBM bytes) in
# launch order, to be aligned with a serialized rocprofv3 kernel trace.
_SHAPE_LOG = os.environ.get("CLOUD_AMD_SHAPE_LOG") or None


def _log(kind, M, N, K, nbytes, **kw):
    if _SHAPE_LOG is None:
        return
    with open(_SHAPE_LOG, "a") as f:
        f.write(json.dumps(dict(kind=kind, M=int(M), N=int(N), K=int(K), bytes=int(nbytes), **kw)) + "\n")


def _nb(*ts):
    if _SHAPE_LOG is None:  # the byte counts only feed the shape log (evaluated per launch)
        return 0
    return sum(t.numel() * t.element_size() for t in ts if t is not None)


def _st(dev):
    return _ext.stream_handle(dev)


def out_hw(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def is_gemm_conv(w, stride, padding):
    return w.shape[1] == 1 and w.shape[2] == 1 and stride == 1 and padding == 0


def stats_buffer(rows, channels, device):
    return torch.empty(((rows + 127) // 128, 2, channels), dtype=torch.float32, device=device)


def gemm_stats_buffer(M, N, K, device, lda=None, ldb=None, ldc=None):
    """Partials buffer for a forward (NT) GEMM with the BN-statistics epilogue: the
    persistent resident-weight core writes one row per workgroup, the tiled cores one per
    128 rows (``ext.gemm_stat_rows`` says which)."""
    ext = _ext.load(required=True)
    rows = ext.gemm_stat_rows(int(M), int(N), int(K), int(lda or K), int(ldb or K), int(ldc or N))
    return torch.empty((rows, 2, N), dtype=torch.float32, device=device)


def conv_stats_buffer(x_shape, w, stride, padding, device):
    """Partials buffer for :func:`conv_fwd` ``stats=`` of x [N, H, W, Cin] * w [Cout, KH, KW, Cin]."""
    N, H, W, Cin = x_shape
    Cout, KH, KW, _ = w.shape
    if is_gemm_conv(w, stride, padding):
        return gemm_stats_buffer(N * H * W, Cout, Cin, device)
    if device.type == "cuda":  # the kernel that will run decides (one row per workgroup on the halo kernel)
        rows = _ext.load(required=True).conv_stat_rows(N, H, W, Cin, Cout, KH, KW, stride, stride, padding, padding)
        return torch.empty((rows, 2, Cout), dtype=torch.float32, device=device)
    return stats_buffer(N * out_hw(H, KH, stride, padding) * out_hw(W, KW, stride, padding), Cout, device)


_WGRAD_BLOCKS = None
_GWS_ROWS = 512  # BN statistics group workspace rows (bn.hip group_count)
_WGRAD_BLOCKS_SMALLM = None
_DENSE_WGRAD_BLOCKS = None


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
        _log("fwd1x1", N * H * W, Cout, Cin, _nb(x, w, y))
        return y
    OH, OW = out_hw(H, KH, stride, padding), out_hw(W, KW, stride, padding)
    y = torch.empty((N, OH, OW, Cout), dtype=torch.bfloat16, device=x.device)
    ext.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), N, H, W, Cin, Cout, KH, KW, stride, stride, padding,
                 padding, _ext.ptr(stats), _st(x.device))
    _log("fwd%dx%ds%d" % (KH, KW, stride), N * OH * OW, Cout, KH * KW * Cin, _nb(x, w, y))
    return y


def conv_dgrad(dy, w, x_shape, stride, padding, out=None, beta=0.0, bn=None, res=None, beta_stride=1,
               skip_empty=False):
    """dx (+= beta * out) for y = conv(x, w).

    ``skip_empty`` (strided convolutions, beta 0): the output-parity classes no filter tap
    reaches -- for a 1x1 / stride-s / pad-0 projection shortcut, every pixel but those with h
    and w multiples of s -- are left UNWRITTEN instead of zero-filled.  ``beta_stride`` = s
    (1x1 convolutions with beta): ``out`` is such a tensor; its unwritten pixels are read as
    zeros (never loaded), so the pair writes dx once instead of zero-filling (s^2-1)/s^2 of it
    and reading those zeros back.

    ``bn=(z, mask)``: dx is the gradient of a BatchNorm(+ReLU) output whose input was
    ``z`` (``mask``: its ReLU bitmask, or None).  The GEMM epilogue then also writes the
    BN-backward statistics partials [tiles][2][Cin] = [sum g | sum g*z], g = dx * relu',
    and ``(dx, partials)`` is returned: :func:`bn_bwd` takes them and skips its own
    reduction pass over dx and z.

    ``res=(src, mask)`` (1x1 convolutions): dx = dgrad + beta * relu'(mask) * src -- a
    residual-path gradient gated on the fly from the block's output gradient instead of
    being materialised by the BN backward first.  With ``res``, ``bn`` may carry a third
    entry ``z2``: the input of a second BN fed by the same gated gradient (a projection
    shortcut's BN); ``(dx, partials, partials2)`` is then returned."""
    ext = _ext.load(required=True)
    N, H, W, Cin = x_shape
    Cout, KH, KW, _ = w.shape
    dx = out if out is not None else torch.empty(x_shape, dtype=torch.bfloat16, device=dy.device)
    if beta_stride > 1:
        assert is_gemm_conv(w, stride, padding) and res is None and out is not None and beta != 0, \
            "beta_stride: a 1x1 input gradient accumulated into a skip_empty strided one"
    if res is not None:
        src, rmask = res
        assert is_gemm_conv(w, stride, padding) and src.shape == dx.shape and src.is_contiguous()
        assert rmask is None or rmask.shape == (N * H * W, Cin // 8)
        part, part2, zp, mp, z2p = None, None, 0, 0, 0
        if bn is not None:
            z, mask = bn[0], bn[1]
            assert z.shape == dx.shape and z.is_contiguous()
            part = torch.empty(((N * H * W + 127) // 128, 2, Cin), dtype=torch.float32, device=dy.device)
            zp, mp = z.data_ptr(), _ext.ptr(mask)
            if len(bn) > 2 and bn[2] is not None:
                assert bn[2].shape == dx.shape and bn[2].is_contiguous()
                part2 = torch.empty_like(part)
                z2p = bn[2].data_ptr()
        ext.dgrad_gemm(NN, dy.data_ptr(), Cout, w.data_ptr(), Cin, dx.data_ptr(), Cin, N * H * W, Cin, Cout,
                       float(beta), src.data_ptr(), _ext.ptr(rmask), zp, mp, _ext.ptr(part), _st(dy.device), z2p,
                       _ext.ptr(part2))
        _log("dgrad1x1_res", N * H * W, Cin, Cout, _nb(dy, w, dx, src, rmask, *(bn or ())) + (2 * _nb(dx) if beta else 0))
        if bn is None:
            return dx
        return (dx, part, part2) if len(bn) > 2 else (dx, part)
    if bn is not None:
        z, mask = bn[0], bn[1]
        assert len(bn) == 2 or bn[2] is None, "second-BN statistics need the residual-gated (res=) form"
        assert z.shape == dx.shape and z.is_contiguous() and (mask is None or mask.shape == (N * H * W, Cin // 8))
        if is_gemm_conv(w, stride, padding):
            part = torch.empty(((N * H * W + 127) // 128, 2, Cin), dtype=torch.float32, device=dy.device)
            if beta_stride > 1:
                ext.dgrad_gemm(NN, dy.data_ptr(), Cout, w.data_ptr(), Cin, dx.data_ptr(), Cin, N * H * W, Cin, Cout,
                               float(beta), 0, 0, z.data_ptr(), _ext.ptr(mask), part.data_ptr(), _st(dy.device),
                               par_s=int(beta_stride), par_h=H, par_w=W)
            else:
                ext.gemm_bf16_bnstats(NN, dy.data_ptr(), Cout, w.data_ptr(), Cin, dx.data_ptr(), Cin, N * H * W, Cin,
                                      Cout, float(beta), z.data_ptr(), _ext.ptr(mask), part.data_ptr(), _st(dy.device))
            _log("dgrad1x1_bn", N * H * W, Cin, Cout, _nb(dy, w, dx, z, mask) + (_nb(dx) if beta else 0))
        else:
            rows = ext.conv_dgrad_stat_rows(N, H, W, Cin, Cout, KH, KW, stride, stride, padding, padding,
                                            float(beta))
            part = torch.empty((rows, 2, Cin), dtype=torch.float32, device=dy.device)
            ext.conv_dgrad_bnstats(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), N, H, W, Cin, Cout, KH, KW, stride,
                                   stride, padding, padding, float(beta), z.data_ptr(), _ext.ptr(mask),
                                   part.data_ptr(), _st(dy.device))
            _log("dgrad%dx%ds%d_bn" % (KH, KW, stride), N * H * W, Cin, Cout * KH * KW, _nb(dy, w, dx, z, mask),
                 launches=stride * stride)
        return dx, part
    if is_gemm_conv(w, stride, padding):
        if beta_stride > 1:
            ext.dgrad_gemm(NN, dy.data_ptr(), Cout, w.data_ptr(), Cin, dx.data_ptr(), Cin, N * H * W, Cin, Cout,
                           float(beta), 0, 0, 0, 0, 0, _st(dy.device), par_s=int(beta_stride), par_h=H, par_w=W)
        else:
            ext.gemm_bf16(NN, dy.data_ptr(), Cout, w.data_ptr(), Cin, dx.data_ptr(), Cin, N * H * W, Cin, Cout, 0,
                          float(beta), _st(dy.device))
        _log("dgrad1x1", N * H * W, Cin, Cout, _nb(dy, w, dx) + (_nb(dx) // beta_stride ** 2 if beta else 0))
        return dx
    if skip_empty:
        assert beta == 0 and stride > 1, "skip_empty: strided convolutions, beta 0"
    ext.conv_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), N, H, W, Cin, Cout, KH, KW, stride, stride, padding,
                   padding, float(beta), _st(dy.device), skip_empty=int(bool(skip_empty)))
    _log("dgrad%dx%ds%d" % (KH, KW, stride), N * H * W, Cin, Cout * KH * KW, _nb(dy, w, dx), launches=stride * stride)
    return dx


def conv_wgrad(dy, x, w_shape, stride, padding, out, beta=1.0, blocks=None):
    """out (bf16 or fp32, shape of w) = wgrad + beta * out, split-K over N*OH*OW.
    ``blocks``: split-K workgroup target overriding the configured one."""
    global _WGRAD_BLOCKS, _WGRAD_BLOCKS_SMALLM
    ext = _ext.load(required=True)
    if _WGRAD_BLOCKS is None:
        from .. import config

        _WGRAD_BLOCKS = config.get("CLOUD_AMD_WGRAD_BLOCKS")
        _WGRAD_BLOCKS_SMALLM = config.get("CLOUD_AMD_WGRAD_BLOCKS_SMALLM")
    N, H, W, Cin = x.shape
    Cout, KH, KW, _ = w_shape
    OH, OW = dy.shape[1], dy.shape[2]
    kred = N * OH * OW
    ncols = KH * KW * Cin
    # <= 128 output channels: one row of tiles, so the grid is mostly K splits; the fp32
    # slabs stay small next to the pixel operands, and more splits fill the CUs
    target = blocks or (_WGRAD_BLOCKS_SMALLM if Cout <= 128 else _WGRAD_BLOCKS)
    splits = ext.gemm_splitk_effective(kred, wgrad_splits(Cout, ncols, kred, target_blocks=target))
    if not (KH == 1 and KW == 1):  # the kernel that will run decides (one slab per workgroup on the halo kernel)
        splits = ext.conv_wgrad_splits(N, H, W, Cin, Cout, KH, KW, stride, stride, padding, padding, splits)
    ws = torch.empty(splits * Cout * ncols, dtype=torch.float32, device=x.device)
    obf = int(out.dtype == torch.bfloat16)
    if KH == 1 and KW == 1 and stride == 1 and padding == 0:
        ext.gemm_splitk(TN, dy.data_ptr(), Cout, x.data_ptr(), Cin, out.data_ptr(), obf, float(beta), Cout, Cin,
                        kred, splits, ws.data_ptr(), _st(x.device))
    else:
        ext.conv_wgrad(dy.data_ptr(), x.data_ptr(), out.data_ptr(), obf, float(beta), N, H, W, Cin, Cout, KH, KW,
                       stride, stride, padding, padding, splits, ws.data_ptr(), _st(x.device))
    _log("wgrad%dx%ds%d" % (KH, KW, stride), Cout, ncols, kred, _nb(dy, x, out) + (2 * _nb(ws) if splits > 1 else 0),
         splits=splits)
    return out


# ------------------------------------------- BN folded into the consuming 1x1 GEMM
XA_BN_RELU, XA_BN_RES_RELU, XA_BN_BWD, XA_BN_RESBN_RELU = 0, 1, 2, 3


def conv1x1_dgrad_bnbwd(dy, z, mask, coef, w, side, out=None, beta=0.0, bn=None, res=None):
    """Input gradient of a 1x1 convolution (``w`` [Cout, 1, 1, Cin]) whose output gradient is
    a BatchNorm(+ReLU) backward: ``dz = A*(dy * relu'(mask)) + B*z + D`` with ``coef`` = [A | B | D]
    (:func:`bn_bwd_coef`).  ``dz`` is computed in the GEMM's operand fetch (``ca_gemm_xa.h``),
    never read back; it is also written to ``side`` (the weight gradient's operand).  Epilogue
    options and return values are :func:`conv_dgrad`'s (``bn=``, ``res=``, ``out=`` / ``beta``)."""
    ext = _ext.load(required=True)
    N, H, W, Cout = z.shape
    Cin = w.shape[3]
    M = N * H * W
    x_shape = (N, H, W, Cin)
    assert dy.shape == z.shape and side.shape == z.shape and w.shape[1:3] == (1, 1)
    assert dy.is_contiguous() and z.is_contiguous() and side.is_contiguous() and coef.numel() == 3 * Cout
    assert mask is None or mask.shape == (M, Cout // 8)
    dx = out if out is not None else torch.empty(x_shape, dtype=torch.bfloat16, device=dy.device)
    src, rmask, zp, mp, part, part2, z2p = 0, 0, 0, 0, None, None, 0
    if res is not None:
        src_t, rm_t = res
        assert src_t.shape == dx.shape and src_t.is_contiguous()
        src, rmask = src_t.data_ptr(), _ext.ptr(rm_t)
    if bn is not None:
        zb, mb = bn[0], bn[1]
        assert zb.shape == dx.shape and zb.is_contiguous() and (mb is None or mb.shape == (M, Cin // 8))
        part = torch.empty(((M + 127) // 128, 2, Cin), dtype=torch.float32, device=dy.device)
        zp, mp = zb.data_ptr(), _ext.ptr(mb)
        if len(bn) > 2 and bn[2] is not None:
            assert res is not None, "second-BN statistics need the residual-gated (res=) form"
            part2 = torch.empty_like(part)
            z2p = bn[2].data_ptr()
    cp = coef.data_ptr()
    ext.gemm_xa(NN, XA_BN_BWD, dy.data_ptr(), z.data_ptr(), _ext.ptr(mask), cp, cp + 4 * Cout, cp + 8 * Cout, 0,
                side.data_ptr(), 0, Cout, w.data_ptr(), Cin, dx.data_ptr(), Cin, M, Cin, Cout, float(beta), src, rmask,
                zp, mp, _ext.ptr(part), z2p, _ext.ptr(part2), _st(dy.device))
    _log("dgrad1x1_xa", M, Cin, Cout, _nb(dy, z, mask, side, w, dx) + (_nb(dx) if beta else 0))
    if bn is None:
        return dx
    return (dx, part, part2) if (len(bn) > 2 and bn[2] is not None) else (dx, part)


def conv1x1_strided_dgrad_bnbwd(dy, z, mask, coef, w, side, x_shape, stride):
    """Input gradient of a stride-``stride`` 1x1 / pad-0 convolution (``w`` [Cout, 1, 1, Cin]; a
    ResNet projection shortcut) whose output gradient is a BatchNorm backward: ``dz = A*(dy *
    relu'(mask)) + B*z + D`` is produced in the GEMM's operand fetch and written to ``side`` (the
    weight gradient's operand); ``dz W`` lands on the one non-empty output-parity class of a new
    ``x_shape`` tensor, whose other pixels are left UNWRITTEN -- the pair of
    ``conv_dgrad(..., skip_empty=True)`` after a separate BN backward, in one pass.  The caller's
    next input-gradient GEMM into it must use ``beta_stride=stride``."""
    ext = _ext.load(required=True)
    N, Ho, Wo, Cout = z.shape
    Nx, H, W, Cin = x_shape
    assert Nx == N and w.shape == (Cout, 1, 1, Cin) and stride > 1
    assert Ho == (H - 1) // stride + 1 and Wo == (W - 1) // stride + 1
    assert dy.shape == z.shape and side.shape == z.shape and dy.is_contiguous() and z.is_contiguous()
    assert side.is_contiguous() and coef.numel() == 3 * Cout and Cout <= 2048
    M = N * Ho * Wo
    assert mask is None or mask.shape == (M, Cout // 8)
    dx = torch.empty(x_shape, dtype=torch.bfloat16, device=dy.device)
    cp = coef.data_ptr()
    ext.gemm_xa_bwd_strided(dy.data_ptr(), z.data_ptr(), _ext.ptr(mask), cp, cp + 4 * Cout, cp + 8 * Cout,
                            side.data_ptr(), Cout, w.data_ptr(), Cin, dx.data_ptr(), Cin, M, Cin, Cout, N, H, W,
                            int(stride), _st(dy.device))
    _log("dgrad1x1s_xa", M, Cin, Cout, _nb(dy, z, mask, side, w) + _nb(dx) // stride ** 2)
    return dx


def dgrad_wgrad_fusable(cout, cin):
    """Shapes the fused input+weight gradient kernel (:func:`conv1x1_dgrad_wgrad_bnbwd`) takes
    (``ca_gemm_xa_dw``): 64 input channels with 64 / 128 / 256 output channels (ResNet stage-1
    conv3), 64 output channels with 256 input channels (stage-1 conv1), 128 input channels with
    512 output channels (stage-2 conv3, 8-wave workgroups)."""
    return (cin == 64 and cout in (64, 128, 256)) or (cout == 64 and cin == 256) or (cin == 128 and cout == 512)


def conv1x1_dgrad_wgrad_bnbwd(dy, z, mask, coef, w, y, dw, out=None, beta=0.0, bn=None, res=None, dw_beta=1.0,
                              blocks=None):
    """:func:`conv1x1_dgrad_bnbwd` with the WEIGHT gradient in the same pass: the transformed
    ``dz = A*(dy * relu'(mask)) + B*z + D`` feeds both ``dx = dz W`` and ``dw (+)= dz^T y``
    (``y``: the convolution's input, NHWC) while it is in LDS, so it is never written
    (``ca_gemm_xa.h mfma_gemm_xa_dw``).  ``dw`` ([Cout, 1, 1, Cin], bf16 or fp32) = dz^T y +
    ``dw_beta`` * dw, reduced deterministically from one fp32 slab per workgroup.  Input-gradient
    epilogue options and return values are :func:`conv1x1_dgrad_bnbwd`'s (``bn=`` (z, mask[, z2]),
    ``res=``, ``out=`` / ``beta``).  Shapes: :func:`dgrad_wgrad_fusable`."""
    ext = _ext.load(required=True)
    N, H, W, Cout = z.shape
    Cin = w.shape[3]
    M = N * H * W
    assert dgrad_wgrad_fusable(Cout, Cin), (Cout, Cin)
    assert dy.shape == z.shape and w.shape[1:3] == (1, 1) and dw.shape == w.shape and dw.is_contiguous()
    assert dy.is_contiguous() and z.is_contiguous() and coef.numel() == 3 * Cout
    assert y.shape == (N, H, W, Cin) and y.is_contiguous() and (mask is None or mask.shape == (M, Cout // 8))
    dx = out if out is not None else torch.empty((N, H, W, Cin), dtype=torch.bfloat16, device=dy.device)
    src, rmask, zp, mp, part, part2, z2p = 0, 0, 0, 0, None, None, 0
    if res is not None:
        src_t, rm_t = res
        assert src_t.shape == dx.shape and src_t.is_contiguous()
        src, rmask = src_t.data_ptr(), _ext.ptr(rm_t)
    if bn is not None:
        zb, mb = bn[0], bn[1]
        assert zb.shape == dx.shape and zb.is_contiguous() and (mb is None or mb.shape == (M, Cin // 8))
        part = torch.empty(((M + 127) // 128, 2, Cin), dtype=torch.float32, device=dy.device)
        zp, mp = zb.data_ptr(), _ext.ptr(mb)
        if len(bn) > 2 and bn[2] is not None:
            assert res is not None, "second-BN statistics need the residual-gated (res=) form"
            part2 = torch.empty_like(part)
            z2p = bn[2].data_ptr()
    if blocks is None:  # 4-wave workgroups two per CU, 8-wave (Cin 128) one per CU
        blocks = (1 if Cin == 128 else 2) * _cu_count(dy.device)
    blocks = max(1, min(int(blocks), (M + 127) // 128))
    ws = torch.empty(blocks * Cout * Cin, dtype=torch.float32, device=dy.device)
    cp = coef.data_ptr()
    g = ext.gemm_xa_dw(dy.data_ptr(), z.data_ptr(), _ext.ptr(mask), cp, cp + 4 * Cout, cp + 8 * Cout, Cout,
                       w.data_ptr(), Cin, dx.data_ptr(), Cin, M, Cin, Cout, float(beta), src, rmask, zp, mp,
                       _ext.ptr(part), z2p, _ext.ptr(part2), y.data_ptr(), Cin, dw.data_ptr(),
                       int(dw.dtype == torch.bfloat16), float(dw_beta), ws.data_ptr(), blocks, _st(dy.device))
    _log("dgrad_wgrad1x1_xa", M, Cin, Cout, _nb(dy, z, mask, w, dx, y) + (_nb(dx) if beta else 0)
         + 2 * g * Cout * Cin * 4)
    if bn is None:
        return dx
    return (dx, part, part2) if part2 is not None else (dx, part)


_CU_COUNT = {}


def _cu_count(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _CU_COUNT:
        _CU_COUNT[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _CU_COUNT[idx]


def conv1x1_fwd_bnapply(z, ss, w, side, mask_out, res=None, res_ss=None, stats=None):
    """Forward 1x1 convolution (``w`` [Cout, 1, 1, Cin]) of a BatchNorm(+residual)+ReLU output
    that is never written by a separate pass: ``y = relu(z*scale + shift [+ r | + bf16(r*rscale +
    rshift)])`` is computed in the GEMM's operand fetch (``ca_gemm_xa.h``) from ``ss`` = [scale |
    shift] (and ``res_ss`` for a projection shortcut's BN), and written once to ``side`` with its
    ReLU bitmask ``mask_out`` ([M, Cin/8]) -- bit for bit what bn_fwd would have stored.
    ``stats``: the BN-forward statistics partials of the output ([ceil(M/128)][2][Cout])."""
    ext = _ext.load(required=True)
    N, H, W, Cin = z.shape
    Cout = w.shape[0]
    M = N * H * W
    assert w.shape[1:] == (1, 1, Cin) and z.is_contiguous() and side.shape == z.shape and side.is_contiguous()
    assert ss.numel() == 2 * Cin and mask_out.shape == (M, Cin // 8)
    mode, src1, c2, c3 = XA_BN_RELU, 0, 0, 0
    if res is not None:
        assert res.shape == z.shape and res.is_contiguous()
        src1 = res.data_ptr()
        mode = XA_BN_RES_RELU
        if res_ss is not None:
            assert res_ss.numel() == 2 * Cin
            mode, c2, c3 = XA_BN_RESBN_RELU, res_ss.data_ptr(), res_ss.data_ptr() + 4 * Cin
    assert stats is None or stats.shape == ((M + 127) // 128, 2, Cout)
    y = torch.empty((N, H, W, Cout), dtype=torch.bfloat16, device=z.device)
    sp = ss.data_ptr()
    ext.gemm_xa(NT, mode, z.data_ptr(), src1, 0, sp, sp + 4 * Cin, c2, c3, side.data_ptr(), mask_out.data_ptr(), Cin,
                w.data_ptr(), Cin, y.data_ptr(), Cout, M, Cout, Cin, 0.0, 0, 0, 0, 0, _ext.ptr(stats), 0, 0,
                _st(z.device))
    _log("fwd1x1_xa", M, Cout, Cin, _nb(z, res, side, mask_out, w, y))
    return y


def uses_prw(M, N, K):
    """Whether a forward NT GEMM with statistics runs on the persistent resident-weight core
    (its statistics partials are then one row per workgroup, not per 128 rows)."""
    ext = _ext.load(required=True)
    return ext.gemm_stat_rows(int(M), int(N), int(K), int(K), int(K), int(N)) != (M + 127) // 128


def bn_bwd_coef(C, M, gamma, stats, partials, dgamma=None, dbeta=None, accumulate=0):
    """BN backward statistics finalize only (no apply pass): dgamma / dbeta written (or
    accumulated) from the dgrad epilogue's ``partials``; returns the [A | B | D] coefficients
    of ``dz = A*g + B*z + D`` for :func:`conv1x1_dgrad_bnbwd`."""
    ext = _ext.load(required=True)
    dev = partials.device
    assert partials.shape[1:] == (2, C)
    coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
    gws = torch.empty(_GWS_ROWS * 2 * C, dtype=torch.float32, device=dev) if partials.shape[0] > 64 else None
    sp = stats.data_ptr()
    ext.bn_bwd_partials(0, 0, 0, 0, int(M), int(C), partials.data_ptr(), partials.shape[0], _ext.ptr(gamma), sp,
                        sp + 4 * C, 0, 0, _ext.ptr(dgamma), _ext.ptr(dbeta), coef.data_ptr(), _ext.ptr(gws),
                        1 | (2 if accumulate else 0), _st(dev))
    return coef


# ------------------------------------------------------------------ batchnorm
def bn_fwd_stats(x, gamma, beta, running_mean, running_var, eps, momentum, partials):
    """Training BN statistics only (no apply pass): returns stats[4C] = mean, rstd, scale,
    shift -- for a BN whose output is consumed on the fly (:func:`bn_fwd` ``residual_ss``)."""
    ext = _ext.load(required=True)
    C = x.shape[-1]
    M = x.numel() // C
    dev = x.device
    stats = torch.empty(4 * C, dtype=torch.float32, device=dev)
    gws = torch.empty(_GWS_ROWS * 2 * C, dtype=torch.float32, device=dev) if partials.shape[0] > 64 else None
    sp = stats.data_ptr()
    ext.bn_fwd_partials_ex(x.data_ptr(), 0, 0, 0, M, C, partials.data_ptr(), partials.shape[0], _ext.ptr(gamma),
                           _ext.ptr(beta), float(eps), float(momentum), _ext.ptr(running_mean),
                           _ext.ptr(running_var), sp, sp + 4 * C, sp + 8 * C, 0, 0, _ext.ptr(gws), _st(dev))
    return stats


def bn_fwd(x, gamma, beta, running_mean, running_var, eps, momentum, relu, residual=None, partials=None,
           keep_mask=False, residual_ss=None):
    """Training BN(+res)(+ReLU).  Returns (y, stats[4C] = mean, rstd, scale, shift, mask) where
    ``mask`` is the ReLU bitmask ([M, C/8] uint8, bit j = channel 8c+j active) when
    ``keep_mask`` and ``relu`` (else None): the backward then reads it instead of y."""
    ext = _ext.load(required=True)
    C = x.shape[-1]
    M = x.numel() // C
    dev = x.device
    y = torch.empty_like(x)
    stats = torch.empty(4 * C, dtype=torch.float32, device=dev)
    mask = torch.empty((M, C // 8), dtype=torch.uint8, device=dev) if (keep_mask and relu) else None
    sp = stats.data_ptr()
    if residual_ss is not None:  # residual = input of another BN with [scale | shift] = residual_ss
        assert partials is not None and residual is not None and residual_ss.numel() == 2 * C
        gws = torch.empty(_GWS_ROWS * 2 * C, dtype=torch.float32, device=dev) if partials.shape[0] > 64 else None
        ext.bn_fwd_partials_ex(x.data_ptr(), residual.data_ptr(), residual_ss.data_ptr(), y.data_ptr(), M, C,
                               partials.data_ptr(), partials.shape[0], _ext.ptr(gamma), _ext.ptr(beta), float(eps),
                               float(momentum), _ext.ptr(running_mean), _ext.ptr(running_var), sp, sp + 4 * C,
                               sp + 8 * C, int(relu), _ext.ptr(mask), _ext.ptr(gws), _st(dev))
        return y, stats, mask
    if partials is not None:
        gws = torch.empty(_GWS_ROWS * 2 * C, dtype=torch.float32, device=dev) if partials.shape[0] > 64 else None
        ext.bn_fwd_partials(x.data_ptr(), _ext.ptr(residual), y.data_ptr(), M, C, partials.data_ptr(),
                            partials.shape[0], _ext.ptr(gamma), _ext.ptr(beta), float(eps), float(momentum),
                            _ext.ptr(running_mean), _ext.ptr(running_var), sp, sp + 4 * C, sp + 8 * C, int(relu),
                            _ext.ptr(mask), _ext.ptr(gws), _st(dev))
    else:
        ws = torch.empty(ext.bn_workspace_floats(M, C), dtype=torch.float32, device=dev)
        ext.bn_fwd(x.data_ptr(), _ext.ptr(residual), y.data_ptr(), M, C, _ext.ptr(gamma), _ext.ptr(beta),
                   float(eps), float(momentum), _ext.ptr(running_mean), _ext.ptr(running_var), sp, sp + 4 * C,
                   sp + 8 * C, ws.data_ptr(), int(relu), _ext.ptr(mask), _st(dev))
    return y, stats, mask


def bn_bwd(dy, y, x, gamma, stats, relu, dgamma=None, dbeta=None, want_dres=False, dx_out=None, accumulate=0,
           mask=None, partials=None):
    """BN(+res)(+ReLU) backward.  The ReLU gate comes from ``mask`` (forward bitmask) or
    ``y``.  dgamma/dbeta (fp32 [C]) are written, or accumulated into when
    ``accumulate`` is set.  ``partials``: the [tiles][2][C] statistics written by the
    epilogue of the dgrad that produced ``dy`` (:func:`conv_dgrad` ``bn=``) -- the
    reduction pass is skipped.  Returns (dx, dres-or-None)."""
    ext = _ext.load(required=True)
    C = x.shape[-1]
    M = x.numel() // C
    dev = x.device
    dx = dx_out if dx_out is not None else torch.empty_like(x)
    dres = torch.empty_like(x) if want_dres else None
    coef = torch.empty(3 * C, dtype=torch.float32, device=dev)
    sp = stats.data_ptr()
    if partials is not None:
        assert partials.shape[1:] == (2, C)
        gws = torch.empty(_GWS_ROWS * 2 * C, dtype=torch.float32, device=dev) if partials.shape[0] > 64 else None
        ext.bn_bwd_partials(dy.data_ptr(), _ext.ptr(y), _ext.ptr(mask), x.data_ptr(), M, C, partials.data_ptr(),
                            partials.shape[0], _ext.ptr(gamma), sp, sp + 4 * C, dx.data_ptr(), _ext.ptr(dres),
                            _ext.ptr(dgamma), _ext.ptr(dbeta), coef.data_ptr(), _ext.ptr(gws),
                            int(relu) | (2 if accumulate else 0), _st(dev))
        return dx, dres
    ws = torch.empty(ext.bn_workspace_floats(M, C), dtype=torch.float32, device=dev)
    ext.bn_bwd(dy.data_ptr(), _ext.ptr(y), _ext.ptr(mask), x.data_ptr(), M, C, _ext.ptr(gamma), sp, sp + 4 * C,
               dx.data_ptr(), _ext.ptr(dres), _ext.ptr(dgamma), _ext.ptr(dbeta), coef.data_ptr(), ws.data_ptr(),
               int(relu) | (2 if accumulate else 0), _st(dev))
    return dx, dres


# ------------------------------------------------------- dense / transformer
ACT = {None: 0, "none": 0, "linear": 0, "gelu": 1, "relu": 2, "tanh": 3, "gelu_tanh": 4}


class PlainGemmPolicy:
    """Which engine runs a PLAIN bf16 GEMM -- no activation, no pre-activation store, no
    act' multiply, no statistics; optional bias and C accumulate (beta = 1): the in-tree
    MFMA kernels or the vendor library (hipBLASLt through torch), the one the task's
    rules reserve for "plain library GEMMs".  Every fused GEMM (bias + GELU + pre-activation,
    GELU' backward, BN statistics, split-K weight gradients into the fp32 arena) stays on
    the in-tree kernels.

    ``CLOUD_AMD_GEMM_LIB``: ``never`` (default) = in-tree only, so every box and every rank runs
    the same kernels; ``auto`` (a diagnostic) times both engines once per (layout, M, N, K,
    bias, beta) key on the first call -- on scratch outputs, outside any stream capture --
    and keeps the faster (``decisions`` records the timings); ``always`` = library for every
    plain GEMM."""

    def __init__(self):
        self.mode = None
        self.decisions = {}

    def _mode(self):
        if self.mode is None:
            from .. import config

            self.mode = config.get("CLOUD_AMD_GEMM_LIB")
        return self.mode

    @staticmethod
    def _time(fn, reps=5):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / reps

    def use_library(self, key, ours, lib):
        mode = self._mode()
        if mode == "never":
            return False
        if mode == "always":
            return True
        d = self.decisions.get(key)
        if d is None:
            if torch.cuda.is_current_stream_capturing():
                return False
            t_ours, t_lib = self._time(ours), self._time(lib)
            d = self.decisions[key] = {"library": t_lib < 0.97 * t_ours, "ours_us": round(t_ours, 1),
                                       "lib_us": round(t_lib, 1)}
        return d["library"]


PLAIN_GEMM = PlainGemmPolicy()


def _plain_lib(a, w, bias, out, beta, layout):
    """The library form of a plain GEMM into ``out`` (bias added in bf16, as autocast does)."""
    wm = w.t() if layout == NT else w
    if beta:
        out.addmm_(a, wm)
        if bias is not None:
            out.add_(bias.to(out.dtype))
    elif bias is not None:
        torch.addmm(bias.to(out.dtype), a, wm, out=out)
    else:
        torch.mm(a, wm, out=out)
    return out


def gemm(a, w, bias=None, act=None, preact=None, out=None, beta=0.0, layout=NT, dact_src=None, stats=None):
    """Fused dense GEMM.  NT: out[M,N] = act(a[M,K] @ w[N,K]^T + bias); NN: a[M,K] @ w[K,N].
    ``preact`` receives the pre-activation; ``dact_src`` switches to the backward
    form out = (a @ w) * act'(dact_src).  Row strides of ``a`` are honoured.  Plain GEMMs
    (see :class:`PlainGemmPolicy`) may run on the vendor library when it measures faster."""
    ext = _ext.load(required=True)
    M, K = a.shape
    N = w.shape[0] if layout == NT else w.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if (PLAIN_GEMM._mode() != "never" and act in (None, "none", "linear") and preact is None and dact_src is None
            and stats is None and beta in (0.0, 1.0) and layout in (NT, NN) and a.is_cuda and a.stride(1) == 1
            and w.is_contiguous() and out.is_contiguous() and (bias is None or layout == NT)):
        key = (layout, M, N, K, bias is not None, float(beta))
        if key not in PLAIN_GEMM.decisions and PLAIN_GEMM._mode() == "auto":
            scratch = torch.zeros_like(out)

            def ours_fn():
                ext.gemm_ex(layout, a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), scratch.data_ptr(), N, M,
                            N, K, 0, float(beta), _ext.ptr(bias), 0, 0, 0, 0, _st(a.device))

            use = PLAIN_GEMM.use_library(key, ours_fn, lambda: _plain_lib(a, w, bias, scratch, beta, layout))
            del scratch
        else:
            use = PLAIN_GEMM.use_library(key, None, None)
        if use:
            _log("lib_nt" if layout == NT else "lib_nn", M, N, K, _nb(a, w, out, bias) + (_nb(out) if beta else 0))
            return _plain_lib(a, w, bias, out, beta, layout)
    aux = preact if preact is not None else dact_src
    ld_aux = aux.stride(0) if aux is not None else 0
    ext.gemm_ex(layout, a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0), M, N, K,
                _ext.ptr(stats), float(beta), _ext.ptr(bias), ACT[act], _ext.ptr(preact), _ext.ptr(dact_src), ld_aux,
                _st(a.device))
    _log("dense_nt" if layout == NT else "dense_nn", M, N, K, _nb(a, w, out, bias, preact, dact_src) +
         (_nb(out) if beta else 0))
    return out


class GradFinalizeBatch:
    """Deferred gradient finalisation (csrc/kernels/gradfin.hip): while active (see
    ``deferred_finalize``), ``wgrad_into`` / ``colsum_into`` / ``ln_bwd`` launch only their
    partial-producing kernels and queue the fixed-order reductions here; ``flush`` runs them
    all in one launch (per 8 jobs) on the current stream.  Results are bitwise those of the
    immediate path.  Workspaces stay referenced until the flush and are recorded on the
    flushing stream (side-stream allocations must not be reused before it runs)."""

    def __init__(self):
        self.groups = {}  # issuing stream -> (stream, jobs, betas, keep)

    def _group(self, t):
        # keyed by the raw handle of the issuing stream (no Stream object per job)
        key = _ext.stream_handle(t.device) if t.device.type == "cuda" else None
        g = self.groups.get(key)
        if g is None:
            g = self.groups[key] = (key, [], [], [])
        return g

    def add_splitk(self, ws, splits, n, out, beta):
        _, jobs, betas, keep = self._group(ws)
        jobs += [0, ws.data_ptr(), splits, n, n, out.data_ptr(), 0, 0, int(out.dtype == torch.bfloat16), 0, 0, 0]
        betas.append(float(beta))
        keep.append(ws)

    def add_cols(self, part, nparts, stride, n, out0, out1=None, out2=None, accumulate=True):
        _, jobs, betas, keep = self._group(part)
        jobs += [1, part.data_ptr(), nparts, stride, n, _ext.ptr(out0), _ext.ptr(out1), _ext.ptr(out2), 0,
                 int(accumulate), 0, 0]
        betas.append(0.0)
        keep.append(part)

    def flush(self):
        """One launch per issuing stream, on that stream (a job runs after the kernel that
        produced its partials, and its workspace was allocated from that stream's pool)."""
        ext = _ext.load(required=True)
        for handle, jobs, betas, keep in self.groups.values():
            if betas:
                ext.grad_finalize_multi(jobs, betas, handle or 0)
        self.groups = {}


_FIN_BATCH = None


class deferred_finalize:
    """``with raw.deferred_finalize() as b: ...; b.flush()`` -- batch the gradient
    finalisations issued inside (nesting keeps the outer batch)."""

    def __init__(self, enabled=True):
        self.enabled = enabled
        self.batch = None
        self.prev = None

    def __enter__(self):
        global _FIN_BATCH
        self.prev = _FIN_BATCH
        if self.enabled:
            self.batch = _FIN_BATCH = GradFinalizeBatch() if self.prev is None else self.prev
        return self.batch

    def __exit__(self, *exc):
        global _FIN_BATCH
        if self.enabled and self.prev is None and self.batch is not None:
            self.batch.flush()
        _FIN_BATCH = self.prev
        return False


def _wgrad_splits_256(n_out, k_in, kred):
    """Split count that puts a dense weight gradient on ONE round of the two-phase 256 x 256
    core (csrc/kernels/gemm.hip use_256: 224-256 workgroups of 256 x 256 tiles, >= 512
    reduction rows each), e.g. BERT's QKV (27 tiles x 9 splits), FFN1 / FFN2 (36 x 7); 0 when
    the shape does not fit one round (``CLOUD_AMD_DENSE_WGRAD_256=0``: never)."""
    from .. import config

    if not config.get("CLOUD_AMD_DENSE_WGRAD_256"):
        return 0
    t256 = -(-n_out // 256) * -(-k_in // 256)
    if t256 > 128:
        return 0
    ext = _ext.load(required=True)
    s = ext.gemm_splitk_effective(kred, 256 // t256)
    if not 224 <= t256 * s <= 256 or kred // s < 512:
        return 0
    return s


def wgrad_into(dy, x, out, beta=1.0):
    """out[N_out, K_in] (+)= dy[M, N_out]^T @ x[M, K_in] (split-K over M), bf16 or fp32 out."""
    global _DENSE_WGRAD_BLOCKS
    ext = _ext.load(required=True)
    if _DENSE_WGRAD_BLOCKS is None:
        from .. import config

        _DENSE_WGRAD_BLOCKS = config.get("CLOUD_AMD_DENSE_WGRAD_BLOCKS")
    M, n_out = dy.shape
    k_in = x.shape[1]
    # dense layers: K = tokens is moderate, so fewer/larger K slices (less slab traffic).
    splits = ext.gemm_splitk_effective(M, wgrad_splits(n_out, k_in, M, target_blocks=_DENSE_WGRAD_BLOCKS, min_k=1024))
    s256 = _wgrad_splits_256(n_out, k_in, M)
    if s256:
        splits = s256
    ws = torch.empty(splits * n_out * k_in, dtype=torch.float32, device=dy.device)
    fb = _FIN_BATCH
    ext.gemm_splitk(TN, dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr(),
                    -1 if fb is not None else int(out.dtype == torch.bfloat16), float(beta), n_out, k_in, M, splits,
                    ws.data_ptr(), _st(dy.device))
    if fb is not None:
        fb.add_splitk(ws, splits, n_out * k_in, out, beta)
    _log("dense_wgrad", n_out, k_in, M, _nb(dy, x, out) + (2 * _nb(ws) if splits > 1 else 0), splits=splits)
    return out


def colsum_into(x, out, accumulate=True):
    """out[N] (+)= sum over rows of bf16 x[M, N] (bias gradient)."""
    ext = _ext.load(required=True)
    M, N = x.shape
    ws = torch.empty(ext.colsum_workspace_floats(M, N), dtype=torch.float32, device=x.device)
    fb = _FIN_BATCH
    ext.colsum(x.data_ptr(), M, N, x.stride(0), out.data_ptr(), -1 if fb is not None else int(accumulate),
               ws.data_ptr(), _st(x.device))
    if fb is not None:
        ry = min(max((M + 63) // 64, 1), 256)  # = ca_colsum's partial rows
        fb.add_cols(ws, ry, N, N, out, accumulate=accumulate)
    return out


def ln_fwd(x, gamma, beta, eps, residual=None, p_in=0.0, seed_in=0, p_out=0.0, seed_out=0, keep_h=True,
           x_bias=None):
    """y = drop_out(LN(residual + drop_in(x + x_bias))).  Returns (y, h, mean, rstd); h is
    the pre-norm sum (None when it equals x: no residual, no input dropout, no bias, or
    keep_h=False).  ``x_bias`` (fp32 [C]): the bias of the GEMM that produced x, added here
    so that GEMM runs without a bias epilogue."""
    ext = _ext.load(required=True)
    C = x.shape[-1]
    M = x.numel() // C
    y = torch.empty_like(x)
    if x_bias is not None and (x_bias.dtype != torch.float32 or x_bias.numel() != C or not x_bias.is_contiguous()
                               or x_bias.data_ptr() % 16):
        raise ValueError("ln_fwd x_bias: contiguous 16-byte-aligned fp32 [C] expected")
    need_h = keep_h and (residual is not None or p_in > 0 or x_bias is not None)
    h = torch.empty_like(x) if need_h else None
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty(M, dtype=torch.float32, device=x.device)
    ext.ln_fwd(x.data_ptr(), _ext.ptr(residual), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), _ext.ptr(h),
               mean.data_ptr(), rstd.data_ptr(), M, C, float(eps), float(p_in), int(seed_in), float(p_out),
               int(seed_out), _st(x.device), _ext.ptr(x_bias))
    return y, h, mean, rstd


def ln_bwd(dy, h, mean, rstd, gamma, dgamma=None, dbeta=None, p_in=0.0, seed_in=0, p_out=0.0, seed_out=0,
           want_dx=False, accumulate=True, dsum=None):
    """Returns (dh, dx): dh = grad wrt the pre-norm sum (also the residual grad); dx =
    drop_in'(dh) when ``want_dx`` (else None).  ``dsum`` (fp32 [C]) receives the column
    sums of dx (else dh) -- the bias gradient of the layer that fed the LN -- from the
    same pass (accumulated when ``accumulate``)."""
    ext = _ext.load(required=True)
    C = dy.shape[-1]
    M = dy.numel() // C
    dh = torch.empty_like(dy)
    dx = torch.empty_like(dy) if want_dx else None
    nws = ext.ln_workspace_floats(M, C)
    ws = torch.empty(nws, dtype=torch.float32, device=dy.device)
    fb = _FIN_BATCH if (dgamma is not None or dbeta is not None or dsum is not None) else None
    ext.ln_bwd(dy.data_ptr(), h.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(), dh.data_ptr(),
               _ext.ptr(dx), _ext.ptr(dgamma), _ext.ptr(dbeta), -1 if fb is not None else int(accumulate),
               ws.data_ptr(), M, C, float(p_in), int(seed_in), float(p_out), int(seed_out), _st(dy.device),
               _ext.ptr(dsum))
    if fb is not None:
        fb.add_cols(ws, nws // (3 * C), 3 * C, C, dgamma, dbeta, dsum, accumulate=accumulate)
    return dh, dx


def cls_head_fwd(pooled, wc, bc, p_drop=0.0, seed=0):
    """logits[B, L] (fp32) = drop(pooled) @ wc^T + bc  (csrc/kernels/head.hip)."""
    ext = _ext.load(required=True)
    B, C = pooled.shape
    L = wc.shape[0]
    logits = torch.empty((B, L), dtype=torch.float32, device=pooled.device)
    ext.cls_head_fwd(pooled.data_ptr(), pooled.stride(0), wc.data_ptr(), bc.data_ptr(), logits.data_ptr(), B, C, L,
                     float(p_drop), int(seed), _st(pooled.device))
    return logits


def cls_head_bwd(dlogits, pooled, wc, gwc=None, gbc=None, p_drop=0.0, seed=0):
    """dpre[B, C] (bf16) = (dlogits @ wc) * drop' * (1 - pooled^2); gwc / gbc (+)= the
    classifier's weight / bias gradients."""
    ext = _ext.load(required=True)
    B, C = pooled.shape
    L = wc.shape[0]
    dl = dlogits.float().contiguous()
    dpre = torch.empty((B, C), dtype=torch.bfloat16, device=pooled.device)
    ext.cls_head_bwd(dl.data_ptr(), pooled.data_ptr(), pooled.stride(0), wc.data_ptr(), dpre.data_ptr(),
                     _ext.ptr(gwc), _ext.ptr(gbc), B, C, L, float(p_drop), int(seed), _st(pooled.device))
    return dpre


def embed_sum(ids, tts, word, pos, type_, seq_len, pos_offset=0):
    ext = _ext.load(required=True)
    M = ids.numel()
    C = word.shape[1]
    h = torch.empty((M, C), dtype=torch.bfloat16, device=word.device)
    ext.embed_sum(ids.data_ptr(), _ext.ptr(tts), word.data_ptr(), pos.data_ptr(), _ext.ptr(type_), h.data_ptr(), M,
                  seq_len, C, pos_offset, _st(word.device))
    return h


# embed_bwd's deterministic token-type workspace: per (device, stream) -- a ticket must
# never be shared by kernels that can run concurrently -- taken from the caching allocator
# and kept; the kernel's last block resets the ticket to 0 for the next launch.
_EMBED_WS = {}
# how many embed_bwd calls took the order-dependent float-atomic path (tests assert 0 where
# the step must be bitwise reproducible; CLOUD_AMD_DETERMINISTIC=1 makes it an error)
EMBED_NONDETERMINISTIC_CALLS = 0


def _embed_ws(C, device):
    stream = torch.cuda.current_stream(device)
    key = (device.index, stream.cuda_stream)
    ws = _EMBED_WS.get(key)
    if ws is None or ws[0].numel() < 64 * 2 * C:
        # a tensor owned by this stream: the caching allocator ties its reuse to the stream
        ws = (torch.empty(64 * 2 * C, dtype=torch.float32, device=device),
              torch.zeros(1, dtype=torch.int32, device=device))
        _EMBED_WS[key] = ws
    return ws


def embed_bwd(dh, ids, tts, dword, dpos, dtype_, seq_len, n_types, pos_offset=0, pad_id=-1):
    """Scatter-add into dword (deterministic owner-row kernel; ids outside [0, vocab) and
    ``pad_id`` get nothing), dpos / dtype_ reduced -- the token-type rows by a fixed-order
    reduction over a workspace from the caching allocator.  A gradient that must take the
    float-atomic path (more than two token types, rows wider than the owner kernel holds) is
    counted in ``EMBED_NONDETERMINISTIC_CALLS`` and raises under ``CLOUD_AMD_DETERMINISTIC=1``."""
    global EMBED_NONDETERMINISTIC_CALLS
    ext = _ext.load(required=True)
    M, C = dh.shape
    V = dword.shape[0] if dword is not None else 0
    tws = tk = None
    if dtype_ is not None and n_types <= 2:
        tws, tk = _embed_ws(C, dh.device)
    nondet = ext.embed_bwd(dh.data_ptr(), ids.data_ptr(), _ext.ptr(tts), _ext.ptr(dword), _ext.ptr(dpos),
                           _ext.ptr(dtype_), M, seq_len, C, n_types, pos_offset, int(pad_id), int(V), _ext.ptr(tws),
                           _ext.ptr(tk), _st(dh.device))
    if nondet:
        EMBED_NONDETERMINISTIC_CALLS += 1
        if os.environ.get("CLOUD_AMD_DETERMINISTIC") == "1":
            raise RuntimeError("embed_bwd: C=%d, %d token types has no deterministic kernel "
                               "(CLOUD_AMD_DETERMINISTIC=1)" % (C, n_types))


def attn_fwd(qkv, B, S, H, key_len=None, p_drop=0.0, seed=0, scale=None):
    """qkv [B*S, 3*H*64] -> (ctx [B*S, H*64], lse [B, H, S])."""
    ext = _ext.load(required=True)
    C = H * 64
    ctx = torch.empty((B * S, C), dtype=torch.bfloat16, device=qkv.device)
    lse = torch.empty((B, H, S), dtype=torch.float32, device=qkv.device)
    scale = 1.0 / 8.0 if scale is None else scale
    ext.attn_fwd(qkv.data_ptr(), ctx.data_ptr(), lse.data_ptr(), _ext.ptr(key_len), B, S, H, float(scale),
                 float(p_drop), int(seed), _st(qkv.device))
    return ctx, lse


def attn_bwd(qkv, ctx, dctx, lse, B, S, H, key_len=None, p_drop=0.0, seed=0, scale=None):
    ext = _ext.load(required=True)
    dqkv = torch.empty_like(qkv)
    dvec = torch.empty_like(lse)
    scale = 1.0 / 8.0 if scale is None else scale
    ext.attn_bwd(qkv.data_ptr(), ctx.data_ptr(), dctx.data_ptr(), lse.data_ptr(), dvec.data_ptr(), dqkv.data_ptr(),
                 _ext.ptr(key_len), B, S, H, float(scale), float(p_drop), int(seed), _st(qkv.device))
    return dqkv


def dropout(x, p, seed, out=None):
    ext = _ext.load(required=True)
    y = out if out is not None else torch.empty_like(x)
    ext.dropout(x.data_ptr(), y.data_ptr(), x.numel(), float(p), int(seed), _st(x.device))
    return y


def dropout_mask(n, p, seed, base=0, device="cuda"):
    """The keep-mask (uint8) the kernels use for elements base..base+n-1 (tests / references)."""
    ext = _ext.load(required=True)
    m = torch.empty(n, dtype=torch.uint8, device=device)
    ext.dropout_mask(m.data_ptr(), n, base, float(p), int(seed), _st(m.device))
    return m
