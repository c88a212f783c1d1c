"""Hand-scheduled forward/backward of a ResNet bottleneck block on the gfx950 kernels.

Running the block through per-op autograd Functions costs, per block, one full
read-read-write pass over the block input's gradient (autograd sums the
identity-path gradient and conv1's input gradient with a separate add kernel)
plus six tiny ``AccumulateGrad`` adds for the BatchNorm parameters.  On
ResNet-50 at batch 256 those adds are ~2 ms of a ~34 ms step, all HBM traffic.

This module runs the whole block as ONE autograd node:

* forward: conv (+fused BN statistics epilogue) -> BN+ReLU apply, three times,
  plus the projection shortcut; only the tensors the backward needs are kept
  (the shortcut BN output is dropped as soon as it is consumed);
* backward: BN backward emits the residual gradient directly; conv1's input
  gradient is accumulated *into* that buffer by the dgrad GEMM epilogue
  (``beta = 1``) -- no separate add; every weight gradient goes split-K into
  its slice of the flat gradient arena and the BN ``dgamma/dbeta`` are summed
  into their arena slots by the BN finalize kernel; the DDP engine is notified
  per parameter so bucketed all-reduces still overlap with the rest of the
  backward;
* the weight-gradient GEMMs (compute bound) run on a second HIP stream so they
  overlap the memory-bound BN-backward / dgrad chain of the main stream; the
  block joins that stream before reporting its conv weights to DDP
  (``CLOUD_AMD_WGRAD_STREAM``);
* the BN-backward statistics come from the dgrad GEMM epilogues: the GEMM that
  produces a BN output's gradient also sums g = dy * relu' and g * z per column
  and tile (``raw.conv_dgrad(..., bn=(z, mask))``), so the BN backward skips its
  own read pass over dy and z.  Inside a block that covers bn2 (conv3's dgrad)
  and bn1 (conv2's dgrad); across blocks, conv1's dgrad of block i+1 -- the
  launch that completes the block-input gradient -- computes block i's bn3
  statistics and parks them for block i's backward (``CLOUD_AMD_BN_BWD_EPILOGUE``);
* no shortcut tensor is materialised in either direction: the projection
  shortcut's BN is folded into bn3's apply (its statistics pass only; the affine
  is applied to the shortcut conv output in registers, rounded to bf16 exactly as
  a stored copy would be), and the residual gradient ``dout * relu'(mask3)`` is
  gated on load -- by conv1's dgrad epilogue in identity blocks (``res=``), by the
  shortcut BN backward in projection blocks.

Parity: the block computes exactly what :class:`cloud_amd.models.resnet.Bottleneck`
computes op by op (same kernels, same order) -- tests compare the two.
"""
from __future__ import annotations

import torch

from .. import config
from ..ops import _ext, raw
from ..runtime.side_stream import SideWork


# Cross-block hand-off of bn3 statistics (one slot: blocks run backward one after
# another).  The parked gradient is held so its memory cannot be reused by another
# tensor while parked; the consumer checks identity (storage, shape, version).
_HANDOFF = {"grad": None, "version": -1, "partials": None, "partials2": None}


def _park(grad, partials, partials2=None):
    _HANDOFF.update(grad=grad, version=grad._version, partials=partials, partials2=partials2)


def _take(dout):
    """(bn3 partials, projection-shortcut BN partials) parked for this block's output
    gradient ``dout`` by the next block's conv1 dgrad epilogue, else (None, None)."""
    g, ver = _HANDOFF["grad"], _HANDOFF["version"]
    part, part2 = _HANDOFF["partials"], _HANDOFF["partials2"]
    _HANDOFF.update(grad=None, version=-1, partials=None, partials2=None)
    if g is None or part is None:
        return None, None
    if g.data_ptr() != dout.data_ptr() or g.shape != dout.shape or dout._version != ver:
        return None, None
    return part, part2


def _arena_grad(p, dtype):
    g = getattr(p, "grad", None)
    if g is None or not getattr(p, "_ca_arena", False) or g.dtype != dtype or not g.is_contiguous():
        return None
    return g


def block_params(blk):
    ps = [blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias,
          blk.conv3.weight, blk.bn3.weight, blk.bn3.bias]
    if blk.downsample is not None:
        ps += [blk.downsample["conv"].weight, blk.downsample["bn"].weight, blk.downsample["bn"].bias]
    return ps


def can_fuse(blk, x):
    """The fused schedule needs the native kernels, bf16 NHWC, training mode and
    every parameter gradient resident in the flat arena (so it can be written in place)."""
    if not (blk.training and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()):
        return False
    if not _ext.use_native(x) or x.shape[-1] % 8:
        return False
    for p in block_params(blk):
        want = torch.bfloat16 if p.dim() == 4 else torch.float32
        if not p.requires_grad or _arena_grad(p, want) is None:
            return False
    convs = [blk.conv1, blk.conv2, blk.conv3] + ([blk.downsample["conv"]] if blk.downsample is not None else [])
    return all(c.bias is None for c in convs)


def _conv_bn(conv, bn, x, residual=None):
    part = raw.conv_stats_buffer(x.shape, conv.weight, conv.stride, conv.padding, x.device)
    z = raw.conv_fwd(x, conv.weight, conv.stride, conv.padding, stats=part)
    y, st, mask = raw.bn_fwd(z, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, bn.momentum,
                             bn.relu, residual=residual, partials=part, keep_mask=True)
    return z, y, (st, mask)


def _bn_stats(bn, z, part, res_ss=None):
    """BN-forward statistics + finalize only (running stats updated, [mean|rstd|scale|shift])."""
    return raw.bn_fwd_stats(z, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, bn.momentum, part)


def _fold_site(K, N):
    """Whether a BN apply is folded into a 1x1 GEMM of reduction K and N output channels.
    The transform-A core (ca_gemm_xa.h) repeats the BN transform for every N tile and has no
    operand pipeline for a single K tile; measured on MI355X (ResNet-50, b1024) only the long-K,
    narrow-N sites beat the separate BN pass (docs/performance.md, round 4); since round 6 stage 3's
    N = 256 sites run on 128 x 256 tiles with two K tiles in flight (ca_gemm_xa.h mfma_gemm_xa_deep)
    and pay too."""
    if config.get("CLOUD_AMD_BN_FOLD_ALL"):
        return True
    return K >= 2 * N and N <= config.get("CLOUD_AMD_BN_FOLD_MAX_N")


def _fold_conv(conv, src, ss, side, mask, res=None, res_ss=None):
    """1x1 forward conv whose input BN(+residual)+ReLU apply runs in its operand fetch; the
    applied input is written once to ``side`` (+ ReLU bitmask ``mask``).  Returns (z, partials)."""
    N, H, W, _ = src.shape
    part = raw.stats_buffer(N * H * W, conv.cout, src.device)
    z = raw.conv1x1_fwd_bnapply(src, ss, conv.weight, side, mask, res=res, res_ss=res_ss, stats=part)
    return z, part


class _BottleneckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blk, prev_src, pend, defer, *params):
        # prev_src: (z, mask) of the BatchNorm+ReLU that produced x (the previous fused
        # block's bn3), or None -- this block's backward computes its statistics.
        # pend: the previous block's bn3 apply, deferred into this block's conv1 (x is its
        # still-unwritten output buffer); defer: leave this block's own bn3 apply to the next.
        ctx.prev_src = prev_src
        ds = blk.downsample
        fold = config.get("CLOUD_AMD_BN_FOLD_FWD")
        if pend is not None:
            z1, part1 = _fold_conv(blk.conv1, pend["z"], pend["ss"], x, pend["mask"], res=pend["res"],
                                   res_ss=pend["res_ss"])
            y1, st1, m1 = raw.bn_fwd(z1, blk.bn1.weight, blk.bn1.bias, blk.bn1.running_mean, blk.bn1.running_var,
                                     blk.bn1.eps, blk.bn1.momentum, blk.bn1.relu, partials=part1, keep_mask=True)
            s1 = (st1, m1)
        else:
            z1, y1, s1 = _conv_bn(blk.conv1, blk.bn1, x)
        c2, c3 = blk.conv2, blk.conv3
        N, H2, W2 = x.shape[0], raw.out_hw(x.shape[1], 3, c2.stride, 1), raw.out_hw(x.shape[2], 3, c2.stride, 1)
        if fold and not raw.uses_prw(N * H2 * W2, c3.cout, c2.cout) and _fold_site(c2.cout, c3.cout):
            # bn2 + ReLU applied in conv3's operand fetch (y2 written once, by that GEMM)
            part2 = raw.conv_stats_buffer(y1.shape, c2.weight, c2.stride, c2.padding, x.device)
            z2 = raw.conv_fwd(y1, c2.weight, c2.stride, c2.padding, stats=part2)
            st2 = _bn_stats(blk.bn2, z2, part2)
            y2 = torch.empty_like(z2)
            m2 = torch.empty((z2.numel() // z2.shape[-1], z2.shape[-1] // 8), dtype=torch.uint8, device=x.device)
            s2 = (st2, m2)
            C2 = z2.shape[-1]
            z3_part = _fold_conv(c3, z2, st2[2 * C2:4 * C2], y2, m2)
        else:
            z2, y2, s2 = _conv_bn(blk.conv2, blk.bn2, y1)
            z3_part = None
        if ds is not None:
            # projection shortcut: its BN is folded into bn3's apply (statistics only here;
            # the shortcut BN output is never written)
            c, bnd = ds["conv"], ds["bn"]
            part_d = raw.conv_stats_buffer(x.shape, c.weight, c.stride, c.padding, x.device)
            zd = raw.conv_fwd(x, c.weight, c.stride, c.padding, stats=part_d)
            st_d = raw.bn_fwd_stats(zd, bnd.weight, bnd.bias, bnd.running_mean, bnd.running_var, bnd.eps,
                                    bnd.momentum, part_d)
            sd = (st_d, None)
            bn3 = blk.bn3
            if z3_part is not None:
                z3, part3 = z3_part
            else:
                part3 = raw.conv_stats_buffer(y2.shape, c3.weight, c3.stride, c3.padding, x.device)
                z3 = raw.conv_fwd(y2, c3.weight, c3.stride, c3.padding, stats=part3)
            C3 = c3.cout
            res, res_ss = zd, st_d[2 * C3:4 * C3]
        else:
            zd, sd = None, None
            bn3 = blk.bn3
            if z3_part is not None:
                z3, part3 = z3_part
            else:
                part3 = raw.conv_stats_buffer(y2.shape, c3.weight, c3.stride, c3.padding, x.device)
                z3 = raw.conv_fwd(y2, c3.weight, c3.stride, c3.padding, stats=part3)
            C3 = c3.cout
            res, res_ss = x, None
        if defer:
            # bn3 (+ residual) + ReLU is applied by the next block's conv1 operand fetch, which
            # also writes `out` and the ReLU mask: only the statistics here
            st3 = _bn_stats(bn3, z3, part3)
            out = torch.empty_like(z3)
            mask3 = torch.empty((z3.numel() // C3, C3 // 8), dtype=torch.uint8, device=x.device)
            blk._ca_pending = {"z": z3, "res": res, "ss": st3[2 * C3:4 * C3], "res_ss": res_ss, "mask": mask3}
        else:
            out, st3, mask3 = raw.bn_fwd(z3, bn3.weight, bn3.bias, bn3.running_mean, bn3.running_var, bn3.eps,
                                         bn3.momentum, bn3.relu, residual=res, partials=part3, keep_mask=True,
                                         residual_ss=res_ss)
        s3 = (st3, mask3)
        if ds is None:
            sd = None
        ctx.blk = blk
        (s1, m1), (s2, m2), (s3, m3) = s1, s2, s3
        ctx.save_for_backward(x, z1, y1, z2, y2, z3, s1, m1, s2, m2, s3, m3,
                              *((zd, sd[0]) if ds is not None else ()))
        # (z3, m3[, zd]): the next block's conv1 dgrad epilogue computes this block's bn3
        # backward statistics -- and the shortcut BN's, whose input zd sees the same gradient
        blk._ca_out_src = (z3, m3, zd) if ds is not None else (z3, m3)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..parallel import ddp

        blk = ctx.blk
        ds = blk.downsample
        saved = ctx.saved_tensors
        x, z1, y1, z2, y2, z3, s1, m1, s2, m2, s3, m3 = saved[:12]
        dout = dout.contiguous()

        epi = config.get("CLOUD_AMD_BN_BWD_EPILOGUE")

        def bn_back(bn, dy, z, st, want_dres=False, partials=None, gate=None):
            """``gate``: a ReLU bitmask applied to dy on load (the shortcut BN of a projection
            block gets dout gated by the block's output ReLU, never a materialised copy)."""
            stats, mask = st
            relu = bn.relu
            if gate is not None:
                assert not bn.relu
                relu, mask = True, gate
            r = raw.bn_bwd(dy, None, z, bn.weight, stats, relu, dgamma=bn.weight.grad, dbeta=bn.bias.grad,
                           want_dres=want_dres, accumulate=1, mask=mask, partials=partials)
            ddp.notify_grad_ready(bn.weight)
            ddp.notify_grad_ready(bn.bias)
            return r

        def dgrad(conv, dz, shape, bn_src, out=None, beta=0.0, res=None, beta_stride=1):
            """Input gradient; with ``bn_src`` = (z, mask[, z2]) of the BN(s) that consume it,
            also their backward statistics from the epilogue.  Returns (dx, partials,
            partials2); z2 is honoured by the residual-gated (``res``) form only."""
            bn = bn_src if (epi and bn_src is not None) else None
            if bn is not None and res is None:
                bn = bn[:2]
            r = raw.conv_dgrad(dz, conv.weight, shape, conv.stride, conv.padding, out=out, beta=beta, bn=bn,
                               res=res, beta_stride=beta_stride)
            if bn is None:
                return r, None, None
            return (r[0], r[1], r[2] if len(r) > 2 else None)

        side = SideWork(x.device)
        deferred = []

        def wgrad(conv, dz, inp):
            side.run(lambda: raw.conv_wgrad(dz, inp, conv.weight.shape, conv.stride, conv.padding,
                                            out=conv.weight.grad, beta=1.0), dz, inp)
            if side.enabled:
                deferred.append(conv.weight)
            else:
                ddp.notify_grad_ready(conv.weight)

        # the residual gradient dout * relu'(m3) is never materialised: identity blocks gate
        # it in conv1's dgrad epilogue (res=), projection blocks in the shortcut BN backward
        gate_res = m3 is not None
        p3, p_short = _take(dout) if epi else (None, None)
        fold = epi and config.get("CLOUD_AMD_BN_FOLD")

        def bn_coef(bn, z, st, partials):
            """BN backward finalize only: dgamma / dbeta into the arena, [A | B | D] for the
            apply that runs in the consuming dgrad GEMM's operand fetch (ca_gemm_xa.h)."""
            C = z.shape[-1]
            coef = raw.bn_bwd_coef(C, z.numel() // C, bn.weight, st, partials, dgamma=bn.weight.grad,
                                   dbeta=bn.bias.grad, accumulate=1)
            ddp.notify_grad_ready(bn.weight)
            ddp.notify_grad_ready(bn.bias)
            return coef

        if fold and p3 is not None and gate_res and _fold_site(blk.conv3.cout, blk.conv3.cin):
            # bn3's backward apply folded into conv3's input-gradient GEMM: dz3 is produced in
            # its operand fetch (and written once, for the weight gradient), never read back
            coef3 = bn_coef(blk.bn3, z3, s3, p3)
            dres = None
            c3 = blk.conv3
            if (config.get("CLOUD_AMD_BN_FOLD_WGRAD") and raw.dgrad_wgrad_fusable(c3.cout, c3.cin)
                    and (c3.cin == 64 or config.get("CLOUD_AMD_BN_FOLD_WGRAD2"))):
                # ... and conv3's weight gradient in the same pass: dz3 never reaches memory
                dy2, p2 = raw.conv1x1_dgrad_wgrad_bnbwd(dout, z3, m3, coef3, c3.weight, y2, c3.weight.grad,
                                                        bn=(z2, m2), dw_beta=1.0)
                ddp.notify_grad_ready(c3.weight)
                dz3 = None
            else:
                dz3 = torch.empty_like(z3)
                dy2, p2 = raw.conv1x1_dgrad_bnbwd(dout, z3, m3, coef3, c3.weight, dz3, bn=(z2, m2))
        else:
            dz3, dres = bn_back(blk.bn3, dout, z3, (s3, m3), want_dres=not gate_res, partials=p3)
            dy2, p2, _ = dgrad(blk.conv3, dz3, y2.shape, (z2, m2))
        if dz3 is not None:
            wgrad(blk.conv3, dz3, y2)
        del dz3
        dz2, _ = bn_back(blk.bn2, dy2, z2, (s2, m2), partials=p2)
        del dy2, p2
        dy1, p1, _ = dgrad(blk.conv2, dz2, y1.shape, (z1, m1))
        wgrad(blk.conv2, dz2, y1)
        del dz2
        coef1 = None
        c1 = blk.conv1
        # stage 1: bn1's backward apply, conv1's input gradient AND its weight gradient in one
        # pass (dz1 never written); elsewhere the long-K fold or the separate passes
        fuse1 = (fold and p1 is not None and config.get("CLOUD_AMD_BN_FOLD_WGRAD1")
                 and raw.dgrad_wgrad_fusable(c1.cout, c1.cin))
        if fuse1:
            coef1 = bn_coef(blk.bn1, z1, s1, p1)
            dz1 = None
        elif fold and p1 is not None and _fold_site(blk.conv1.cout, blk.conv1.cin):
            coef1 = bn_coef(blk.bn1, z1, s1, p1)  # bn1's apply runs in conv1's dgrad below
            dz1 = torch.empty_like(z1)
        else:
            dz1, _ = bn_back(blk.bn1, dy1, z1, (s1, m1), partials=p1)
            del dy1
        del p1
        dx_stride = 1  # > 1: dx holds the strided shortcut's one parity class only (below)
        if ds is not None:
            zd, sd = saved[12], saved[13]
            c = ds["conv"]
            if (fold and gate_res and p_short is not None and config.get("CLOUD_AMD_BN_FOLD_WGRAD_DS")
                    and raw.is_gemm_conv(c.weight, c.stride, c.padding) and raw.dgrad_wgrad_fusable(c.cout, c.cin)):
                # stage-1 projection shortcut: its BN backward (gated by the block output's ReLU),
                # the shortcut conv's input gradient and its weight gradient in one pass -- the
                # shortcut's dz is never written
                coefd = bn_coef(ds["bn"], zd, sd, p_short)
                dx = raw.conv1x1_dgrad_wgrad_bnbwd(dout, zd, m3, coefd, c.weight, x, c.weight.grad, dw_beta=1.0)
                ddp.notify_grad_ready(c.weight)
                del dres
            else:
                # strided 1x1 shortcut: only its one non-empty parity class is written; conv1's
                # input gradient below reads the other pixels as zeros (never stored)
                sparse = (coef1 is None and c.stride > 1 and c.padding == 0 and c.weight.shape[1:3] == (1, 1)
                          and config.get("CLOUD_AMD_DS_SPARSE_DGRAD"))
                if (sparse and fold and gate_res and p_short is not None and c.cout <= 2048
                        and config.get("CLOUD_AMD_BN_FOLD_DS")):
                    # ... and its BN backward (gated by the block output's ReLU) in that GEMM's
                    # operand fetch: dzd is written once (the weight gradient's operand), never read
                    coefd = bn_coef(ds["bn"], zd, sd, p_short)
                    dzd = torch.empty_like(zd)
                    dx = raw.conv1x1_strided_dgrad_bnbwd(dout, zd, m3, coefd, c.weight, dzd, x.shape, c.stride)
                else:
                    if gate_res:
                        dzd, _ = bn_back(ds["bn"], dout, zd, (sd, None), gate=m3, partials=p_short)
                    else:
                        dzd, _ = bn_back(ds["bn"], dres, zd, (sd, None))
                    dx = raw.conv_dgrad(dzd, c.weight, x.shape, c.stride, c.padding, skip_empty=sparse)
                del dres
                dx_stride = c.stride if sparse else 1
                wgrad(c, dzd, x)
                del dzd
        elif gate_res:
            dx = torch.empty_like(x)  # = conv1's input gradient + dout * relu'(m3), one epilogue
        else:
            dx = dres  # identity gradient; conv1's input gradient is summed into it below
        # the last write of dx: its epilogue sees the complete block-input gradient
        res1 = (dout, m3) if (gate_res and ds is None) else None
        if coef1 is not None:
            bn_src = ctx.prev_src
            if bn_src is not None and res1 is None:
                bn_src = bn_src[:2]
            if fuse1:
                r = raw.conv1x1_dgrad_wgrad_bnbwd(dy1, z1, m1, coef1, c1.weight, x, c1.weight.grad, out=dx, beta=1.0,
                                                  bn=bn_src, res=res1, dw_beta=1.0)
                ddp.notify_grad_ready(c1.weight)
            else:
                r = raw.conv1x1_dgrad_bnbwd(dy1, z1, m1, coef1, c1.weight, dz1, out=dx, beta=1.0, bn=bn_src,
                                            res=res1)
            del dy1
            p_prev, p_prev2 = (None, None) if bn_src is None else (r[1], r[2] if len(r) > 2 else None)
        else:
            _, p_prev, p_prev2 = dgrad(blk.conv1, dz1, x.shape, ctx.prev_src, out=dx, beta=1.0, res=res1,
                                       beta_stride=dx_stride)
        del dout
        if p_prev is not None:
            _park(dx, p_prev, p_prev2)
        ctx.prev_src = None
        if dz1 is not None:
            wgrad(blk.conv1, dz1, x)
        # join: later kernels on the main stream (and DDP's bucket events recorded on it)
        # are ordered after this block's weight gradients
        side.join()
        for w in deferred:
            ddp.notify_grad_ready(w)
        return (dx, None, None) + (None,) * (len(ctx.needs_input_grad) - 3)


def _global_hooks():
    """Module hooks registered for EVERY module (``register_module_forward_hook`` / ``_pre_hook``)
    would see a deferred block output before the next block's conv1 writes it."""
    from torch.nn.modules import module as _m

    return bool(_m._global_forward_hooks or _m._global_forward_pre_hooks)


def bottleneck_forward(blk, x, next_blk=None):
    """Run ``blk`` as one autograd node.  ``next_blk``: the fused block that will consume this
    block's output next (ResNet.forward passes it): this block's bn3 apply is then left to that
    block's conv1 (CLOUD_AMD_BN_FOLD_FWD), which writes the output tensor returned here."""
    prev = getattr(x, "_ca_bn_src", None) if config.get("CLOUD_AMD_BN_BWD_EPILOGUE") else None
    pend = x.__dict__.pop("_ca_pending", None)
    defer = (next_blk is not None and config.get("CLOUD_AMD_BN_FOLD_FWD") and not blk._forward_hooks
             and not next_blk._forward_pre_hooks and not _global_hooks()
             and getattr(next_blk, "fused_block", False)
             and can_fuse(next_blk, x) and _fold_site(next_blk.conv1.cin, next_blk.conv1.cout)
             and raw.is_gemm_conv(next_blk.conv1.weight, next_blk.conv1.stride,
                                                            next_blk.conv1.padding))
    out = _BottleneckFn.apply(x, blk, prev, pend, defer, *block_params(blk))
    src = blk.__dict__.pop("_ca_out_src", None)
    if src is not None:
        out._ca_bn_src = src  # (z3, mask3): the next fused block computes bn3's backward statistics
    pending = blk.__dict__.pop("_ca_pending", None)
    if pending is not None:
        out._ca_pending = pending  # `out` is written by next_blk's conv1
    return out


def check_not_pending(x):
    """A tensor whose BN apply was deferred to a fused consumer must never reach another op."""
    if "_ca_pending" in getattr(x, "__dict__", {}):
        raise RuntimeError("internal error: a deferred BatchNorm output reached a non-fused consumer")
