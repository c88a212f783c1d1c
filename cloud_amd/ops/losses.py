"""Fused softmax + sparse categorical cross-entropy (K3/K12).

The HIP kernel computes loss rows, the correct-prediction flags AND the logits
gradient in the forward pass (one read of the logits); backward just scales
the stored gradient by the incoming loss-gradient.  Parity target:
``tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True)`` with
``SUM_OVER_BATCH_SIZE`` / ``compute_average_loss(global_batch_size=...)``
(reference ``core/tests/testdata/mnist_example_using_ctl.py:93-101``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext


# batches up to this many logits take the one-block kernel that also reduces the mean
# loss and the metric sums in place (xent.hip xent_batch_kernel): Keras fit batches, the
# BERT classifier head.  Larger ones (the ResNet-50 head, 1024 x 1000 per GPU) take the
# row-parallel kernel: one workgroup on 1M logits measured 0.98 ms vs 0.013 ms
# (profiles/r3_s14/rn_step_kernels.txt).
_BATCH_KERNEL_MAX = 1 << 17
_UNIT = {}


def unit_seed(device):
    """A persistent 1.0 to pass as ``torch.autograd.backward(loss, grad_tensors=...)``: the
    fused loss recognises it and hands its stored gradient on unscaled (no fill kernel for
    autograd's implicit ones, no multiply)."""
    key = str(device)
    t = _UNIT.get(key)
    if t is None:
        t = _UNIT[key] = torch.ones((), dtype=torch.float32, device=device)
    return t


def backward_with_seed(loss, seed):
    """``torch.autograd.backward(loss, grad_tensors=seed)`` without its Python-side shape
    check: in this torch that check imports ``torch.fx.experimental.symbolic_shapes`` -- and
    with it sympy, 0.86 s cold on the GPU box -- on the first seeded backward of every process
    (every tuner worker's first trial; scripts/debug/cold_trial.py)."""
    if loss.shape != seed.shape:
        raise ValueError(f"seed shape {tuple(seed.shape)} != loss shape {tuple(loss.shape)}")
    try:
        from torch.autograd.graph import _engine_run_backward
    except ImportError:  # pragma: no cover - other torch versions
        return torch.autograd.backward(loss, grad_tensors=seed)
    _engine_run_backward((loss,), (seed,), False, False, (), allow_unreachable=True, accumulate_grad=True)


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, denom, label_smoothing, acc, acc_w):
        # the `correct` output never receives a gradient: no zero tensor materialised for it
        ctx.set_materialize_grads(False)
        ext = _ext.load(required=True)
        B, C = logits.shape
        small = B * C <= _BATCH_KERNEL_MAX
        # the one-block kernel takes strided rows (a padded head's [:, :C] view: no copy)
        z = logits if (small and logits.stride(1) == 1) else logits.contiguous()
        dev = z.device
        correct = torch.empty(B, dtype=torch.float32, device=dev)
        dz = torch.empty((B, C), dtype=z.dtype, device=dev)
        lab = labels.contiguous()
        if small:
            mean = torch.empty(1, dtype=torch.float32, device=dev)
            ext.softmax_xent_batch(z.data_ptr(), z.stride(0), int(z.dtype == torch.bfloat16), lab.data_ptr(), B, C,
                                   1.0 / float(denom), float(label_smoothing), mean.data_ptr(), correct.data_ptr(),
                                   dz.data_ptr(), _ext.ptr(acc), float(acc_w), _ext.stream_handle(dev))
            out = mean.view(())
        else:
            loss = torch.empty(B, dtype=torch.float32, device=dev)
            ext.softmax_xent(z.data_ptr(), int(z.dtype == torch.bfloat16), lab.data_ptr(), B, C,
                             1.0 / float(denom), float(label_smoothing), loss.data_ptr(), correct.data_ptr(),
                             dz.data_ptr(), _ext.stream_handle(dev))
            if acc is not None:
                acc += torch.stack([loss.sum(), correct.sum(), loss.new_tensor(float(B))]) * float(acc_w)
            out = loss.sum() / float(denom)
        ctx.save_for_backward(dz)
        ctx.mark_non_differentiable(correct)
        return out, correct

    @staticmethod
    def backward(ctx, gloss, _gcorrect):
        (dz,) = ctx.saved_tensors
        if gloss is None:  # (grads are not materialised)
            return None, None, None, None, None, None
        u = _UNIT.get(str(gloss.device))
        if u is not None and gloss.data_ptr() == u.data_ptr():
            return dz, None, None, None, None, None
        return dz * gloss.to(dz.dtype), None, None, None, None, None


def softmax_cross_entropy(logits, labels, *, denom=None, label_smoothing=0.0, acc=None, acc_weight=1.0):
    """Return ``(mean_loss, correct_flags)``.

    ``denom`` defaults to the local batch size; pass the GLOBAL batch size to get
    the MultiWorkerMirrored ``compute_average_loss`` convention.  ``acc`` (fp32 [3] on the
    device): ``acc += [sum of row losses, sum of correct flags, rows] * acc_weight``
    inside the loss kernel (Keras loss / accuracy metric state without per-step syncs).
    """
    B = logits.shape[0]
    denom = B if denom is None else denom
    labels = labels.long()
    if logits.dtype in (torch.bfloat16, torch.float32) and _ext.use_native(logits, labels):
        return _XentFn.apply(logits, labels, denom, label_smoothing, acc, acc_weight)
    lf = logits.float()
    per = F.cross_entropy(lf, labels, reduction="none", label_smoothing=label_smoothing)
    correct = (lf.argmax(-1) == labels).float()
    if acc is not None:
        with torch.no_grad():
            acc += torch.stack([per.sum(), correct.sum(), per.new_tensor(float(B))]).to(acc.device) * float(acc_weight)
    return per.sum() / float(denom), correct
