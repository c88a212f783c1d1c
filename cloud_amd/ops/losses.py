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


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, denom, label_smoothing):
        ext = _ext.load(required=True)
        z = logits.contiguous()
        B, C = z.shape
        dev = z.device
        loss = torch.empty(B, dtype=torch.float32, device=dev)
        correct = torch.empty(B, dtype=torch.float32, device=dev)
        dz = torch.empty_like(z)
        ext.softmax_xent(z.data_ptr(), int(z.dtype == torch.bfloat16), labels.contiguous().data_ptr(), B, C,
                         1.0 / float(denom), float(label_smoothing), loss.data_ptr(), correct.data_ptr(),
                         dz.data_ptr(), _ext.stream_handle(dev))
        ctx.save_for_backward(dz)
        ctx.mark_non_differentiable(correct)
        return loss.sum() / float(denom), correct

    @staticmethod
    def backward(ctx, gloss, _gcorrect):
        (dz,) = ctx.saved_tensors
        return dz * gloss.to(dz.dtype), None, None, None


def softmax_cross_entropy(logits, labels, *, denom=None, label_smoothing=0.0):
    """Return ``(mean_loss, correct_flags)``.

    ``denom`` defaults to the local batch size; pass the GLOBAL batch size to get
    the MultiWorkerMirrored ``compute_average_loss`` convention.
    """
    B = logits.shape[0]
    denom = B if denom is None else denom
    labels = labels.long()
    if logits.dtype in (torch.bfloat16, torch.float32) and _ext.use_native(logits, labels):
        return _XentFn.apply(logits, labels, denom, label_smoothing)
    lf = logits.float()
    per = F.cross_entropy(lf, labels, reduction="none", label_smoothing=label_smoothing)
    correct = (lf.argmax(-1) == labels).float()
    return per.sum() / float(denom), correct
