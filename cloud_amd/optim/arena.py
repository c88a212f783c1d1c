"""Flat parameter/gradient arenas.

All trainable parameters of one dtype live in ONE contiguous buffer, and so do
their gradients.  This is the memory layout the whole MI355X step is built on:

* the fused optimizer (``csrc/kernels/optim.hip``) is one launch per arena
  segment instead of one per tensor;
* the data-parallel engine (:mod:`cloud_amd.parallel.ddp`) all-reduces
  contiguous SLICES of the gradient arena -- the buckets ARE the gradients, so
  there is no flatten/unflatten copy (K14 becomes a no-op);
* checkpoints are a handful of large tensors.

Layout per arena: ``[decayed params | non-decayed params]`` (weight decay is a
per-segment hyper-parameter), each parameter padded to ``ALIGN`` elements so
every slice starts 128-byte aligned for 16-byte vector access.  Parameters are
ordered in REVERSE registration order (≈ reverse forward order) so backward
fills the arena front to back and buckets become ready in order.

For bf16 compute the arena also keeps an fp32 master copy; the module's
parameter ``.data`` is a bf16 view into the model copy that the optimizer
rewrites after each update.  fp32 parameters (BatchNorm, biases of fp32
layers) use the master buffer directly.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

ALIGN = 64


def _pad(n, a=ALIGN):
    return (n + a - 1) // a * a


@dataclass
class Slot:
    param: torch.nn.Parameter
    name: str
    offset: int
    numel: int
    decay: bool
    seq: int = 0  # position in reverse registration order (~ the order backward produces gradients)


@dataclass
class Arena:
    dtype: torch.dtype
    device: torch.device
    slots: list = field(default_factory=list)
    n: int = 0            # total padded elements
    n_decay: int = 0      # elements [0, n_decay) belong to decayed params
    master: torch.Tensor = None   # fp32 [n]
    model: torch.Tensor = None    # dtype [n] (None when dtype is fp32: master IS the model)
    grad: torch.Tensor = None     # dtype [n]

    @property
    def low_precision(self):
        return self.dtype != torch.float32

    def model_flat(self):
        return self.model if self.model is not None else self.master


def default_decay(name: str, p: torch.Tensor) -> bool:
    return p.ndim > 1


def build_arenas(named_params, decay_fn=default_decay):
    """Move ``named_params`` (list of (name, Parameter)) into flat arenas, one per dtype."""
    named_params = [(n, p) for n, p in named_params if p.requires_grad]
    groups: dict = {}
    seq = {}
    for i, (name, p) in enumerate(reversed(named_params)):
        groups.setdefault((p.dtype, p.device), []).append((name, p))
        seq[id(p)] = i
    arenas = []
    for (dtype, device), items in groups.items():
        a = Arena(dtype=dtype, device=device)
        ordered = [it for it in items if decay_fn(*it)] + [it for it in items if not decay_fn(*it)]
        off = 0
        for name, p in ordered:
            d = decay_fn(name, p)
            a.slots.append(Slot(p, name, off, p.numel(), d, seq[id(p)]))
            off += _pad(p.numel())
            if d:
                a.n_decay = off
        a.n = off
        a.master = torch.zeros(a.n, dtype=torch.float32, device=device)
        if dtype != torch.float32:
            a.model = torch.zeros(a.n, dtype=dtype, device=device)
        a.grad = torch.zeros(a.n, dtype=dtype, device=device)
        flat = a.model_flat()
        with torch.no_grad():
            for s in a.slots:
                src = s.param.detach()
                a.master[s.offset:s.offset + s.numel].copy_(src.reshape(-1).float())
                if a.model is not None:
                    a.model[s.offset:s.offset + s.numel].copy_(src.reshape(-1))
                s.param.data = flat[s.offset:s.offset + s.numel].view_as(src)
                s.param.grad = a.grad[s.offset:s.offset + s.numel].view_as(src)
                s.param._ca_arena = True
        arenas.append(a)
    return arenas


def zero_grads(arenas):
    for a in arenas:
        a.grad.zero_()


def reattach_grads(arenas):
    """Re-point ``param.grad`` at the arena slices (if user code replaced them)."""
    for a in arenas:
        for s in a.slots:
            g = s.param.grad
            if g is None or g.data_ptr() != a.grad[s.offset:].data_ptr():
                if g is not None:
                    a.grad[s.offset:s.offset + s.numel].copy_(g.reshape(-1))
                s.param.grad = a.grad[s.offset:s.offset + s.numel].view_as(s.param)


def sync_model_from_master(arenas):
    with torch.no_grad():
        for a in arenas:
            if a.model is not None:
                a.model.copy_(a.master)
