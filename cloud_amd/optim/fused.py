"""Fused optimizers over flat arenas (K4 Adam/AdamW, K5 SGD(+momentum), K6 RMSprop).

One HIP launch per arena segment (decayed / non-decayed) updates the fp32
master weights, the optimizer state and the bf16 model copy in a single pass.
``step()`` passes the hyper-parameters by value in the kernel arguments (no
host-to-device copy, no stream synchronisation per step); the hipGraph-capturable
path (:meth:`prepare_step` + :meth:`step_kernels`) reads them from a tiny device
array refreshed before each replay.  With ``fuse_zero_grad`` (default) the update
kernel also zeroes the gradient elements it consumed, and the next ``zero_grad()``
skips its fill pass (the arena is known clean).
On CPU the same math runs as PyTorch ops on the flat buffers (reference path
for the numerics tests).

API parity: ``tf.keras.optimizers.{SGD, Adam, RMSprop}`` as used by the
reference workloads (``mnist_example_using_fit.py:67``,
``cloud_fit/tests/unit/client_test.py:87-89``,
``keras_tuner_cifar_example.py:66-77``) -- ``learning_rate`` may be a float or
a schedule callable ``lr(step)``.
"""
from __future__ import annotations

import math
import weakref

import torch

from ..ops import _ext
from .arena import build_arenas, reattach_grads, zero_grads


class _OwnerRef:
    """``param._ca_opt``: a weak reference to the optimizer whose arenas hold the parameter.
    Pickles (model save via cloudpickle, checkpoints) as a dead reference: an optimizer is
    never serialised through its parameters."""

    __slots__ = ("_ref",)

    def __init__(self, opt=None):
        self._ref = weakref.ref(opt) if opt is not None else None

    def __call__(self):
        return self._ref() if self._ref is not None else None

    def __reduce__(self):
        return (_OwnerRef, ())


class FusedOptimizer:
    kind = "base"

    def __init__(self, params, learning_rate=1e-3, weight_decay=0.0, grad_scale=1.0, decay_fn=None,
                 clipnorm=None):
        from ..runtime import host

        host.configure()
        if isinstance(params, torch.nn.Module):
            named = list(params.named_parameters())
        else:
            named = [(f"p{i}", p) for i, p in enumerate(params)]
        kw = {} if decay_fn is None else {"decay_fn": decay_fn}
        self.arenas = build_arenas(named, **kw)
        self.learning_rate = learning_rate
        self.weight_decay = float(weight_decay)
        self.grad_scale = float(grad_scale)
        self.clipnorm = clipnorm
        self.iterations = 0
        self.state = [self._init_state(a) for a in self.arenas]
        self._hp = {}
        self.fuse_zero_grad = True
        self._grads_clean = True  # arenas are allocated zeroed
        # gradient all-reduce engine attached by the training loop that owns this optimizer
        # (Keras fit, apply_gradients); tf.GradientTape finds it through the parameters
        self.reducer = None
        owner = _OwnerRef(self)
        for a in self.arenas:
            for s in a.slots:
                s.param._ca_opt = owner
        # Bounded host run-ahead as a property of the step itself (runtime/step_pacer.py):
        # every loop that steps this optimizer -- Keras fit, custom loops, strategy.run,
        # user scripts -- queues at most CLOUD_AMD_MAX_STEPS_IN_FLIGHT steps ahead of the GPU.
        self.pacer = None
        if self.arenas and self.arenas[0].master.is_cuda:
            from ..runtime.step_pacer import StepPacer

            self.pacer = StepPacer(self.arenas[0].device)

    # -- hyper-parameters ---------------------------------------------------
    @property
    def lr(self) -> float:
        lr = self.learning_rate
        return float(lr(self.iterations)) if callable(lr) else float(lr)

    @lr.setter
    def lr(self, v):
        self.learning_rate = v

    def _hp_values(self, wd):  # pragma: no cover - overridden
        raise NotImplementedError

    def _hp_tensor(self, ai, seg, wd):
        vals = self._hp_values(wd)
        key = (ai, seg)
        dev = self.arenas[ai].device
        t = self._hp.get(key)
        host = torch.tensor(vals, dtype=torch.float32)
        if t is None:
            t = host.to(dev)
            self._hp[key] = t
        else:
            t.copy_(host, non_blocking=False)
        return t

    def _segments(self, a):
        segs = []
        if a.n_decay > 0:
            segs.append((0, a.n_decay, self.weight_decay))
        if a.n > a.n_decay:
            segs.append((a.n_decay, a.n, 0.0))
        return segs

    # -- public API -----------------------------------------------------------
    def zero_grad(self, set_to_none=False):
        if self._grads_clean:
            # the last native step zeroed every gradient it consumed; skip the fill once
            # (a second zero_grad before the next step fills as usual)
            self._grads_clean = False
            return
        zero_grads(self.arenas)

    def parameters(self):
        for a in self.arenas:
            for s in a.slots:
                yield s.param

    def prepare_step(self):
        """Refresh device hyper-parameters (call OUTSIDE a graph capture)."""
        for ai, a in enumerate(self.arenas):
            for seg, (_, _, wd) in enumerate(self._segments(a)):
                self._hp_tensor(ai, seg, wd)

    def step_kernels(self):
        """Launch the update kernels (graph-capturable; uses current device hp)."""
        for ai, a in enumerate(self.arenas):
            for seg, (lo, hi, wd) in enumerate(self._segments(a)):
                hp = self._hp.get((ai, seg))
                if hp is None:
                    hp = self._hp_tensor(ai, seg, wd)
                self._update(ai, a, lo, hi, hp, None)
        self._after_update()

    # -- per-slice update (driven by the DP engine, parallel/ddp.attach_optimizer) ------------
    def sliced_begin(self):
        """Open a step whose update is issued slice by slice: count the iteration and freeze
        this step's hyper-parameters (one host computation per distinct weight decay)."""
        self.iterations += 1
        self._slice_hv = {}
        self._slice_ai = {id(a): i for i, a in enumerate(self.arenas)}

    def sliced_update(self, arena, lo, hi):
        """Update elements [lo, hi) of ``arena`` (a gradient bucket) on the current stream;
        a slice that straddles the decayed / non-decayed boundary is split there."""
        ai = self._slice_ai[id(arena)]
        for slo, shi, wd in self._segments(arena):
            a, b = max(lo, slo), min(hi, shi)
            if a >= b:
                continue
            hv = self._slice_hv.get(wd)
            if hv is None:
                hv = self._slice_hv[wd] = [float(v) for v in self._hp_values(wd)]
            self._update(ai, arena, a, b, None, hv)

    def update_bytes_per_elem(self, arena):
        """HBM bytes one element of ``arena`` moves through the fused update (master read +
        write, optimizer state read + write, gradient read + in-kernel zero, model-copy
        write): the DP engine's overlap budget prices an update slice with it."""
        ai = self.arenas.index(arena)
        st = self.state[ai]
        b = 2 * arena.master.element_size() + 2 * arena.grad.element_size()
        b += sum(2 * t.element_size() for t in st.values() if t.numel() == arena.n)
        if arena.model is not None:
            b += arena.model.element_size()
        return b

    def sliced_end_pending(self):
        """Every slice of this step has been issued: the next ``step()`` only closes it."""
        self._sliced_done = True

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if getattr(self, "_sliced_done", False):
            # the DP engine already issued this step's update bucket by bucket (and the compute
            # stream joined it); only the bookkeeping and the run-ahead bound remain
            self._sliced_done = False
            self._after_update()
            if self.pacer is not None:
                self.pacer.step_done()
            return loss
        if self.clipnorm is not None:
            self._clip()
        self.iterations += 1
        for ai, a in enumerate(self.arenas):
            for lo, hi, wd in self._segments(a):
                self._update(ai, a, lo, hi, None, [float(v) for v in self._hp_values(wd)])
        self._after_update()
        if self.pacer is not None:
            self.pacer.step_done()
        return loss

    def _zero_in_kernel(self, a):
        return self.fuse_zero_grad and self._use_native(a)

    def _after_update(self):
        self._grads_clean = bool(self.arenas) and all(self._zero_in_kernel(a) for a in self.arenas)

    def _clip(self):
        tot = 0.0
        for a in self.arenas:
            tot += float(a.grad.float().pow(2).sum())
        norm = math.sqrt(tot) * self.grad_scale
        if norm > self.clipnorm:
            for a in self.arenas:
                a.grad.mul_(self.clipnorm / (norm + 1e-6))

    def reattach(self):
        reattach_grads(self.arenas)

    # -- checkpointing ---------------------------------------------------------
    def state_dict(self):
        return {
            "kind": self.kind,
            "iterations": self.iterations,
            "masters": [a.master.detach().cpu() for a in self.arenas],
            "state": [{k: v.detach().cpu() for k, v in st.items()} for st in self.state],
        }

    def load_state_dict(self, sd):
        self.iterations = int(sd["iterations"])
        with torch.no_grad():
            for a, m, st_src, st in zip(self.arenas, sd["masters"], sd["state"], self.state):
                a.master.copy_(m)
                if a.model is not None:
                    a.model.copy_(a.master)
                for k, v in st_src.items():
                    st[k].copy_(v)

    def _use_native(self, a):
        return a.master.is_cuda and _ext.use_native(a.master)


class SGD(FusedOptimizer):
    kind = "sgd"

    def __init__(self, params, learning_rate=0.01, momentum=0.0, nesterov=False, dampening=0.0, **kw):
        self.momentum, self.nesterov, self.dampening = float(momentum), bool(nesterov), float(dampening)
        super().__init__(params, learning_rate=learning_rate, **kw)

    def _init_state(self, a):
        return {"momentum": torch.zeros(a.n, dtype=torch.float32, device=a.device)} if self.momentum else {}

    def _hp_values(self, wd):
        return [self.lr, self.momentum, self.dampening, wd, self.grad_scale, 1.0 if self.iterations <= 1 else 0.0]

    def _update(self, ai, a, lo, hi, hp, hv):
        st = self.state[ai]
        m = st.get("momentum")
        if self._use_native(a):
            ext = _ext.load(required=True)
            es = a.grad.element_size()
            ext.sgd_step(a.master.data_ptr() + 4 * lo, a.grad.data_ptr() + es * lo, int(a.grad.dtype == torch.bfloat16),
                         0 if m is None else m.data_ptr() + 4 * lo,
                         0 if a.model is None else a.model.data_ptr() + a.model.element_size() * lo,
                         0 if hp is None else hp.data_ptr(), hv or [], hi - lo, int(self.nesterov),
                         int(self._zero_in_kernel(a)), _ext.stream_handle(a.device))
            return
        lr, mom, damp, wdv, gs, first = hp.tolist() if hp is not None else hv
        p = a.master[lo:hi]
        g = a.grad[lo:hi].float() * gs + wdv * p
        if mom:
            mm = m[lo:hi]
            if first:
                mm.copy_(g)
            else:
                mm.mul_(mom).add_(g, alpha=1 - damp)
            g = g + mom * mm if self.nesterov else mm
        p.sub_(lr * g)
        if a.model is not None:
            a.model[lo:hi].copy_(p)


class Adam(FusedOptimizer):
    kind = "adam"

    def __init__(self, params, learning_rate=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7, decoupled=False, **kw):
        self.beta_1, self.beta_2, self.epsilon, self.decoupled = float(beta_1), float(beta_2), float(epsilon), decoupled
        super().__init__(params, learning_rate=learning_rate, **kw)

    def _init_state(self, a):
        return {"m": torch.zeros(a.n, dtype=torch.float32, device=a.device),
                "v": torch.zeros(a.n, dtype=torch.float32, device=a.device)}

    def _hp_values(self, wd):
        t = max(self.iterations, 1)
        return [self.lr, self.beta_1, self.beta_2, self.epsilon, wd, self.grad_scale,
                1.0 - self.beta_1 ** t, 1.0 - self.beta_2 ** t]

    def _update(self, ai, a, lo, hi, hp, hv):
        st = self.state[ai]
        if self._use_native(a):
            ext = _ext.load(required=True)
            es = a.grad.element_size()
            ext.adam_step(a.master.data_ptr() + 4 * lo, a.grad.data_ptr() + es * lo, int(a.grad.dtype == torch.bfloat16),
                          st["m"].data_ptr() + 4 * lo, st["v"].data_ptr() + 4 * lo,
                          0 if a.model is None else a.model.data_ptr() + a.model.element_size() * lo,
                          0 if hp is None else hp.data_ptr(), hv or [], hi - lo, int(self.decoupled),
                          int(self._zero_in_kernel(a)), _ext.stream_handle(a.device))
            return
        lr, b1, b2, eps, wdv, gs, bc1, bc2 = hp.tolist() if hp is not None else hv
        p = a.master[lo:hi]
        g = a.grad[lo:hi].float() * gs
        if not self.decoupled:
            g = g + wdv * p
        m, v = st["m"][lo:hi], st["v"][lo:hi]
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        upd = (m / bc1) / ((v / bc2).sqrt() + eps)
        if self.decoupled:
            upd = upd + wdv * p
        p.sub_(lr * upd)
        if a.model is not None:
            a.model[lo:hi].copy_(p)


class AdamW(Adam):
    kind = "adamw"

    def __init__(self, params, learning_rate=1e-3, weight_decay=0.01, **kw):
        super().__init__(params, learning_rate=learning_rate, weight_decay=weight_decay, decoupled=True, **kw)


class RMSprop(FusedOptimizer):
    kind = "rmsprop"

    def __init__(self, params, learning_rate=1e-3, rho=0.9, momentum=0.0, epsilon=1e-7, **kw):
        self.rho, self.momentum, self.epsilon = float(rho), float(momentum), float(epsilon)
        super().__init__(params, learning_rate=learning_rate, **kw)

    def _init_state(self, a):
        st = {"ms": torch.zeros(a.n, dtype=torch.float32, device=a.device)}
        if self.momentum:
            st["mom"] = torch.zeros(a.n, dtype=torch.float32, device=a.device)
        return st

    def _hp_values(self, wd):
        return [self.lr, self.rho, self.epsilon, wd, self.grad_scale, self.momentum]

    def _update(self, ai, a, lo, hi, hp, hv):
        st = self.state[ai]
        buf = st.get("mom")
        if self._use_native(a):
            ext = _ext.load(required=True)
            es = a.grad.element_size()
            ext.rmsprop_step(a.master.data_ptr() + 4 * lo, a.grad.data_ptr() + es * lo,
                             int(a.grad.dtype == torch.bfloat16), st["ms"].data_ptr() + 4 * lo,
                             0 if buf is None else buf.data_ptr() + 4 * lo,
                             0 if a.model is None else a.model.data_ptr() + a.model.element_size() * lo,
                             0 if hp is None else hp.data_ptr(), hv or [], hi - lo, int(self._zero_in_kernel(a)),
                             _ext.stream_handle(a.device))
            return
        lr, rho, eps, wdv, gs, mom = hp.tolist() if hp is not None else hv
        p = a.master[lo:hi]
        g = a.grad[lo:hi].float() * gs + wdv * p
        ms = st["ms"][lo:hi]
        ms.mul_(rho).addcmul_(g, g, value=1 - rho)
        upd = g / (ms.sqrt() + eps)
        if mom:
            b = buf[lo:hi]
            b.mul_(mom).add_(upd)
            upd = b
        p.sub_(lr * upd)
        if a.model is not None:
            a.model[lo:hi].copy_(p)


OPTIMIZERS = {"sgd": SGD, "adam": Adam, "adamw": AdamW, "rmsprop": RMSprop}


def get(identifier, params, **kw):
    """Keras-style lookup: ``get("adam", model.parameters(), learning_rate=...)``."""
    if isinstance(identifier, FusedOptimizer):
        return identifier
    cls = OPTIMIZERS[str(identifier).lower()]
    return cls(params, **kw)
