"""Keras optimizer front-ends (``tf.keras.optimizers``) bound lazily to a model.

``compile(optimizer=Adam(1e-3))`` only records hyper-parameters; at the first
``fit`` the model's parameters are moved into flat arenas and one of the
fused HIP optimizers of :mod:`cloud_amd.optim` is created with
``grad_scale = 1 / num_replicas`` (the data-parallel mean folded into the
update kernel).  Learning-rate schedules are callables ``schedule(step)``.
"""
from __future__ import annotations

from .. import optim as fused


class schedules:  # namespace parity: tf.keras.optimizers.schedules
    class LearningRateSchedule:
        def __call__(self, step):  # pragma: no cover - abstract
            raise NotImplementedError

    class ExponentialDecay(LearningRateSchedule):
        def __init__(self, initial_learning_rate, decay_steps, decay_rate, staircase=False):
            self.lr0, self.steps, self.rate, self.staircase = initial_learning_rate, decay_steps, decay_rate, staircase

        def __call__(self, step):
            p = step / self.steps
            if self.staircase:
                p = int(p)
            return self.lr0 * self.rate ** p

    class PiecewiseConstantDecay(LearningRateSchedule):
        def __init__(self, boundaries, values):
            self.b, self.v = list(boundaries), list(values)

        def __call__(self, step):
            for b, v in zip(self.b, self.v):
                if step <= b:
                    return v
            return self.v[-1]

    class CosineDecay(LearningRateSchedule):
        def __init__(self, initial_learning_rate, decay_steps, alpha=0.0, warmup_steps=0):
            self.lr0, self.steps, self.alpha, self.warm = initial_learning_rate, decay_steps, alpha, warmup_steps

        def __call__(self, step):
            import math

            if self.warm and step < self.warm:
                return self.lr0 * (step + 1) / self.warm
            t = min(step - self.warm, self.steps) / max(self.steps, 1)
            return self.lr0 * ((1 - self.alpha) * 0.5 * (1 + math.cos(math.pi * t)) + self.alpha)


class _Scalar(float):
    """A float that also answers ``.numpy()`` (``model.optimizer.lr.numpy()`` in TF scripts)."""

    def numpy(self):
        return float(self)


class Optimizer:
    fused_cls = None

    def __init__(self, learning_rate=0.001, name=None, clipnorm=None, **kw):
        self.learning_rate = learning_rate
        self.clipnorm = clipnorm
        self.kw = kw
        self.name = name or type(self).__name__
        self._impl = None

    def bind(self, model, grad_scale=1.0):
        self._impl = self.fused_cls(model, learning_rate=self.learning_rate, grad_scale=grad_scale,
                                    clipnorm=self.clipnorm, **self.kw)
        return self._impl

    @property
    def impl(self):
        return self._impl

    def apply_gradients(self, grads_and_vars):
        """Custom-training-loop update (``optimizer.apply_gradients(zip(grads, vars))``).

        On first use the variables move into flat arenas, replicas adopt rank 0's
        weights (TF mirrors variables at creation; here before the first update), and the
        fused HIP optimizer is created with ``grad_scale = 1``: as under TF's
        MirroredStrategy, per-replica gradients are SUMMED across replicas (the loss is
        already divided by the global batch via ``compute_average_loss``).

        The optimizer's :class:`~cloud_amd.parallel.ddp.GradAllReducer` is the hook-driven,
        backward-overlapped one that ``fit`` uses.  Gradients from ``tf.GradientTape`` over
        arena-resident variables arrive already reduced (the tape joined the buckets) and as
        views of the arena: no copy, no second reduction.  Any other gradient tensor is
        copied into its arena slot (a variable given ``None`` gets a zero gradient), and the
        arena is all-reduced here unless the tape already did.
        Reference: ``TFC/core/tests/testdata/mnist_example_using_ctl.py:124-129,150-157``.
        """
        pairs = [(g, v) for g, v in grads_and_vars]
        first = self._impl is None
        if first:
            self._impl = self.fused_cls([v for _, v in pairs], learning_rate=self.learning_rate, grad_scale=1.0,
                                        clipnorm=self.clipnorm, **self.kw)
            self._reducer = None
            from ..parallel.strategy import get_strategy

            if get_strategy().num_replicas_in_sync > 1:
                from ..parallel.ddp import GradAllReducer

                self._reducer = GradAllReducer(self._impl.arenas)
                self._reducer.broadcast_parameters()
                self._impl.reducer = self._reducer
        impl = self._impl
        red = getattr(self, "_reducer", None)
        reduced = red is not None and red.tape_reduced
        if not getattr(impl, "_ca_tape_fresh", False):
            # the arena was not written by a tape this step: slots of variables missing from
            # this call would keep last step's gradient where the update kernel does not zero
            # it (CPU path, fuse_zero_grad=False) -- clear them; a gradient that IS its slot
            # is saved first
            pairs = [(g.clone() if g is not None and v.grad is not None and g.data_ptr() == v.grad.data_ptr()
                      else g, v) for g, v in pairs]
            impl.zero_grad()
        impl._ca_tape_fresh = False
        n_slots = sum(len(a.slots) for a in impl.arenas)
        if len(pairs) < n_slots:
            # a variable left out of this call keeps its weights, as in TF: no gradient
            # (neither a stale one nor the tape's) reaches its slot
            given = {id(v) for _, v in pairs}
            for a in impl.arenas:
                for sl in a.slots:
                    if id(sl.param) not in given and sl.param.grad is not None:
                        sl.param.grad.zero_()
        for g, v in pairs:
            slot = v.grad
            if g is None:
                if slot is not None:
                    slot.zero_()  # TF skips such a variable; a zero gradient is the closest
                continue
            if slot is not None and g.data_ptr() == slot.data_ptr() and g.dtype == slot.dtype \
                    and g.numel() == slot.numel():
                continue  # the tape's in-arena gradient: already in place
            slot.copy_(g.detach().to(slot.dtype).reshape(slot.shape))
        if red is not None:
            if not reduced:
                red.finish()
            red.tape_reduced = False
        impl.step()
        return impl.iterations

    @property
    def lr(self):
        if self._impl is not None:
            return _Scalar(self._impl.lr)
        lr = self.learning_rate
        return _Scalar(lr(0) if callable(lr) else lr)

    @lr.setter
    def lr(self, v):
        self.learning_rate = v
        if self._impl is not None:
            self._impl.lr = v

    @property
    def iterations(self):
        return self._impl.iterations if self._impl is not None else 0

    def get_config(self):
        lr = self.learning_rate
        return {"name": self.name, "learning_rate": lr if not callable(lr) else None, **self.kw}


class SGD(Optimizer):
    fused_cls = fused.SGD

    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, name=None, **kw):
        super().__init__(learning_rate, name, momentum=momentum, nesterov=nesterov, **kw)


class Adam(Optimizer):
    fused_cls = fused.Adam

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, amsgrad=False, name=None, **kw):
        super().__init__(learning_rate, name, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon, **kw)


class AdamW(Optimizer):
    fused_cls = fused.AdamW

    def __init__(self, learning_rate=0.001, weight_decay=0.004, beta_1=0.9, beta_2=0.999, epsilon=1e-7, name=None,
                 **kw):
        super().__init__(learning_rate, name, weight_decay=weight_decay, beta_1=beta_1, beta_2=beta_2,
                         epsilon=epsilon, **kw)


class RMSprop(Optimizer):
    fused_cls = fused.RMSprop

    def __init__(self, learning_rate=0.001, rho=0.9, momentum=0.0, epsilon=1e-7, name=None, **kw):
        super().__init__(learning_rate, name, rho=rho, momentum=momentum, epsilon=epsilon, **kw)


_ALIASES = {"sgd": SGD, "adam": Adam, "adamw": AdamW, "rmsprop": RMSprop}


def get(identifier):
    if isinstance(identifier, Optimizer):
        return identifier
    try:
        return _ALIASES[str(identifier).lower()]()
    except KeyError as e:
        raise ValueError(f"Unknown optimizer {identifier!r}") from e
