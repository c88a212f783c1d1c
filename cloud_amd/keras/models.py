"""Keras ``Model`` / ``Sequential`` with a data-parallel ``fit`` on MI355X.

Functional (``Model(inputs, outputs)``), sequential and subclassed models are
supported.  ``fit``/``evaluate``/``predict`` run under the current
distribution strategy (:mod:`cloud_amd.parallel.strategy`, installed by the
``run()`` wrapper or by ``strategy.scope()``):

* one process per GPU; the model is broadcast from rank 0 at the first fit;
* ``batch_size`` is the GLOBAL batch -- each replica trains on its
  1/num_replicas slice of every global batch (MirroredStrategy semantics);
* gradients live in the fused optimizer's flat arena and are all-reduced in
  buckets overlapped with backward (:mod:`cloud_amd.parallel.ddp`); the
  1/num_replicas mean is folded into the fused update kernel;
* metric states are all-reduced once per epoch (not per step);
* a final softmax + ``SparseCategoricalCrossentropy`` is trained through the
  fused softmax-xent HIP kernel on the pre-softmax logits;
* checkpoints are written by the chief only and load under any strategy
  (reference ``core/tests/testdata/save_and_load.py:89-125``).
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch

from .. import monitoring, ops
from ..parallel import strategy as strat
from ..utils import trace
from . import callbacks as cbks
from . import losses as losses_mod
from . import metrics as metrics_mod
from . import optimizers as opt_mod
from .data import Dataset
from .engine import KerasTensor, Layer, global_policy

FORMAT = "cloud_amd.keras/1"


def _to_torch(x, device, dtype=None):
    if isinstance(x, dict):
        return {k: _to_torch(v, device, dtype) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_torch(v, device, dtype) for v in x)
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
    if dtype is not None and t.is_floating_point():
        t = t.to(dtype)
    return t.to(device, non_blocking=True)


def _plain_array(a):
    return a is not None and not isinstance(a, (dict, list, tuple, Dataset))


def _device_arrays(x, y, dev, dtype):
    """Array inputs go to the device ONCE per fit (x in the compute dtype, integer labels as
    int64): every step then trains on views of them -- no per-step host slicing, cast or
    host-to-device copy."""
    xt = _to_torch(x, dev, dtype)
    yt = None
    if y is not None:
        yt = _to_torch(y, dev)
        if not yt.is_floating_point():
            yt = yt.long()
    return xt, yt


def _grouped_to_device(items, dev, dtype, group=16):
    """Dataset batches -> device in groups: ``group`` consecutive host batches of one shape
    are concatenated into one pinned buffer and uploaded with ONE asynchronous copy; the
    steps get views.  Pipeline order is unchanged (the group is filled in order)."""
    def key(it):
        xb, yb = np.asarray(it[0]), None if it[1] is None else np.asarray(it[1])
        return (xb.shape[1:], xb.dtype.str, None if yb is None else (yb.shape[1:], yb.dtype.str))

    def emit(buf):
        X = torch.as_tensor(np.concatenate([np.asarray(b[0]) for b in buf]))
        if X.is_floating_point() and dtype is not None:
            X = X.to(dtype)
        X = X.pin_memory().to(dev, non_blocking=True)
        Y = None
        if buf[0][1] is not None:
            Y = torch.as_tensor(np.concatenate([np.asarray(b[1]) for b in buf]))
            if not Y.is_floating_point():
                Y = Y.long()
            Y = Y.pin_memory().to(dev, non_blocking=True)
        off = 0
        for b in buf:
            n = len(np.asarray(b[0]))
            yield X[off:off + n], (None if Y is None else Y[off:off + n]), b[2], b[3]
            off += n

    buf = []
    for it in items:
        if not (_plain_array(it[0]) and (it[1] is None or _plain_array(it[1]))) or \
                isinstance(it[0], torch.Tensor) and it[0].is_cuda:
            yield from emit(buf) if buf else ()
            buf = []
            yield it
            continue
        if buf and (len(buf) == group or key(it) != key(buf[0])):
            yield from emit(buf)
            buf = []
        buf.append(it)
    if buf:
        yield from emit(buf)


def _first(x):
    while isinstance(x, (list, tuple)):
        x = x[0]
    if isinstance(x, dict):
        return next(iter(x.values()))
    return x


def _slice(x, idx):
    if isinstance(x, dict):
        return {k: _slice(v, idx) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_slice(v, idx) for v in x)
    return x[idx]


def _replica_range(n, world, rank):
    """[lo, hi) of replica ``rank``'s slice of an ``n``-row global batch: contiguous
    ceil(n/world) chunks (the last replicas may get fewer rows, or none)."""
    per = -(-n // world)
    lo = min(rank * per, n)
    return lo, min(lo + per, n)


def _length(x):
    return len(_first(x))


class Model(Layer):
    def __init__(self, inputs=None, outputs=None, name=None, **kw):
        super().__init__(name=name, **kw)
        self.stop_training = False
        self.optimizer = None
        self.loss = None
        self.compiled_metrics = []
        self.history = None
        self._strategy = None
        self._dev_acc = None
        self._reducer = None
        self._fused_xent = False
        self._graph = None
        if inputs is not None and outputs is not None:
            self._init_graph(inputs, outputs)

    # ------------------------------------------------------------ functional API
    def _init_graph(self, inputs, outputs):
        ins = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        outs = list(outputs) if isinstance(outputs, (list, tuple)) else [outputs]
        order, seen = [], set()

        def visit(kt):
            if kt.id in seen:
                return
            seen.add(kt.id)
            for p in kt.inputs:
                visit(p)
            order.append(kt)

        for o in outs:
            visit(o)
        layers, lids = [], set()
        for kt in order:
            if kt.layer is not None and not getattr(kt, "is_input", False) and id(kt.layer) not in lids:
                lids.add(id(kt.layer))
                layers.append(kt.layer)
        self._layer_list = torch.nn.ModuleList(layers)
        self._graph = (ins, outs, order)
        self._multi_out = isinstance(outputs, (list, tuple))
        self.built = True

    @property
    def inputs(self):
        if getattr(self, "_sym_in", None) is not None:
            return [self._sym_in]
        return list(self._graph[0]) if self._graph is not None else None

    @property
    def outputs(self):
        if getattr(self, "_sym_out", None) is not None:
            return [self._sym_out]
        return list(self._graph[1]) if self._graph is not None else None

    @property
    def input(self):
        ins = self.inputs
        if not ins:
            raise AttributeError("model has no symbolic input (not built on Input tensors)")
        return ins[0] if len(ins) == 1 else ins

    @property
    def output(self):
        outs = self.outputs
        if not outs:
            raise AttributeError("model has no symbolic output (not built on Input tensors)")
        return outs[0] if len(outs) == 1 else outs

    @property
    def layers(self):
        if self._graph is not None:
            return list(self._layer_list)
        return [m for m in self.children() if isinstance(m, Layer)]

    def get_layer(self, name=None, index=None):
        if index is not None:
            return self.layers[index]
        for layer in self.layers:
            if layer.name == name:
                return layer
        raise ValueError(f"No such layer: {name}")

    def call(self, inputs, training=None):
        if self._graph is None:
            raise NotImplementedError("subclassed models must implement call()")
        ins, outs, order = self._graph
        vals = {}
        xs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
        for kt, x in zip(ins, xs):
            vals[kt.id] = x
        for kt in order:
            if kt.id in vals:
                continue
            args = [vals[p.id] for p in kt.inputs]
            vals[kt.id] = kt.layer(args if len(args) > 1 else args[0], training=training)
        res = [vals[o.id] for o in outs]
        return res if self._multi_out else res[0]

    def __call__(self, inputs, *args, **kwargs):
        out = super().__call__(inputs, *args, **kwargs)
        if isinstance(out, torch.Tensor) and global_policy().name != "float32" and out.is_floating_point() \
                and not getattr(self, "_raw_logits", False):
            out = out.float()
        return out

    def build(self, input_shape):
        self.built = True

    def _dry_build(self, sample_x):
        """Create lazily-built weights with one CPU forward on a single example."""
        if all(getattr(m, "built", True) for m in self.modules() if isinstance(m, Layer)) and \
                any(True for _ in self.parameters()):
            return
        x = _slice(sample_x, slice(0, 1))
        x = _to_torch(x, "cpu", torch.float32)
        was = self.training
        self.eval()
        with torch.no_grad():
            self(x)
        self.train(was)

    # ------------------------------------------------------------------- compile
    def compile(self, optimizer="rmsprop", loss=None, metrics=None, loss_weights=None, run_eagerly=None,
                steps_per_execution=None, **kwargs):
        self.optimizer = opt_mod.get(optimizer)
        self.loss = losses_mod.get(loss) if loss is not None else None
        self.compiled_metrics = [metrics_mod.get(m, self.loss) for m in (metrics or [])]
        self._compiled = True

    def _final_softmax_layer(self):
        from .layers import Activation, Dense

        last = None
        if self._graph is not None:
            last = self._graph[1][0].layer
        elif self.layers:
            last = self.layers[-1]
        if isinstance(last, (Dense, Activation)) and getattr(last.activation, "__name__", "") == "softmax":
            return last
        return None

    # ----------------------------------------------------------------- training
    def _setup(self, sample_x):
        s = strat.get_strategy()
        if self._strategy is s and self.optimizer is not None and self.optimizer.impl is not None:
            return s
        self._strategy = s
        self._dry_build(sample_x)
        self.to(s.device)
        if self.optimizer is None:
            raise RuntimeError("You must compile your model before training/testing.")
        world = s.num_replicas_in_sync
        impl = self.optimizer.bind(self, grad_scale=1.0 / world)
        pend = getattr(self, "_pending_optimizer_state", None)
        if pend and os.path.exists(pend):
            impl.load_state_dict(torch.load(pend, map_location="cpu", weights_only=True))
            self._pending_optimizer_state = None
        from ..parallel.ddp import GradAllReducer

        self._reducer = GradAllReducer(impl.arenas) if world > 1 else None
        impl.reducer = self._reducer
        if self._reducer is not None:
            self._reducer.attach_optimizer(impl)  # RCCL: the update runs per bucket as it joins
            self._reducer.broadcast_parameters()
            self._broadcast_buffers()
        sm = self._final_softmax_layer()
        self._fused_xent = (isinstance(self.loss, losses_mod.SparseCategoricalCrossentropy)
                            and (self.loss.from_logits or sm is not None) and not self._multi_output())
        return s

    def _multi_output(self):
        return self._graph is not None and self._multi_out

    def _broadcast_buffers(self):
        import torch.distributed as dist

        for b in self.buffers():
            t = b.data if b.device.type == "cuda" or dist.get_backend() == "gloo" else b.data.cpu()
            dist.broadcast(t, 0)
            if t is not b.data:
                b.data.copy_(t)

    def _forward_train(self, x, training=True):
        """Logits for the fused loss, in the compute dtype (the kernel reads bf16 directly:
        no fp32 cast of the model output)."""
        sm = self._final_softmax_layer() if (self._fused_xent and not self.loss.from_logits) else None
        if sm is not None:
            sm._emit_logits = True
        self._raw_logits = True
        try:
            return self(x, training=training)
        finally:
            self._raw_logits = False
            if sm is not None:
                sm._emit_logits = False

    def _metrics_fusable(self):
        """Loss and accuracy state kept by the fused loss kernel itself (device accumulator,
        read once per log): fused sparse-xent with only sparse-categorical-accuracy metrics."""
        return self._fused_xent and all(type(m) is metrics_mod.SparseCategoricalAccuracy
                                        for m in self.compiled_metrics)

    def train_step(self, xb, yb, sample_weight=None, loss_weight=1.0, n_real=None):
        """One replica step.  ``loss_weight`` rescales this replica's mean loss so that the
        cross-replica gradient SUM (times the optimizer's 1/world) is the gradient of the
        mean over the GLOBAL batch, whatever the per-replica slice sizes were;
        ``n_real=0`` marks a stand-in batch of a replica whose slice of the global batch
        was empty: it still runs forward/backward (zero-weighted) so every replica
        issues the same collectives, but it does not count in the metrics."""
        dev = self._strategy.device
        x = _to_torch(xb, dev, self._input_dtype())
        y = _to_torch(yb, dev) if yb is not None else None
        impl = self.optimizer.impl
        impl.zero_grad()
        n = _length(x) if n_real is None else n_real
        fused_metrics = False
        with trace.range("forward"):
            if self._fused_xent:
                logits = self._forward_train(x)
                fused_metrics = self._metrics_fusable()
                if fused_metrics and self._dev_acc is None:
                    self._dev_acc = torch.zeros(3, dtype=torch.float32, device=logits.device)
                loss, _ = self.loss.fused_logits_loss(logits, y, acc=self._dev_acc if fused_metrics else None,
                                                      acc_weight=1.0 if n else 0.0)
                pred = logits
            else:
                pred = self(x, training=True)
                loss = self.loss(y, pred, sample_weight)
            reg = self._regularization()
            scaled = loss * loss_weight if loss_weight != 1.0 else loss
            total = scaled + reg if reg is not None else scaled
        with trace.range("backward"):
            if total is loss and self._fused_xent:
                # the fused loss hands its stored gradient on as-is for the unit seed
                ops.backward_with_seed(total, ops.unit_seed(total.device))
            else:
                total.backward()
        if self._reducer is not None:
            with trace.range("allreduce_join"):
                self._reducer.finish()
        with trace.range("optimizer"):
            impl.step()
        if n and not fused_metrics:
            self._loss_tracker.update_state(loss.detach().float().reshape(1), sample_weight=[n])
            with torch.no_grad():
                for m in self.compiled_metrics:
                    m.update_state(y, pred.detach())
        return loss

    def _regularization(self):
        # layers without regularizers report a plain 0.0: leave them out, so an unregularized
        # model's loss stays the fused loss tensor itself (no add kernel, and the unit-seed
        # backward path of train_step applies)
        regs = [r for r in (m.regularization_loss() for m in self.modules() if hasattr(m, "regularization_loss"))
                if torch.is_tensor(r) or r != 0]
        return sum(regs) if regs else None

    def _input_dtype(self):
        return global_policy().compute_dtype

    def _logs(self, prefix="", reduce=True):
        if getattr(self, "_dev_acc", None) is not None:
            # loss / accuracy state accumulated by the fused loss kernel (one sync per log)
            tl, tc, rows = self._dev_acc.tolist()
            self._loss_tracker.set_state([tl, rows])
            for m in self.compiled_metrics:
                m.set_state([tc, rows])
        trackers = [self._loss_tracker] + list(self.compiled_metrics)
        if reduce and self._strategy is not None and self._strategy.num_replicas_in_sync > 1:
            state = torch.tensor([v for m in trackers for v in m.state()], dtype=torch.float64)
            state = self._strategy.reduce(strat.ReduceOp.SUM, state)
            for i, m in enumerate(trackers):
                m.set_state(state[2 * i:2 * i + 2].tolist())
        logs = {prefix + "loss": float(self._loss_tracker.result())}
        for m in self.compiled_metrics:
            logs[prefix + m.name] = float(m.result())
        return logs

    def _reset_metrics(self):
        self._dev_acc = None
        self._loss_tracker = metrics_mod.Mean(name="loss")
        for m in self.compiled_metrics:
            m.reset_state()

    def _batches(self, x, y, batch_size, shuffle, epoch, seed=1234):
        """Yield ``(x, y, n_local, n_global)``: this replica's slice of every global batch.

        Every replica walks the SAME sequence of global batches (arrays: one shared
        permutation; datasets: every replica iterates the dataset, whose unseeded
        shuffles are job-seeded, and cuts its slice) and yields once per global batch,
        so all replicas run the same number of steps and issue the same collectives
        -- the lock-step that TF's MirroredStrategy/MWMS input pipelines guarantee.
        A replica whose slice is empty (global batch smaller than the replica count)
        gets ``n_local == 0`` and a one-row stand-in it trains on with zero weight."""
        s = self._strategy
        world, rank = s.num_replicas_in_sync, s.rank
        if isinstance(x, Dataset):
            for el in x:
                if isinstance(el, (tuple, list)) and len(el) >= 2:
                    ex, ey = el[0], el[1]
                else:
                    ex, ey = el, None
                n = _length(ex)
                if world == 1:
                    yield ex, ey, n, n
                    continue
                lo, hi = _replica_range(n, world, rank)
                if hi > lo:
                    yield _slice(ex, slice(lo, hi)), _slice(ey, slice(lo, hi)), hi - lo, n
                else:
                    yield _slice(ex, slice(0, 1)), _slice(ey, slice(0, 1)), 0, n
            return
        n = _length(x)
        bs = batch_size or 32
        idx = np.random.default_rng(seed + epoch).permutation(n) if shuffle else np.arange(n)
        if isinstance(x, torch.Tensor) and x.is_cuda and (y is None or isinstance(y, torch.Tensor)):
            # device-resident arrays: ONE gather per epoch, then every batch is a view
            if shuffle:
                perm = torch.from_numpy(idx).to(x.device)
                x = x.index_select(0, perm)
                y = y.index_select(0, perm) if y is not None else None
            for start in range(0, n, bs):
                stop = min(start + bs, n)
                gn = stop - start
                if world == 1:
                    yield x[start:stop], (y[start:stop] if y is not None else None), gn, gn
                    continue
                lo, hi = _replica_range(gn, world, rank)
                a, b, real = (start + lo, start + hi, hi - lo) if hi > lo else (start, start + 1, 0)
                yield x[a:b], (y[a:b] if y is not None else None), real, gn
            return
        for start in range(0, n, bs):
            gb = idx[start:start + bs]
            if world == 1:
                yield _slice(x, gb), (_slice(y, gb) if y is not None else None), len(gb), len(gb)
                continue
            lo, hi = _replica_range(len(gb), world, rank)
            mine, real = (np.sort(gb[lo:hi]), hi - lo) if hi > lo else (gb[:1], 0)
            yield _slice(x, mine), (_slice(y, mine) if y is not None else None), real, len(gb)

    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose="auto", callbacks=None, validation_split=0.0,
            validation_data=None, shuffle=True, class_weight=None, sample_weight=None, initial_epoch=0,
            steps_per_epoch=None, validation_steps=None, validation_batch_size=None, validation_freq=1, **kw):
        if validation_split and not isinstance(x, Dataset):
            n = _length(x)
            cut = int(n * (1 - validation_split))
            validation_data = (_slice(x, slice(cut, None)), _slice(y, slice(cut, None)))
            x, y = _slice(x, slice(0, cut)), _slice(y, slice(0, cut))
        sample = x if not isinstance(x, Dataset) else next(iter(x))[0]
        s = self._setup(sample)
        on_gpu = s.device.type == "cuda"
        if on_gpu and _plain_array(x) and (y is None or _plain_array(y)):
            x, y = _device_arrays(x, y, s.device, self._input_dtype())
        verbose = 1 if verbose == "auto" else verbose
        history = cbks.History()
        cb_list = list(callbacks or []) + ([cbks.ProgbarLogger()] if verbose else []) + [history]
        steps = steps_per_epoch
        if steps is None and not isinstance(x, Dataset):
            steps = -(-_length(x) // (batch_size or 32))
        callbacks_ = cbks.CallbackList(cb_list, model=self, params={"epochs": epochs, "steps": steps,
                                                                        "verbose": verbose})
        self.stop_training = False
        self.train()
        callbacks_.on_train_begin({})
        persistent = None

        def batches(epoch):
            it = self._batches(x, y, batch_size, shuffle, epoch)
            if on_gpu and isinstance(x, Dataset):
                it = _grouped_to_device(it, s.device, self._input_dtype())
            return it

        if steps_per_epoch is not None:
            persistent = iter(batches(0))
        from ..utils import faults

        global_step = 0
        from ..runtime import gc_control

        # (the fused optimizer's step() bounds the host run-ahead: runtime/step_pacer.py)
        if getattr(self, "_ca_gc_frozen", False):  # a previous fit ended by an exception
            gc_control.unfreeze()
            self._ca_gc_frozen = False
        for epoch in range(initial_epoch, epochs):
            self._reset_metrics()
            callbacks_.on_epoch_begin(epoch, {})
            it = persistent if persistent is not None else batches(epoch)
            step = 0
            t0 = time.time()
            mon = monitoring.enabled()
            t_prev = time.perf_counter()
            while True:
                if steps_per_epoch is not None and step >= steps_per_epoch:
                    break
                t_get = time.perf_counter()
                try:
                    xb, yb, n_local, n_global = next(it)
                except StopIteration:
                    break
                if mon:
                    monitoring.observe(monitoring.GETNEXT, (time.perf_counter() - t_get) * 1e6)
                callbacks_.on_train_batch_begin(step, {})
                faults.maybe_inject(global_step, rank=s.rank)
                world = s.num_replicas_in_sync
                w = (n_local * world / n_global) if world > 1 else 1.0
                loss = self.train_step(xb, yb, loss_weight=w, n_real=n_local)
                if mon:  # host-side step period (the device queue evens it out over steps)
                    now = time.perf_counter()
                    monitoring.observe(monitoring.STEP_TIME, (now - t_prev) * 1e3)
                    t_prev = now
                callbacks_.on_train_batch_end(step, {"loss": float(loss.detach())} if step % 50 == 0 else {})
                step += 1
                global_step += 1
                if global_step == 3 and gc_control.frozen_count() == 0:
                    # model, optimizer state and kernel caches exist now.  Only when nothing is
                    # frozen yet: gc.unfreeze() at the end is process-wide and must not hand back
                    # objects the caller froze itself (e.g. to keep pages shared after fork)
                    self._ca_gc_frozen = gc_control.freeze() > 0
                if self.stop_training:
                    break
            logs = self._logs()
            logs["epoch_time_s"] = time.time() - t0
            if validation_data is not None and (epoch + 1) % validation_freq == 0:
                vx, vy = (validation_data, None) if isinstance(validation_data, Dataset) else validation_data[:2]
                vlogs = self.evaluate(vx, vy, batch_size=validation_batch_size or batch_size, verbose=0,
                                      steps=validation_steps, return_dict=True, _internal=True)
                logs.update({"val_" + k: v for k, v in vlogs.items()})
                self.train()
            callbacks_.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        callbacks_.on_train_end({})
        if getattr(self, "_ca_gc_frozen", False):
            gc_control.unfreeze()  # this fit's objects may become garbage (tuner workers run many fits)
            self._ca_gc_frozen = False
        self.history = history
        return history

    def evaluate(self, x=None, y=None, batch_size=None, verbose="auto", sample_weight=None, steps=None,
                 callbacks=None, return_dict=False, _internal=False, **kw):
        sample = x if not isinstance(x, Dataset) else next(iter(x))[0]
        if not _internal:
            self._setup(sample)
        dev = self._strategy.device
        saved = (self._loss_tracker, [m.state() for m in self.compiled_metrics], self._dev_acc) \
            if hasattr(self, "_loss_tracker") else None
        self._reset_metrics()
        self.eval()
        if dev.type == "cuda" and _plain_array(x) and (y is None or _plain_array(y)):
            x, y = _device_arrays(x, y, dev, self._input_dtype())  # one upload, not one per batch
        # the training step's fused softmax-xent kernel scores the batch too (loss + accuracy
        # into the device accumulator): no separate softmax / log / nll / argmax kernels
        fused = self._metrics_fusable() and self.loss is not None and sample_weight is None
        with torch.no_grad():
            for i, (xb, yb, n_local, _) in enumerate(self._batches(x, y, batch_size, False, 0)):
                if steps is not None and i >= steps:
                    break
                if n_local == 0:
                    continue  # stand-in row of an empty replica slice: nothing to score
                xt = _to_torch(xb, dev, self._input_dtype())
                yt = _to_torch(yb, dev) if yb is not None else None
                if fused and yt is not None:
                    logits = self._forward_train(xt, training=False)
                    if self._dev_acc is None:
                        self._dev_acc = torch.zeros(3, dtype=torch.float32, device=logits.device)
                    self.loss.fused_logits_loss(logits, yt, acc=self._dev_acc)
                    continue
                pred = self(xt, training=False)
                if self.loss is not None and yt is not None:
                    loss = self.loss(yt, pred)
                    self._loss_tracker.update_state(loss.detach().float().reshape(1), sample_weight=[_length(xt)])
                for m in self.compiled_metrics:
                    m.update_state(yt, pred)
        logs = self._logs()
        if saved is not None and _internal:
            self._loss_tracker = saved[0]
            for m, st in zip(self.compiled_metrics, saved[1]):
                m.set_state(st)
            self._dev_acc = saved[2]
        if return_dict:
            return logs
        vals = list(logs.values())
        return vals[0] if len(vals) == 1 else vals

    def predict(self, x, batch_size=None, verbose="auto", steps=None, callbacks=None, **kw):
        s = strat.get_strategy()
        sample = x if not isinstance(x, Dataset) else next(iter(x))[0]
        if not any(True for _ in self.parameters()):
            self._dry_build(sample)
        dev = s.device
        self.to(dev)
        self.eval()
        outs = []
        bs = batch_size or 32
        with torch.no_grad():
            if isinstance(x, Dataset):
                batches = (el[0] if isinstance(el, (tuple, list)) else el for el in x)
            else:
                n = _length(x)
                batches = (_slice(x, slice(i, i + bs)) for i in range(0, n, bs))
            for i, xb in enumerate(batches):
                if steps is not None and i >= steps:
                    break
                outs.append(self(_to_torch(xb, dev, self._input_dtype()), training=False).float().cpu().numpy())
        return np.concatenate(outs) if outs else np.zeros((0,))

    def predict_on_batch(self, x):
        return self.predict(x, batch_size=_length(x))

    def train_on_batch(self, x, y):
        self._setup(x)
        self._reset_metrics()
        self.train()
        self.train_step(x, y)
        return list(self._logs(reduce=False).values())

    # --------------------------------------------------------------- weights I/O
    def get_weights(self):
        return [t.detach().float().cpu().numpy() for t in list(self.parameters()) + list(self.buffers())]

    def set_weights(self, weights):
        tensors = list(self.parameters()) + list(self.buffers())
        with torch.no_grad():
            for t, w in zip(tensors, weights):
                t.copy_(torch.as_tensor(np.asarray(w)).to(t.dtype).reshape(t.shape))
        self._sync_master()

    def _sync_master(self):
        impl = self.optimizer.impl if self.optimizer is not None else None
        if impl is None:
            return
        with torch.no_grad():
            for a in impl.arenas:
                for sl in a.slots:
                    a.master[sl.offset:sl.offset + sl.numel].copy_(sl.param.detach().reshape(-1).float())

    def save_weights(self, filepath, overwrite=True, save_format=None):
        from .saving import chief_only

        sd = {k: v.detach().cpu() for k, v in self.state_dict().items()}

        def write():
            os.makedirs(os.path.dirname(os.path.abspath(filepath)), exist_ok=True)
            torch.save(sd, filepath)

        chief_only(write)

    def load_weights(self, filepath, by_name=False, skip_mismatch=False):
        sd = torch.load(filepath, map_location="cpu", weights_only=True)
        self._load_state(sd)

    def _load_state(self, sd):
        own = self.state_dict()
        if any(k not in own for k in sd) and any(True for _ in self.parameters()) is False:
            raise ValueError("model must be built before loading weights")
        if not own:
            raise ValueError("model has no weights yet: build it (call it once or fit) before load_weights")
        with torch.no_grad():
            for k, v in sd.items():
                if k in own:
                    own[k].copy_(v.to(own[k].dtype))
        self._sync_master()

    def save(self, filepath, overwrite=True, include_optimizer=True, save_format=None):
        from . import saving

        saving.save_model(self, filepath, include_optimizer=include_optimizer)

    # ---------------------------------------------------------------- summary
    def count_params(self):
        return int(sum(p.numel() for p in self.parameters()))

    def summary(self, print_fn=print):
        print_fn(f'Model: "{self.name}"')
        print_fn("_" * 65)
        print_fn(f"{'Layer (type)':<34}{'Param #':>12}")
        print_fn("=" * 65)
        for layer in self.layers:
            print_fn(f"{layer.name + ' (' + type(layer).__name__ + ')':<34}{layer.count_params():>12,}")
        print_fn("=" * 65)
        tot = self.count_params()
        tr = sum(p.numel() for p in self.parameters() if p.requires_grad)
        print_fn(f"Total params: {tot:,}")
        print_fn(f"Trainable params: {tr:,}")
        print_fn(f"Non-trainable params: {tot - tr:,}")

    def get_config(self):
        if isinstance(self, Sequential):
            return {"name": self.name, "layers": [{"class_name": type(layer).__name__,
                                                   "config": layer.get_config()} for layer in self.layers]}
        raise NotImplementedError("config serialisation is implemented for Sequential models")

    def to_json(self):
        return json.dumps({"class_name": type(self).__name__, "config": self.get_config(), "format": FORMAT})


class Sequential(Model):
    def __init__(self, layers=None, name=None, **kw):
        super().__init__(name=name, **kw)
        self._seq = torch.nn.ModuleList()
        for layer in layers or []:
            self.add(layer)

    @property
    def layers(self):
        return list(self._seq)

    def add(self, layer):
        if isinstance(layer, KerasTensor):
            return
        self._seq.append(layer)
        first = self._seq[0]
        shape = getattr(first, "_input_shape_arg", None)
        if shape is not None:
            self._build_from_shape(shape)

    def pop(self):
        self._seq = torch.nn.ModuleList(list(self._seq)[:-1])

    def _build_from_shape(self, shape):
        x = torch.zeros((1,) + tuple(shape))
        was = self.training
        self.eval()
        with torch.no_grad():
            for layer in self._seq:
                x = layer(x)
        self.train(was)

    def call(self, x, training=None):
        for layer in self._seq:
            x = layer(x, training=training)
        return x

    @classmethod
    def from_config(cls, config):
        from .layers import LAYERS

        m = cls(name=config.get("name"))
        for lc in config["layers"]:
            m.add(LAYERS[lc["class_name"]].from_config(lc["config"]))
        return m


def clone_model(model):
    import copy

    return copy.deepcopy(model)


def load_model(filepath, custom_objects=None, compile=True):
    from . import saving

    return saving.load_model(filepath, compile=compile)
