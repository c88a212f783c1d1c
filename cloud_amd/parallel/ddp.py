"""Bucketed gradient all-reduce overlapped with backward (C1/C2/C14 in SURVEY.md).

Gradients live in the optimizer's flat arenas (:mod:`cloud_amd.optim.arena`),
so a bucket is simply a contiguous slice ``arena.grad[lo:hi]``: no
flatten/unflatten copies.  Parameters were laid out in reverse forward order,
so backward produces gradients roughly front-to-back through the arena.

Mechanics (one process per GPU, ``torch.distributed`` over RCCL/xGMI):

* a ``post_accumulate_grad`` hook per parameter counts down its bucket;
* a full bucket is launched as an async ``all_reduce(SUM)`` -- RCCL runs it on
  its own stream, ordered after the producing kernels on the compute stream,
  so communication overlaps the rest of backward;
* buckets launch strictly in index order (a ready bucket waits for its
  predecessors), which keeps the collective sequence identical on every rank;
* :meth:`finish` launches whatever is left (unused params) and makes the
  compute stream wait for all outstanding collectives -- no host sync;
* the 1/world mean is NOT a separate pass: it is folded into the optimizer
  kernel's ``grad_scale``.

Transport: ``torch.distributed`` (RCCL backend) by default, or the native C++
RCCL communicator (:mod:`cloud_amd.parallel.comm`, ``CLOUD_AMD_COMM=rccl``) whose
collectives run on a dedicated high-priority stream joined once before the
optimizer step.

Timing (bench JSON ``comm`` / monitoring): every transport records, per bucket, when
its collective started (gradients ready and the comm path free) and when it completed --
GPU events on the comm stream for RCCL (torch.distributed or the native communicator),
host clocks from the work's completion future for gloo / CPU.  ``allreduce_ms`` is the
time the (serial) comm path was busy, ``exposed_comm_ms`` the time from the end of
backward to the last bucket joined; both are finite on every transport.

Bucket size: xGMI on MI355X is 7 point-to-point links per GPU; a ring
all-reduce moves 2(N-1)/N of the bucket per link, so ~25-64 MB buckets keep
RCCL's multi-channel rings busy while leaving enough buckets (>= 4-8 for
ResNet-50's 51 MB of bf16 grads) to overlap with backward.  Default 16 MB
keeps the first bucket ready early in backward; tune with
``CLOUD_AMD_BUCKET_MB``.
"""
from __future__ import annotations

import os
import time
import weakref

import torch
import torch.distributed as dist

from ..utils import trace
from . import comm as _comm

_ACTIVE = weakref.WeakSet()
# "event" (default): explicit compute->comm-stream event per bucket; "sync": also
# host-synchronise (debug); "backend": leave ordering to the process-group backend.
_DDP_ORDER = os.environ.get("CLOUD_AMD_DDP_ORDER", "event")


# notify_grad_ready runs for every parameter of every step (~150 times per BERT step): it walks
# a cached tuple of weak references instead of iterating the WeakSet (~2 us per call).  The
# cache is rebuilt when a reducer is activated (_activate) or collected (the set shrinks).
_SNAP = [(), -1]


def _activate(r):
    _ACTIVE.add(r)
    _SNAP[1] = -1


def notify_grad_ready(param):
    """Called by ops that write a parameter's gradient straight into its arena
    slice (bypassing autograd's AccumulateGrad, hence its hooks)."""
    n = len(_ACTIVE)
    if n != _SNAP[1]:
        _SNAP[0], _SNAP[1] = tuple(weakref.ref(r) for r in _ACTIVE), n
    for ref in _SNAP[0]:
        r = ref()
        if r is not None:
            r._on_grad(param)


def _busy_ms(evs):
    """Time the collectives of one step kept the (serial) comm path busy: each bucket
    counts from max(its gradients ready, previous collective done) to its completion."""
    total, prev_end = 0.0, None
    for start, end in evs:
        begin = start if prev_end is None or start.elapsed_time(prev_end) <= 0 else prev_end
        total += max(begin.elapsed_time(end), 0.0)
        prev_end = end
    return total


def _busy_host_ms(spans):
    """Host-clock version of :func:`_busy_ms` over (start_s, end_s) pairs."""
    total, prev_end = 0.0, None
    for start, end in spans:
        begin = start if prev_end is None else max(start, prev_end)
        total += max(end - begin, 0.0)
        prev_end = end if prev_end is None else max(prev_end, end)
    return total * 1e3


class _TorchTransport:
    """``torch.distributed`` all-reduce (RCCL on GPU, gloo on CPU); a fake with the same
    ``all_reduce(tensor) -> work`` contract can be injected (tests)."""

    def __init__(self, pg):
        self.pg = pg

    def all_reduce(self, t):
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)


class Bucket:
    __slots__ = ("arena", "lo", "hi", "slots", "pending", "work", "launched", "index", "wire", "wire_buf", "ev",
                 "span", "ready_ev", "wire_dtype", "part")

    def __init__(self, arena, lo, hi, slots, index, wire_dtype=None, part=None):
        self.arena, self.lo, self.hi, self.slots, self.index = arena, lo, hi, slots, index
        self.wire_dtype = wire_dtype  # per-bucket wire dtype (None: the reducer's)
        self.part = part  # (k, n): chunk k of n of one split parameter, else None
        self.pending = len(slots)
        self.work = None
        self.launched = False
        self.wire = None   # this step's reduce-dtype copy on the wire (None: reduced in place)
        self.wire_buf = None  # persistent storage of that copy (allocated on first use)
        self.ev = None     # (start, end) timing events of this step's collective (GPU)
        self.span = None   # [start_s, end_s] host clock of this step's collective (gloo / CPU)
        self.ready_ev = None  # compute-stream event: this step's last gradient of the bucket produced

    @property
    def tensor(self):
        return self.arena.grad[self.lo:self.hi]


class GradAllReducer:
    def __init__(self, arenas, process_group=None, bucket_mb=None, overlap=True, reduce_dtype=None,
                 transport=None, world=None, wire_dtypes=None):
        self.arenas = arenas
        # per-parameter wire dtype overrides {param: dtype} (see _param_wire)
        self._wire_overrides = {id(p): dt for p, dt in (wire_dtypes or {}).items()}
        self.pg = process_group
        if world is None:
            world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.world = world
        mb = float(bucket_mb if bucket_mb is not None else os.environ.get("CLOUD_AMD_BUCKET_MB", 16))
        self.bucket_mb = mb
        self.bucket_bytes = int(mb * (1 << 20))
        self.overlap = overlap
        # Wire dtype of the reduction (CLOUD_AMD_GRAD_REDUCE_DTYPE, default "auto"):
        #   bf16   -- every bucket reduced in bf16: bf16 arenas in place, fp32 arenas (BERT's
        #             word-embedding table, BatchNorm / LayerNorm parameters) through a bf16
        #             copy cast back into the fp32 gradient -- half the xGMI bytes of fp32;
        #   fp32   -- every bucket reduced in fp32 (bf16 arenas through an fp32 copy);
        #   native -- each arena in its own dtype;
        #   auto   -- native: bf16 arenas on a bf16 wire, fp32 arenas (master-weight gradients:
        #             BatchNorm / LayerNorm parameters, BERT's word-embedding table) in fp32, as
        #             the reference's MirroredStrategy reduces each gradient in its variable's
        #             dtype.  The all-bf16 wire (half the fp32 arenas' xGMI bytes, ~3 bf16 ulp of
        #             error on their sums) is an explicit opt-in.
        # The casts run on the comm stream, next to the collective, into a wire buffer kept
        # per bucket (allocated once).  RCCL adds bf16 operands in fp32 and rounds each hop's
        # partial sum to bf16 (error: tests/test_grad_reduce_precision.py).
        rd = reduce_dtype if reduce_dtype is not None else os.environ.get("CLOUD_AMD_GRAD_REDUCE_DTYPE", "auto")
        if rd == "auto":
            rd = "native"
        if isinstance(rd, str):
            rd = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
                  "bfloat16": torch.bfloat16, "native": None}[rd]
        self.reduce_dtype = rd
        # Per-step communication timing (bench / monitoring): see timing_start/timing_summary.
        # With the metrics exporter on, every step is timed and completed steps are drained
        # into the ALLREDUCE / EXPOSED_COMM histograms by event query (never a host sync).
        from .. import monitoring as _mon

        self._mon = _mon if (_mon.enabled() and self.world > 1) else None
        self.timing = self._mon is not None
        self._timing_log = []
        self.check_every = int(os.environ.get("CLOUD_AMD_GRAD_CHECK_EVERY", "0"))
        self._steps = 0
        self.comm = None
        self._side = None
        self._comm_stream = None
        on_gpu = bool(self.arenas) and self.arenas[0].grad.is_cuda
        self.transport = transport
        injected = transport is not None
        if transport is None and self.world > 1:
            self.transport = _TorchTransport(process_group)
        # GPU-event timing needs a collective that the comm stream can wait on without
        # blocking the host: RCCL.  gloo (CPU tensors, or the shared-GPU rehearsal) is timed
        # on the host clock from each work's completion future.
        backend = dist.get_backend(process_group) if (dist.is_initialized() and not injected) else "fake"
        self._device_timed = on_gpu and backend == "nccl"
        if (self.world > 1 and on_gpu and not injected and _comm.backend() != "rccl"
                and _DDP_ORDER != "backend"):
            self._side = torch.cuda.Stream(self.arenas[0].grad.device, priority=-1)
        if (self.world > 1 and not injected and _comm.backend() == "rccl" and self.arenas
                and self.arenas[0].grad.is_cuda):
            self.comm = _comm.RcclComm()  # native communicator: side stream + events
            self.comm.start_watchdog()
            self._comm_stream = torch.cuda.ExternalStream(self.comm.c.stream, device=self.arenas[0].grad.device)
            self._device_timed = True
        self.buckets = []
        self._param_bucket = {}
        self._next = 0
        self._seen = set()
        self._sync_enabled = True
        self.tape_reduced = False  # tf.GradientTape joined this step's buckets (cloud_amd/tf.py)
        self._hooks = []
        # overlap budget (bench JSON): per bucket, a compute-stream event when its last gradient
        # was produced, and one at the end of backward -- recorded at ANY world size
        self._probe = False
        self._ready_log = []
        # per-slice optimizer (attach_optimizer): bucket k's fused update runs on its own
        # stream as soon as bucket k's collective completes, overlapping bucket k+1's
        self.optimizer = None
        self._opt_stream = None
        self._sliced_step = False
        self._build()
        if self.world > 1 and overlap:
            self._install_hooks()
            _activate(self)

    def _param_wire(self, p):
        """Wire dtype override of one parameter: ``wire_dtypes[p]`` given to the reducer, or
        the parameter's ``_ca_wire_dtype`` attribute (e.g. BERT's word-embedding table)."""
        dt = self._wire_overrides.get(id(p)) if self._wire_overrides else None
        return dt if dt is not None else getattr(p, "_ca_wire_dtype", None)

    def _build(self):
        # An arena is in reverse forward order, so its LAST bucket holds the first layers,
        # whose gradients exist only when backward ends: that all-reduce is never hidden
        # behind compute.  Each arena's final bucket is capped at CLOUD_AMD_TAIL_BUCKET_MB
        # (split off the end of the arena) so the exposed collectives are small ones.
        #
        # A parameter larger than CLOUD_AMD_SPLIT_PARAM_MB (default 2 buckets) is cut into
        # sub-buckets of about one bucket each (at least CLOUD_AMD_SPLIT_PARAM_MIN chunks): all
        # become ready together (one gradient), then go on the wire one after another, so with
        # the per-bucket optimizer chunk k's update runs while chunk k+1 is in flight -- BERT's
        # 91 MB word-embedding gradient, produced last in backward, is otherwise one
        # collective followed by one serial AdamW over the whole table.
        tail = int(float(os.environ.get("CLOUD_AMD_TAIL_BUCKET_MB", 1.0)) * (1 << 20))
        split_mb = float(os.environ.get("CLOUD_AMD_SPLIT_PARAM_MB") or 0) or 2 * self.bucket_mb
        split_bytes = int(split_mb * (1 << 20))
        min_chunks = max(int(os.environ.get("CLOUD_AMD_SPLIT_PARAM_MIN", 4)), 1)
        for a in self.arenas:
            es = a.grad.element_size()
            cur, lo = [], 0
            for s in a.slots:
                end = s.offset + ((s.numel + 63) // 64) * 64
                nbytes = (end - s.offset) * es
                if split_bytes > 0 and nbytes > split_bytes:
                    # close the open bucket at this slot, then the slot's own chunks
                    if cur:
                        self.buckets.append(Bucket(a, lo, s.offset, cur, len(self.buckets)))
                    n = max(-(-nbytes // self.bucket_bytes), min_chunks)
                    step = -(-((end - s.offset) // 64) // n) * 64
                    cuts = list(range(s.offset, end, step)) + [end]
                    wd = self._param_wire(s.param)
                    for k in range(len(cuts) - 1):
                        self.buckets.append(Bucket(a, cuts[k], cuts[k + 1], [s], len(self.buckets), wire_dtype=wd,
                                                   part=(k, len(cuts) - 1)))
                    cur, lo = [], end
                    continue
                cur.append(s)
                if (end - lo) * es >= self.bucket_bytes:
                    self.buckets.append(Bucket(a, lo, end, cur, len(self.buckets)))
                    cur, lo = [], end
            if cur:
                if tail > 0 and len(cur) > 1 and (a.n - lo) * es > tail:
                    k = len(cur) - 1  # keep at least one slot in the tail
                    while k > 1 and (a.n - cur[k - 1].offset) * es <= tail:
                        k -= 1
                    cut = cur[k].offset
                    self.buckets.append(Bucket(a, lo, cut, cur[:k], len(self.buckets)))
                    cur, lo = cur[k:], cut
                self.buckets.append(Bucket(a, lo, a.n, cur, len(self.buckets)))
        # buckets of whole slots take a per-parameter wire dtype only when every slot agrees
        for b in self.buckets:
            if b.part is None:
                dts = {self._param_wire(s.param) for s in b.slots}
                if len(dts) == 1:
                    b.wire_dtype = dts.pop()
        # Launch order = the order buckets COMPLETE in backward (their last slot in reverse
        # registration order), across arenas -- not arena by arena: BERT's fp32 arena starts
        # with the word-embedding table, whose gradient is the very last one backward produces,
        # and a strictly ordered launch would hold every bf16 bucket behind it (nothing
        # overlapped; overlap_budget showed ~1.5 ms exposed at 300 GB/s).  Every rank builds the
        # same order from the same model.  (Chunks of one parameter keep their order.)
        if os.environ.get("CLOUD_AMD_BUCKET_ORDER", "ready") == "ready":
            self.buckets.sort(key=lambda b: (max(s.seq for s in b.slots), b.index))
            for i, b in enumerate(self.buckets):
                b.index = i
        for b in self.buckets:
            for s in b.slots:
                ent = self._param_bucket.setdefault(id(s.param), (s.param, []))
                ent[1].append(b)

    def _install_hooks(self):
        for b in self.buckets:
            for s in b.slots:
                self._hooks.append(s.param.register_post_accumulate_grad_hook(self._on_hook))

    def _on_hook(self, p):
        # autograd's post-accumulate hook fires when the Function that took ``p`` returns --
        # also when it returned no gradient for it.  A parameter whose gradient is finished
        # LATER by deferred side-stream work (runtime/side_stream.defer marks it) must be
        # counted only by that work's explicit notify_grad_ready, or its bucket would launch
        # (all-reduce / optimizer slice) before the weight-gradient GEMM has written it.
        if getattr(p, "_ca_explicit_notify", False):
            return
        self._on_grad(p)

    def _on_grad(self, p):
        # A parameter can be reported twice per step: explicitly by an op that wrote its
        # arena gradient in place (notify_grad_ready), and again by autograd's
        # post-accumulate hook (which fires for Function inputs even when the Function
        # returned no gradient for them).  Count each parameter once per step, or a
        # bucket would launch before all its gradients exist.
        if not self._sync_enabled or id(p) in self._seen:
            return
        self._seen.add(id(p))
        pb = self._param_bucket.get(id(p))
        # (identity checked: a dead reducer's id(param) keys can be reused by another model's
        # parameters while the dead one still sits in _ACTIVE awaiting cycle collection)
        bs = pb[1] if pb is not None and pb[0] is p else ()
        ready = False
        for b in bs:  # one bucket, or every chunk of a split parameter
            if b.launched:
                continue
            b.pending -= 1
            if b.pending <= 0:
                ready = True
                if self._probe:
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record(torch.cuda.current_stream(b.tensor.device))
                    b.ready_ev = ev
        # world 1: hooks exist for the readiness probe and / or the per-slice optimizer
        if ready and (self.world > 1 or self.optimizer is not None or not self._probe):
            self._launch_ready()

    def _wire_dtype(self, b):
        return b.wire_dtype if b.wire_dtype is not None else (self.reduce_dtype or b.tensor.dtype)

    def _wire(self, b):
        """The tensor this bucket's collective reduces; runs on the comm stream."""
        dt = self._wire_dtype(b)
        if dt == b.tensor.dtype:
            return b.tensor
        if b.wire_buf is None:
            b.wire_buf = torch.empty(b.hi - b.lo, dtype=dt, device=b.tensor.device)
        b.wire_buf.copy_(b.tensor)
        b.wire = b.wire_buf
        return b.wire

    def _launch(self, b):
        trace.mark("bucket%d" % b.index)
        if self.world <= 1:
            # nothing to reduce: the bucket's gradients are final, so its slice of the fused
            # update can start now, on the optimizer stream, beside the rest of backward
            self._update_slice(b, torch.cuda.current_stream(b.tensor.device))
            b.launched = True
            return
        if self.comm is not None:
            # native communicator: the copy to the wire dtype, the collective and the copy
            # back all run on the communicator's stream, after the gradients' producers
            dev = b.tensor.device
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(dev))
            self._comm_stream.wait_event(ready)
            with torch.cuda.stream(self._comm_stream):
                if self.timing:
                    b.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    b.ev[0].record(self._comm_stream)
                wire = self._wire(b)
                self.comm.all_reduce(wire)
                if b.wire is not None:
                    b.tensor.copy_(b.wire)
                if self.timing:
                    b.ev[1].record(self._comm_stream)
            self._update_slice(b, self._comm_stream)
        elif self._side is not None:
            # Explicit ordering: the collective is issued from a dedicated comm stream that
            # first waits on an event recorded on the compute stream (where the kernels that
            # wrote this bucket's gradients were queued).  Do not rely on the backend picking
            # up the caller's stream: hooks and notify_grad_ready() run on autograd threads.
            mode = _DDP_ORDER
            if mode == "sync":
                torch.cuda.current_stream(b.tensor.device).synchronize()
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(b.tensor.device))
            self._side.wait_event(ev)
            with torch.cuda.stream(self._side):
                if self.timing and self._device_timed:
                    # start: the comm stream has caught up with this bucket's gradients
                    b.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    b.ev[0].record(self._side)
                b.work = self.transport.all_reduce(self._wire(b))
                if self._device_timed:
                    # RCCL: the side stream waits for the collective's stream (no host block),
                    # so the end event marks its completion and the copy back follows it
                    b.work.wait()
                    b.work = None
                    if b.wire is not None:
                        b.tensor.copy_(b.wire)
                    if b.ev is not None:
                        b.ev[1].record(self._side)
                elif self.timing:
                    self._host_span(b)
            if self._device_timed:
                self._update_slice(b, self._side)
        else:
            b.work = self.transport.all_reduce(self._wire(b))
            if self.timing:
                self._host_span(b)
        b.launched = True

    def _host_span(self, b):
        """Host-clock span of a gloo / fake collective: launch -> completion future."""
        b.span = [time.perf_counter(), None]
        fut = b.work.get_future() if hasattr(b.work, "get_future") else None
        if fut is not None:
            def done(_f, span=b.span):
                span[1] = time.perf_counter()
                return None

            fut.then(done)

    def _launch_ready(self):
        while self._next < len(self.buckets) and self.buckets[self._next].pending <= 0:
            self._launch(self.buckets[self._next])
            self._next += 1

    def finish(self):
        """Launch remaining buckets in order and join them onto the compute stream."""
        if self._probe:
            self._log_ready()
        if self.world <= 1:
            if self.optimizer is not None:
                while self._next < len(self.buckets):
                    self._launch(self.buckets[self._next])
                    self._next += 1
                self._join_sliced()
            self.reset()
            return
        dev_timed = self.timing and self._device_timed
        if self.timing:  # backward done (compute stream) -> comm joined = exposed communication
            if dev_timed:
                t_bwd = torch.cuda.Event(enable_timing=True)
                t_bwd.record(torch.cuda.current_stream(self.arenas[0].grad.device))
            else:
                t_bwd = time.perf_counter()
        while self._next < len(self.buckets):
            self._launch(self.buckets[self._next])
            self._next += 1
        if self.comm is not None:
            self.comm.join()  # compute stream waits for the comm stream (collectives + copies)
            self._join_sliced()
        elif self._side is not None:
            with torch.cuda.stream(self._side):
                for b in self.buckets:
                    if b.work is not None:  # gloo on device tensors: a host-side wait
                        b.work.wait()
                        self._close_span(b)
                        if b.wire is not None:
                            b.tensor.copy_(b.wire)
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)
            self._join_sliced()
        else:
            for b in self.buckets:
                if b.work is not None:
                    b.work.wait()
                    self._close_span(b)
                if b.wire is not None:
                    b.tensor.copy_(b.wire)
        if self.timing:
            if dev_timed:
                t_join = torch.cuda.Event(enable_timing=True)
                t_join.record(torch.cuda.current_stream(self.arenas[0].grad.device))
                self._timing_log.append((t_bwd, t_join, [b.ev for b in self.buckets if b.ev is not None]))
            else:
                t_join = time.perf_counter()
                spans = [tuple(b.span) for b in self.buckets if b.span is not None]
                self._timing_log.append(((t_join - t_bwd) * 1e3, _busy_host_ms(spans), None))
            if self._mon is not None:
                self._drain_to_monitoring()
        self.reset()
        self._steps += 1
        if self.check_every and self._steps % self.check_every == 0:
            self.check_consistency()

    @staticmethod
    def _close_span(b):
        if b.span is not None and b.span[1] is None:  # no completion callback ran (fake work)
            b.span[1] = time.perf_counter()

    def no_sync(self):
        """Gradient accumulation: backward passes inside this context only accumulate into
        the arena; the all-reduce happens on the first backward after it (DDP.no_sync)."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            prev, self._sync_enabled = self._sync_enabled, False
            try:
                yield
            finally:
                self._sync_enabled = prev

        return ctx()

    def check_consistency(self, rtol=0.0):
        """Desync detector: after the all-reduce every replica must hold
        the same gradients, and every replica the same master weights.  Compares an fp64
        (sum, sum of squares, sum of |x|) fingerprint of every arena's gradients and master
        weights across ranks; raises RuntimeError on mismatch.  Cheap -- meant to
        run every N steps (``CLOUD_AMD_GRAD_CHECK_EVERY``)."""
        if self.world <= 1:
            return True
        fp = []
        for a in self.arenas:
            # the master weights are compared too: after a fused step the gradient arena is
            # zero (the update kernel clears it), while the weights must agree at all times
            for t in (a.grad, a.master):
                t = t.double()
                fp += [t.sum(), (t * t).sum(), t.abs().sum()]
        mine = torch.stack(fp)
        allfp = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(allfp, mine, group=self.pg)
        ref = allfp[0]
        for r, other in enumerate(allfp[1:], 1):
            tol = rtol * ref.abs() + 1e-12
            if bool(((other - ref).abs() > tol).any()):
                raise RuntimeError("gradient desync: rank %d fingerprint %s != rank 0 %s"
                                   % (r, other.tolist(), ref.tolist()))
        return True

    def reset(self):
        self._seen = set()
        for b in self.buckets:
            b.pending = len(b.slots)
            b.work = None
            b.launched = False
            b.wire = None
            b.ev = None
            b.span = None
            b.ready_ev = None
        self._next = 0

    def _drain_to_monitoring(self):
        """Observe the per-step comm times of every finished step (event.query(): no sync)."""
        keep = []
        for entry in self._timing_log:
            t_bwd, t_join, evs = entry
            if evs is None:  # host-timed: (exposed_ms, allreduce_ms, None)
                self._mon.observe(self._mon.ALLREDUCE, t_join)
                self._mon.observe(self._mon.EXPOSED_COMM, t_bwd)
                continue
            if not t_join.query():
                keep.append(entry)
                continue
            self._mon.observe(self._mon.EXPOSED_COMM, t_bwd.elapsed_time(t_join))
            self._mon.observe(self._mon.ALLREDUCE, _busy_ms(evs) if evs else 0.0)
        self._timing_log = keep[-64:]

    def timing_start(self):
        """Record communication timing for every following step (events only; no sync)."""
        self.timing = True
        self._timing_log = []

    def timing_summary(self):
        """Mean per-step ``allreduce_ms`` (time the serial comm path was busy with this
        step's collectives) and ``exposed_comm_ms`` (end of backward on the compute stream
        -> all buckets joined).  Call after a device synchronize.  Always finite."""
        self.timing = self._mon is not None
        if self.world <= 1 or not self._timing_log:
            return {"allreduce_ms": 0.0, "exposed_comm_ms": 0.0, "steps": len(self._timing_log),
                    "timing": "none"}
        ar, ex = [], []
        host = False
        for t_bwd, t_join, evs in self._timing_log:
            if evs is None:
                host = True
                ex.append(t_bwd)
                ar.append(t_join)
                continue
            ex.append(t_bwd.elapsed_time(t_join))
            ar.append(_busy_ms(evs) if evs else 0.0)
        n = len(ex)
        return {"allreduce_ms": round(sum(ar) / n, 3), "exposed_comm_ms": round(sum(ex) / n, 3), "steps": n,
                "timing": "host_clock" if host else "device_events"}

    def describe(self):
        """Bucket layout for reports: count, target size, wire dtype, transport."""
        transport = ("native RcclComm" if self.comm is not None else
                     "torch.distributed(%s)" % (dist.get_backend(self.pg) if dist.is_initialized() else "none"))
        def name(dt):
            return str(dt).replace("torch.", "")

        wire = sorted({name(self._wire_dtype(b)) for b in self.buckets})
        wire_mb = sum((b.hi - b.lo) * self._wire_dtype(b).itemsize for b in self.buckets) / 2 ** 20
        split = sorted({(b.part[1], name(self._wire_dtype(b))) for b in self.buckets if b.part is not None})
        return {"buckets": len(self.buckets), "bucket_mb": self.bucket_mb,
                "reduce_dtype": wire[0] if len(wire) == 1 else "mixed(%s)" % ",".join(wire),
                "grad_dtypes": sorted({name(a.grad.dtype) for a in self.arenas}),
                "split_params": [{"chunks": n, "wire": w} for n, w in split],
                "wire_mb_per_step": round(wire_mb, 2), "transport": transport, "world": self.world}

    # -- per-slice optimizer ---------------------------------------------------------
    def attach_optimizer(self, optimizer):
        """Run ``optimizer``'s fused update per bucket, as each bucket's collective completes
        (RCCL transports; opt-in at world 1, as soon as the bucket's gradients are final --
        only for loops that do not touch gradients between backward and ``step()``): bucket
        k's update runs on a dedicated stream while bucket k+1 is
        still on the wire and backward is still running, so after the last collective only the
        last bucket's update remains -- for BERT that is the word-embedding tail instead of the
        whole-arena AdamW.  The elementwise update is the same per element, so the weights are
        bitwise those of the whole-arena ``step()`` (tests/test_rccl_dataplane_gpu.py).
        ``optimizer.step()`` after ``finish()`` then only closes the step.  Off when the
        transport is not stream-ordered (gloo / CPU), with ``clipnorm`` (needs the global norm
        first), and unless opted in: ``CLOUD_AMD_SLICED_OPT=1`` (world > 1) /
        ``CLOUD_AMD_SLICED_OPT_WORLD1=1`` (world 1).  Returns True when enabled."""
        from .. import config

        cuda = bool(self.arenas) and self.arenas[0].grad.is_cuda
        # world 1 (opt-in, CLOUD_AMD_SLICED_OPT_WORLD1): no collective, so each bucket's update
        # starts as soon as backward has produced its last gradient, beside the rest of
        # backward.  Measured SLOWER on one MI355X -- BERT 6,927 vs 6,969 seq/s, ResNet-50
        # 15,231 vs 15,278 img/s (profiles/r5_s22/): the bandwidth-bound update competes with
        # backward's own memory traffic and adds a launch per bucket
        wire_ok = ((self.world > 1 and self._device_timed)
                   or (self.world == 1 and cuda and config.get("CLOUD_AMD_SLICED_OPT_WORLD1")))
        ok = (wire_ok and getattr(optimizer, "clipnorm", None) is None
              and (self.world == 1 or config.get("CLOUD_AMD_SLICED_OPT")) and hasattr(optimizer, "sliced_begin"))
        self.optimizer = optimizer if ok else None
        if ok and self._opt_stream is None:
            self._opt_stream = torch.cuda.Stream(self.arenas[0].grad.device)
        if ok and self.world == 1 and not self._hooks:
            self._install_hooks()
            _activate(self)
        return bool(ok)

    def _update_slice(self, b, after_stream):
        opt = self.optimizer
        if opt is None:
            return
        if not self._sliced_step:
            opt.sliced_begin()  # iteration count / hyper-parameters of this step, once
            self._sliced_step = True
        done = torch.cuda.Event()
        done.record(after_stream)
        self._opt_stream.wait_event(done)
        with torch.cuda.stream(self._opt_stream):
            opt.sliced_update(b.arena, b.lo, b.hi)

    def _join_sliced(self):
        if self.optimizer is not None and self._sliced_step:
            torch.cuda.current_stream(self._opt_stream.device).wait_stream(self._opt_stream)
            self.optimizer.sliced_end_pending()
            self._sliced_step = False

    # -- overlap budget ------------------------------------------------------------------
    def probe_readiness(self, on=True):
        """Record, for every following step, when each bucket's gradients were complete on the
        compute stream and when backward ended (device events, no sync; any world size -- at
        world 1 the hooks are installed for the probe only).  Read with :meth:`overlap_budget`."""
        self._probe = bool(on) and bool(self.arenas) and self.arenas[0].grad.is_cuda
        self._ready_log = []
        if self._probe and not self._hooks:
            self._install_hooks()
            _activate(self)

    def _log_ready(self):
        end = torch.cuda.Event(enable_timing=True)
        end.record(torch.cuda.current_stream(self.arenas[0].grad.device))
        self._ready_log.append((end, [b.ready_ev for b in self.buckets]))
        self._ready_log = self._ready_log[-64:]

    def overlap_budget(self, busbw_gbs=(150.0, 300.0), world=None, optimizer=None, hbm_gbs=5000.0):
        """Per bucket: wire MB and how many ms before the end of backward its gradients were
        ready (mean over the probed steps; 0 for buckets completed only by ``finish``), and the
        exposed communication PREDICTED for a serial comm path at each bus bandwidth (nccl-tests
        convention: a bucket of B bytes takes B * 2(n-1)/n / busbw) with n = ``world`` (default:
        this job's world, 8 at world 1).

        With an ``optimizer`` (default: the attached per-bucket one) the prediction also prices
        the update slices at ``hbm_gbs``: ``predicted_exposed_step_ms`` is the time from the end
        of backward until the last slice has run when each bucket's slice follows its collective
        on one optimizer stream (the per-bucket optimizer), and ``predicted_exposed_whole_ms``
        the same with the whole-arena update after the last collective -- both beyond the
        backward; the difference is what slicing buys.  Call after a device synchronize."""
        if not self._ready_log:
            return None
        n = world or (self.world if self.world > 1 else 8)
        nb = len(self.buckets)
        before = [0.0] * nb
        for end, evs in self._ready_log:
            for i, ev in enumerate(evs):
                if ev is not None:
                    before[i] += max(ev.elapsed_time(end), 0.0)
        before = [v / len(self._ready_log) for v in before]
        mb = [(b.hi - b.lo) * self._wire_dtype(b).itemsize / 2 ** 20 for b in self.buckets]
        opt = optimizer if optimizer is not None else self.optimizer
        upd = None
        if opt is not None and hasattr(opt, "update_bytes_per_elem"):
            upd = [(b.hi - b.lo) * opt.update_bytes_per_elem(b.arena) / (hbm_gbs * 1e9) * 1e3 for b in self.buckets]
        pred, pred_step, pred_whole = {}, {}, {}
        for bw in busbw_gbs:
            t_end = None
            t_opt = None  # end of the last update slice issued (one optimizer stream)
            for i in range(nb):  # launch order = bucket order
                dur = mb[i] * 2 ** 20 * 2.0 * (n - 1) / n / (bw * 1e9) * 1e3
                start = -before[i] if t_end is None else max(-before[i], t_end)
                t_end = start + dur
                if upd is not None:
                    t_opt = max(t_end, t_opt if t_opt is not None else t_end) + upd[i]
            pred["%g" % bw] = round(max(t_end or 0.0, 0.0), 3)
            if upd is not None:
                pred_step["%g" % bw] = round(max(t_opt or 0.0, 0.0), 3)
                pred_whole["%g" % bw] = round(max(t_end or 0.0, 0.0) + sum(upd), 3)
        out = {"world_predicted": n, "steps": len(self._ready_log),
               "buckets": [{"mb": round(m, 2), "ready_before_bwd_end_ms": round(v, 3),
                            "wire": str(self._wire_dtype(b)).replace("torch.", "")}
                           for m, v, b in zip(mb, before, self.buckets)],
               "predicted_exposed_comm_ms": pred}
        if upd is not None:
            out.update({"hbm_gbs": hbm_gbs, "update_ms_total": round(sum(upd), 3),
                        "predicted_exposed_step_ms": pred_step, "predicted_exposed_whole_ms": pred_whole})
        return out

    def broadcast_parameters(self, src=0):
        """C2: make every rank start from rank ``src``'s weights (one call per arena)."""
        if self.world <= 1:
            return
        for a in self.arenas:
            if self.comm is not None:
                self.comm.broadcast(a.master, src)
                if a.model is not None:
                    self.comm.broadcast(a.model, src)
            else:
                dist.broadcast(a.master, src, group=self.pg)
                if a.model is not None:
                    dist.broadcast(a.model, src, group=self.pg)
        if self.comm is not None:
            self.comm.join()

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
