"""Distribution strategies (P1-P5 in SURVEY.md section 2.4).

Same names and surface as the ``tf.distribute`` strategies the reference
injects (``TFC/core/preprocess.py:124-149``): ``OneDeviceStrategy``,
``MirroredStrategy``, ``MultiWorkerMirroredStrategy``; ``scope()``,
``run(fn, args)``, ``reduce(op, value, axis)``, ``experimental_distribute_dataset``,
``num_replicas_in_sync``, ``experimental_set_strategy`` / ``get_strategy``.

MI355X design: always ONE PROCESS PER GPU.  Mirrored (one node, many GPUs)
and MultiWorkerMirrored (many "machines") are the same engine -- a
``torch.distributed`` process group over RCCL (xGMI inside the node) with
the bucketed, backward-overlapped gradient all-reduce of
:mod:`cloud_amd.parallel.ddp` on the flat gradient arena.  The global batch is
split across replicas (per-replica batch = global / world); models train in
the strategy's ``device`` (``cuda:LOCAL_RANK``, or CPU + gloo on CPU nodes).
"""
from __future__ import annotations

import contextlib
import enum
import json
import os

import torch
import torch.distributed as dist

from ..utils import dist_env

_CURRENT = None


class ReduceOp(enum.Enum):
    SUM = "SUM"
    MEAN = "MEAN"


class Strategy:
    """Common base: a process-group-backed data-parallel strategy."""

    name = "Strategy"

    def __init__(self, device=None):
        from ..runtime import host

        host.configure()
        self._device = torch.device(device) if device is not None else None
        self._prev = None

    # -- topology -------------------------------------------------------------
    @property
    def num_replicas_in_sync(self) -> int:
        return dist.get_world_size() if dist.is_initialized() else 1

    @property
    def rank(self) -> int:
        return dist.get_rank() if dist.is_initialized() else 0

    @property
    def device(self) -> torch.device:
        return self._device

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    @property
    def cluster_resolver(self):
        return ClusterResolver.from_env()

    # -- scope ----------------------------------------------------------------
    @contextlib.contextmanager
    def scope(self):
        global _CURRENT
        prev, _CURRENT = _CURRENT, self
        try:
            yield self
        finally:
            _CURRENT = prev

    # -- execution ------------------------------------------------------------
    def run(self, fn, args=(), kwargs=None):
        """Run ``fn`` on this replica (one process == one replica)."""
        return fn(*args, **(kwargs or {}))

    experimental_run_v2 = run

    def reduce(self, reduce_op, value, axis=None):
        """Cross-replica reduction of a per-replica value (C3)."""
        op = ReduceOp(reduce_op.value if isinstance(reduce_op, ReduceOp) else str(reduce_op).upper().split(".")[-1])
        t = value if isinstance(value, torch.Tensor) else torch.tensor(value, dtype=torch.float64)
        if axis is not None:
            t = t.sum(dim=axis) if op == ReduceOp.SUM else t.sum(dim=axis)
        t = t.detach().clone()
        n_local = value.shape[axis] if (axis is not None and isinstance(value, torch.Tensor)) else 1
        if dist.is_initialized() and self.num_replicas_in_sync > 1:
            comm = t.to(self._comm_device())
            dist.all_reduce(comm, op=dist.ReduceOp.SUM)
            t = comm.to(t.device)
            if op == ReduceOp.MEAN:
                cnt = torch.tensor([float(n_local)], device=self._comm_device())
                dist.all_reduce(cnt)
                return t / cnt.item()
            return t
        if op == ReduceOp.MEAN:
            return t / n_local
        return t

    def gather(self, value, axis=0):
        if not (dist.is_initialized() and self.num_replicas_in_sync > 1):
            return value
        t = value.to(self._comm_device()).contiguous()
        outs = [torch.empty_like(t) for _ in range(self.num_replicas_in_sync)]
        dist.all_gather(outs, t)
        return torch.cat(outs, dim=axis).to(value.device)

    def _comm_device(self):
        if dist.is_initialized() and dist.get_backend() == "nccl":
            return self.device
        return torch.device("cpu")

    def barrier(self):
        if dist.is_initialized():
            dist.barrier()

    # -- the data-parallel engine ----------------------------------------------
    def gradient_reducer(self, arenas, **kwargs):
        """The strategy's gradient all-reduce engine over the optimizer's flat arenas
        (:class:`cloud_amd.parallel.ddp.GradAllReducer`: buckets overlapped with backward
        on a side stream).  With one replica it is a no-op, so training code is the same
        under every strategy."""
        from .ddp import GradAllReducer

        if self.num_replicas_in_sync <= 1:
            kwargs["world"] = 1
        return GradAllReducer(arenas, **kwargs)

    # -- data -----------------------------------------------------------------
    def experimental_distribute_dataset(self, dataset):
        """Shard a dataset across replicas (C4): rank-strided, no communication."""
        if hasattr(dataset, "shard") and self.num_replicas_in_sync > 1:
            return dataset.shard(self.num_replicas_in_sync, self.rank)
        return dataset

    distribute_dataset = experimental_distribute_dataset

    def distribute_datasets_from_function(self, dataset_fn):
        ctx = InputContext(self.num_replicas_in_sync, self.rank)
        return dataset_fn(ctx)

    def __repr__(self):
        return "{}(device={}, replicas={})".format(self.name, self.device, self.num_replicas_in_sync)


class InputContext:
    def __init__(self, num_input_pipelines, input_pipeline_id):
        self.num_input_pipelines = num_input_pipelines
        self.input_pipeline_id = input_pipeline_id
        self.num_replicas_in_sync = num_input_pipelines

    def get_per_replica_batch_size(self, global_batch_size):
        if global_batch_size % self.num_replicas_in_sync:
            raise ValueError("global batch {} not divisible by {} replicas".format(global_batch_size,
                                                                                 self.num_replicas_in_sync))
        return global_batch_size // self.num_replicas_in_sync


def _parse_device(device):
    if device is None:
        return None
    if isinstance(device, torch.device):
        return device
    if os.environ.get("CLOUD_AMD_DEVICE") == "cpu":  # CPU rehearsal of a GPU-shaped job
        return torch.device("cpu")
    d = str(device).lower().strip("/")
    if d.startswith("device:"):
        d = d[len("device:"):]
    if d.startswith("gpu") or d.startswith("cuda"):
        idx = int(d.split(":")[1]) if ":" in d else 0
        if torch.cuda.is_available():
            return torch.device("cuda", idx)
        return torch.device("cpu")
    return torch.device("cpu")


class OneDeviceStrategy(Strategy):
    """P1: one device, no collectives.  ``'/gpu:0'`` falls back to CPU on CPU hosts."""

    name = "OneDeviceStrategy"

    def __init__(self, device=None):
        dev = _parse_device(device)
        if dev is None:
            dev = torch.device("cuda", dist_env.local_rank()) if torch.cuda.is_available() else torch.device("cpu")
        super().__init__(dev)

    @property
    def num_replicas_in_sync(self):
        return 1

    @property
    def rank(self):
        return 0


class MirroredStrategy(Strategy):
    """P2: synchronous DP over the GPUs of one node, one process per GPU (RCCL/xGMI)."""

    name = "MirroredStrategy"

    def __init__(self, devices=None, cross_device_ops=None):
        forced = os.environ.get("CLOUD_AMD_DEVICE")
        use_gpu = torch.cuda.is_available() and forced != "cpu"
        # GPU: init_distributed picks cuda:LOCAL_RANK (cuda:0 for every rank of the
        # CLOUD_AMD_SHARED_GPU rehearsal on a one-GPU box)
        _, _, dev = dist_env.init_distributed(device=None if use_gpu else torch.device("cpu"))
        super().__init__(dev)
        self.cross_device_ops = cross_device_ops


class MultiWorkerMirroredStrategy(MirroredStrategy):
    """P3: the same engine, world = every rank of every worker (TF_CONFIG-shaped roles kept)."""

    name = "MultiWorkerMirroredStrategy"

    def __init__(self, cluster_resolver=None, communication_options=None):
        super().__init__()
        self._resolver = cluster_resolver

    @property
    def cluster_resolver(self):
        return self._resolver or ClusterResolver.from_env()


class TPUStrategy(Strategy):
    name = "TPUStrategy"

    def __init__(self, *a, **k):
        raise NotImplementedError("TPUStrategy has no MI355X analogue; use MirroredStrategy / "
                                  "MultiWorkerMirroredStrategy on MI355X GPUs.")


class ClusterResolver:
    """TF_CONFIG view (reference ``cloud_fit/remote.py:148-156`` reads the same JSON)."""

    def __init__(self, cfg):
        self.cfg = cfg or {}

    @classmethod
    def from_env(cls):
        raw = os.environ.get("TF_CONFIG")
        return cls(json.loads(raw) if raw else {})

    @property
    def task_type(self):
        return self.cfg.get("task", {}).get("type")

    @property
    def task_id(self):
        return self.cfg.get("task", {}).get("index")

    def cluster_spec(self):
        return self.cfg.get("cluster", {})


def is_chief_task(tf_config=None):
    """Reference quirk kept: chief role OR task index 0 counts as chief (remote.py:148-156)."""
    cfg = tf_config if tf_config is not None else json.loads(os.environ.get("TF_CONFIG", "{}") or "{}")
    if not cfg:
        raise ValueError("TF_CONFIG is not set")
    task = cfg.get("task", {})
    if task.get("type") == "chief":
        return True
    # reference quirk (remote.py:151-154): index 0 counts as chief -- kept for
    # worker-only clusters; with an explicit chief only the chief writes.
    return task.get("index") == 0 and "chief" not in cfg.get("cluster", {})


def experimental_set_strategy(strategy):
    global _CURRENT
    _CURRENT = strategy


def get_strategy():
    global _CURRENT
    if _CURRENT is None:
        _CURRENT = _default_strategy()
    return _CURRENT


def has_strategy():
    return _CURRENT is not None


def _default_strategy():
    """No strategy installed (a rank started by torchrun, or a plain script): Mirrored
    when every rank is on this node, MultiWorkerMirrored across nodes, else OneDevice."""
    w = dist_env.world_size()
    if w > 1:
        if dist_env.env_int("LOCAL_WORLD_SIZE", w) == w:
            return MirroredStrategy()
        return MultiWorkerMirroredStrategy()
    forced = os.environ.get("CLOUD_AMD_DEVICE")
    return OneDeviceStrategy(forced if forced else None)


def auto_strategy(chief_gpus=None, worker_count=0):
    """Strategy from the launcher environment (what the generated wrapper picks)."""
    if worker_count > 0:
        return MultiWorkerMirroredStrategy()
    if (chief_gpus or 0) > 1 or dist_env.world_size() > 1:
        return MirroredStrategy()
    return OneDeviceStrategy()


STRATEGIES = {
    "OneDeviceStrategy": OneDeviceStrategy,
    "MirroredStrategy": MirroredStrategy,
    "MultiWorkerMirroredStrategy": MultiWorkerMirroredStrategy,
}
