"""A small ``tf.data``-style input pipeline (``cloud_amd.keras.data.Dataset``).

Covers what the reference workloads use (``mnist_example_using_fit.py:31-51``,
``mnist_example_using_ctl.py:55-69``): ``from_tensor_slices``, ``map``,
``cache``, ``shuffle``, ``batch``, ``repeat``, ``take``, ``prefetch`` and the
``shard`` used by ``Strategy.experimental_distribute_dataset`` (rank-strided
element sharding, no communication -- C4 in SURVEY.md).  Elements are numpy
pytrees; batching stacks them.  A background thread implements ``prefetch``.
"""
from __future__ import annotations

import os
import queue
import threading

import numpy as np

AUTOTUNE = -1


def _map_tree(fn, x):
    if isinstance(x, dict):
        return {k: _map_tree(fn, v) for k, v in x.items()}
    if isinstance(x, (tuple, list)):
        return type(x)(_map_tree(fn, v) for v in x)
    return fn(x)


def _stack(items):
    first = items[0]
    if isinstance(first, dict):
        return {k: _stack([it[k] for it in items]) for k in first}
    if isinstance(first, (tuple, list)):
        return type(first)(_stack([it[i] for it in items]) for i in range(len(first)))
    try:
        import torch

        if isinstance(first, torch.Tensor):
            return torch.stack(items)
    except ImportError:  # pragma: no cover
        pass
    return np.stack([np.asarray(i) for i in items])


def _to_numpy(x):
    try:
        import torch

        if isinstance(x, torch.Tensor):
            return x.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(x)


class Dataset:
    def __init__(self, gen_fn, length=None):
        self._gen_fn = gen_fn
        self._length = length

    # -- sources --------------------------------------------------------------
    @staticmethod
    def from_tensor_slices(tensors):
        arrs = _map_tree(_to_numpy, tensors)
        leaves = []
        _map_tree(leaves.append, arrs)
        n = len(leaves[0])

        def gen():
            for i in range(n):
                yield _map_tree(lambda a: a[i], arrs)

        ds = Dataset(gen, n)
        ds._slices = arrs
        return ds

    @staticmethod
    def from_tensors(tensors):
        return Dataset(lambda: iter([tensors]), 1)

    @staticmethod
    def range(*args):
        r = range(*args)
        return Dataset(lambda: (np.int64(i) for i in r), len(r))

    @staticmethod
    def from_generator(generator, output_signature=None, output_types=None, output_shapes=None):
        return Dataset(lambda: iter(generator()), None)

    # -- transformations --------------------------------------------------------
    def map(self, fn, num_parallel_calls=None, deterministic=None):
        src = self

        def gen():
            for el in src:
                yield fn(*el) if isinstance(el, tuple) else fn(el)

        return Dataset(gen, self._length)

    def filter(self, pred):
        src = self
        return Dataset(lambda: (el for el in src if (pred(*el) if isinstance(el, tuple) else pred(el))), None)

    def batch(self, batch_size, drop_remainder=False):
        src = self

        def gen():
            buf = []
            for el in src:
                buf.append(el)
                if len(buf) == batch_size:
                    yield _stack(buf)
                    buf = []
            if buf and not drop_remainder:
                yield _stack(buf)

        n = None
        if self._length is not None:
            n = self._length // batch_size if drop_remainder else -(-self._length // batch_size)
        ds = Dataset(gen, n)
        ds._batch_size = batch_size
        return ds

    def unbatch(self):
        src = self

        def gen():
            for b in src:
                leaves = []
                _map_tree(leaves.append, b)
                for i in range(len(leaves[0])):
                    yield _map_tree(lambda a: a[i], b)

        return Dataset(gen, None)

    def shuffle(self, buffer_size, seed=None, reshuffle_each_iteration=True):
        """Buffered shuffle.  An unseeded shuffle inside a launched job draws its seed
        from the job id, so every replica sees the same global order (the replicas of
        a data-parallel job each iterate the pipeline and cut their slice of every
        global batch: they must agree on what the global batches are)."""
        src = self
        state = {"epoch": 0}
        if seed is None:
            seed = _job_seed()

        def gen():
            rng = np.random.default_rng(None if seed is None else seed + (state["epoch"] if reshuffle_each_iteration
                                                                          else 0))
            state["epoch"] += 1
            buf = []
            for el in src:
                buf.append(el)
                if len(buf) >= buffer_size:
                    j = rng.integers(len(buf))
                    buf[j], buf[-1] = buf[-1], buf[j]
                    yield buf.pop()
            rng.shuffle(buf)
            yield from buf

        return Dataset(gen, self._length)

    def repeat(self, count=None):
        src = self

        def gen():
            i = 0
            while count is None or count < 0 or i < count:
                yield from src
                i += 1

        return Dataset(gen, None if count in (None, -1) else (self._length * count if self._length else None))

    def take(self, count):
        src = self

        def gen():
            for i, el in enumerate(src):
                if i >= count:
                    break
                yield el

        n = count if self._length is None else min(count, self._length)
        return Dataset(gen, n)

    def skip(self, count):
        src = self

        def gen():
            for i, el in enumerate(src):
                if i >= count:
                    yield el

        return Dataset(gen, None if self._length is None else max(self._length - count, 0))

    def cache(self, filename=""):
        src = self
        store = {"items": None}

        def gen():
            if store["items"] is None:
                items = []
                for el in src:
                    items.append(el)
                    yield el
                store["items"] = items
            else:
                yield from store["items"]

        return Dataset(gen, self._length)

    def prefetch(self, buffer_size=AUTOTUNE):
        src = self
        depth = 4 if buffer_size in (None, AUTOTUNE) else max(1, int(buffer_size))

        def gen():
            q = queue.Queue(depth)
            end = object()

            def worker():
                try:
                    for el in src:
                        q.put(el)
                finally:
                    q.put(end)

            t = threading.Thread(target=worker, daemon=True)
            t.start()
            while True:
                el = q.get()
                if el is end:
                    break
                yield el

        return Dataset(gen, self._length)

    def shard(self, num_shards, index):
        """Every num_shards-th element starting at ``index``; on a batched dataset the
        *batches* are split instead (each replica gets a 1/num_shards slice of every
        global batch, the MirroredStrategy convention)."""
        src = self
        if getattr(self, "_batch_size", None):
            def gen():
                for b in src:
                    def cut(a):
                        n = len(a)
                        per = -(-n // num_shards)
                        return a[index * per:(index + 1) * per]
                    yield _map_tree(cut, b)

            ds = Dataset(gen, self._length)
            ds._batch_size = -(-self._batch_size // num_shards)
            return ds
        return Dataset(lambda: (el for i, el in enumerate(src) if i % num_shards == index),
                       None if self._length is None else len(range(index, self._length, num_shards)))

    def with_options(self, options):
        return self

    # -- iteration ----------------------------------------------------------------
    def __iter__(self):
        return iter(self._gen_fn())

    def __len__(self):
        if self._length is None:
            raise TypeError("dataset length is unknown")
        return self._length

    def cardinality(self):
        return -2 if self._length is None else self._length

    def as_numpy_iterator(self):
        return iter(self)


def _job_seed():
    """A seed shared by all ranks of a launched job (None outside one)."""
    job = os.environ.get("CLOUD_AMD_JOB_ID") or os.environ.get("TORCHELASTIC_RUN_ID")
    if not job:
        return None
    import zlib

    return zlib.crc32(job.encode()) & 0x7FFFFFFF


class Options:
    def __init__(self):
        self.experimental_distribute = type("D", (), {"auto_shard_policy": None})()
