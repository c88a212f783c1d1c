"""Input pipeline for one-process-per-GPU training on MI355X.

Host side -- :class:`NpyBatchLoader` over the C++ module ``cloud_amd._data``
(``csrc/data/loader.cpp``):

* the sample arrays are ``.npy`` files (first dim = samples) memory-mapped once;
* every epoch draws one permutation from ``(seed, epoch)`` -- identical on every
  rank -- and rank r takes elements r, r+world, ... of it (equal share per rank,
  the tail dropped), so the ranks see disjoint samples with no communication
  (``strategy.experimental_distribute_dataset``);
* C++ worker threads gather the samples of upcoming batches into a ring of
  caller-owned slot buffers (pinned host tensors), ahead of the consumer.

Device side -- :class:`DeviceLoader`: the next batch's host->device copy and the
uint8 -> bf16 normalisation kernel (``csrc/kernels/input.hip``, K9) run on a
separate copy stream while the current batch trains; the training stream waits
on an event, never on the host.

The loader does not decode images: datasets are stored as decoded uint8 arrays
(as the synthetic ImageNet-shaped set of :func:`write_npy_dataset`).
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from .. import monitoring

_DTYPES = {"u1": torch.uint8, "i1": torch.int8, "i2": torch.int16, "i4": torch.int32, "i8": torch.int64,
           "f2": torch.float16, "f4": torch.float32, "f8": torch.float64, "b1": torch.bool}


def _native():
    """The C++ module; built in-tree on first use when missing (host-only, g++, seconds)."""
    import importlib

    try:
        return importlib.import_module("cloud_amd._data")
    except ImportError:
        from .. import _build

        _build.build_data()
        importlib.invalidate_caches()
        return importlib.import_module("cloud_amd._data")


def _torch_dtype(descr):
    key = descr[1:]
    if key not in _DTYPES:
        raise ValueError(f"unsupported .npy dtype {descr}")
    return _DTYPES[key]


class NpyBatchLoader:
    """Shuffled, rank-sharded batches of one or more aligned ``.npy`` arrays.

    ``for slot, arrays in loader.epoch(e): ...; loader.release(slot)`` -- ``arrays``
    are views of the slot's (pinned) buffers, valid until ``release``.
    """

    def __init__(self, paths, batch_size, shuffle=True, seed=0, rank=None, world=None, drop_remainder=True,
                 threads=4, slots=4, pin_memory=None):
        from ..utils import dist_env

        self.paths = [os.fspath(p) for p in paths]
        self.batch_size = int(batch_size)
        self.rank = dist_env.rank() if rank is None else int(rank)
        self.world = dist_env.world_size() if world is None else int(world)
        if slots < 2:
            raise ValueError("NpyBatchLoader needs >= 2 slots (one held by the consumer, one being filled)")
        if pin_memory is None:
            pin_memory = torch.cuda.is_available()
        nat = _native()
        infos = [nat.npy_info(p) for p in self.paths]
        self.shapes = [tuple(i["shape"]) for i in infos]
        self.dtypes = [_torch_dtype(i["descr"]) for i in infos]
        self._slots = [[torch.empty((self.batch_size,) + s[1:], dtype=d, pin_memory=pin_memory)
                        for s, d in zip(self.shapes, self.dtypes)] for _ in range(slots)]
        ptrs = [[t.data_ptr() for t in slot] for slot in self._slots]
        self._L = nat.Loader(self.paths, self.batch_size, bool(shuffle), int(seed), self.rank, self.world,
                             bool(drop_remainder), int(threads), ptrs)
        self._held = set()

    @property
    def num_samples(self):
        return self.shapes[0][0]

    def batches_per_epoch(self, drop_remainder=True):
        per = self.num_samples // self.world
        return per // self.batch_size if drop_remainder else -(-per // self.batch_size)

    def epoch(self, epoch):
        for s in list(self._held):  # a new epoch recycles every slot
            self.release(s)
        n = self._L.start_epoch(int(epoch))
        mon = monitoring.enabled()
        for _ in range(n):
            t0 = time.perf_counter()
            slot, count = self._L.next()
            if mon:
                monitoring.observe(monitoring.GETNEXT, (time.perf_counter() - t0) * 1e6, source="native_loader")
            if slot < 0:
                return
            self._held.add(slot)
            yield slot, [t[:count] for t in self._slots[slot]]

    def release(self, slot):
        self._held.discard(slot)
        self._L.release(int(slot))


class DeviceLoader:
    """Batches on the GPU: ``x`` normalised to bf16 (array 0, uint8 images), the other
    arrays copied as they are (labels).  H2D + normalisation of batch k+1 overlap
    the training of batch k (copy stream + event)."""

    def __init__(self, host: NpyBatchLoader, device=None, mean=(0.0,), std=(255.0,)):
        self.host = host
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.mean = [float(m) for m in mean]
        self.std = [float(s) for s in std]
        self.copy_stream = torch.cuda.Stream(self.device)

    def _stage(self, arrays):
        from ..ops import _ext

        ext = _ext.load(required=True)
        out = []
        with torch.cuda.stream(self.copy_stream):
            for i, a in enumerate(arrays):
                d = torch.empty(a.shape, dtype=a.dtype, device=self.device)
                d.copy_(a, non_blocking=True)
                if i == 0 and a.dtype == torch.uint8:
                    C = a.shape[-1]
                    mean = self.mean * C if len(self.mean) == 1 else self.mean
                    std = self.std * C if len(self.std) == 1 else self.std
                    y = torch.empty(a.shape, dtype=torch.bfloat16, device=self.device)
                    ext.u8_normalize(d.data_ptr(), y.data_ptr(), d.numel(), mean, std,
                                     self.copy_stream.cuda_stream)
                    d = y
                out.append(d)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        return out, ev

    def epoch(self, epoch):
        main = torch.cuda.current_stream(self.device)
        it = self.host.epoch(epoch)
        pending = None
        for slot, arrays in it:
            staged = (slot,) + self._stage(arrays)
            if pending is not None:
                yield self._hand_over(pending, main)
            pending = staged
        if pending is not None:
            yield self._hand_over(pending, main)

    def _hand_over(self, staged, main):
        slot, out, ev = staged
        main.wait_event(ev)
        for t in out:
            t.record_stream(main)  # allocated on the copy stream, consumed on the training stream
        ev.synchronize()  # the pinned slot may be refilled only after its copy has landed
        self.host.release(slot)
        return out


def write_npy_dataset(directory, n, image_shape=(224, 224, 3), classes=1000, seed=0, chunk=1024):
    """Synthetic uint8 image set + int64 labels as ``x.npy`` / ``y.npy`` (written in chunks
    through a memory map, so n x 150 KB images never sit in memory at once)."""
    os.makedirs(directory, exist_ok=True)
    xp, yp = os.path.join(directory, "x.npy"), os.path.join(directory, "y.npy")
    rng = np.random.default_rng(seed)
    x = np.lib.format.open_memmap(xp, mode="w+", dtype=np.uint8, shape=(n,) + tuple(image_shape))
    for i in range(0, n, chunk):
        j = min(n, i + chunk)
        x[i:j] = rng.integers(0, 256, size=(j - i,) + tuple(image_shape), dtype=np.uint8)
    x.flush()
    del x
    np.save(yp, rng.integers(0, classes, size=n).astype(np.int64))
    return xp, yp
