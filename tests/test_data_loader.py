"""Native input pipeline (csrc/data/loader.cpp via cloud_amd.data): sharding,
shuffling, determinism, drop_remainder, .npy parsing, error paths."""
import numpy as np
import pytest
import torch

from cloud_amd.data import NpyBatchLoader, write_npy_dataset


def _files(tmp_path, n=103):
    x = np.arange(n * 2 * 3, dtype=np.uint8).reshape(n, 2, 3) % 251
    x[:, 0, 0] = np.arange(n) % 256  # identify the sample
    y = np.arange(n, dtype=np.int64) * 7
    xp, yp = tmp_path / "x.npy", tmp_path / "y.npy"
    np.save(xp, x)
    np.save(yp, y)
    return x, y, xp, yp


def _collect(ld, epoch):
    ys, sizes = [], []
    for slot, (xb, yb) in ld.epoch(epoch):
        ys.append(yb.clone())
        sizes.append(len(yb))
        # the gathered rows are the right samples
        assert torch.equal(xb[:, 0, 0].long(), (yb // 7) % 256)
        ld.release(slot)
    return torch.cat(ys) if ys else torch.empty(0, dtype=torch.long), sizes


def test_two_ranks_disjoint_and_cover(tmp_path):
    x, y, xp, yp = _files(tmp_path)
    seen = []
    for r in range(2):
        ld = NpyBatchLoader([xp, yp], 10, shuffle=True, seed=3, rank=r, world=2, threads=3, slots=3)
        got, sizes = _collect(ld, 0)
        assert sizes == [10] * 5  # 103 // 2 = 51 per rank -> 5 full batches
        seen.append(set((got // 7).tolist()))
    assert not (seen[0] & seen[1])
    assert len(seen[0]) == len(seen[1]) == 50


def test_shuffle_deterministic_and_epoch_dependent(tmp_path):
    _, _, xp, yp = _files(tmp_path)
    a = NpyBatchLoader([xp, yp], 8, seed=5, rank=0, world=1, threads=4)
    b = NpyBatchLoader([xp, yp], 8, seed=5, rank=0, world=1, threads=1)
    e0a, _ = _collect(a, 0)
    e0b, _ = _collect(b, 0)
    e1a, _ = _collect(a, 1)
    assert torch.equal(e0a, e0b)  # thread count does not change the order
    assert not torch.equal(e0a, e1a)
    assert sorted(e0a.tolist()) != e0a.tolist()


def test_no_shuffle_strided_and_remainder(tmp_path):
    _, y, xp, yp = _files(tmp_path, n=23)
    ld = NpyBatchLoader([xp, yp], 4, shuffle=False, rank=1, world=2, drop_remainder=False, slots=2)
    got, sizes = _collect(ld, 0)
    assert got.tolist() == list(y[1:22:2])  # 23 // 2 = 11 per rank
    assert sizes == [4, 4, 3]


def test_mismatched_arrays_and_bad_args(tmp_path):
    x, y, xp, yp = _files(tmp_path)
    np.save(tmp_path / "short.npy", y[:5])
    with pytest.raises(Exception):
        NpyBatchLoader([xp, tmp_path / "short.npy"], 4, rank=0, world=1)
    with pytest.raises(ValueError):
        NpyBatchLoader([xp, yp], 4, rank=0, world=1, slots=1)
    np.save(tmp_path / "f.npy", np.asfortranarray(np.ones((4, 3, 2), dtype=np.float32)))
    with pytest.raises(Exception):
        NpyBatchLoader([tmp_path / "f.npy"], 2, rank=0, world=1)


def test_write_npy_dataset_roundtrip(tmp_path):
    xp, yp = write_npy_dataset(tmp_path / "ds", 37, image_shape=(8, 8, 3), classes=10, chunk=16)
    x = np.load(xp)
    assert x.shape == (37, 8, 8, 3) and x.dtype == np.uint8
    ld = NpyBatchLoader([xp, yp], 5, seed=1, rank=0, world=1)
    n = 0
    for slot, (xb, yb) in ld.epoch(0):
        assert xb.dtype == torch.uint8 and yb.dtype == torch.int64
        n += len(yb)
        ld.release(slot)
    assert n == 35
