"""``tf.keras.datasets``-shaped loaders.

There is no network on MI355X job nodes, so these return SYNTHETIC data of the
real datasets' shapes and dtypes (deterministic, class-conditional patterns so
small models can actually learn them).  If a real ``.npz`` is present at
``$CLOUD_AMD_DATA/<name>.npz`` (keys x_train, y_train, x_test, y_test) it is
loaded instead (numpy, no pickle).
"""
from __future__ import annotations

import os

import numpy as np


def _real(name):
    root = os.environ.get("CLOUD_AMD_DATA")
    if root:
        p = os.path.join(root, f"{name}.npz")
        if os.path.exists(p):
            d = np.load(p)
            return (d["x_train"], d["y_train"]), (d["x_test"], d["y_test"])
    return None


def _synthetic_images(n, shape, classes, seed, proto_seed=1234):
    protos = np.random.default_rng(proto_seed).integers(0, 256, size=(classes,) + shape).astype(np.float32)
    rng = np.random.default_rng(seed)
    y = rng.integers(0, classes, size=n).astype(np.uint8)
    noise = rng.normal(0, 40, size=(n,) + shape).astype(np.float32)
    x = np.clip(protos[y] * 0.6 + noise + 50, 0, 255).astype(np.uint8)
    return x, y


class mnist:
    @staticmethod
    def load_data(path="mnist.npz", n_train=60000, n_test=10000):
        real = _real("mnist")
        if real is not None:
            return real
        xtr, ytr = _synthetic_images(n_train, (28, 28), 10, 0)
        xte, yte = _synthetic_images(n_test, (28, 28), 10, 1)
        return (xtr, ytr), (xte, yte)


class fashion_mnist(mnist):
    pass


class cifar10:
    @staticmethod
    def load_data(n_train=50000, n_test=10000):
        real = _real("cifar10")
        if real is not None:
            return real
        xtr, ytr = _synthetic_images(n_train, (32, 32, 3), 10, 2)
        xte, yte = _synthetic_images(n_test, (32, 32, 3), 10, 3)
        return (xtr, ytr.reshape(-1, 1)), (xte, yte.reshape(-1, 1))
