#!/usr/bin/env python3
"""Which PyTorch ops still run in a steady-state Keras fit step (reference MNIST CNN)?
Logs every aten op of 3 fit steps through a TorchDispatchMode (autograd backward included)
with the innermost cloud_amd frame that issued it."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cloud_amd import keras  # noqa: E402


def main():
    model = keras.Sequential([
        keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
        keras.layers.MaxPooling2D(),
        keras.layers.Flatten(),
        keras.layers.Dense(64, activation="relu"),
        keras.layers.Dense(10, activation="softmax"),
    ])
    model.compile(loss="sparse_categorical_crossentropy", optimizer=keras.optimizers.Adam(), metrics=["accuracy"])
    (x, y), _ = keras.datasets.mnist.load_data(n_train=4096, n_test=64)
    x = (x[..., None] / np.float32(255)).astype("float32")
    model.fit(x, y, batch_size=64, epochs=1, verbose=0)  # warm
    import traceback

    from torch.utils._python_dispatch import TorchDispatchMode

    skip = {"view", "reshape", "_reshape_alias", "as_strided", "detach", "t", "transpose", "slice", "expand",
            "empty", "empty_strided", "select", "unsqueeze", "squeeze", "alias", "permute", "_unsafe_view",
            "empty_like", "new_empty", "new_empty_strided", "lift_fresh", "_local_scalar_dense", "is_nonzero",
            "set_", "resize_", "clone_", "split", "unbind", "narrow", "view_as", "_to_copy_noop"}
    seen = {}

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            name = func.overloadpacket.__name__
            if name not in skip:
                fr = [f for f in traceback.extract_stack()[:-1] if "cloud_amd" in f.filename]
                where = ("%s:%d %s" % (fr[-1].filename.split("cloud_amd/")[-1], fr[-1].lineno, fr[-1].name)
                         if fr else "?")
                seen[(name, where)] = seen.get((name, where), 0) + 1
            return out

    steps = 3
    with Log():
        model.fit(x[:64 * steps], y[:64 * steps], batch_size=64, epochs=1, verbose=0)
    print("aten ops per fit() of %d steps (view ops skipped); count, op, innermost cloud_amd frame" % steps)
    for (name, fr), n in sorted(seen.items(), key=lambda kv: -kv[1]):
        print("%4d  %-24s %s" % (n, name, fr))


if __name__ == "__main__":
    main()
