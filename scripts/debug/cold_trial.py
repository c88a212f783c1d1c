#!/usr/bin/env python3
"""Where a tuner worker's first (cold) trial spends its time: one process, the tuner
bench's MNIST CNN, phase wall times and a cProfile of the first fit (top entries by
cumulative time), then a second, warm trial for comparison."""
import cProfile
import os
import pstats
import sys
import time

t0 = time.time()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

t_torch = time.time()
from bench.tuner_8trials import build_model  # noqa: E402
from cloud_amd import keras  # noqa: E402
from cloud_amd.tuner import HyperParameters  # noqa: E402

t_imp = time.time()
torch.cuda.set_device(0)
t_dev = time.time()
(x, y), (xt, yt) = keras.datasets.mnist.load_data(n_train=8192, n_test=1024)
x = (x[..., None] / np.float32(255)).astype("float32")
xt = (xt[..., None] / np.float32(255)).astype("float32")
t_data = time.time()
print(f"import torch {t_torch - t0:.3f}s  cloud_amd+keras {t_imp - t_torch:.3f}s  set_device {t_dev - t_imp:.3f}s  "
      f"data {t_data - t_dev:.3f}s", flush=True)
for trial in range(2):
    hp = HyperParameters()
    ta = time.time()
    model = build_model(hp)
    tb = time.time()
    prof = cProfile.Profile() if trial == 0 else None
    if prof:
        prof.enable()
    model.fit(x, y, epochs=2, batch_size=128, validation_data=(xt, yt), verbose=0)
    torch.cuda.synchronize()
    if prof:
        prof.disable()
    tc = time.time()
    print(f"trial {trial}: build {tb - ta:.3f}s fit {tc - tb:.3f}s", flush=True)
    if prof:
        pstats.Stats(prof).sort_stats("cumulative").print_stats(45)
