#!/usr/bin/env python3
"""Native input pipeline throughput on MI355X (cloud_amd.data):

1. host loader alone (C++ workers: mmap'd .npy -> shuffled batches in pinned slots);
2. DeviceLoader alone (+ H2D on the copy stream + uint8 -> bf16 normalisation);
3. ResNet-50 training (bench.py's step, batch --batch) fed by the DeviceLoader,
   against the same step on a resident synthetic batch.

The dataset is synthetic uint8 ImageNet-shaped data written to --dir first
(no network, no decode).  One JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/cloud_amd_synth_imagenet")
    ap.add_argument("--images", type=int, default=8192)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--steps", type=int, default=12)
    a = ap.parse_args()
    from cloud_amd.data import DeviceLoader, NpyBatchLoader, write_npy_dataset

    t0 = time.time()
    xp, yp = write_npy_dataset(a.dir, a.images, image_shape=(224, 224, 3), classes=1000, seed=0)
    print(json.dumps({"stage": "write_dataset", "images": a.images, "s": round(time.time() - t0, 2)}), flush=True)
    host = NpyBatchLoader([xp, yp], a.batch, seed=0, rank=0, world=1, threads=a.threads, slots=4)
    n = 0
    t0 = time.time()
    for slot, (xb, yb) in host.epoch(0):
        n += len(yb)
        host.release(slot)
    dt = time.time() - t0
    print(json.dumps({"stage": "host_loader", "images_per_s": round(n / dt, 1), "threads": a.threads}), flush=True)

    dev = torch.device("cuda", 0)
    dl = DeviceLoader(host, device=dev, mean=(123.7, 116.3, 103.5), std=(58.4, 57.1, 57.4))
    torch.cuda.synchronize()
    n = 0
    t0 = time.time()
    for x, y in dl.epoch(1):
        n += x.shape[0]
    torch.cuda.synchronize()
    dt = time.time() - t0
    print(json.dumps({"stage": "device_loader", "images_per_s": round(n / dt, 1)}), flush=True)

    from cloud_amd.models import resnet50
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD

    model = resnet50(num_classes=1000, dtype=torch.bfloat16, device=dev)
    opt = SGD(model, learning_rate=0.1, momentum=0.9, weight_decay=5e-5)

    def step(x, y):
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(model(x), y, denom=x.shape[0])
        loss.backward()
        opt.step()
        return loss

    xs = torch.randn(a.batch, 224, 224, 3, device=dev).to(torch.bfloat16)
    ys = torch.randint(0, 1000, (a.batch,), device=dev)
    for _ in range(3):
        step(xs, ys)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(a.steps):
        step(xs, ys)
    torch.cuda.synchronize()
    synth = a.steps * a.batch / (time.time() - t0)
    epoch, done, t0 = 2, 0, None
    while done < a.steps + 3:
        for x, y in dl.epoch(epoch):
            if done == 3:
                torch.cuda.synchronize()
                t0 = time.time()
            step(x, y)
            done += 1
            if done >= a.steps + 3:
                break
        epoch += 1
    torch.cuda.synchronize()
    fed = a.steps * a.batch / (time.time() - t0)
    print(json.dumps({"stage": "resnet50_train", "batch": a.batch, "synthetic_images_per_s": round(synth, 1),
                      "loader_fed_images_per_s": round(fed, 1)}), flush=True)


if __name__ == "__main__":
    main()
