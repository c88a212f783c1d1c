#!/usr/bin/env python3
"""Stock PyTorch-ROCm comparator for the headline metric (BASELINE.md "Stock").

Plain ``torch.nn`` ResNet-50 v1.5 (no torchvision in this image, so the module
tree is written out here), ``channels_last`` memory format, bf16 autocast with
fp32 weights, ``torch.optim.SGD(momentum=0.9, foreach=True)``, and
``DistributedDataParallel`` (RCCL, default 25 MB buckets) when WORLD_SIZE > 1.
Same synthetic data and same JSON line as ../bench.py, launched the same way: through
``cloud_amd.run()`` (``--via-run 1``, the default; one rank per GPU) or in-process.
MIOpen compiles its kernels during the first steps (minutes at batch 1024): a heartbeat
line every 30 s shows the run is alive.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        o = F.relu(self.bn1(self.conv1(x)))
        o = F.relu(self.bn2(self.conv2(o)))
        return F.relu(self.bn3(self.conv3(o)) + idt)


class ResNet50(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        blocks, cin = [], 64
        for i, (n, w) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
            for j in range(n):
                blocks.append(Bottleneck(cin, w, 2 if (j == 0 and i > 0) else 1))
                cin = w * 4
        self.layers = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, classes)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.layers(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024, help="per-GPU batch (bench.py's default)")
    ap.add_argument("--layout", default="nhwc", choices=["nhwc", "nchw"])
    ap.add_argument("--precision", default="amp", choices=["amp", "bf16"])
    ap.add_argument("--benchmark", type=int, default=0, help="torch.backends.cudnn.benchmark (MIOpen find)")
    ap.add_argument("--via-run", type=int, default=1, help="1: launch the ranks through cloud_amd.run()")
    args = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from cloud_amd.utils import benchlaunch

    if args.via_run and not benchlaunch.inside_launched_rank():
        return benchlaunch.launch_via_run(os.path.abspath(__file__), args.gpus, tag="stock_resnet50")
    t_start = time.time()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    benchlaunch.check_world(args.gpus, world, tag="stock_resnet50")
    phase = {"what": "setup", "t": time.time()}
    done = threading.Event()

    def heartbeat():
        while not done.wait(30.0):
            print("[stock_resnet50] rank %d: %s, %.0f s" % (rank, phase["what"], time.time() - phase["t"]), flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    lr = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", lr)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = bool(args.benchmark)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.distributed.init_process_group("nccl")
    mf = torch.channels_last if args.layout == "nhwc" else torch.contiguous_format
    model = ResNet50().to(dev, memory_format=mf)
    if args.precision == "bf16":
        model = model.to(torch.bfloat16)
    ddp = model
    if world > 1:
        ddp = nn.parallel.DistributedDataParallel(model, device_ids=[lr])
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)
    x = torch.randn(args.batch, 3, 224, 224, device=dev).to(memory_format=mf)
    if args.precision == "bf16":
        x = x.to(torch.bfloat16)
    y = torch.randint(0, 1000, (args.batch,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.precision == "amp"):
            loss = F.cross_entropy(ddp(x).float(), y)
        loss.backward()
        opt.step()
        return loss

    phase.update(what="first step (MIOpen kernel compilation)", t=time.time())
    step()
    torch.cuda.synchronize()
    first = time.time() - t_start
    for i in range(args.warmup - 1):
        phase.update(what="warmup step %d" % (i + 2), t=time.time())
        step()
        torch.cuda.synchronize()
    phase.update(what="timed steps", t=time.time())
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t)
    if rank == 0:
        print(json.dumps({"metric": "images/sec ResNet-50 (stock torch comparator)",
                          "value": round(args.batch * world * args.steps / el, 2), "unit": "images/sec",
                          "n_gpus": world, "ms_per_step": round(el / args.steps * 1000, 3),
                          "config": {"layout": args.layout, "precision": args.precision, "batch": args.batch,
                                     "benchmark": args.benchmark},
                          "first_step_latency_s": round(first, 3), "launched_via": benchlaunch.launched_via(),
                          "run_to_first_step_s": (round(t_start + first - float(os.environ["CLOUD_AMD_RUN_T0"]), 3)
                                                  if os.environ.get("CLOUD_AMD_RUN_T0") else None),
                          "loss": float(loss)}), flush=True)
    done.set()


if __name__ == "__main__":
    main()
