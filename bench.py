#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 training throughput on synthetic ImageNet.

Metric (BASELINE.json): images/sec of ResNet-50 training at 1/2/4/8 MI355X,
one process per GPU, data parallel over RCCL/xGMI, bf16 compute with fp32
master weights, SGD(momentum 0.9) -- plus ``first_step_latency_s`` (process
start -> end of first optimizer step) and, with ``--via-run 1``, the launch
through ``cloud_amd.run()`` and ``run_to_first_step_s`` (run() call -> end of
the first step on every rank, max over ranks).

    python bench.py --gpus 1 --steps 20 --warmup 10
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 10

Weak scaling: the per-GPU batch is fixed (``--batch``, default 512), global batch =
batch x N.  512 images per GPU is sized for 288 GB of HBM3E (``peak_mem_gb`` in the
JSON line reports the step's peak) and halves the per-image share of the step's fixed
costs (~570 kernel boundaries at ~1.8 us each, per-layer BN finalize kernels)
relative to 256; the sweep 128..1024 and the stock comparator at 256 and 512
are in BASELINE.md.
Synthetic data: random NHWC bf16 images and random labels, generated once on
the device (no input pipeline in the timed region, as in tf_cnn_benchmarks'
synthetic mode).  Random-init weights.  Every timed step runs the full forward,
backward, gradient all-reduce and fused optimizer update.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_START = time.time()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("CLOUD_AMD_BENCH_BATCH", 512)),
                    help="per-GPU batch")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--graph", type=int, default=int(os.environ.get("CLOUD_AMD_GRAPH", "0")),
                    help="capture the training step in a HIP graph (1-GPU only unless forced)")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--via-run", type=int, default=0,
                    help="launch through cloud_amd.run() (stage -> spawn one rank per GPU) and report "
                         "run()->first-step latency; the ranks' JSON line is streamed from rank 0's log")
    return ap.parse_args()


def via_run(args):
    """The BASELINE metric's 'via run()' form: this process only stages and launches
    (it never touches the GPU); every rank re-runs this file with remote() True."""
    import cloud_amd as tfc

    argv = [a for a in sys.argv[1:]]
    if "--via-run" in argv:
        i = argv.index("--via-run")
        del argv[i:i + 2]
    cfg = tfc.COMMON_MACHINE_CONFIGS["MI355X_%dX" % args.gpus]
    os.chdir(os.path.dirname(os.path.abspath(__file__)))
    job = tfc.run(entry_point="bench.py", distribution_strategy=None, chief_config=cfg, worker_count=0,
                  entry_point_args=argv, stream_logs=True, exit=False, wait=True)
    sys.exit(job.returncode or 0)


def main():
    args = parse()
    if args.via_run and not (os.environ.get("CLOUD_AMD_RUNNING_REMOTELY") or os.environ.get("TORCHELASTIC_RUN_ID")):
        return via_run(args)
    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cloud_amd.models import resnet50
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD
    from cloud_amd.parallel.ddp import GradAllReducer
    from cloud_amd.utils import dist_env

    rank, world, device = dist_env.init_distributed()
    if world != args.gpus and rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.manual_seed(1234)  # identical init on every rank (also broadcast below)
    B, S = args.batch, args.image_size
    model = resnet50(num_classes=args.classes, dtype=torch.bfloat16, device=device)
    opt = SGD(model, learning_rate=args.lr, momentum=0.9, weight_decay=5e-5, grad_scale=1.0 / world)
    reducer = GradAllReducer(opt.arenas)
    reducer.broadcast_parameters()

    gen = torch.Generator(device=device)
    gen.manual_seed(1000 + rank)
    x = torch.randn((B, S, S, 3), generator=gen, device=device, dtype=torch.float32).to(torch.bfloat16)
    y = torch.randint(0, args.classes, (B,), generator=gen, device=device)
    global_batch = B * world

    from cloud_amd.utils import trace

    def fwd_bwd():
        with trace.range("forward"):
            logits = model(x)
            loss, _ = softmax_cross_entropy(logits, y, denom=B)
        with trace.range("backward"):
            loss.backward()
        return loss.detach()  # never keep the autograd graph alive across steps (graph capture)

    def train_step():
        opt.zero_grad()
        loss = fwd_bwd()
        with trace.range("allreduce_join"):
            reducer.finish()
        with trace.range("optimizer"):
            opt.step()
        return loss

    # first step = end-to-end "first-step latency" (process start -> step done)
    loss = train_step()
    torch.cuda.synchronize()
    first_step_latency = time.time() - T_START
    run_t0 = os.environ.get("CLOUD_AMD_RUN_T0")
    run_to_first = (time.time() - float(run_t0)) if run_t0 else None

    use_graph = bool(args.graph) and (world == 1 or os.environ.get("CLOUD_AMD_GRAPH_FORCE") == "1")
    step_fn = train_step
    if use_graph:
        loss = None
        from cloud_amd.runtime.graph import capture_train_step

        step_fn = capture_train_step(fwd_bwd, opt, reducer, warmup=3)

    for _ in range(max(args.warmup - 1, 0)):
        loss = step_fn()
    dist_env.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step_fn()
    torch.cuda.synchronize()
    dist_env.barrier()
    t1 = time.perf_counter()
    elapsed = dist_env.all_reduce_max(t1 - t0, device)
    ms = elapsed / args.steps * 1000.0
    ips = global_batch * args.steps / elapsed
    first_lat = dist_env.all_reduce_max(first_step_latency, device)
    if run_to_first is not None:
        run_to_first = dist_env.all_reduce_max(run_to_first, device)
    final_loss = float(loss.detach().float().item()) if loss is not None else float("nan")
    try:
        from cloud_amd import monitoring

        monitoring.gauge(monitoring.THROUGHPUT, ips)
        monitoring.gauge(monitoring.FIRST_STEP, first_lat)
        monitoring.observe(monitoring.STEP_TIME, ms)
    except Exception:
        pass
    if rank == 0:
        out = {
            "metric": "images/sec ResNet-50 via run() at 1/2/4/8 MI355X; run()→first-step latency",
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random NHWC bf16 images + random labels, random-init weights)",
            "config": {"model": "resnet50", "global_batch": global_batch, "seq_len": None,
                       "image_size": S, "per_gpu_batch": B, "parallelism": f"dp{world}",
                       "optimizer": "sgd_momentum0.9_fused", "hip_graph": use_graph},
            "first_step_latency_s": round(first_lat, 3),
            "run_to_first_step_s": round(run_to_first, 3) if run_to_first is not None else None,
            "launched_via": "cloud_amd.run()" if run_t0 else "direct",
            "final_loss": round(final_loss, 4),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 2**30, 2),
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
