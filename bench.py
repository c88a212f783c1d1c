#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 training throughput on synthetic ImageNet, launched
through ``cloud_amd.run()``.

Metric (BASELINE.json): images/sec of ResNet-50 training **via run()** at 1/2/4/8
MI355X, one process per GPU, data parallel over RCCL/xGMI, bf16 compute with fp32
master weights, SGD(momentum 0.9) -- plus ``run_to_first_step_s`` (``run()`` call ->
end of the first optimizer step on every rank, max over ranks).

    python bench.py --gpus 8 --steps 20 --warmup 10          # stages + spawns 8 ranks via run()
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 10   # ranks started by torchrun

Launch modes:

* **not inside a launched job** (no ``WORLD_SIZE`` / ``CLOUD_AMD_RUNNING_REMOTELY`` /
  ``TORCHELASTIC_RUN_ID``): this process only stages the job and spawns ``--gpus``
  ranks through ``cloud_amd.run(chief_config=MI355X_<N>X)`` -- the reference's
  ``run()`` -> strategy auto-selection -> multi-replica job path
  (reference ``TFC/core/preprocess.py:137-146``, ``TFC/core/deploy.py:98-167``).  It
  never touches the GPU: the launcher counts devices from KFD sysfs.  A node with
  fewer GPUs than ``--gpus`` fails validation and exits non-zero.
* **inside a rank** (spawned by run() or torchrun): trains; the world size actually
  seen by torch.distributed MUST equal ``--gpus`` or the rank exits non-zero.

Weak scaling: the per-GPU batch is fixed (``--batch``, default 1024), global batch =
batch x N.  1024 images per GPU use 41 GB of the 288 GB of HBM3E and make the 8-GPU
global batch 8,192 -- the large-batch ImageNet setting (Goyal et al., 2017).  Measured on
one MI355X (``profiles/r2_batch_sweep``): 11,603 / 12,098 / 12,436 / 12,671 / 12,727 img/s
at 512 / 768 / 1024 / 1536 / 2048 per GPU; larger batches amortise the fixed part of a step
(kernel boundaries, per-layer statistics finalize kernels).  Synthetic data: random NHWC bf16 images and random labels generated once
on the device; random-init weights.  Every timed step runs the full forward,
backward, bucketed gradient all-reduce (overlapped with backward) and fused
optimizer update.  The JSON line carries the communication breakdown of the timed
steps: bucket count, all-reduce ms and exposed (not overlapped) communication ms.

``--model tiny --device cpu`` runs the same code path on a small bottleneck ResNet on
CPU ranks over gloo (CPU tests of the launch contract); its numbers are not a metric.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_START = time.time()
METRIC = "images/sec ResNet-50 via run() at 1/2/4/8 MI355X; run()→first-step latency"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per MI355X)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (ResNet-50 default 1024 or CLOUD_AMD_BENCH_BATCH: 41 GB of the 288 GB "
                         "HBM3E; 8 GPUs -> the 8,192-image global batch of large-batch ImageNet training; "
                         "--model tiny default 8)")
    ap.add_argument("--image-size", type=int, default=None, help="default 224 (ResNet-50), 32 (--model tiny)")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--model", choices=("resnet50", "tiny"), default="resnet50")
    ap.add_argument("--device", choices=("auto", "cpu"), default="auto")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="gradient all-reduce bucket size (default CLOUD_AMD_BUCKET_MB or 16)")
    ap.add_argument("--grad-reduce-dtype", choices=("auto", "bf16", "fp32", "native"), default=None,
                    help="wire dtype of the gradient all-reduce (default auto: bf16 for every bucket of a bf16 model)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--ab", type=int, default=1,
                    help="N > 1: after the timed region, a <= 5-step A/B per DP-engine cell (per-bucket optimizer "
                         "on/off x buckets 16/32/64 MB x torch/native RCCL; CLOUD_AMD_BENCH_AB selects cells)")
    ap.add_argument("--ab-steps", type=int, default=5)
    ap.add_argument("--via-run", type=int, default=int(os.environ.get("CLOUD_AMD_BENCH_VIA_RUN", "1")),
                    help="1 (default): launch the ranks through cloud_amd.run(); 0: train in this process")
    return ap.parse_args(argv)


def _finite(o):
    """NaN / inf -> None: the JSON line must be strict JSON (json.dumps allow_nan=False)."""
    if isinstance(o, float):
        return o if o == o and o not in (float("inf"), float("-inf")) else None
    if isinstance(o, dict):
        return {k: _finite(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_finite(v) for v in o]
    return o


def via_run(args):
    """Stage this script and launch ``--gpus`` ranks through ``cloud_amd.run()``.
    This process never initialises HIP; rank 0's log (ending in the JSON line) is
    streamed to stdout and the job's exit code becomes ours."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cloud_amd.utils import benchlaunch

    benchlaunch.launch_via_run(os.path.abspath(__file__), args.gpus, device=args.device)


def main():
    args = parse()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cloud_amd.utils import benchlaunch

    if args.via_run and not benchlaunch.inside_launched_rank():
        return via_run(args)
    import torch

    from cloud_amd import config
    from cloud_amd.models import resnet50
    from cloud_amd.models.resnet import resnet18_like_small
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD
    from cloud_amd.parallel import strategy as strategy_mod
    from cloud_amd.runtime import gc_control
    from cloud_amd.utils import dist_env, trace

    if args.device == "cpu":
        os.environ.setdefault("CLOUD_AMD_DEVICE", "cpu")
    # The DP engine comes from the distribution strategy: the one run()'s generated wrapper
    # installed (distribution_strategy="auto": MirroredStrategy at N > 1, OneDeviceStrategy at
    # 1 -- reference TFC/core/preprocess.py:137-146), or the default for a torchrun rank.
    strategy = strategy_mod.get_strategy()
    device = strategy.device
    rank, world = strategy.rank, strategy.num_replicas_in_sync
    benchlaunch.check_world(args.gpus, world)
    on_gpu = device.type == "cuda"
    if not on_gpu and args.model == "resnet50" and os.environ.get("CLOUD_AMD_BENCH_ALLOW_CPU") != "1":
        print("[bench] error: ResNet-50 bench needs a GPU (use --model tiny --device cpu for CPU runs)",
              file=sys.stderr)
        sys.exit(3)
    dtype = torch.bfloat16 if on_gpu else torch.float32
    torch.manual_seed(1234)  # identical init on every rank (also broadcast below)
    if args.batch is None:
        args.batch = int(os.environ.get("CLOUD_AMD_BENCH_BATCH", 1024)) if args.model == "resnet50" else 8
    if args.image_size is None:
        args.image_size = 224 if args.model == "resnet50" else 32
    B, S = args.batch, args.image_size
    build = resnet50 if args.model == "resnet50" else resnet18_like_small
    model = build(num_classes=args.classes, dtype=dtype, device=device)
    # mean over the GLOBAL batch: every rank holds B samples, so 1/world folds into the optimizer
    opt = SGD(model, learning_rate=args.lr, momentum=0.9, weight_decay=5e-5, grad_scale=1.0 / world)
    reducer = strategy.gradient_reducer(opt.arenas, bucket_mb=args.bucket_mb, reduce_dtype=args.grad_reduce_dtype)
    reducer.broadcast_parameters()
    # world > 1 (RCCL): bucket k's fused update runs as its all-reduce completes
    sliced = reducer.attach_optimizer(opt)

    gen = torch.Generator(device=device)
    gen.manual_seed(1000 + rank)
    x = torch.randn((B, S, S, 3), generator=gen, device=device, dtype=torch.float32).to(dtype)
    y = torch.randint(0, args.classes, (B,), generator=gen, device=device)
    global_batch = B * world

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def fwd_bwd():
        with trace.range("forward"):
            logits = model(x)
            loss, _ = softmax_cross_entropy(logits, y, denom=B)
        with trace.range("backward"):
            loss.backward()
        return loss.detach()  # never keep the autograd graph alive across steps

    holder = {"red": reducer}  # the DP A/B cells after the timed region swap reducers

    def train_step():
        opt.zero_grad()
        loss = fwd_bwd()
        with trace.range("allreduce_join"):
            holder["red"].finish()
        with trace.range("optimizer"):
            opt.step()
        return loss

    # first step = end-to-end "first-step latency" (process start -> step done)
    loss = train_step()
    sync()
    t_first_done = time.time()
    first_step_latency = t_first_done - T_START
    phases = benchlaunch.startup_phases(T_START, t_first_done)
    run_t0 = os.environ.get("CLOUD_AMD_RUN_T0")
    run_to_first = (time.time() - float(run_t0)) if run_t0 else None

    # (HIP-graph capture of this step measured slower than eager on ROCm 7.2 at b256/b512:
    # kernel boundaries cost the same in a graph; not offered here -- docs/performance.md)
    step_fn = train_step
    # the fused optimizer's step() keeps at most CLOUD_AMD_MAX_STEPS_IN_FLIGHT steps queued ahead
    # of the GPU (warmup and timed steps alike, runtime/step_pacer.py), so the caching allocator's
    # pool is complete before the timed region
    pacer = opt.pacer
    for _ in range(max(args.warmup - 1, 0)):
        loss = step_fn()
    # desync check once after warmup (world > 1): every replica must hold identical
    # all-reduced gradients (fp64 fingerprint over all arenas, all-gathered)
    replicas_consistent = None
    if world > 1:
        try:
            replicas_consistent = bool(reducer.check_consistency())
        except RuntimeError as e:
            replicas_consistent = False
            print("[bench] %s" % e, file=sys.stderr, flush=True)
    dist_env.barrier()
    sync()
    # everything alive now (model, optimizer state, imports) leaves the collector's full passes
    gc_frozen = gc_control.freeze()
    reducer.timing_start()
    reducer.probe_readiness()  # per-bucket gradient-ready events -> overlap budget (any world size)
    host0 = benchlaunch.host_state()
    step_probe = benchlaunch.StepProbe(cuda=on_gpu)
    # per-step device time from events on the compute stream and per-step host launch time
    # (no added synchronisation: events are read after the closing sync)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if on_gpu else None
    host_ms = []
    paced_ms = []  # per step: host time blocked in the run-ahead bound (host_ms minus this = launch time)
    t0 = time.perf_counter()
    if evs:
        evs[0].record()
    for i in range(args.steps):
        th = time.perf_counter()
        w0 = pacer.wait_ms if pacer is not None else 0.0
        loss = step_fn()
        if evs:
            evs[i + 1].record()
        host_ms.append((time.perf_counter() - th) * 1e3)
        paced_ms.append((pacer.wait_ms if pacer is not None else 0.0) - w0)
        step_probe.mark()
    sync()
    dist_env.barrier()
    t1 = time.perf_counter()
    step_stats = benchlaunch.step_stats(
        [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)] if evs else None, host_ms,
        host0, benchlaunch.host_state(), probe=step_probe.close(), paced_ms=paced_ms)
    comm = reducer.timing_summary()
    budget = reducer.overlap_budget(optimizer=opt)
    per_rank_ms = [v / args.steps * 1000.0 for v in dist_env.all_gather_floats(t1 - t0, device)]
    elapsed = dist_env.all_reduce_max(t1 - t0, device)
    ms = elapsed / args.steps * 1000.0
    busbw = dist_env.allreduce_busbw(device) if world > 1 else None  # after the timed steps
    # both transports on the same buffers: decides the default data plane (CLOUD_AMD_COMM)
    probe = dist_env.comm_probe(device) if world > 1 else None
    ips = global_batch * args.steps / elapsed
    first_lat = dist_env.all_reduce_max(first_step_latency, device)
    if run_to_first is not None:
        run_to_first = dist_env.all_reduce_max(run_to_first, device)
    comm["allreduce_ms"] = dist_env.all_reduce_max(comm["allreduce_ms"], device)
    comm["exposed_comm_ms"] = dist_env.all_reduce_max(comm["exposed_comm_ms"], device)
    final_loss = float(loss.detach().float().item()) if loss is not None else float("nan")
    try:
        from cloud_amd import monitoring

        monitoring.gauge(monitoring.THROUGHPUT, ips)
        monitoring.gauge(monitoring.FIRST_STEP, first_lat)
        monitoring.observe(monitoring.STEP_TIME, ms)
    except Exception:
        pass
    out = None
    if rank == 0:
        launched = benchlaunch.launched_via()
        backend = "none"
        if world > 1:
            import torch.distributed as dist

            backend = dist.get_backend()
        out = {
            "metric": METRIC,
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic (random NHWC images + random labels, random-init weights)",
            "config": {"model": "resnet50" if args.model == "resnet50" else "tiny_bottleneck_resnet_cpu_test",
                       "global_batch": global_batch, "seq_len": None,
                       "image_size": S, "per_gpu_batch": B, "parallelism": f"dp{world}",
                       "optimizer": "sgd_momentum0.9_fused"},
            "device": device.type,
            "backend": backend if world > 1 else None,
            "shared_gpu": bool(config.get("CLOUD_AMD_SHARED_GPU")),
            "strategy": strategy.name,
            "comm": dict(reducer.describe(), allreduce_ms=comm["allreduce_ms"],
                         exposed_comm_ms=comm["exposed_comm_ms"], timing=comm.get("timing"),
                         busbw_gbs=busbw, comm_probe=probe, sliced_optimizer=sliced),
            "overlap_budget": budget,
            "replicas_consistent": replicas_consistent,
            "step_stats_rank0": step_stats,
            "gc_frozen_objects": gc_frozen,
            "max_steps_in_flight": pacer.depth if (pacer is not None and pacer.enabled) else None,
            "pacer_step_ms": round(pacer.step_ms, 3) if (pacer is not None and pacer.step_ms) else None,
            "warnings": step_stats.pop("warnings"),
            "rank_ms_per_step": {"min": round(min(per_rank_ms), 3), "max": round(max(per_rank_ms), 3)},
            "first_step_latency_s": round(first_lat, 3),
            "run_to_first_step_s": round(run_to_first, 3) if run_to_first is not None else None,
            "startup_phases_rank0": phases,
            "launched_via": launched,
            "final_loss": round(final_loss, 4),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 2**30, 2) if on_gpu else None,
        }

    def emit(ab=None):
        if out is None:
            return
        if ab is not None:
            out["dp_ab"] = {"cells": ab, "best": dp_ab.best(ab), "steps_per_cell": args.ab_steps,
                            "note": "after the timed region; value above is the default configuration"}
        line = json.dumps(_finite(out), allow_nan=False)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")

    # N > 1: a bounded step-level A/B of the DP knobs no one-GPU box can settle (per-bucket
    # optimizer, bucket size, transport) -- cloud_amd/utils/dp_ab.py
    from cloud_amd.utils import dp_ab

    cells = dp_ab.cells_from_env() if (world > 1 and args.ab) else []
    if cells:
        dp_ab.teardown(reducer)
        ab = []

        def build(bucket_mb):
            return strategy.gradient_reducer(opt.arenas, bucket_mb=bucket_mb, reduce_dtype=args.grad_reduce_dtype)

        dp_ab.run_cells(build, lambda r: holder.__setitem__("red", r), train_step, opt, device, cells,
                        steps=args.ab_steps, on_timeout=lambda res: emit(list(res)), results=ab)
        emit(ab)
    else:
        emit()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
