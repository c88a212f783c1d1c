#!/usr/bin/env python3
"""BASELINE.json config 5: BERT-base fine-tune on synthetic GLUE (sequence
classification), data parallel, bf16 compute, fused AdamW.

    python bench/bert_base_synth.py --steps 20 --warmup 5            # 1 rank via cloud_amd.run()
    python bench/bert_base_synth.py --gpus 8                         # 8 ranks via cloud_amd.run()
    python bench/bert_base_synth.py --stock 1 --steps 20 --warmup 5  # HF transformers + torch AdamW, autocast bf16
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/bert_base_synth.py --gpus 8

Launch contract as bench.py (:mod:`cloud_amd.utils.benchlaunch`): outside a launched
job the script stages itself and spawns ``--gpus`` ranks through ``cloud_amd.run()``
(``--via-run 0`` trains in-process); inside a rank, WORLD_SIZE != --gpus is an error.

Synthetic GLUE: random token ids (vocab 30522), segment ids (A|B split), a
right-padded attention mask with per-example lengths in [S/2, S], 2 labels;
random-init BERT-base weights.  Metric: sequences/s over all ranks (weak
scaling, fixed per-GPU batch).  Same JSON contract as bench.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_START = time.time()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--lr", type=float, default=2e-5)
    ap.add_argument("--stock", type=int, default=0)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--grad-reduce-dtype", choices=("auto", "bf16", "fp32", "native"), default=None)
    ap.add_argument("--ab", type=int, default=1, help="N > 1: DP-engine A/B cells after the timed region")
    ap.add_argument("--ab-steps", type=int, default=5)
    ap.add_argument("--embed-wire", choices=("bf16", "native"), default="bf16",
                    help="wire dtype of the word-embedding table's gradient all-reduce (split into pipelined "
                         "sub-buckets; bf16 halves its bytes -- error bound: tests/test_grad_reduce_precision.py)")
    ap.add_argument("--via-run", type=int, default=int(os.environ.get("CLOUD_AMD_BENCH_VIA_RUN", "1")))
    return ap.parse_args()


def synthetic_glue(B, S, device, seed):
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    ids = torch.randint(1000, 30522, (B, S), generator=g, device=device)
    ids[:, 0] = 101  # [CLS]
    lens = torch.randint(S // 2, S + 1, (B,), generator=g, device=device)
    pos = torch.arange(S, device=device)[None]
    am = (pos < lens[:, None]).long()
    split = (lens // 2)[:, None]
    tts = ((pos >= split) & (am == 1)).long()
    ids = ids * am
    labels = torch.randint(0, 2, (B,), generator=g, device=device)
    return ids, tts, am, labels


def _finite(o):
    """NaN / inf -> None (the result line is strict JSON)."""
    if isinstance(o, float):
        return o if o == o and o not in (float("inf"), float("-inf")) else None
    if isinstance(o, dict):
        return {k: _finite(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_finite(v) for v in o]
    return o


def _plain_gemm_summary():
    """Per plain-GEMM shape: which engine the measured policy kept (ops/raw.py PlainGemmPolicy)."""
    try:
        from cloud_amd.ops import raw
    except Exception:  # pragma: no cover
        return None
    out = {}
    for (layout, M, N, K, bias, beta), d in raw.PLAIN_GEMM.decisions.items():
        name = "%s %dx%dx%d%s%s" % ("NT" if layout == 0 else "NN", M, N, K, "+bias" if bias else "",
                                    "+C" if beta else "")
        out[name] = "%s (ours %.1f us, hipBLASLt %.1f us)" % ("hipBLASLt" if d["library"] else "ours", d["ours_us"],
                                                             d["lib_us"])
    return out or None


def main():
    args = parse()
    from cloud_amd.utils import benchlaunch

    if args.via_run and not benchlaunch.inside_launched_rank():
        return benchlaunch.launch_via_run(os.path.abspath(__file__), args.gpus, tag="bert")
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F

    from cloud_amd import config
    from cloud_amd.parallel import strategy as strategy_mod
    from cloud_amd.utils import dist_env

    # DP engine from the strategy run()'s wrapper installed (auto: Mirrored at N > 1,
    # OneDevice at 1), or the default strategy of a torchrun rank
    strategy = strategy_mod.get_strategy()
    device = strategy.device
    rank, world = strategy.rank, strategy.num_replicas_in_sync
    benchlaunch.check_world(args.gpus, world, tag="bert")
    reducer = None
    torch.manual_seed(1234)
    B, S = args.batch, args.seq
    ids, tts, am, labels = synthetic_glue(B, S, device, 1000 + rank)

    if args.stock:
        from transformers import BertConfig as HFConfig
        from transformers import BertForSequenceClassification as HFBert

        cfg = HFConfig(num_hidden_layers=args.layers, num_labels=2)
        model = HFBert(cfg).to(device)
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[device.index])
        opt = torch.optim.AdamW(model.parameters(), lr=args.lr, weight_decay=0.01, fused=True)

        def train_step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = model(input_ids=ids, token_type_ids=tts, attention_mask=am).logits
            loss = F.cross_entropy(logits.float(), labels)
            loss.backward()
            opt.step()
            return loss
        impl = "stock: transformers BertForSequenceClassification + torch.autocast(bf16) + AdamW(fused)"
    else:
        from cloud_amd.models.bert import BertConfig, BertForSequenceClassification
        from cloud_amd.ops import softmax_cross_entropy
        from cloud_amd.optim import AdamW

        cfg = BertConfig.base(num_hidden_layers=args.layers, num_labels=2)
        model = BertForSequenceClassification(cfg, device=device)
        if args.embed_wire == "bf16":
            # the table's gradient is the last one backward produces: its collective is exposed
            model.embeddings.word._ca_wire_dtype = torch.bfloat16
        opt = AdamW(model, learning_rate=args.lr, weight_decay=0.01, grad_scale=1.0 / world)
        reducer = strategy.gradient_reducer(opt.arenas, bucket_mb=args.bucket_mb,
                                            reduce_dtype=args.grad_reduce_dtype)
        reducer.broadcast_parameters()
        reducer.attach_optimizer(opt)  # world > 1: AdamW per bucket as each all-reduce completes

        holder = {"red": reducer}  # the DP A/B cells after the timed region swap reducers

        def train_step():
            opt.zero_grad()
            logits = model(ids, tts, am)
            loss, _ = softmax_cross_entropy(logits, labels, denom=B)
            loss.backward()
            holder["red"].finish()
            opt.step()
            return loss
        impl = "cloud_amd: fused layer fwd/bwd, MFMA GEMM epilogues, fused attention/LN, AdamW arena"

    loss = train_step()
    torch.cuda.synchronize()
    t_first_done = time.time()
    first = t_first_done - T_START
    phases = benchlaunch.startup_phases(T_START, t_first_done)
    run_t0 = os.environ.get("CLOUD_AMD_RUN_T0")
    run_to_first = (time.time() - float(run_t0)) if run_t0 else None
    # (cloud_amd: the fused optimizer's step() bounds the host run-ahead, runtime/step_pacer.py,
    # so the allocator's pool is complete after warmup)
    for _ in range(max(args.warmup - 1, 0)):
        loss = train_step()
    replicas_consistent = None
    if world > 1 and reducer is not None:
        try:
            replicas_consistent = bool(reducer.check_consistency())
        except RuntimeError as e:
            replicas_consistent = False
            print("[bert] %s" % e, file=sys.stderr, flush=True)
    dist_env.barrier()
    torch.cuda.synchronize()
    gc_frozen = None
    if not args.stock:
        from cloud_amd.runtime import gc_control

        gc_frozen = gc_control.freeze()  # model / optimizer / imports leave the collector's full passes
    if reducer is not None:
        reducer.timing_start()
        reducer.probe_readiness()  # per-bucket gradient-ready events -> overlap budget
    # per-step host time, and the part of it spent blocked in the fused optimizer's run-ahead
    # bound: host_ms - paced = the host's own launch cost (host-bound if it nears ms_per_step)
    pacer = getattr(opt, "pacer", None) if not args.stock else None
    host_ms, paced_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        th = time.perf_counter()
        w0 = pacer.wait_ms if pacer is not None else 0.0
        loss = train_step()
        host_ms.append((time.perf_counter() - th) * 1e3)
        paced_ms.append((pacer.wait_ms if pacer is not None else 0.0) - w0)
    torch.cuda.synchronize()
    dist_env.barrier()
    dt = time.perf_counter() - t0
    unpaced = sorted(h - w for h, w in zip(host_ms, paced_ms))
    host_launch = {"unpaced_median_ms": round(unpaced[len(unpaced) // 2], 3),
                   "unpaced_max_ms": round(unpaced[-1], 3)} if unpaced else None
    per_rank = [v / args.steps * 1000.0 for v in dist_env.all_gather_floats(dt, device)]
    elapsed = dist_env.all_reduce_max(dt, device)
    busbw = dist_env.allreduce_busbw(device) if world > 1 else None
    probe = dist_env.comm_probe(device) if world > 1 else None  # torch.distributed vs native RcclComm
    sps = B * world * args.steps / elapsed
    first = dist_env.all_reduce_max(first, device)
    if run_to_first is not None:
        run_to_first = dist_env.all_reduce_max(run_to_first, device)
    comm = None
    if reducer is not None:
        t = reducer.timing_summary()
        comm = dict(reducer.describe(), allreduce_ms=dist_env.all_reduce_max(t["allreduce_ms"], device),
                    exposed_comm_ms=dist_env.all_reduce_max(t["exposed_comm_ms"], device), timing=t.get("timing"),
                    busbw_gbs=busbw, comm_probe=probe, sliced_optimizer=reducer.optimizer is not None,
                    overlap_budget=reducer.overlap_budget(optimizer=opt), embed_wire=args.embed_wire)
    out = None
    if rank == 0:
        out = ({
            "metric": "sequences/sec BERT-base fine-tune synthetic GLUE (seq %d)" % S,
            "value": round(sps, 2), "unit": "sequences/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1000, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic GLUE (random ids/segments/prefix masks/labels, random-init weights)",
            "config": {"model": "bert-base" if args.layers == 12 else "bert-%dL" % args.layers,
                       "global_batch": B * world, "seq_len": S, "per_gpu_batch": B, "parallelism": "dp%d" % world,
                       "optimizer": "adamw"},
            "impl": impl, "gc_frozen_objects": gc_frozen, "first_step_latency_s": round(first, 3),
            "run_to_first_step_s": round(run_to_first, 3) if run_to_first is not None else None,
            "startup_phases_rank0": phases, "host_launch_rank0": host_launch,
            "max_steps_in_flight": pacer.depth if (pacer is not None and pacer.enabled) else None,
            "pacer_step_ms": round(pacer.step_ms, 3) if (pacer is not None and pacer.step_ms) else None,
            "launched_via": benchlaunch.launched_via(), "comm": comm,
            "backend": dist.get_backend() if world > 1 else None,
            "shared_gpu": bool(config.get("CLOUD_AMD_SHARED_GPU")),
            "tokens_per_sec": round(sps * S, 1), "final_loss": round(float(loss.detach().float()), 4),
            "strategy": strategy.name, "replicas_consistent": replicas_consistent,
            "rank_ms_per_step": {"min": round(min(per_rank), 3), "max": round(max(per_rank), 3)},
            "plain_gemm_engine": _plain_gemm_summary()})

    def emit(ab=None):
        if out is None:
            return
        if ab is not None:
            out["dp_ab"] = {"cells": ab, "best": dp_ab.best(ab), "steps_per_cell": args.ab_steps,
                            "note": "after the timed region; value above is the default configuration"}
        print(json.dumps(_finite(out), allow_nan=False), flush=True)

    # N > 1: bounded step-level A/B of the DP knobs (cloud_amd/utils/dp_ab.py)
    from cloud_amd.utils import dp_ab

    cells = dp_ab.cells_from_env() if (world > 1 and args.ab and reducer is not None) else []
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
