"""Two ranks on one GPU over gloo: per-parameter gradient fingerprints after the
bucketed all-reduce (must match across ranks)."""
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from cloud_amd.models.resnet import ResNet
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD
    from cloud_amd.parallel.ddp import GradAllReducer

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = ResNet((1, 1, 1, 1), num_classes=10, stem_channels_pad=5, device="cuda")
    opt = SGD(m, learning_rate=0.05, momentum=0.9, grad_scale=1.0 / world)
    red = GradAllReducer(opt.arenas, bucket_mb=float(os.environ.get("PROBE_BUCKET_MB", "0.05")))
    red.broadcast_parameters()
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(8 * world, 32, 32, 3, device="cuda", generator=g).to(torch.bfloat16)
    Y = torch.randint(0, 10, (8 * world,), device="cuda", generator=g)
    xb, yb = X[rank * 8:(rank + 1) * 8].contiguous(), Y[rank * 8:(rank + 1) * 8].contiguous()
    names = {id(p): n for n, p in m.named_parameters()}
    if rank == 0:
        print("mode", os.environ.get("CLOUD_AMD_DDP_ORDER", "event"), "main stream", torch.cuda.current_stream().cuda_stream,
              flush=True)
    log = []
    orig_on, orig_launch = red._on_grad, red._launch

    def on(p):
        b = red._param_bucket.get(id(p))
        log.append(("notify", names.get(id(p), "?"), b.index if b else None, b.pending if b else None,
                    b.launched if b else None))
        return orig_on(p)

    def la(b):
        log.append(("launch", b.index, [names.get(id(s.param), "?") for s in b.slots]))
        return orig_launch(b)

    red._on_grad, red._launch = on, la
    import cloud_amd.parallel.ddp as ddpmod
    for h in red._hooks:
        h.remove()
    red._hooks = [s.param.register_post_accumulate_grad_hook(lambda p: on(p)) for b in red.buckets for s in b.slots]
    for step in range(2):
        log.clear()
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(m(xb), yb, denom=8)
        loss.backward()
        if rank == 0 and step == 0:
            for e in log:
                print("LOG", e, flush=True)
        red.finish()
        torch.cuda.synchronize()
        rows = []
        for a in opt.arenas:
            for sl in a.slots:
                gsl = a.grad[sl.offset:sl.offset + sl.numel].double()
                rows.append((names.get(id(sl.param), sl.name), float(gsl.sum()), float(gsl.abs().sum())))
        fps = [None] * world
        dist.all_gather_object(fps, rows)
        if rank == 0:
            bad = [(r0[0], r0[1], r1[1]) for r0, r1 in zip(fps[0], fps[1]) if r0[1:] != r1[1:]]
            print("step", step, "mismatching params:", len(bad), bad[:6], flush=True)
            print("buckets", [(b.index, b.lo, b.hi, len(b.slots)) for b in red.buckets][:40], flush=True)
        opt.step()
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(worker, args=(2, 29811), nprocs=2, join=True)
