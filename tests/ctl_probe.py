"""Custom-training-loop probe shared by the CPU and GPU CTL tests.

The reference's MultiWorkerMirrored custom loop (``TFC/core/tests/testdata/
mnist_example_using_ctl.py:124-129,150-157``: ``tf.GradientTape`` + ``apply_gradients``
inside ``strategy.run``, loss summed with ``strategy.reduce``) on a small Conv2D + Dense
model with Adam, trained for ``--steps`` steps on ONE fixed global batch (so the loss must
fall).  Every rank takes its slice of the global batch; rank 0 writes the final weights
(fp32) and the per-step losses to ``--out`` (``.npz``).

Run directly for one rank, or with RANK / WORLD_SIZE / MASTER_* set for a
MultiWorkerMirroredStrategy job (gloo on CPU, or the shared-GPU rehearsal).
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--global-batch", type=int, default=32)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--optimizer", default="adam")
    ap.add_argument("--mode", choices=("ctl", "reference"), default="ctl",
                    help="reference: one rank, plain autograd backward + torch.optim.Adam on fp32 master copies")
    ap.add_argument("--alloc-warmup", type=int, default=0,
                    help="> 0: keep the per-step losses on the device (no host sync in the loop) and report "
                         "the caching allocator's device allocations made after this many steps")
    args = ap.parse_args(argv)

    import torch

    from cloud_amd import tf

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    strategy = (tf.distribute.MultiWorkerMirroredStrategy() if world_env > 1
                else tf.distribute.OneDeviceStrategy(os.environ.get("CLOUD_AMD_DEVICE") or "/gpu:0"))
    rank, world = strategy.rank, strategy.num_replicas_in_sync
    G = args.global_batch
    per = G // world
    rng = np.random.default_rng(7)
    X = rng.random((G, 12, 12, 1), dtype=np.float32)
    Y = rng.integers(0, 10, (G,)).astype(np.int64)
    xb, yb = X[rank * per:(rank + 1) * per], Y[rank * per:(rank + 1) * per]

    torch.manual_seed(0)  # identical initial weights on every rank and in every run
    with strategy.scope():
        model = tf.keras.Sequential([
            tf.keras.layers.Conv2D(8, 3, activation="relu"),
            tf.keras.layers.MaxPooling2D(),
            tf.keras.layers.Flatten(),
            tf.keras.layers.Dense(16, activation="relu"),
            tf.keras.layers.Dense(10, activation="softmax"),
        ])
        loss_object = tf.keras.losses.SparseCategoricalCrossentropy(reduction=tf.keras.losses.Reduction.NONE)
        opt = {"adam": tf.keras.optimizers.Adam, "sgd": tf.keras.optimizers.SGD}[args.optimizer](
            learning_rate=args.lr)

    def train_step(inputs):
        images, labels = inputs
        with tf.GradientTape() as tape:
            predictions = model(images, training=True)
            loss = tf.nn.compute_average_loss(loss_object(labels, predictions), global_batch_size=G)
        gradients = tape.gradient(loss, model.trainable_variables)
        opt.apply_gradients(zip(gradients, model.trainable_variables))
        return loss

    with torch.no_grad():
        model(xb[:1], training=True)  # build: the initial weights are part of the record
    init = {"i%d" % i: w.astype(np.float32) for i, w in enumerate(model.get_weights())}
    if args.mode == "reference":
        return _reference(args, model, loss_object, xb, yb, G, init)
    losses = []
    on_gpu = torch.cuda.is_available() and strategy.device is not None and strategy.device.type == "cuda"
    allocs0 = None
    for step in range(args.steps):
        if args.alloc_warmup and step == args.alloc_warmup and on_gpu:
            allocs0 = torch.cuda.memory_stats().get("num_device_alloc", 0)
        per_replica = strategy.run(train_step, args=((xb, yb),))
        if args.alloc_warmup:
            losses.append(per_replica.detach())  # no host sync: the optimizer's step bounds the run-ahead
        else:
            losses.append(float(strategy.reduce(tf.distribute.ReduceOp.SUM, per_replica, axis=None)))
    if args.alloc_warmup:
        if on_gpu:
            torch.cuda.synchronize()
            new = torch.cuda.memory_stats().get("num_device_alloc", 0) - (allocs0 or 0)
            pacer = opt.impl.pacer
            print("RESULT ctl_alloc dev_alloc_after_warmup=%d pacer_waits=%d depth=%s" % (
                new, pacer.waits if pacer else -1, pacer.depth if pacer else None), flush=True)
        losses = [float(v) * world for v in losses]
    if rank == 0:
        weights = [w.astype(np.float32) for w in model.get_weights()]
        np.savez(args.out, losses=np.asarray(losses), **init, **{"w%d" % i: w for i, w in enumerate(weights)})
    print("RESULT ctl_probe rank=%d world=%d losses=%s" % (rank, world, ",".join("%.5f" % v for v in losses)),
          flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


def _reference(args, model, loss_object, xb, yb, G, init):
    """Plain PyTorch training of the same model: autograd gradients (no arena), fp32 master
    weights updated by torch.optim.Adam (eps 1e-7 as Keras), copied back to the model dtype."""
    import torch

    from cloud_amd import tf

    params = list(model.trainable_variables)
    masters = [p.detach().float().clone().requires_grad_(True) for p in params]
    opt = torch.optim.Adam(masters, lr=args.lr, betas=(0.9, 0.999), eps=1e-7)
    losses = []
    for _ in range(args.steps):
        for p in params:
            p.grad = None
        pred = model(xb, training=True)
        loss = tf.nn.compute_average_loss(loss_object(yb, pred), global_batch_size=G)
        loss.backward()
        for m, p in zip(masters, params):
            m.grad = p.grad.float()
        opt.step()
        with torch.no_grad():
            for m, p in zip(masters, params):
                p.copy_(m.to(p.dtype))
        losses.append(float(loss))
    weights = [w.astype(np.float32) for w in model.get_weights()]
    np.savez(args.out, losses=np.asarray(losses), **init, **{"w%d" % i: w for i, w in enumerate(weights)})
    print("RESULT ctl_probe reference losses=%s" % ",".join("%.5f" % v for v in losses), flush=True)


if __name__ == "__main__":
    main()
