"""Multi-process data parallelism on CPU (gloo): the DP engine must make every
rank's update equal the single-process large-batch update, and a Keras job
launched through run() must stay replica-consistent."""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def _free_port():
    """An unused TCP port on 127.0.0.1 (bind to 0): fixed pid-based formulas collide across
    test cases and pytest-xdist workers."""
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]

def _worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from cloud_amd.optim import SGD
    from cloud_amd.parallel.ddp import GradAllReducer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    if rank == 1:  # different init on purpose: broadcast must fix it
        for p in model.parameters():
            p.data.add_(1.0)
    opt = SGD(model, learning_rate=0.1, momentum=0.9, grad_scale=1.0 / world)
    red = GradAllReducer(opt.arenas, bucket_mb=0.0005)
    assert len(red.buckets) > 1
    red.broadcast_parameters()
    g = torch.Generator().manual_seed(1)
    X = torch.randn(8 * world, 16, generator=g)
    Y = torch.randn(8 * world, 4, generator=g)
    for _ in range(3):
        opt.zero_grad()
        xb, yb = X[rank * 8:(rank + 1) * 8], Y[rank * 8:(rank + 1) * 8]
        loss = torch.nn.functional.mse_loss(model(xb), yb)
        loss.backward()
        red.finish()
        opt.step()
    torch.save({k: v.detach().clone() for k, v in model.state_dict().items()}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_matches_single_process(tmp_path):
    world = 2
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    for k in r0:
        torch.testing.assert_close(r0[k], r1[k])
    # single-process reference on the full batch
    sys.path.insert(0, ROOT)
    from cloud_amd.optim import SGD

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    opt = SGD(model, learning_rate=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(1)
    X = torch.randn(16, 16, generator=g)
    Y = torch.randn(16, 4, generator=g)
    for _ in range(3):
        opt.zero_grad()
        loss = 0.5 * (torch.nn.functional.mse_loss(model(X[:8]), Y[:8]) + torch.nn.functional.mse_loss(model(X[8:]), Y[8:]))
        loss.backward()
        opt.step()
    for k, v in model.state_dict().items():
        torch.testing.assert_close(r0[k], v, atol=1e-5, rtol=1e-5)


def test_keras_job_via_run_two_workers(tmp_path):
    env = dict(os.environ, CLOUD_AMD_EXAMPLE_CPU="1", CLOUD_AMD_NUM_GPUS="0", CLOUD_AMD_JOBS_DIR=str(tmp_path),
               WORKERS="1", EPOCHS="2", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "mnist_mlp.py")], env=env,
                       capture_output=True, text=True, timeout=600, cwd=os.path.join(ROOT, "examples"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Job submitted successfully." in r.stdout
    # stream_logs tails every rank, lines tagged with the rank's role (the chief's first)
    res = [json.loads(ln[len("[chief-0] RESULT "):]) for ln in r.stdout.splitlines()
           if ln.startswith("[chief-0] RESULT ")]
    assert any(ln.startswith("[worker-0] ") for ln in r.stdout.splitlines())
    assert res and res[0]["replicas"] == 2 and res[0]["strategy"] == "MultiWorkerMirroredStrategy"
    assert res[0]["loss"][-1] < res[0]["loss"][0] and res[0]["test_acc"] > 0.8
    logs = os.listdir(os.path.join(tmp_path, os.listdir(tmp_path)[0], "logs"))
    assert sorted(logs) == ["chief-0.log", "worker-0.log"]
    other = [json.loads(ln[7:]) for ln in open(os.path.join(tmp_path, os.listdir(tmp_path)[0], "logs", "worker-0.log"))
             if ln.startswith("RESULT ")]
    assert abs(other[0]["weights_checksum"] - res[0]["weights_checksum"]) < 1e-6


def _desync_worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), CLOUD_AMD_GRAD_CHECK_EVERY="1")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from cloud_amd.optim import SGD
    from cloud_amd.parallel.ddp import GradAllReducer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = torch.nn.Linear(8, 4)
    opt = SGD(model, learning_rate=0.1, grad_scale=1.0 / world)
    red = GradAllReducer(opt.arenas)
    red.broadcast_parameters()
    opt.zero_grad()
    model(torch.randn(4, 8)).sum().backward()
    red.finish()  # check_every=1: the post-all-reduce fingerprints agree
    ok = True
    if rank == 1:
        opt.arenas[0].grad[0] += 1.0  # simulate a desynchronised replica
    try:
        red.check_consistency()
    except RuntimeError as e:
        ok = "desync" in str(e)
    else:
        ok = False
    with open(os.path.join(out_dir, f"desync{rank}"), "w") as f:
        f.write("caught" if ok else "missed")
    dist.destroy_process_group()


def test_grad_desync_detector(tmp_path):
    world = 2
    port = _free_port()
    mp.spawn(_desync_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    assert [open(tmp_path / f"desync{r}").read() for r in range(world)] == ["caught", "caught"]


def test_trace_ranges_are_noops_when_disabled():
    sys.path.insert(0, ROOT)
    from cloud_amd.utils import trace

    with trace.range("fwd"):
        trace.mark("x")
    assert trace.enabled() in (False, True)


def test_grad_ready_counts_each_param_once():
    """A parameter reported both by notify_grad_ready (in-place arena write) and by
    autograd's post-accumulate hook must only count once towards its bucket."""
    sys.path.insert(0, ROOT)
    from cloud_amd.optim import SGD
    from cloud_amd.parallel.ddp import GradAllReducer

    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 8))
    opt = SGD(model, learning_rate=0.1)
    red = GradAllReducer(opt.arenas, bucket_mb=1000)  # one bucket per arena
    launched = []
    red._launch = lambda b: (launched.append(b.index), setattr(b, "launched", True))
    params = list(model.parameters())
    for p in params[:-1]:
        red._on_grad(p)
        red._on_grad(p)  # duplicate report
    assert launched == []  # the last parameter has not been reported yet
    red._on_grad(params[-1])
    assert launched == [0]
    with red.no_sync():
        red._on_grad(params[0])
    assert launched == [0]


def test_init_distributed_backend_and_shared_gpu_overrides(monkeypatch):
    """CLOUD_AMD_DIST_BACKEND picks the process-group backend; CLOUD_AMD_SHARED_GPU maps
    every local rank onto device 0 (the one-GPU rehearsal of the multi-rank bench)."""
    import torch.distributed as dist

    from cloud_amd.utils import dist_env

    seen = {}

    def fake_init(backend, rank, world_size, timeout, **kw):
        seen.update(backend=backend, rank=rank, world=world_size)

    monkeypatch.setattr(dist, "is_initialized", lambda: False)
    monkeypatch.setattr(dist, "init_process_group", fake_init)
    monkeypatch.setattr(dist_env.atexit, "register", lambda fn: None)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: seen.update(device=d))
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("CLOUD_AMD_DIST_BACKEND", "gloo")
    monkeypatch.setenv("CLOUD_AMD_SHARED_GPU", "1")
    r, w, dev = dist_env.init_distributed()
    assert (r, w) == (1, 2)
    assert dev == torch.device("cuda", 0) and seen["device"] == dev
    assert seen["backend"] == "gloo" and seen["world"] == 2
    monkeypatch.delenv("CLOUD_AMD_DIST_BACKEND")
    monkeypatch.delenv("CLOUD_AMD_SHARED_GPU")
    r, w, dev = dist_env.init_distributed()
    assert dev == torch.device("cuda", 1) and seen["backend"] == "nccl"
