"""Helpers for the custom-training-loop tests (tests/ctl_probe.py runs)."""
import os
import socket
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tests", "ctl_probe.py")


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def run_probe(out, world=1, env_extra=None, args=(), timeout=240):
    """Run the probe on ``world`` ranks (subprocesses, MultiWorkerMirroredStrategy when > 1)."""
    base = dict(os.environ)
    base.pop("CLOUD_AMD_DEVICE", None)
    base.update({"PYTHONPATH": ROOT})
    base.update(env_extra or {})
    cmd = [sys.executable, PROBE, "--out", str(out), *args]
    if world == 1:
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
            base.pop(k, None)
        p = subprocess.run(cmd, env=base, capture_output=True, text=True, timeout=timeout)
        assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
        return p.stdout
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(base, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            outs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-4000:]
    return "\n".join(outs)


def load(out):
    z = np.load(str(out))
    n = len([k for k in z.files if k.startswith("w")])
    return ([z["i%d" % i] for i in range(n)], [z["w%d" % i] for i in range(n)], z["losses"])


def rel_to_update(a, ref):
    """max over tensors of |w_a - w_ref| / |w_ref - w_init| (L2): the error relative to how far
    training moved the weights -- zeroed gradients after step 1 leave a large fraction."""
    ia, wa, _ = a
    ir, wr, _ = ref
    worst = 0.0
    for i0, x, y in zip(ir, wa, wr):
        moved = float(np.linalg.norm(y - i0))
        worst = max(worst, float(np.linalg.norm(x - y)) / max(moved, 1e-12))
    return worst
