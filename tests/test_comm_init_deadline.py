"""Native RCCL communicator bootstrap deadline (round-4 verdict item 7).

A peer that HANGS before joining must fail the job within ``CLOUD_AMD_COMM_INIT_TIMEOUT_S``
instead of stalling every rank:

* CPU: the unique-id exchange (``parallel/comm.exchange_unique_id``) over a real c10d
  TCPStore whose rank 0 never publishes raises ``TimeoutError`` within the deadline;
* GPU: ``ncclCommInitRankConfig`` (non-blocking, polled) for a 2-rank communicator that only
  rank 0 ever joins is aborted at the deadline and raises ``TimeoutError``.
"""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _store(port=0):
    import datetime

    from torch.distributed import TCPStore

    return TCPStore("127.0.0.1", port, 2, True, datetime.timedelta(seconds=30), wait_for_workers=False)


def test_missing_rank0_unique_id_raises_within_deadline():
    from cloud_amd.parallel.comm import exchange_unique_id

    st = _store()
    t0 = time.time()
    with pytest.raises(TimeoutError, match="not published by rank 0"):
        exchange_unique_id(st, "cloud_amd/rccl_uid/t", 1, lambda: b"x" * 128, 1.0)
    assert time.time() - t0 < 10.0


def test_unique_id_exchange_roundtrip():
    from cloud_amd.parallel.comm import exchange_unique_id

    st = _store()
    uid = exchange_unique_id(st, "k", 0, lambda: b"\x01" * 128, 1.0)
    assert exchange_unique_id(st, "k", 1, lambda: b"never", 1.0) == uid == b"\x01" * 128


def test_init_timeout_env(monkeypatch):
    from cloud_amd.parallel import comm

    monkeypatch.setenv("CLOUD_AMD_COMM_INIT_TIMEOUT_S", "7.5")
    assert comm.init_timeout_s() == 7.5


_GPU_PROBE = r"""
import sys, time
sys.path.insert(0, %r)
import torch
from cloud_amd.parallel.comm import RcclComm
torch.cuda.init()
t0 = time.time()
try:
    RcclComm(rank=0, world=2, device="cuda:0", store=False, timeout_s=3.0)
    print("NO_TIMEOUT")
except TimeoutError as e:
    print("TIMEOUT %%.2f %%s" %% (time.time() - t0, e))
"""


@pytest.mark.gpu
def test_rccl_init_with_missing_peer_times_out():
    p = subprocess.run([sys.executable, "-c", _GPU_PROBE % ROOT], capture_output=True, text=True, timeout=90,
                       env=dict(os.environ, NCCL_DEBUG="WARN"))
    out = p.stdout + p.stderr
    line = [ln for ln in p.stdout.splitlines() if ln.startswith(("TIMEOUT", "NO_TIMEOUT"))]
    assert line and line[-1].startswith("TIMEOUT"), out[-3000:]
    assert float(line[-1].split()[1]) < 30.0, line
