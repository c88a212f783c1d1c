"""Host launch path (runtime/host.py) without a GPU: the process-wide autograd threading switch."""
import torch

from cloud_amd.runtime import host


def test_configure_disables_autograd_worker_threads(monkeypatch):
    monkeypatch.setattr(host, "_DONE", [False])
    calls = []
    monkeypatch.setattr(torch.autograd, "set_multithreading_enabled", lambda mode: calls.append(mode))
    monkeypatch.delenv("CLOUD_AMD_AUTOGRAD_MT", raising=False)
    host.configure()
    host.configure()  # idempotent
    assert calls == [False]
    monkeypatch.setattr(host, "_DONE", [False])
    monkeypatch.setenv("CLOUD_AMD_AUTOGRAD_MT", "1")
    host.configure()
    assert calls == [False]  # kept torch's default
