"""runtime.step_pacer: the host never runs more than ``depth`` steps ahead of the GPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pacer_bounds_steps_in_flight():
    from cloud_amd.runtime.step_pacer import StepPacer

    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    pacer = StepPacer(torch.device("cuda"), depth=2)
    assert pacer.enabled
    ends = []
    for _ in range(8):
        for _ in range(20):  # a "step" of ~a few ms of GPU work, enqueued in microseconds
            a = (a @ a).clamp_(-1, 1)
        ev = torch.cuda.Event()
        ev.record()
        ends.append(ev)
        pacer.step_done()
        # after step_done at most `depth` steps are unfinished
        assert sum(not e.query() for e in ends) <= 2
    assert pacer.waits > 0  # the host was held back
    torch.cuda.synchronize()


def test_pacer_disabled_by_config(monkeypatch):
    from cloud_amd.runtime.step_pacer import StepPacer

    monkeypatch.setenv("CLOUD_AMD_MAX_STEPS_IN_FLIGHT", "0")
    p = StepPacer(torch.device("cuda"))
    assert not p.enabled
    p.step_done()
