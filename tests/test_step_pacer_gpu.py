"""runtime.step_pacer: the host never runs more than ``depth`` steps ahead of the GPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pacer_bounds_steps_in_flight():
    from cloud_amd.runtime.step_pacer import StepPacer

    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    pacer = StepPacer(torch.device("cuda"), depth=2, run_ahead_ms=0)
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


@pytest.mark.parametrize("run_ahead_ms", [1000.0, 1e-3])
def test_pacer_depth_adapts_to_step_time_early(run_ahead_ms):
    """CLOUD_AMD_RUN_AHEAD_MS: the depth is settled from the GPU time between two completed
    step ends during the first steps -- short steps deepen the queue (capped), long ones keep
    the configured minimum -- and the bound then holds at the settled depth."""
    from cloud_amd.runtime.step_pacer import StepPacer

    a = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    pacer = StepPacer(torch.device("cuda"), depth=2, run_ahead_ms=run_ahead_ms)
    ends = []
    for i in range(10):
        for _ in range(10):
            a = (a @ a).clamp_(-1, 1)
        ev = torch.cuda.Event()
        ev.record()
        ends.append(ev)
        pacer.step_done()
        if i + 1 >= StepPacer.CALIBRATE_AT:
            assert not pacer._calibrating
        assert sum(not e.query() for e in ends) <= pacer.depth
    assert pacer.step_ms is not None and pacer.step_ms > 0
    want = StepPacer.MAX_ADAPTIVE_DEPTH if run_ahead_ms > 100 else 2
    assert pacer.depth == want, (pacer.depth, pacer.step_ms)
    torch.cuda.synchronize()
