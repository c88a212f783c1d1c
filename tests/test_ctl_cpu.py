"""The reference's custom training loop (tf.GradientTape + apply_gradients under
MultiWorkerMirroredStrategy; TFC/core/tests/testdata/mnist_example_using_ctl.py:124-129,150-157)
on CPU: after the variables have moved into the optimizer's arenas (step 2 on) the tape must
still return the real gradients, and two gloo replicas over halves of the global batch must
train exactly like one process over all of it (and like plain autograd + torch.optim.Adam)."""
import numpy as np

from _ctl_util import load, rel_to_update, run_probe

CPU = {"CLOUD_AMD_DEVICE": "cpu", "CLOUD_AMD_DIST_BACKEND": "gloo"}


def test_ctl_matches_plain_autograd_reference(tmp_path):
    run_probe(tmp_path / "ref.npz", env_extra=CPU, args=("--mode", "reference", "--steps", "6"))
    run_probe(tmp_path / "ctl.npz", env_extra=CPU, args=("--steps", "6"))
    ref, ctl = load(tmp_path / "ref.npz"), load(tmp_path / "ctl.npz")
    np.testing.assert_allclose(ctl[2], ref[2], rtol=1e-4, atol=1e-5)
    assert rel_to_update(ctl, ref) < 1e-3
    assert ctl[2][-1] < ctl[2][0]  # one fixed batch: the loss falls


def test_ctl_two_replicas_equal_one_process_over_global_batch(tmp_path):
    run_probe(tmp_path / "one.npz", env_extra=CPU, args=("--steps", "6"))
    out = run_probe(tmp_path / "two.npz", world=2, env_extra=CPU, args=("--steps", "6"))
    assert out.count("world=2") == 2, out
    one, two = load(tmp_path / "one.npz"), load(tmp_path / "two.npz")
    np.testing.assert_allclose(two[2], one[2], rtol=1e-4, atol=1e-5)
    assert rel_to_update(two, one) < 1e-3
    assert two[2][-1] < two[2][0]
