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


def test_ctl_replica_semantics_two_replicas(tmp_path):
    """``CLOUD_AMD_TAPE_REDUCE=replica`` (TF MirroredStrategy semantics: the tape returns
    per-replica gradients, apply_gradients sums them) trains like one process too."""
    run_probe(tmp_path / "one.npz", env_extra=CPU, args=("--steps", "6"))
    out = run_probe(tmp_path / "two.npz", world=2, env_extra=dict(CPU, CLOUD_AMD_TAPE_REDUCE="replica"),
                    args=("--steps", "6"))
    assert out.count("world=2") == 2, out
    one, two = load(tmp_path / "one.npz"), load(tmp_path / "two.npz")
    np.testing.assert_allclose(two[2], one[2], rtol=1e-4, atol=1e-5)
    assert rel_to_update(two, one) < 1e-3


def test_persistent_tape_returns_copies_and_stale_slots_are_cleared():
    """A persistent tape's second gradient() must not overwrite the first's result, and an
    apply_gradients that skips a variable must not re-apply its previous gradient."""
    import os

    os.environ["CLOUD_AMD_DEVICE"] = "cpu"
    import torch

    import cloud_amd.tf as tf
    from cloud_amd import keras

    torch.manual_seed(0)
    model = keras.Sequential([keras.layers.Dense(4, input_shape=(3,)), keras.layers.Dense(2)])
    opt = keras.optimizers.SGD(learning_rate=0.1)
    x = torch.randn(8, 3)
    variables = list(model.trainable_variables)
    with tf.GradientTape() as tape:
        loss = model(x).square().mean()
    opt.apply_gradients(zip(tape.gradient(loss, variables), variables))  # variables move into arenas
    with tf.GradientTape(persistent=True) as tape:
        l1 = model(x).square().mean()
        l2 = (2.0 * model(x)).square().mean()
    g1 = [g.clone() for g in tape.gradient(l1, variables)]
    g1b = tape.gradient(l1, variables)
    g2 = tape.gradient(l2, variables)
    for a, b, c in zip(g1, g1b, g2):
        assert torch.allclose(a, b) and torch.allclose(4 * a, c, rtol=1e-4, atol=1e-6)
    # skip the last variable: its weights must not move by a stale gradient
    last = variables[-1].detach().clone()
    opt.apply_gradients([(g, v) for g, v in zip(g1b, variables)][:-1])
    assert torch.equal(variables[-1].detach(), last)
