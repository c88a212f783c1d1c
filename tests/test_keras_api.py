"""Keras-compatible API on CPU: the reference workloads' model/compile/fit/save
patterns (README MLP, MNIST CNN, save_and_load.py, callbacks, functional API)."""
import json
import os

import numpy as np
import pytest
import torch

from cloud_amd import keras
from cloud_amd.keras import layers
from cloud_amd.parallel import strategy as S


@pytest.fixture(autouse=True)
def _one_device():
    S.experimental_set_strategy(S.OneDeviceStrategy("/cpu:0"))
    yield
    S.experimental_set_strategy(None)


def _mnist(n=2048):
    (x, y), (xt, yt) = keras.datasets.mnist.load_data(n_train=n, n_test=512)
    return (x.reshape(-1, 784).astype("float32") / 255, y), (xt.reshape(-1, 784).astype("float32") / 255, yt)


def test_readme_mlp_fit_evaluate():
    """README.md:71-81 MLP: Dense(512 relu) - Dropout(0.2) - Dense(10 softmax), SCCE, Adam."""
    (x, y), (xt, yt) = _mnist()
    model = keras.Sequential([layers.Dense(512, activation="relu", input_shape=(784,)), layers.Dropout(0.2),
                              layers.Dense(10, activation="softmax")])
    model.compile(loss="sparse_categorical_crossentropy", optimizer=keras.optimizers.Adam(1e-3),
                  metrics=["accuracy"])
    assert model.count_params() == 784 * 512 + 512 + 5130
    h = model.fit(x, y, epochs=3, batch_size=128, verbose=0)
    assert h.history["loss"][-1] < h.history["loss"][0]
    loss, acc = model.evaluate(xt, yt, verbose=0)
    assert acc > 0.8, acc
    p = model.predict(xt[:10])
    assert p.shape == (10, 10) and np.allclose(p.sum(-1), 1, atol=1e-4)


def test_cnn_with_dataset_and_callbacks(tmp_path):
    (x, y), _ = keras.datasets.mnist.load_data(n_train=512, n_test=64)
    x = x[..., None].astype("float32") / 255
    ds = keras.Dataset.from_tensor_slices((x, y.astype("int64"))).shuffle(512, seed=1).batch(64).prefetch(2)
    model = keras.Sequential([
        layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)), layers.MaxPooling2D(),
        layers.Flatten(), layers.Dense(64, activation="relu"), layers.Dense(10)])
    model.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer="adam",
                  metrics=["accuracy"])
    seen = []
    sched = keras.callbacks.LearningRateScheduler(lambda e: 1e-3 if e < 1 else 5e-4)
    ckpt = keras.callbacks.ModelCheckpoint(str(tmp_path / "ckpt_{epoch}.pt"), save_weights_only=True)
    tb = keras.callbacks.TensorBoard(str(tmp_path / "tb"))
    lam = keras.callbacks.LambdaCallback(on_epoch_end=lambda e, logs: seen.append(logs["loss"]))
    h = model.fit(ds, epochs=2, callbacks=[sched, ckpt, tb, lam], verbose=0)
    assert len(seen) == 2 and h.history["lr"] == [1e-3, 5e-4]
    assert os.path.exists(tmp_path / "ckpt_2.pt")
    rows = [json.loads(ln) for ln in open(tmp_path / "tb" / "train" / "scalars.jsonl")]
    assert rows[-1]["epoch"] == 1 and "accuracy" in rows[-1]


def test_early_stopping_and_validation():
    (x, y), (xt, yt) = _mnist(1024)
    model = keras.Sequential([layers.Dense(16, activation="relu", input_shape=(784,)), layers.Dense(10)])
    model.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer="sgd")
    es = keras.callbacks.EarlyStopping(monitor="val_loss", patience=0, min_delta=10.0)
    h = model.fit(x, y, epochs=5, validation_data=(xt, yt), callbacks=[es], verbose=0)
    assert len(h.history["loss"]) == 2 and "val_loss" in h.history


def test_save_and_load_roundtrip(tmp_path):
    """save_and_load.py: weights/model saved, reloaded, evaluated and trained further."""
    (x, y), (xt, yt) = _mnist(1024)
    model = keras.Sequential([layers.Dense(64, activation="relu", input_shape=(784,)),
                              layers.BatchNormalization(), layers.Dense(10, activation="softmax")])
    model.compile(loss="sparse_categorical_crossentropy", optimizer="adam", metrics=["accuracy"])
    model.fit(x, y, epochs=1, batch_size=64, verbose=0)
    ref = model.evaluate(xt, yt, verbose=0)
    model.save(str(tmp_path / "saved"))
    m2 = keras.models.load_model(str(tmp_path / "saved"))
    np.testing.assert_allclose(m2.evaluate(xt, yt, verbose=0), ref, rtol=1e-5, atol=1e-5)
    m2.fit(x, y, epochs=1, batch_size=64, verbose=0)
    model.save_weights(str(tmp_path / "w" / "cp.ckpt"))
    m3 = keras.Sequential([layers.Dense(64, activation="relu", input_shape=(784,)),
                           layers.BatchNormalization(), layers.Dense(10, activation="softmax")])
    m3.load_weights(str(tmp_path / "w" / "cp.ckpt"))
    m3.compile(loss="sparse_categorical_crossentropy", optimizer="adam", metrics=["accuracy"])
    np.testing.assert_allclose(m3.evaluate(xt, yt, verbose=0), ref, rtol=1e-5, atol=1e-5)


def test_functional_api_and_summary(capsys):
    inp = keras.Input(shape=(20,))
    a = layers.Dense(8, activation="relu")(inp)
    b = layers.Dense(8, activation="tanh")(inp)
    out = layers.Dense(3)(layers.Concatenate()([a, b]))
    model = keras.Model(inp, out)
    assert out.shape == (None, 3)
    model.compile(optimizer="rmsprop", loss="mse", metrics=["mae"])
    x = np.random.randn(64, 20).astype("float32")
    y = np.random.randn(64, 3).astype("float32")
    h = model.fit(x, y, epochs=2, batch_size=16, verbose=0)
    assert "mae" in h.history
    model.summary()
    assert "Total params" in capsys.readouterr().out


def test_custom_training_loop_semantics():
    """mnist_example_using_ctl.py: reduction NONE + compute_average_loss + strategy.reduce."""
    loss_obj = keras.losses.SparseCategoricalCrossentropy(from_logits=True, reduction=keras.losses.Reduction.NONE)
    logits = torch.randn(8, 10)
    y = torch.randint(0, 10, (8,))
    per = loss_obj(y, logits)
    assert per.shape == (8,)
    avg = keras.losses.compute_average_loss(per, global_batch_size=16)
    torch.testing.assert_close(avg, per.sum() / 16)
    s = S.get_strategy()
    assert float(s.reduce(S.ReduceOp.SUM, torch.tensor(3.0))) == 3.0
    acc = keras.metrics.SparseCategoricalAccuracy()
    acc.update_state(y, torch.nn.functional.one_hot(y, 10).float())
    assert acc.result() == 1.0


def test_mixed_bfloat16_policy_cpu():
    keras.mixed_precision.set_global_policy("mixed_bfloat16")
    try:
        model = keras.Sequential([layers.Dense(16, activation="relu", input_shape=(8,)), layers.Dense(2)])
        assert model.layers[0].kernel.dtype == torch.bfloat16
        model.compile(optimizer="sgd", loss="mse")
        model.fit(np.random.randn(32, 8).astype("float32"), np.random.randn(32, 2).astype("float32"),
                  epochs=1, verbose=0)
        assert model.predict(np.zeros((2, 8), "float32")).dtype == np.float32
    finally:
        keras.mixed_precision.set_global_policy("float32")


def test_regularizers_and_constant_initializer():
    """kernel_regularizer adds its penalty to the training loss; Constant takes Keras-layout
    values (the reference cloud_fit model: Dense(1, Constant([[0.5]]), l2(0.01)))."""
    import numpy as np
    import torch

    from cloud_amd import tf

    d = tf.keras.layers.Dense(2, kernel_initializer=tf.keras.initializers.Constant([[1.0, 2.0], [3.0, 4.0],
                                                                                   [5.0, 6.0]]),
                              bias_initializer=tf.keras.initializers.Constant(0.5),
                              kernel_regularizer=tf.keras.regularizers.l2(0.1))
    inp = tf.keras.layers.Input(shape=(3,))
    m = tf.keras.Model(inp, d(inp))
    k = d.kernel.detach().float()
    assert torch.equal(k, torch.tensor([[1.0, 3.0, 5.0], [2.0, 4.0, 6.0]]))  # Keras [in, out] -> [out, in]
    assert torch.equal(d.bias.detach().float(), torch.full((2,), 0.5))
    assert abs(float(d.regularization_loss()) - 0.1 * float((k * k).sum())) < 1e-4
    assert abs(float(m._regularization()) - 0.1 * float((k * k).sum())) < 1e-4
    m.compile(loss="mse", optimizer=tf.keras.optimizers.SGD(0.01))
    x = np.ones((4, 3), np.float32)
    m.fit(x, np.zeros((4, 2), np.float32), epochs=1, verbose=0)
    assert float((d.kernel.detach().float() ** 2).sum()) < float((k * k).sum())  # data + L2 both shrink it
    assert isinstance(tf.keras.regularizers.get("l1_l2"), tf.keras.regularizers.L1L2)


@pytest.mark.parametrize("kernel,strides,padding", [((3, 5), (1, 2), "same"), ((1, 7), (1, 1), "same"),
                                                    ((5, 3), (2, 1), "valid")])
def test_conv2d_rectangular_kernels_and_strides(kernel, strides, padding):
    """Keras Conv2D with rectangular kernels / strides (TF semantics, incl. SAME's asymmetric
    split) against torch's conv of the same weights."""
    import torch.nn.functional as F

    torch.manual_seed(0)
    layer = layers.Conv2D(6, kernel, strides=strides, padding=padding, activation="relu")
    x = torch.randn(2, 11, 14, 3)
    y = layer(x)
    w = layer.kernel.detach().float().permute(0, 3, 1, 2)
    xin = x.permute(0, 3, 1, 2)
    if padding == "same":
        (pt, pb), (pl, pr) = layer._same_pads(11, 14)
        xin = F.pad(xin, (pl, pr, pt, pb))
    ref = torch.relu(F.conv2d(xin, w, layer.bias.detach().float(), stride=strides)).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    torch.testing.assert_close(y.float(), ref, atol=1e-4, rtol=1e-4)
    if padding == "same":
        assert y.shape[1] == -(-11 // strides[0]) and y.shape[2] == -(-14 // strides[1])


def test_evaluate_on_fused_loss_matches_reference_and_keeps_train_logs():
    """evaluate() scores with the training step's fused softmax-xent (loss + accuracy into
    the device accumulator); the numbers equal the plain formulas on predict()'s
    probabilities, and fit's validation pass leaves the epoch's TRAIN logs intact."""
    from cloud_amd import keras

    rng = np.random.default_rng(5)
    x = rng.normal(size=(200, 12)).astype("float32")
    y = (x[:, 0] + 0.5 * x[:, 1] > 0).astype("int64") + (x[:, 2] > 1).astype("int64")
    model = keras.Sequential([keras.layers.Dense(16, activation="relu", input_shape=(12,)),
                              keras.layers.Dense(3, activation="softmax")])
    model.compile(loss="sparse_categorical_crossentropy", optimizer=keras.optimizers.Adam(1e-2),
                  metrics=["accuracy"])
    from cloud_amd.keras import losses as L

    def banned(*a, **k):
        raise AssertionError("unfused loss path reached")

    orig = L.SparseCategoricalCrossentropy.per_example
    L.SparseCategoricalCrossentropy.per_example = banned
    try:
        hist = model.fit(x, y, batch_size=32, epochs=2, validation_data=(x[:96], y[:96]), verbose=0)
    finally:
        L.SparseCategoricalCrossentropy.per_example = orig
    h = hist.history
    assert h["loss"][-1] != h["val_loss"][-1]  # train logs not overwritten by the eval accumulator
    loss, acc = model.evaluate(x[:96], y[:96], batch_size=40, verbose=0)
    p = model.predict(x[:96], batch_size=96).astype("float64")
    ref_loss = float(np.mean(-np.log(np.clip(p[np.arange(96), y[:96]], 1e-7, None))))
    ref_acc = float(np.mean(p.argmax(-1) == y[:96]))
    assert abs(loss - ref_loss) < 2e-2 * max(1.0, ref_loss), (loss, ref_loss)
    assert abs(acc - ref_acc) <= 1.0 / 96 + 1e-9, (acc, ref_acc)
    assert abs(h["val_loss"][-1] - loss) < 1e-5 and abs(h["val_accuracy"][-1] - acc) < 1e-6


def test_backward_with_seed_matches_autograd_and_skips_sympy():
    """ops.backward_with_seed == torch.autograd.backward(loss, grad_tensors=seed), without the
    Python shape check that imports sympy on a process's first seeded backward."""
    import subprocess
    import sys

    import torch

    from cloud_amd import ops

    w = torch.randn(5, 3, requires_grad=True)
    x = torch.randn(4, 5)
    ops.backward_with_seed((x @ w).square().mean(), torch.tensor(2.0))
    g1 = w.grad.clone()
    w.grad = None
    torch.autograd.backward((x @ w).square().mean(), grad_tensors=torch.tensor(2.0))
    torch.testing.assert_close(g1, w.grad)
    with pytest.raises(ValueError):
        ops.backward_with_seed((x @ w).sum(), torch.ones(2))
    code = ("import sys, torch; from cloud_amd import ops; w = torch.ones(3, requires_grad=True); "
            "ops.backward_with_seed((w * 2).sum(), torch.tensor(1.0)); print('sympy' in sys.modules)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.stdout.strip().splitlines()[-1] == "False", out.stdout + out.stderr
