"""The reference workloads' Dense / Conv2D layers on the hand-written kernels (VERDICT r1
item 3): fused bias + activation epilogues, skinny / odd widths (N in {2, 10, 64},
K = 20), first-layer convolutions with Cin in {1, 3} -- forward, input gradient,
weight and bias gradients against a plain PyTorch fp32 reference of the same op on
the same bf16-rounded operands; and a Keras MNIST CNN whose training step runs with
the PyTorch library GEMM / convolution entry points disabled."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_act(y, act):
    return {None: lambda t: t, "relu": torch.relu, "elu": F.elu, "tanh": torch.tanh, "gelu": F.gelu}[act](y)


@pytest.mark.parametrize("act", [None, "relu", "elu", "tanh", "gelu"])
@pytest.mark.parametrize("M,K,N", [(64, 784, 512), (64, 512, 10), (37, 1600, 64), (32, 20, 2), (130, 64, 10),
                                   (64, 5408, 64), (200, 4096, 10)])
def test_dense_fused_vs_fp32(M, K, N, act):
    from cloud_amd.ops import _ext
    from cloud_amd.ops.dense import dense

    _ext.load(required=True)
    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16).requires_grad_()
    b = torch.randn(N, device=DEV).requires_grad_()
    y = dense(x, w, b, act)
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    dy = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = _ref_act(xr @ wr.t() + br, act)
    yr.backward(dy.float())
    tol = dict(atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2 * N ** 0.5, rtol=3e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=3e-2 * M ** 0.5, rtol=3e-2)
    torch.testing.assert_close(b.grad, br.grad, atol=3e-2 * M ** 0.5, rtol=3e-2)


@pytest.mark.parametrize("act", [None, "relu", "elu"])
@pytest.mark.parametrize("N,H,Cin,Cout,k,p", [(8, 28, 1, 32, 3, 0), (4, 32, 3, 32, 3, 1), (4, 13, 32, 64, 3, 0),
                                               (2, 16, 3, 16, 3, 1)])
def test_conv_fused_vs_fp32(N, H, Cin, Cout, k, p, act):
    from cloud_amd.ops import _ext
    from cloud_amd.ops.dense import conv2d

    _ext.load(required=True)
    torch.manual_seed(N * H + Cin)
    x = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(Cout, k, k, Cin, device=DEV) / (k * k * Cin) ** 0.5).to(torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(Cout, device=DEV)).requires_grad_()
    y = conv2d(x, w, b, 1, p, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr.permute(0, 3, 1, 2), br, padding=p)
    yr = _ref_act(yr, act).permute(0, 2, 3, 1)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    red = N * H * H
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=3e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=3e-2 * red ** 0.5, rtol=3e-2)
    torch.testing.assert_close(b.grad, br.grad, atol=3e-2 * red ** 0.5, rtol=3e-2)


@pytest.mark.parametrize("kh,kw,stride,pad", [((3, 5), None, (1, 2), (1, 2)), ((1, 7), None, (1, 1), (0, 3)),
                                               ((5, 3), None, (2, 1), (2, 0))])
def test_conv_rectangular_vs_fp32(kh, kw, stride, pad):
    """Rectangular kernels / strides / paddings (Keras Conv2D((3, 5), strides=(1, 2)), the
    7x1 / 1x7 factorised convolutions): the same implicit-GEMM kernels, geometry per axis."""
    from cloud_amd.ops import _ext
    from cloud_amd.ops.dense import conv2d

    _ext.load(required=True)
    KH, KW = kh
    torch.manual_seed(KH * 10 + KW)
    N, H, W, Cin, Cout = 3, 17, 22, 16, 32
    x = torch.randn(N, H, W, Cin, device=DEV).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(Cout, KH, KW, Cin, device=DEV) / (KH * KW * Cin) ** 0.5).to(torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(Cout, device=DEV)).requires_grad_()
    y = conv2d(x, w, b, stride, pad, "relu")
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.relu(F.conv2d(xr.permute(0, 3, 1, 2), wr.permute(0, 3, 1, 2), br, stride=stride, padding=pad))
    yr = yr.permute(0, 2, 3, 1)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    red = y.numel() / Cout
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=3e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=3e-2 * red ** 0.5, rtol=3e-2)
    torch.testing.assert_close(b.grad, br.grad, atol=3e-2 * red ** 0.5, rtol=3e-2)


def test_keras_mnist_cnn_trains_on_native_kernels(monkeypatch):
    """The reference MNIST CNN (mnist_example_using_fit.py:54-68) under the default
    (auto -> mixed_bfloat16) policy: the training step never reaches PyTorch's
    library GEMM / convolution entry points (hipBLASLt / MIOpen)."""
    import numpy as np

    from cloud_amd import keras
    from cloud_amd.keras import engine

    monkeypatch.setattr(engine, "_POLICY", None)
    monkeypatch.delenv("CLOUD_AMD_PRECISION", raising=False)
    rng = np.random.default_rng(0)
    x = rng.random((512, 28, 28, 1), dtype=np.float32)
    y = (x[:, :14].mean(axis=(1, 2, 3)) > x[:, 14:].mean(axis=(1, 2, 3))).astype("int64")
    model = keras.Sequential([
        keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
        keras.layers.MaxPooling2D(),
        keras.layers.Flatten(),
        keras.layers.Dense(64, activation="relu"),
        keras.layers.Dense(10, activation="softmax"),
    ])
    model.compile(loss="sparse_categorical_crossentropy", optimizer=keras.optimizers.Adam(), metrics=["accuracy"])
    assert engine.global_policy().name == "mixed_bfloat16"
    model.train_on_batch(x[:64], y[:64])  # builds arenas etc. outside the guarded region

    def banned(*a, **k):
        raise AssertionError("library GEMM/conv reached in the training step")

    for mod, name in ((F, "linear"), (F, "conv2d"), (torch, "mm"), (torch, "matmul"), (torch, "addmm")):
        monkeypatch.setattr(mod, name, banned)
    hist = model.fit(x, y, batch_size=64, epochs=4, verbose=0)
    losses = hist.history["loss"]
    assert losses[-1] < losses[0], losses
    monkeypatch.undo()
    pred = model.predict(x[:8])
    assert pred.shape == (8, 10) and np.allclose(pred.sum(-1), 1.0, atol=1e-2)


@pytest.mark.parametrize("N,H,W,C", [(4, 7, 7, 64), (3, 5, 9, 24)])
def test_global_max_pool_native_matches_amax(N, H, W, C):
    """Keras GlobalMaxPooling2D on the native kernel: forward = amax, backward splits the
    gradient evenly over ties (all-zero post-ReLU channels are HW-way ties) as amax does."""
    from cloud_amd import ops

    torch.manual_seed(12)
    x = torch.relu(torch.randn(N, H, W, C, device="cuda")).to(torch.bfloat16)
    x[0, :, :, :5] = 0  # whole-channel ties
    x[1, 0, 0, 7] = x[1, 1, 1, 7] = 9.0  # a two-way tie at the max
    xr = x.float().clone().requires_grad_()
    xn = x.clone().requires_grad_()
    y = ops.global_max_pool_nhwc(xn)
    yr = xr.amax(dim=(1, 2))
    assert torch.equal(y.float(), yr)
    g = torch.randn(N, C, device="cuda")
    y.backward(g.to(torch.bfloat16))
    yr.backward(g.to(torch.bfloat16).float())
    torch.testing.assert_close(xn.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


def test_keras_dropout_layer_native():
    """Keras Dropout runs the native stateless-hash kernel on bf16 activations: keep rate,
    1/(1-p) scaling, identity at inference, and the backward reuses the forward mask."""
    from cloud_amd import tf

    layer = tf.keras.layers.Dropout(0.25)
    x = torch.ones(256, 1024, device="cuda", dtype=torch.bfloat16).requires_grad_()
    y = layer(x, training=True)
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.75) < 5e-3
    torch.testing.assert_close(y[y != 0].float(), torch.full_like(y[y != 0].float(), 1 / 0.75), rtol=1e-2, atol=0)
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, y != 0)
    assert torch.equal(layer(x, training=False), x)


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["relu", "elu", "tanh", "gelu", None])
@pytest.mark.parametrize("N,Np", [(64, 64), (10, 16)])
def test_act_grad_kernel_matches_torch(act, N, Np):
    """rowops.hip act_grad (Dense / Conv2D backward through a fused activation) against the
    fp32 PyTorch form of the same expression, including the zero padding of dy to Np."""
    from cloud_amd.ops import dense as D

    torch.manual_seed(3)
    M = 1000
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    src = torch.randn(M, Np, device="cuda").to(torch.bfloat16)
    y = src if act != "gelu" else None
    if act in ("relu", "elu"):
        y = torch.relu(src) if act == "relu" else torch.nn.functional.elu(src.float()).to(torch.bfloat16)
    if act == "tanh":
        y = torch.tanh(src.float()).to(torch.bfloat16)
    s = src if act == "gelu" else y
    got = D._act_grad_dev(dy, s if act is not None else None, N, Np, act)
    ref = D._act_grad(torch.nn.functional.pad(dy, (0, Np - N)), src if y is None else y,
                      src if act == "gelu" else None, act)
    torch.testing.assert_close(got.float(), ref.float(), atol=2e-2, rtol=2e-2)
    assert got[:, N:].abs().max().item() == 0.0 if Np > N else True


def test_keras_evaluate_fused_loss_matches_predict():
    """evaluate() on the GPU scores with the fused softmax-xent kernel (bf16 logits, device
    accumulator); its loss / accuracy equal the plain formulas on predict()'s
    probabilities, and fit's validation numbers equal a standalone evaluate."""
    import numpy as np

    from cloud_amd import keras
    from cloud_amd.keras import losses as L

    rng = np.random.default_rng(4)
    x = rng.random((384, 28, 28, 1), dtype=np.float32)
    y = (x[:, :14].mean(axis=(1, 2, 3)) > x[:, 14:].mean(axis=(1, 2, 3))).astype("int64")
    model = keras.Sequential([
        keras.layers.Conv2D(16, 3, activation="relu", input_shape=(28, 28, 1)),
        keras.layers.MaxPooling2D(),
        keras.layers.Flatten(),
        keras.layers.Dense(10, activation="softmax"),
    ])
    model.compile(loss="sparse_categorical_crossentropy", optimizer=keras.optimizers.Adam(), metrics=["accuracy"])
    orig = L.SparseCategoricalCrossentropy.per_example

    def banned(*a, **k):
        raise AssertionError("unfused loss path reached")

    L.SparseCategoricalCrossentropy.per_example = banned
    try:
        hist = model.fit(x[:256], y[:256], batch_size=64, epochs=2, validation_data=(x[256:], y[256:]), verbose=0)
        loss, acc = model.evaluate(x[256:], y[256:], batch_size=64, verbose=0)
    finally:
        L.SparseCategoricalCrossentropy.per_example = orig
    p = model.predict(x[256:], batch_size=128).astype("float64")
    n = len(p)
    ref_loss = float(np.mean(-np.log(np.clip(p[np.arange(n), y[256:]], 1e-7, None))))
    ref_acc = float(np.mean(p.argmax(-1) == y[256:]))
    assert abs(loss - ref_loss) < 3e-2 * max(1.0, ref_loss), (loss, ref_loss)
    assert abs(acc - ref_acc) <= 2.0 / n + 1e-9, (acc, ref_acc)
    assert abs(hist.history["val_loss"][-1] - loss) < 1e-4 and abs(hist.history["val_accuracy"][-1] - acc) < 1e-6
