"""The residual library paths are never reached by the default workloads (round-4 verdict,
"Residual library paths"): ``ops/gemm.py``'s ``torch.mm`` fallback for unaligned operands,
``models/bert.py``'s ``F.linear`` head for more labels than the fused head kernel takes,
PyTorch convolutions, and the vendor-library engine of ``ops/raw.py PlainGemmPolicy``
(``CLOUD_AMD_GEMM_LIB=never`` by default).  Each entry point is wrapped with a counter
while a training step of ResNet-50, BERT-base (2 layers) and the reference's Keras MNIST
models runs on the native path; every counter must stay at zero."""
import contextlib

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def counted(monkeypatch):
    from cloud_amd.ops import raw

    calls = {}

    def wrap(owner, name):
        orig = getattr(owner, name)

        def f(*a, **k):
            calls[name] = calls.get(name, 0) + 1
            return orig(*a, **k)

        monkeypatch.setattr(owner, name, f)

    for name in ("mm", "matmul", "bmm", "addmm", "conv2d"):
        wrap(torch, name)
    for name in ("linear", "conv2d"):
        wrap(F, name)
    wrap(raw, "_plain_lib")
    yield calls


def test_resnet50_step_uses_no_library_gemm(monkeypatch):
    from cloud_amd.models import resnet50
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD

    torch.manual_seed(0)
    m = resnet50(num_classes=1000, dtype=torch.bfloat16, device="cuda")
    opt = SGD(m, learning_rate=0.1, momentum=0.9)
    x = torch.randn(32, 224, 224, 3, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 1000, (32,), device="cuda")
    with counted(monkeypatch) as calls:
        for _ in range(2):
            opt.zero_grad()
            loss, _ = softmax_cross_entropy(m(x), y)
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
    assert not calls, calls


def test_bert_step_uses_no_library_gemm(monkeypatch):
    from cloud_amd.models.bert import BertConfig, BertForSequenceClassification
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import AdamW

    torch.manual_seed(0)
    cfg = BertConfig.base(num_hidden_layers=2, num_labels=2)
    m = BertForSequenceClassification(cfg, device="cuda")
    opt = AdamW(m, learning_rate=2e-5, weight_decay=0.01)
    ids = torch.randint(1000, 30522, (16, 128), device="cuda")
    tts = torch.zeros_like(ids)
    am = torch.ones_like(ids)
    labels = torch.randint(0, 2, (16,), device="cuda")
    with counted(monkeypatch) as calls:
        for _ in range(2):
            opt.zero_grad()
            loss, _ = softmax_cross_entropy(m(ids, tts, am), labels, denom=16)
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
    assert not calls, calls


def test_keras_mnist_models_use_no_library_gemm(monkeypatch):
    from cloud_amd import keras

    rng = np.random.default_rng(0)
    x = rng.random((256, 28, 28, 1), dtype=np.float32)
    y = rng.integers(0, 10, (256,))
    cnn = keras.Sequential([keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
                            keras.layers.MaxPooling2D(), keras.layers.Flatten(),
                            keras.layers.Dense(64, activation="relu"), keras.layers.Dense(10, activation="softmax")])
    mlp = keras.Sequential([keras.layers.Flatten(input_shape=(28, 28, 1)), keras.layers.Dense(512, activation="relu"),
                            keras.layers.Dropout(0.2), keras.layers.Dense(10, activation="softmax")])
    for m in (cnn, mlp):
        m.compile(optimizer="adam", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
        m.fit(x[:64], y[:64], batch_size=64, epochs=1, verbose=0)  # build + first-step paths outside the count
    with counted(monkeypatch) as calls:
        for m in (cnn, mlp):
            m.fit(x, y, batch_size=64, epochs=1, verbose=0)
        torch.cuda.synchronize()
    assert not calls, calls
