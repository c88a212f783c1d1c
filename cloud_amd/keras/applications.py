"""``tf.keras.applications`` subset backed by the native NHWC model zoo.

``ResNet50`` (reference ``call_run_within_script_with_keras_fit.py:80``) wraps
:class:`cloud_amd.models.resnet.ResNet` -- fused BN/ReLU, MFMA implicit-GEMM
convolutions -- as a Keras model.  ``weights`` must be None (no network: random
init); ``include_top=False`` + ``pooling`` give the feature extractor.
"""
from __future__ import annotations

import torch

from ..models.resnet import ResNet
from .engine import Layer, global_policy
from .models import Model


class _ResNetBody(Layer):
    def __init__(self, include_top, classes, pooling, **kw):
        super().__init__(**kw)
        self.include_top, self.classes, self.pooling = include_top, classes, pooling

    def build(self, input_shape):
        dt = global_policy().compute_dtype
        cin = int(input_shape[-1])
        self.net = ResNet((3, 4, 6, 3), num_classes=self.classes, in_channels=cin,
                          stem_channels_pad=(8 - cin % 8) % 8, dtype=dt)

    def call(self, x, training=None):
        n = self.net
        x = x.to(n.conv1.weight.dtype)
        if n.stem_cin != n.in_channels:
            x = torch.nn.functional.pad(x, (0, n.stem_cin - n.in_channels))
        x = n.maxpool(n.bn1(n.conv1(x.contiguous(), stats=True)))
        x = n.layers(x)
        if self.include_top:
            return torch.softmax(n.fc(n.pool(x)).float(), -1)
        if self.pooling == "avg":
            return n.pool(x)
        if self.pooling == "max":
            return x.amax(dim=(1, 2))
        return x


class ResNet50(Model):
    def __init__(self, include_top=True, weights=None, input_tensor=None, input_shape=None, pooling=None,
                 classes=1000, **kw):
        if weights not in (None, "none"):
            raise ValueError("pretrained weights are not available offline; use weights=None")
        super().__init__(name=kw.pop("name", "resnet50"))
        self.body = _ResNetBody(include_top, classes, pooling)
        self.include_top, self.pooling, self.classes = include_top, pooling, classes
        if input_tensor is not None and input_shape is None:
            input_shape = tuple(input_tensor.shape[1:])
        if input_shape is not None:
            self.body._maybe_build((None,) + tuple(input_shape))
        self._sym_in = self._sym_out = None
        if input_tensor is not None:  # functional use: base_model.output feeds further layers
            self._sym_in = input_tensor
            self._sym_out = self(input_tensor)

    def compute_output_shape(self, input_shape):
        _, h, w, _ = input_shape
        if self.include_top:
            return (None, self.classes)
        if self.pooling in ("avg", "max"):
            return (None, 2048)

        def down(v):
            if v is None:
                return None
            v = (v + 2 * 3 - 7) // 2 + 1       # stem 7x7/2
            v = (v + 2 - 3) // 2 + 1           # maxpool 3x3/2
            for _ in range(3):
                v = (v + 2 - 3) // 2 + 1       # 3x3/2 in layers 2..4
            return v
        return (None, down(h), down(w), 2048)

    def call(self, x, training=None):
        return self.body(x, training=training)


class resnet50:  # namespace parity: tf.keras.applications.resnet50
    @staticmethod
    def preprocess_input(x, data_format=None):
        """Caffe-style: RGB -> BGR, minus the ImageNet channel means (0..255 inputs)."""
        import numpy as np

        mean = [103.939, 116.779, 123.68]
        if isinstance(x, torch.Tensor):
            x = x.float()[..., [2, 1, 0]]
            return x - torch.tensor(mean, dtype=x.dtype, device=x.device)
        x = np.asarray(x, dtype=np.float32)[..., ::-1]
        return (x - np.asarray(mean, dtype=np.float32)).astype(np.float32)
