"""Keras layers (``tf.keras.layers`` names/arguments) on cloud_amd NHWC ops.

Used by the reference workloads: Dense, Conv2D, MaxPooling2D, GlobalMax/Avg
pooling, Flatten, Dropout, BatchNormalization, Activation, Rescaling and the
CIFAR augmentation layers (``keras_tuner_cifar_example.py:24-77``,
``mnist_example_using_fit.py:54-63``, README MLP).  Weight layouts are the
MI355X kernel layouts: Dense ``[units, in]``, Conv2D ``[filters, kh, kw, in]``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import ops
from ..ops.dense import conv2d as conv_act_op
from ..ops.dense import dense as dense_op
from ..ops.dropout import dropout as dropout_op
from . import activations, initializers, regularizers
from .engine import Input, InputLayer, Layer, global_policy  # noqa: F401


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


_ACT_NAMES = {activations.linear: None, activations.relu: "relu", activations.elu: "elu",
              activations.tanh: "tanh", activations.gelu: "gelu"}


def _fused_act(fn):
    """(epilogue activation name, remaining activation fn) for a Keras activation."""
    if fn in _ACT_NAMES:
        return _ACT_NAMES[fn], None
    return None, fn


def _bias_dtype(layer):
    """Biases are variables: fp32 under the mixed policy (the epilogue adds them in fp32)."""
    return layer._dtype_policy.variable_dtype if layer.compute_dtype == torch.bfloat16 else layer.compute_dtype


class _Regularized:
    """kernel/bias regularizers -> ``regularization_loss()`` (summed into the loss by Model)."""

    def _set_regularizers(self, kernel_regularizer, bias_regularizer):
        self.kernel_regularizer = regularizers.get(kernel_regularizer)
        self.bias_regularizer = regularizers.get(bias_regularizer)

    def regularization_loss(self):
        out = None
        for reg, w in ((self.kernel_regularizer, getattr(self, "kernel", None)),
                       (self.bias_regularizer, getattr(self, "bias", None))):
            if reg is not None and w is not None and self.trainable:
                p = reg(w)
                out = p if out is None else out + p
        return out if out is not None else 0.0


class Dense(_Regularized, Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, bias_regularizer=None, **kw):
        super().__init__(**kw)
        self.units = int(units)
        self.activation = activations.get(activation)
        self.use_bias = use_bias
        self.kernel_initializer, self.bias_initializer = kernel_initializer, bias_initializer
        self._set_regularizers(kernel_regularizer, bias_regularizer)

    def build(self, input_shape):
        fin = int(input_shape[-1])
        w = torch.empty(self.units, fin)
        initializers.get(self.kernel_initializer)(w)
        self.kernel = torch.nn.Parameter(w.to(self.compute_dtype))
        if self.use_bias:
            b = torch.empty(self.units)
            initializers.get(self.bias_initializer)(b)
            self.bias = torch.nn.Parameter(b.to(_bias_dtype(self)))
        else:
            self.bias = None

    def call(self, x, training=None):
        x = x.to(self.kernel.dtype)
        if getattr(self, "_emit_logits", False):  # fused softmax-xent training path (Model.fit)
            return dense_op(x, self.kernel, self.bias, None)
        act, rest = _fused_act(self.activation)
        y = dense_op(x, self.kernel, self.bias, act)
        return rest(y) if rest is not None else y

    def get_config(self):
        c = super().get_config()
        c.update(units=self.units, activation=activations.serialize(self.activation), use_bias=self.use_bias,
                 kernel_initializer=self.kernel_initializer if isinstance(self.kernel_initializer, str)
                 else "glorot_uniform")
        return c


class Conv2D(_Regularized, Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None, use_bias=True,
                 kernel_initializer="glorot_uniform", data_format=None, kernel_regularizer=None,
                 bias_regularizer=None, **kw):
        super().__init__(**kw)
        self._set_regularizers(kernel_regularizer, bias_regularizer)
        if data_format not in (None, "channels_last"):
            raise ValueError("cloud_amd layers are channels_last (NHWC) only")
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        self.activation = activations.get(activation)
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer

    def build(self, input_shape):
        cin = int(input_shape[-1])
        kh, kw = self.kernel_size
        w = torch.empty(self.filters, kh, kw, cin)
        initializers.get(self.kernel_initializer)(w)
        self.kernel = torch.nn.Parameter(w.to(self.compute_dtype))
        self.bias = torch.nn.Parameter(torch.zeros(self.filters, dtype=_bias_dtype(self))) if self.use_bias else None

    def _same_pads(self, H, W):
        out = []
        for n, k, s in ((H, self.kernel_size[0], self.strides[0]), (W, self.kernel_size[1], self.strides[1])):
            o = math.ceil(n / s)
            tot = max((o - 1) * s + k - n, 0)
            out.append((tot // 2, tot - tot // 2))
        return out

    def call(self, x, training=None):
        x = x.to(self.kernel.dtype)
        pad = (0, 0)
        if self.padding == "same":
            (pt, pb), (pl, pr) = self._same_pads(x.shape[1], x.shape[2])
            if pt == pb and pl == pr:
                pad = (pt, pl)
            else:  # TF's asymmetric SAME split (extra row/column at the bottom/right)
                x = F.pad(x, (0, 0, pl, pr, pt, pb))
        act, rest = _fused_act(self.activation)
        y = conv_act_op(x.contiguous(), self.kernel, self.bias, tuple(self.strides), pad, act)
        return rest(y) if rest is not None else y

    def get_config(self):
        c = super().get_config()
        c.update(filters=self.filters, kernel_size=list(self.kernel_size), strides=list(self.strides),
                 padding=self.padding, activation=activations.serialize(self.activation), use_bias=self.use_bias)
        return c


class _Pool2D(Layer):
    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", **kw):
        super().__init__(**kw)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        self.padding = padding.lower()

    def get_config(self):
        c = super().get_config()
        c.update(pool_size=list(self.pool_size), strides=list(self.strides), padding=self.padding)
        return c


class MaxPooling2D(_Pool2D):
    def call(self, x, training=None):
        k, s = self.pool_size[0], self.strides[0]
        if self.padding == "same":
            H, W = x.shape[1], x.shape[2]
            ph = max((math.ceil(H / s) - 1) * s + k - H, 0)
            pw = max((math.ceil(W / s) - 1) * s + k - W, 0)
            if ph or pw:
                x = F.pad(x, (0, 0, pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=float("-inf"))
        return ops.max_pool2d_nhwc(x.contiguous(), k, s, 0)


class AveragePooling2D(_Pool2D):
    def call(self, x, training=None):
        y = F.avg_pool2d(x.permute(0, 3, 1, 2), self.pool_size, self.strides)
        return y.permute(0, 2, 3, 1).contiguous()


class GlobalAveragePooling2D(Layer):
    def call(self, x, training=None):
        return ops.global_avg_pool_nhwc(x.contiguous())


class GlobalMaxPooling2D(Layer):
    def call(self, x, training=None):
        return ops.global_max_pool_nhwc(x.contiguous())


class Flatten(Layer):
    def call(self, x, training=None):
        return x.reshape(x.shape[0], -1)


class Reshape(Layer):
    def __init__(self, target_shape, **kw):
        super().__init__(**kw)
        self.target_shape = tuple(target_shape)

    def call(self, x, training=None):
        return x.reshape((x.shape[0],) + self.target_shape)

    def get_config(self):
        c = super().get_config()
        c["target_shape"] = list(self.target_shape)
        return c


class Dropout(Layer):
    def __init__(self, rate, seed=None, **kw):
        super().__init__(**kw)
        self.rate = float(rate)

    def call(self, x, training=None):
        return dropout_op(x, self.rate, training=bool(training))

    def get_config(self):
        c = super().get_config()
        c["rate"] = self.rate
        return c


class Activation(Layer):
    def __init__(self, activation, **kw):
        super().__init__(**kw)
        self.activation = activations.get(activation)

    def call(self, x, training=None):
        if getattr(self, "_emit_logits", False):
            return x
        return self.activation(x)

    def get_config(self):
        c = super().get_config()
        c["activation"] = activations.serialize(self.activation)
        return c


class ReLU(Activation):
    def __init__(self, **kw):
        super().__init__("relu", **kw)

    def get_config(self):
        c = super().get_config()
        c.pop("activation")
        return c


class Softmax(Activation):
    def __init__(self, **kw):
        super().__init__("softmax", **kw)

    def get_config(self):
        c = super().get_config()
        c.pop("activation")
        return c


class BatchNormalization(Layer):
    """Keras semantics: moving = momentum * moving + (1 - momentum) * batch; epsilon 1e-3."""

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, **kw):
        super().__init__(**kw)
        if axis not in (-1, 3):
            raise ValueError("BatchNormalization normalises the channel (last) axis in NHWC")
        self.momentum, self.epsilon, self.center, self.scale = float(momentum), float(epsilon), center, scale

    def build(self, input_shape):
        c = int(input_shape[-1])
        self.gamma = torch.nn.Parameter(torch.ones(c)) if self.scale else None
        self.beta = torch.nn.Parameter(torch.zeros(c)) if self.center else None
        self.register_buffer("moving_mean", torch.zeros(c))
        self.register_buffer("moving_variance", torch.ones(c))

    def call(self, x, training=None):
        return ops.bn_act(x.contiguous(), self.gamma, self.beta, self.moving_mean, self.moving_variance,
                          eps=self.epsilon, momentum=1.0 - self.momentum, relu=False, training=bool(training))

    def get_config(self):
        c = super().get_config()
        c.update(momentum=self.momentum, epsilon=self.epsilon, center=self.center, scale=self.scale)
        return c


class LayerNormalization(Layer):
    def __init__(self, axis=-1, epsilon=1e-3, **kw):
        super().__init__(**kw)
        self.epsilon = float(epsilon)

    def build(self, input_shape):
        c = int(input_shape[-1])
        self.gamma = torch.nn.Parameter(torch.ones(c))
        self.beta = torch.nn.Parameter(torch.zeros(c))

    def call(self, x, training=None):
        y = F.layer_norm(x.float(), (x.shape[-1],), self.gamma, self.beta, self.epsilon)
        return y.to(x.dtype)

    def get_config(self):
        c = super().get_config()
        c["epsilon"] = self.epsilon
        return c


class Embedding(Layer):
    def __init__(self, input_dim, output_dim, **kw):
        super().__init__(**kw)
        self.input_dim, self.output_dim = int(input_dim), int(output_dim)

    def build(self, input_shape):
        w = torch.empty(self.input_dim, self.output_dim)
        torch.nn.init.uniform_(w, -0.05, 0.05)
        self.embeddings = torch.nn.Parameter(w.to(self.compute_dtype))

    def call(self, x, training=None):
        return F.embedding(x.long(), self.embeddings)

    def get_config(self):
        c = super().get_config()
        c.update(input_dim=self.input_dim, output_dim=self.output_dim)
        return c


class Rescaling(Layer):
    def __init__(self, scale, offset=0.0, **kw):
        super().__init__(**kw)
        self.scale, self.offset = float(scale), float(offset)

    def call(self, x, training=None):
        return x.float() * self.scale + self.offset

    def get_config(self):
        c = super().get_config()
        c.update(scale=self.scale, offset=self.offset)
        return c


class Add(Layer):
    def call(self, xs, training=None):
        out = xs[0]
        for t in xs[1:]:
            out = out + t
        return out


class Concatenate(Layer):
    def __init__(self, axis=-1, **kw):
        super().__init__(**kw)
        self.axis = axis

    def call(self, xs, training=None):
        return torch.cat(list(xs), dim=self.axis)

    def get_config(self):
        c = super().get_config()
        c["axis"] = self.axis
        return c


# ---- augmentation (K11): active only in training ------------------------------
class RandomFlip(Layer):
    def __init__(self, mode="horizontal", seed=None, **kw):
        super().__init__(**kw)
        self.mode = mode

    def call(self, x, training=None):
        if not training:
            return x
        B = x.shape[0]
        if "horizontal" in self.mode:
            m = torch.rand(B, device=x.device) < 0.5
            x = torch.where(m[:, None, None, None], x.flip(2), x)
        if "vertical" in self.mode:
            m = torch.rand(B, device=x.device) < 0.5
            x = torch.where(m[:, None, None, None], x.flip(1), x)
        return x

    def get_config(self):
        c = super().get_config()
        c["mode"] = self.mode
        return c


class _RandomAffine(Layer):
    def _affine(self, x, theta):
        grid = F.affine_grid(theta, (x.shape[0], x.shape[3], x.shape[1], x.shape[2]), align_corners=False)
        y = F.grid_sample(x.permute(0, 3, 1, 2).float(), grid, padding_mode="reflection", align_corners=False)
        return y.permute(0, 2, 3, 1).to(x.dtype).contiguous()


class RandomRotation(_RandomAffine):
    def __init__(self, factor, seed=None, **kw):
        super().__init__(**kw)
        self.factor = factor

    def call(self, x, training=None):
        if not training:
            return x
        lo, hi = (-self.factor, self.factor) if not isinstance(self.factor, (tuple, list)) else self.factor
        ang = (torch.rand(x.shape[0], device=x.device) * (hi - lo) + lo) * 2 * math.pi
        c, s = torch.cos(ang), torch.sin(ang)
        z = torch.zeros_like(c)
        theta = torch.stack([torch.stack([c, -s, z], 1), torch.stack([s, c, z], 1)], 1)
        return self._affine(x, theta)

    def get_config(self):
        c = super().get_config()
        c["factor"] = self.factor
        return c


class RandomTranslation(_RandomAffine):
    def __init__(self, height_factor, width_factor, seed=None, **kw):
        super().__init__(**kw)
        self.hf, self.wf = height_factor, width_factor

    def call(self, x, training=None):
        if not training:
            return x
        B = x.shape[0]
        ty = (torch.rand(B, device=x.device) * 2 - 1) * self.hf * 2
        tx = (torch.rand(B, device=x.device) * 2 - 1) * self.wf * 2
        o, z = torch.ones(B, device=x.device), torch.zeros(B, device=x.device)
        theta = torch.stack([torch.stack([o, z, tx], 1), torch.stack([z, o, ty], 1)], 1)
        return self._affine(x, theta)


class RandomZoom(_RandomAffine):
    def __init__(self, height_factor, width_factor=None, seed=None, **kw):
        super().__init__(**kw)
        self.hf = height_factor
        self.wf = width_factor if width_factor is not None else height_factor

    def call(self, x, training=None):
        if not training:
            return x
        B = x.shape[0]
        zy = 1 + (torch.rand(B, device=x.device) * 2 - 1) * abs(self.hf)
        zx = 1 + (torch.rand(B, device=x.device) * 2 - 1) * abs(self.wf)
        z = torch.zeros(B, device=x.device)
        theta = torch.stack([torch.stack([zx, z, z], 1), torch.stack([z, zy, z], 1)], 1)
        return self._affine(x, theta)


class _RandomResize(Layer):
    """Keras RandomHeight / RandomWidth: one factor per batch, the output size changes."""

    axis = 1

    def __init__(self, factor, interpolation="bilinear", seed=None, **kw):
        super().__init__(**kw)
        self.factor = factor
        self.interpolation = interpolation

    def call(self, x, training=None):
        if not training:
            return x
        lo, hi = (-self.factor, self.factor) if not isinstance(self.factor, (tuple, list)) else self.factor
        f = 1.0 + float(torch.empty(()).uniform_(lo, hi))
        size = [x.shape[1], x.shape[2]]
        size[self.axis - 1] = max(1, int(round(size[self.axis - 1] * f)))
        mode = "bilinear" if self.interpolation == "bilinear" else "nearest"
        y = F.interpolate(x.permute(0, 3, 1, 2).float(), size=size, mode=mode,
                          align_corners=False if mode == "bilinear" else None)
        return y.permute(0, 2, 3, 1).to(x.dtype).contiguous()

    def get_config(self):
        c = super().get_config()
        c["factor"] = self.factor
        return c


class RandomHeight(_RandomResize):
    axis = 1


class RandomWidth(_RandomResize):
    axis = 2


class RandomContrast(Layer):
    def __init__(self, factor, seed=None, **kw):
        super().__init__(**kw)
        self.factor = factor

    def call(self, x, training=None):
        if not training:
            return x
        f = 1 + (torch.rand(x.shape[0], 1, 1, 1, device=x.device) * 2 - 1) * self.factor
        m = x.mean(dim=(1, 2), keepdim=True)
        return (x - m) * f + m


class Lambda(Layer):
    def __init__(self, function, **kw):
        super().__init__(**kw)
        self.function = function

    def call(self, x, training=None):
        return self.function(x)


class TorchModule(Layer):
    """Wrap an arbitrary (already-built) ``nn.Module`` as a Keras layer."""

    def __init__(self, module, **kw):
        super().__init__(**kw)
        self.module = module
        self.built = True

    def call(self, x, training=None):
        return self.module(x)


LAYERS = {cls.__name__: cls for cls in [
    Dense, Conv2D, MaxPooling2D, AveragePooling2D, GlobalAveragePooling2D, GlobalMaxPooling2D, Flatten, Reshape,
    Dropout, Activation, ReLU, Softmax, BatchNormalization, LayerNormalization, Embedding, Rescaling, Add,
    Concatenate, RandomFlip, RandomRotation, RandomTranslation, RandomZoom, RandomContrast, InputLayer]}
MaxPool2D = MaxPooling2D
AvgPool2D = AveragePooling2D
GlobalAvgPool2D = GlobalAveragePooling2D
GlobalMaxPool2D = GlobalMaxPooling2D
Convolution2D = Conv2D


class experimental:  # namespace parity: tf.keras.layers.experimental.preprocessing (TF 2.3)
    class preprocessing:
        RandomFlip = RandomFlip
        RandomRotation = RandomRotation
        RandomTranslation = RandomTranslation
        RandomZoom = RandomZoom
        RandomContrast = RandomContrast
        RandomHeight = RandomHeight
        RandomWidth = RandomWidth
        Rescaling = Rescaling
