"""ResNet-50 (v1.5) in NHWC on cloud_amd ops -- the north-star workload.

Reference workload: ``tf.keras.applications.ResNet50`` trained on images in
``TFC/core/tests/examples/call_run_within_script_with_keras_fit.py:80-107``; the
BASELINE.json config is ResNet-50 on synthetic ImageNet (224x224x3, 1000
classes).  Layout is NHWC end to end: every 1x1 convolution runs as a GEMM on
the activation memory as it lies, BatchNorm + residual + ReLU are one fused
HIP kernel pair, pooling and the loss are HIP kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import fused_block
from .. import config
from ..ops import conv as conv_ops
from ..ops import pooling as pool_ops
from .layers import BatchNormAct, Conv2d, GlobalAvgPool, Linear, MaxPool2d


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, dtype=torch.bfloat16, device=None, zero_init_residual=True):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = Conv2d(cin, width, 1, dtype=dtype, device=device)
        self.bn1 = BatchNormAct(width, relu=True, device=device)
        self.conv2 = Conv2d(width, width, 3, stride=stride, padding=1, dtype=dtype, device=device)
        self.bn2 = BatchNormAct(width, relu=True, device=device)
        self.conv3 = Conv2d(width, cout, 1, dtype=dtype, device=device)
        self.bn3 = BatchNormAct(cout, relu=True, zero_init=zero_init_residual, device=device)
        self.fused_stats = True
        self.fused_block = True  # one autograd node per block when the params live in the grad arena
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.ModuleDict({
                "conv": Conv2d(cin, cout, 1, stride=stride, dtype=dtype, device=device),
                "bn": BatchNormAct(cout, relu=False, device=device),
            })

    def forward(self, x, next_block=None):
        if self.fused_block and fused_block.can_fuse(self, x):
            return fused_block.bottleneck_forward(self, x, next_block)
        fused_block.check_not_pending(x)
        identity = x
        fs = self.fused_stats
        if self.downsample is not None:
            identity = self.downsample["bn"](self.downsample["conv"](x, stats=fs))
        out = self.bn1(self.conv1(x, stats=fs))
        out = self.bn2(self.conv2(out, stats=fs))
        return self.bn3(self.conv3(out, stats=fs), residual=identity)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, in_channels=3, stem_channels_pad=0,
                 dtype=torch.bfloat16, device=None, zero_init_residual=True):
        super().__init__()
        self.in_channels = in_channels
        self.stem_cin = in_channels + stem_channels_pad
        self.conv1 = Conv2d(self.stem_cin, 64, 7, stride=2, padding=3, dtype=dtype, device=device)
        self.bn1 = BatchNormAct(64, relu=True, device=device)
        self.maxpool = MaxPool2d(3, 2, 1)
        self.stem_s2d = True  # space-to-depth stem on the native path (ops.conv.stem_conv_s2d)
        blocks = []
        cin = 64
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(Bottleneck(cin, width, stride, dtype=dtype, device=device,
                                         zero_init_residual=zero_init_residual))
                cin = width * Bottleneck.expansion
        self.layers = nn.Sequential(*blocks)
        self.pool = GlobalAvgPool()
        self.fc = Linear(cin, num_classes, dtype=dtype, device=device)

    def forward(self, x):
        """x: NHWC [N, H, W, in_channels] in the compute dtype -> logits [N, classes]."""
        c1 = self.conv1
        if self.stem_s2d and x.shape[-1] == self.in_channels and conv_ops.stem_s2d_ok(x, c1.weight, c1.stride,
                                                                                         c1.padding):
            # 7x7/2 stem as a 4x4/1 conv over the space-to-depth input (no channel pad pass)
            x = self._stem_tail(conv_ops.stem_conv_s2d(x, c1.weight, stats=True))
        else:
            if self.stem_cin != self.in_channels:
                x = torch.nn.functional.pad(x, (0, self.stem_cin - self.in_channels))
            x = self._stem_tail(self.conv1(x, stats=True))
        if self.layers._forward_hooks or self.layers._forward_pre_hooks:
            # hooks on the block Sequential: call it (they fire; no cross-block BN fold)
            x = self.layers(x)
        else:
            blocks = list(self.layers)
            for i, blk in enumerate(blocks):
                # a fused block hands its bn3 apply to the next fused block's conv1 (fused_block)
                x = blk(x, blocks[i + 1] if i + 1 < len(blocks) else None)
        return self.fc(self.pool(x))

    def _stem_tail(self, out):
        """maxpool(bn1(conv1 output)): in training, BN + ReLU + max-pool fused into one pass
        each way (the 112x112x64 BN output is never materialised); else the separate ops."""
        z, part = out if isinstance(out, tuple) else (out, None)
        if config.get("CLOUD_AMD_STEM_TAIL") and pool_ops.stem_tail_ok(z, self.bn1, self.maxpool, part):
            return pool_ops.stem_bn_relu_maxpool(z, self.bn1, part)
        return self.maxpool(self.bn1((z, part) if part is not None else z))


def resnet50(**kw):
    """ResNet-50 v1.5.  The 3-channel input is zero-padded to 8 channels so the 7x7
    stem runs on the implicit-GEMM kernel (16-byte channel chunks)."""
    kw.setdefault("stem_channels_pad", 5)
    return ResNet((3, 4, 6, 3), **kw)


def resnet18_like_small(**kw):
    """Tiny bottleneck ResNet for CPU tests (same code path, few blocks)."""
    return ResNet((1, 1, 1, 1), **kw)
