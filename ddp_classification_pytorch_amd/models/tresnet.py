"""TResNet-M (the BASELINE default ``tresnet_m_miil_in21k``, BASELINE/main.py:29,143-144)
on the gfx950 kernels.

Architecture (timm TResNet; not vendored in the reference):
* SpaceToDepth(4) stem: [N,224,224,3] -> [N,56,56,48] (``space_to_depth`` kernel)
  then conv3x3(48->64) + InplaceABN(leaky 0.01);
* layer1: 3 x BasicBlock(64), layer2: 4 x BasicBlock(128), layer3: 11 x
  Bottleneck(256 -> 1024), layer4: 3 x Bottleneck(512 -> 2048);
  SE in layers 1-3; stride-2 blocks downsample with a stride-1 conv followed
  by an anti-aliased 3x3 blur (reflect pad; ``dwconv`` kernel); the residual
  path downsamples with AvgPool2d(2) + 1x1 conv-BN;
* InplaceABN = BN + leaky-ReLU (slope 1e-3 inside blocks, 1e-2 in the stem) in
  one kernel, with inplace_abn's semantics: effective weight |gamma| + eps, and
  only the activation OUTPUT kept -- the backward inverts the leaky ReLU and the
  affine transform in registers (``bn_bwd_* inv``), so the BN input is freed
  after the forward (one activation per layer less than BN + activation);
* global average pool -> fc.
Input: NHWC activations with 3 channels (``cpad=3``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import functional as Fn
from .layers import BatchNorm2d, Conv2d, ConvBN, Linear

LEAKY_BLOCK = 1e-3
LEAKY_STEM = 1e-2


def _blur_filter():
    f = torch.tensor([1.0, 2.0, 1.0])
    return (f[:, None] * f[None, :]) / 16.0


class AntiAliasDownsample(nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("filt", _blur_filter(), persistent=False)

    def forward(self, x):
        return Fn.blur_pool(x, self.filt.to(x.device), k=3, s=2, p=1, reflect=True)


class AvgPool2x2(nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("filt", torch.full((2, 2), 0.25), persistent=False)

    def forward(self, x, deposit=None):
        return Fn.blur_pool(x, self.filt.to(x.device), k=2, s=2, p=0, reflect=False, deposit=deposit)


class SEModule(nn.Module):
    """avg-pool -> fc(C->R)+ReLU -> fc(R->C)+sigmoid -> channel scale (fused with residual+ReLU)."""

    def __init__(self, channels, reduction_channels):
        super().__init__()
        self.fc1 = Linear(channels, reduction_channels)
        self.fc2 = Linear(reduction_channels, channels)

    def gate(self, x, join=None):
        p = Fn.global_avg_pool(x, link=join)
        if Fn.se_gate_fusable(p, self.fc1.weight, self.fc2.weight):  # small batch: one kernel each way
            return Fn.se_gate(p, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias)
        h = self.fc1(p, relu=True)
        return Fn.linear(h, self.fc2.weight, self.fc2.bias, act="sigmoid")

    def forward(self, x, residual=None, relu=False, link=None):
        # x feeds the pooling and the channel scale: the scale's backward (which runs first)
        # deposits its x-gradient and the pooling's backward adds it while broadcasting
        join = Fn.GradJoin(1)
        return Fn.channel_scale(x, self.gate(x, join), residual, relu, link=link, deposit=join)


class Downsample(nn.Module):
    def __init__(self, inplanes, planes, stride):
        super().__init__()
        self.pool = AvgPool2x2() if stride == 2 else None
        self.conv = ConvBN(inplanes, planes, 1, 1, 0, act="none")

    def forward(self, x):
        if self.pool is not None:
            x = self.pool(x)
        return self.conv(x)

    def raw(self, x, deposit=None):
        """(conv output, BN statistics slabs, BN module): the shortcut before its BN, for a
        consumer that normalises it on the fly (BatchNorm2d(residual_bn=...)).  ``deposit``: the
        block's GradJoin, which receives the shortcut's input gradient."""
        if self.pool is not None:
            x = self.pool(x, deposit=deposit)
            deposit = None
        bn = self.conv.bn
        r, rs = self.conv.conv(x, stats=bn.training and not bn.frozen, deposit=deposit)
        return r, (bn, rs)

    def normed(self, x, deposit=None):
        r, (bn, rs) = self.raw(x, deposit)
        return bn(r, rs, act="none")


def _first_conv(cbn, x, join):
    """A block's first ConvBN as the primary consumer of the block input: its dgrad epilogue adds
    the shortcut's gradient (GradJoin) and fuses the producing BN's backward reduction."""
    y, s = cbn.conv(x, stats=cbn.bn.training and not cbn.bn.frozen, link=join)
    return cbn.bn(y, s, act=cbn.act, slope=cbn.slope)


class TBasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, use_se=True):
        super().__init__()
        self.conv1 = ConvBN(inplanes, planes, 3, 1, act="leaky", slope=LEAKY_BLOCK, inplace_abn=True)
        self.aa = AntiAliasDownsample() if stride == 2 else None
        self.conv2 = ConvBN(planes, planes, 3, 1, act="none")
        self.se = SEModule(planes, max(planes // 4, 64)) if use_se else None
        self.downsample = Downsample(inplanes, planes, stride) if (stride != 1 or inplanes != planes) else None

    def forward(self, x):
        # the block input's second consumer (identity residual / shortcut pool) hands its gradient
        # to conv1 (GradJoin); the shortcut runs after the main path so its backward comes first
        join = Fn.GradJoin(1)
        out = _first_conv(self.conv1, x, join)
        if self.aa is not None:
            out = self.aa(out)
        if self.se is None:
            y, s = self.conv2.conv(out, stats=self.conv2.bn.training and not self.conv2.bn.frozen)
            if self.downsample is not None:
                r, rbn = self.downsample.raw(x, deposit=join)
                return self.conv2.bn(y, s, act="relu", residual=r, residual_bn=rbn)
            return self.conv2.bn(y, s, act="relu", residual=x, link=join)
        out = self.conv2(out)
        if self.downsample is not None:
            return self.se(out, residual=self.downsample.normed(x, deposit=join), relu=True)
        return self.se(out, residual=x, relu=True, link=join)


class TBottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, use_se=True):
        super().__init__()
        self.conv1 = ConvBN(inplanes, planes, 1, 1, 0, act="leaky", slope=LEAKY_BLOCK, inplace_abn=True)
        self.conv2 = ConvBN(planes, planes, 3, 1, act="leaky", slope=LEAKY_BLOCK, inplace_abn=True)
        self.aa = AntiAliasDownsample() if stride == 2 else None
        self.se = SEModule(planes, max(planes * 4 // 8, 64)) if use_se else None
        self.conv3 = ConvBN(planes, planes * 4, 1, 1, 0, act="none")
        self.downsample = (Downsample(inplanes, planes * 4, stride)
                           if (stride != 1 or inplanes != planes * 4) else None)

    def forward(self, x):
        join = Fn.GradJoin(1)
        out = _first_conv(self.conv1, x, join)
        out = self.conv2(out)
        if self.aa is not None:
            out = self.aa(out)
        if self.se is not None:
            out = self.se(out)
        y, s = self.conv3.conv(out, stats=self.conv3.bn.training and not self.conv3.bn.frozen)
        if self.downsample is not None:
            # projection shortcut (after the main path: its backward precedes conv1's); its BN is
            # applied inside conv3's BN pass (no shortcut activation)
            r, rbn = self.downsample.raw(x, deposit=join)
            return self.conv3.bn(y, s, act="relu", residual=r, residual_bn=rbn)
        return self.conv3.bn(y, s, act="relu", residual=x, link=join)


class TResNet(nn.Module):
    def __init__(self, layers=(3, 4, 11, 3), num_classes=1000, width_factor=1.0, in_chans=3):
        super().__init__()
        self.inplanes = self.planes = int(64 * width_factor)
        self.stem = ConvBN(in_chans * 16, self.planes, 3, 1, act="leaky", slope=LEAKY_STEM, inplace_abn=True)
        self.layer1 = self._make(TBasicBlock, self.planes, layers[0], 1, True)
        self.layer2 = self._make(TBasicBlock, self.planes * 2, layers[1], 2, True)
        self.layer3 = self._make(TBottleneck, self.planes * 4, layers[2], 2, True)
        self.layer4 = self._make(TBottleneck, self.planes * 8, layers[3], 2, False)
        self.feat_dim = self.planes * 8 * TBottleneck.expansion
        self.fc = Linear(self.feat_dim, num_classes) if num_classes > 0 else None
        for m in self.modules():  # timm: zero-init the last BN of each residual branch
            if isinstance(m, TBasicBlock):
                nn.init.zeros_(m.conv2.bn.weight)
            elif isinstance(m, TBottleneck):
                nn.init.zeros_(m.conv3.bn.weight)

    def _make(self, block, planes, n, stride, use_se):
        layers = [block(self.inplanes, planes, stride, use_se)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes, 1, use_se) for _ in range(1, n)]
        return nn.Sequential(*layers)

    def forward_features(self, x):
        """x: NHWC [N,H,W,3] (H, W divisible by 32), or already the SpaceToDepth(4) input
        [N,H/4,W/4,48] (``input_layout``: the input kernel writes it straight from the images)."""
        if x.shape[-1] != 48:
            x = Fn.space_to_depth(x, 4)
        x = self.stem(x)
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        return Fn.global_avg_pool(x)

    def forward(self, x):
        f = self.forward_features(x)
        return self.fc(f) if self.fc is not None else f


def tresnet_m(num_classes=1000, **kw):
    return TResNet((3, 4, 11, 3), num_classes=num_classes, **kw)
