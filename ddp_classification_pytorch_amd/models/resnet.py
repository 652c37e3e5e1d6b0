"""ResNet / ResNeXt family in NHWC on the gfx950 conv+BN kernels.

Capabilities of the reference's model zoo:
* ImageNet ResNet-18/34/50/101/152 (NESTED/model/imagenet_resnet.py:102-224 and
  torchvision resnet50 used by BASELINE/main.py:135, ARCFACE/arc_main.py:224,
  CDR/main.py:330): 7x7/2 stem + 3x3/2 max-pool, stride on the 3x3 of the
  bottleneck ("v1.5"), global average pool (any input size >= 32, not the
  fixed AvgPool2d(7) of the local copy), Kaiming fan-out init.
* ResNeXt-50 32x4d (BASELINE.json config 4) via grouped 3x3 convolutions.
* CIFAR ResNets (NESTED/model/cifar_resnet.py:77-160): 3x3/1 stem, no pool.

Module names follow torchvision (conv1, bn1, layer1..4, downsample.0/1, fc)
so torchvision-format checkpoints load through :meth:`Conv2d._load_from_state_dict`.
Input: NHWC activations with the 3 image channels zero-padded to 8
(see :func:`ddp_classification_pytorch_amd.ops.functional.to_device_nhwc`).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops import functional as Fn
from .layers import BatchNorm2d, Conv2d, Linear, bn_relu_conv, conv_bn


# the one-op stem (conv + BN + ReLU + max pool, fused one-pass backward, stem.hip stem_bwd).
# On by default: it removes the full-resolution dz tensor, both BN-backward passes and the stem
# weight-gradient GEMM -- 1.39 ms against 2.25 ms for the unfused maxpool_bn_bwd x 2 + weight-
# gradient chain at R50 b1024 (profiles/stem_bwd_fused_ab.txt).  DCP_FUSED_STEM=0 switches it off.
_FUSED_STEM = [os.environ.get("DCP_FUSED_STEM", "1") == "1"]


def _train_stats(bn: BatchNorm2d) -> bool:
    return bn.training and not bn.frozen


def _folded(*bns) -> bool:
    """Every BN of the block normalises with running statistics and needs no affine gradient:
    run the block as conv launches with the BNs folded into their epilogues (layers.conv_bn)."""
    return all(b is not None and Fn.bn_foldable(b) for b in bns)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 3, stride, 1)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, 3, 1, 1)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x):
        if _folded(self.bn1, self.bn2, self.downsample[1] if self.downsample is not None else self.bn2):
            y = conv_bn(self.conv1, self.bn1, x)
            r = x if self.downsample is None else conv_bn(self.downsample[0], self.downsample[1], x, act="none")
            return conv_bn(self.conv2, self.bn2, y, residual=r)
        t = _train_stats(self.bn1)
        # the block input's second consumer (residual add / downsample conv) hands its
        # gradient to conv1, which sums it in its dgrad epilogue (strided conv1: no join)
        join = Fn.GradJoin(1) if self.conv1.stride == 1 else None
        y, s = self.conv1(x, stats=t, link=join)
        y = self.bn1(y, s, act="relu")
        y, s = self.conv2(y, stats=t)
        if self.downsample is not None:
            r, rs = self.downsample[0](x, stats=t, deposit=join)
            return self.bn2(y, s, act="relu", residual=r, residual_bn=(self.downsample[1], rs))
        return self.bn2(y, s, act="relu", residual=x, link=join)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = Conv2d(inplanes, width, 1, 1, 0)
        self.bn1 = BatchNorm2d(width)
        self.conv2 = Conv2d(width, width, 3, stride, 1, groups=groups)
        self.bn2 = BatchNorm2d(width)
        self.conv3 = Conv2d(width, planes * self.expansion, 1, 1, 0)
        self.bn3 = BatchNorm2d(planes * self.expansion)
        self.downsample = downsample

    def forward(self, x):
        if _folded(self.bn1, self.bn2, self.bn3, self.downsample[1] if self.downsample is not None else self.bn3):
            y = conv_bn(self.conv1, self.bn1, x)
            y = conv_bn(self.conv2, self.bn2, y)
            r = x if self.downsample is None else conv_bn(self.downsample[0], self.downsample[1], x, act="none")
            return conv_bn(self.conv3, self.bn3, y, residual=r)
        t = _train_stats(self.bn1)
        # the block input's second consumer (the residual add of an identity block, the
        # downsample conv of a projection block) hands its gradient to conv1, which sums it
        # in its dgrad epilogue -- fused there with the backward of the BN that produced x.
        # The downsample branch runs after conv3 so its backward precedes conv1's.
        join = Fn.GradJoin(1)
        y, s = self.conv1(x, stats=t, link=join)
        # bn1 + ReLU inside conv2's staged windows where the direct 64-channel 3x3 kernels run
        # (layers.bn_relu_conv); a grouped conv2 (ResNeXt) fuses bn1's backward reduction into its dgrad
        y, s = bn_relu_conv(self.bn1, self.conv2, y, s, stats=t, fuse_bwd=self.conv2.groups > 1)
        # bn2 + ReLU run inside conv3's GEMMs (layers.bn_relu_conv): no activation pass
        y, s = bn_relu_conv(self.bn2, self.conv3, y, s, stats=t)
        if self.downsample is not None:
            r, rs = self.downsample[0](x, stats=t, deposit=join)
            return self.bn3(y, s, act="relu", residual=r, residual_bn=(self.downsample[1], rs))
        return self.bn3(y, s, act="relu", residual=x, link=join)


class ResNet(nn.Module):
    """num_classes=0 -> feature extractor returning pooled features [N, C]."""

    def __init__(self, block, layers, num_classes=1000, variant="imagenet", groups=1, width_per_group=64,
                 zero_init_residual=False, in_chans=3, stem_s2d=True):
        super().__init__()
        self.variant = variant
        self.groups, self.base_width = groups, width_per_group
        self.inplanes = 64
        self.in_chans = in_chans
        # 7x7/2 stem computed as a 4x4/1 conv over the 2x2 space-to-depth input
        # (ops.functional.stem_conv_s2d); the parameter keeps the torchvision 7x7 layout
        self.stem_s2d = bool(stem_s2d) and variant == "imagenet" and in_chans <= 4
        if variant == "imagenet":
            self.conv1 = Conv2d(in_chans, 64, 7, 2, 3)
            if self.stem_s2d:
                self.register_buffer("_stem_w16", torch.zeros(64, 4, 4, 16), persistent=False)
        elif variant == "cifar":
            self.conv1 = Conv2d(in_chans, 64, 3, 1, 1)
        else:
            raise ValueError(variant)
        self.bn1 = BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.feat_dim = 512 * block.expansion
        self.num_classes = num_classes
        self.fc = Linear(self.feat_dim, num_classes) if num_classes > 0 else None
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(Conv2d(self.inplanes, planes * block.expansion, 1, stride, 0),
                                       BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, 1, None, self.groups, self.base_width))
        return nn.Sequential(*layers)

    def forward_features(self, x):
        """x: NHWC [N,H,W,8] (or the s2d stem's [N,H/2,W/2,16]) -> pooled features [N, feat_dim]."""
        t = _train_stats(self.bn1)
        fold = _folded(self.bn1)
        if self.stem_s2d and (x.shape[-1] == 16 or (x.shape[1] % 2 == 0 and x.shape[2] % 2 == 0)):
            if x.shape[-1] != 16:
                x = Fn.nhwc_to_s2d(x)
            if fold:  # eval-mode / frozen stem BN: conv, then BN + ReLU + max pool in one pass
                y, _ = Fn.stem_conv_s2d(x, self.conv1.weight, self._stem_w16, stats=False)
                return self._forward_stages(Fn.bn_eval_act_maxpool(y, self.bn1, act="relu"))
            if (t and self.variant == "imagenet" and _FUSED_STEM[0] and self.bn1.weight is not None
                    and Fn.stem_bn_pool_fusable(x)):
                # conv + BN + ReLU + max pool as one op with the one-pass fused backward
                self.bn1._nbt_pending += 1
                y = Fn.stem_bn_pool(x, self.conv1.weight, self._stem_w16, self.bn1.weight, self.bn1.bias,
                                    self.bn1.running_mean, self.bn1.running_var, self.bn1.momentum, self.bn1.eps,
                                    act="relu", group=self.bn1.process_group)
                return self._forward_stages(y)
            y, s = Fn.stem_conv_s2d(x, self.conv1.weight, self._stem_w16, stats=t)
            s = s if (t and x.is_cuda) else None
        elif fold and self.variant == "cifar":
            return self._forward_stages(conv_bn(self.conv1, self.bn1, x))
        else:
            y, s = self.conv1(x, stats=t)
        if self.variant == "imagenet":
            y = self.bn1.forward_pool(y, s, act="relu", k=3, s=2, p=1)  # BN + ReLU + max pool, one fused op
        else:
            y = self.bn1(y, s, act="relu")
        return self._forward_stages(y)

    def _forward_stages(self, y):
        y = self.layer1(y)
        y = self.layer2(y)
        y = self.layer3(y)
        y = self.layer4(y)
        return Fn.global_avg_pool(y)

    def forward(self, x):
        f = self.forward_features(x)
        return self.fc(f) if self.fc is not None else f


_CFG = {
    "resnet18": (BasicBlock, [2, 2, 2, 2], {}),
    "resnet34": (BasicBlock, [3, 4, 6, 3], {}),
    "resnet50": (Bottleneck, [3, 4, 6, 3], {}),
    "resnet101": (Bottleneck, [3, 4, 23, 3], {}),
    "resnet152": (Bottleneck, [3, 8, 36, 3], {}),
    "resnext50_32x4d": (Bottleneck, [3, 4, 6, 3], {"groups": 32, "width_per_group": 4}),
    "resnext101_32x8d": (Bottleneck, [3, 4, 23, 3], {"groups": 32, "width_per_group": 8}),
}


def build_resnet(name: str, num_classes: int = 1000, variant: str = "imagenet", **kw) -> ResNet:
    if name.startswith("cifar_"):
        name, variant = name[len("cifar_"):], "cifar"
    block, layers, extra = _CFG[name]
    return ResNet(block, layers, num_classes=num_classes, variant=variant, **{**extra, **kw})


def resnet18(num_classes=1000, **kw):
    return build_resnet("resnet18", num_classes, **kw)


def resnet34(num_classes=1000, **kw):
    return build_resnet("resnet34", num_classes, **kw)


def resnet50(num_classes=1000, **kw):
    return build_resnet("resnet50", num_classes, **kw)


def resnet101(num_classes=1000, **kw):
    return build_resnet("resnet101", num_classes, **kw)


def resnet152(num_classes=1000, **kw):
    return build_resnet("resnet152", num_classes, **kw)


def resnext50_32x4d(num_classes=1000, **kw):
    return build_resnet("resnext50_32x4d", num_classes, **kw)


def cifar_resnet18(num_classes=100, **kw):
    return build_resnet("resnet18", num_classes, variant="cifar", **kw)


def cifar_resnet34(num_classes=100, **kw):
    return build_resnet("resnet34", num_classes, variant="cifar", **kw)


def cifar_resnet50(num_classes=100, **kw):
    return build_resnet("resnet50", num_classes, variant="cifar", **kw)


def cifar_resnet101(num_classes=100, **kw):
    return build_resnet("resnet101", num_classes, variant="cifar", **kw)


def cifar_resnet152(num_classes=100, **kw):
    return build_resnet("resnet152", num_classes, variant="cifar", **kw)
