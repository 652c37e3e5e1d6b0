"""NESTED feature network (NESTED/model/model.py:12-61).

``NetFeat`` truncates a ResNet to its pooled features (CIFAR ResNet-18: 512;
ImageNet ResNet-18/50: 512/2048) and overrides ``train(mode, freeze_bn)`` to
run BatchNorm on running statistics with gamma/beta frozen.
"""
from __future__ import annotations

import torch.nn as nn

from .layers import BatchNorm2d
from .resnet import build_resnet


class NetFeat(nn.Module):
    def __init__(self, arch="resnet50", dataset="Clothing1M", pretrained=None):
        super().__init__()
        if "CIFAR" in dataset.upper():
            self.net = build_resnet(arch, num_classes=0, variant="cifar")
        else:
            self.net = build_resnet(arch, num_classes=0, variant="imagenet")
        self.feat_dim = self.net.feat_dim
        self.freeze_bn = False
        if pretrained:
            from .pretrained import load_pretrained

            load_pretrained(self.net, pretrained)

    def train(self, mode=True, freeze_bn=False):
        super().train(mode)
        self.freeze_bn = freeze_bn
        if freeze_bn:
            for m in self.modules():
                if isinstance(m, BatchNorm2d):
                    m.eval()
                    if m.weight is not None:
                        m.weight.requires_grad_(False)
                        m.bias.requires_grad_(False)
        return self

    def forward(self, x):
        return self.net.forward_features(x)
