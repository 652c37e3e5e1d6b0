"""VGG19-bn and its NESTED feature net (NESTED/model/vgg.py:10-75; dead code in
the reference, provided for capability parity).

Convolutions/BN/ReLU/max-pool run on the gfx950 kernels (NHWC); the
classifier flattens in NHWC (H, W, C) order, so torchvision classifier
weights would need a column permutation.  ``VGGNetFeat`` exposes the split
classifier of the reference: features -> fc1 -> ReLU -> [mask / dropout
point] -> fc2 -> ReLU, feature dim 4096.
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

from ..ops import functional as Fn
from .layers import ConvBN, Linear

CFG19 = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]


class VGG(nn.Module):
    def __init__(self, cfg=CFG19, num_classes=1000, in_chans=3, dropout=0.5):
        super().__init__()
        layers, c = [], in_chans
        for v in cfg:
            if v == "M":
                layers.append("M")
            else:
                layers.append(ConvBN(c, v, 3, 1, 1, act="relu"))
                c = v
        self.convs = nn.ModuleList([m for m in layers if m != "M"])
        self.plan = layers
        self.fc1 = Linear(512 * 7 * 7, 4096)
        self.fc2 = Linear(4096, 4096)
        self.fc3 = Linear(4096, num_classes) if num_classes > 0 else None
        self.dropout = dropout
        self.feat_dim = 4096

    def forward_conv(self, x):
        k = 0
        for m in self.plan:
            if m == "M":
                x = Fn.max_pool2d(x, 2, 2, 0)
            else:
                x = self.convs[k](x)
                k += 1
        if x.shape[1] != 7 or x.shape[2] != 7:
            raise ValueError("VGG classifier expects a 7x7 feature map (224px input)")
        return x.reshape(x.shape[0], -1)

    def _drop(self, h):
        return F.dropout(h, self.dropout, self.training) if self.dropout > 0 else h

    def forward_features(self, x):
        h = self._drop(self.fc1(self.forward_conv(x), relu=True))
        return self._drop(self.fc2(h, relu=True))

    def forward(self, x):
        f = self.forward_features(x)
        return self.fc3(f) if self.fc3 is not None else f


def vgg19_bn(num_classes=1000, **kw):
    return VGG(CFG19, num_classes=num_classes, **kw)


class VGGNetFeat(nn.Module):
    """NESTED/model/vgg.py NetFeat: features + first classifier layers (dim 4096)."""

    def __init__(self, pretrained=None):
        super().__init__()
        self.net = vgg19_bn(num_classes=0)
        self.feat_dim = 4096

    def forward(self, x):
        return self.net.forward_features(x)
