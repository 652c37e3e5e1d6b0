"""VGG19-bn and its NESTED feature net (NESTED/model/vgg.py:10-75; dead code in
the reference, provided for capability parity).

Convolutions/BN/ReLU/max-pool run on the gfx950 kernels (NHWC); an adaptive
7x7 average pool (torchvision's ``AdaptiveAvgPool2d((7, 7))``, identity at 224 px)
precedes the classifier, which flattens in NHWC (H, W, C) order, so torchvision
classifier weights would need a column permutation.  Dropout is the Philox HIP
kernel (``Fn.dropout``).  ``VGGNetFeat`` is the reference's split classifier:
features -> avgpool -> fc1 -> ReLU -> [x * mask1] -> [dropout1] -> fc2 -> ReLU ->
[dropout2], feature dim 4096; its dropouts exist only when ``vgg_dropout > 0``
(the reference skips torchvision's p = 0.5 dropouts otherwise, NESTED/model/vgg.py:20-30).
"""
from __future__ import annotations

import torch.nn as nn

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
        x = Fn.adaptive_avg_pool2d(x, 7, 7)
        return x.reshape(x.shape[0], -1)

    def _drop(self, h, p=None):
        p = self.dropout if p is None else p
        return Fn.dropout(h, p, self.training) if p > 0 else h

    def forward_features(self, x, mask1=None, dropout=None):
        """``mask1``: multiplied into the fc1 activations (NESTED's mask point); ``dropout``:
        overrides the classifier dropout probability (the reference NetFeat's ``vgg_dropout``)."""
        h = self.fc1(self.forward_conv(x), relu=True)
        if mask1 is not None:
            h = h * mask1.to(h.dtype)
        h = self._drop(h, dropout)
        return self._drop(self.fc2(h, relu=True), dropout)

    def forward(self, x):
        f = self.forward_features(x)
        return self.fc3(f) if self.fc3 is not None else f


def vgg19_bn(num_classes=1000, **kw):
    return VGG(CFG19, num_classes=num_classes, **kw)


class VGGNetFeat(nn.Module):
    """NESTED/model/vgg.py NetFeat: features + first classifier layers (dim 4096), ``forward(x,
    mask1=None)``, dropout only when ``vgg_dropout > 0``, ``train(mode, freeze_bn)``."""

    def __init__(self, pretrained=None, vgg_dropout=0.0):
        super().__init__()
        self.net = vgg19_bn(num_classes=0)
        self.vgg_dropout = float(vgg_dropout)
        self.feat_dim = 4096
        self.freeze_bn = False
        if pretrained:
            from .pretrained import load_pretrained

            load_pretrained(self.net, pretrained)

    def train(self, mode=True, freeze_bn=False):
        from .layers import BatchNorm2d

        super().train(mode)
        self.freeze_bn = freeze_bn
        if freeze_bn:
            for m in self.modules():
                if isinstance(m, BatchNorm2d):
                    m.eval()
                    m.weight.requires_grad_(False)
                    m.bias.requires_grad_(False)
        return self

    def forward(self, x, mask1=None):
        return self.net.forward_features(x, mask1=mask1, dropout=self.vgg_dropout)
