"""Classifier heads of the reference workloads.

* :class:`MLPHead` — 2048 -> 512 -> ReLU -> C (+ optional LogSoftmax); the
  torchvision-ResNet ``fc`` replacement of BASELINE/main.py:137-142 and
  CDR/main.py:332-337 (which appends LogSoftmax), and the ARCFACE embedding
  head 2048 -> 512 -> ReLU -> 256 -> LogSoftmax (ARCFACE/arc_main.py:226-231).
* :class:`ArcMarginProduct` — additive angular margin head
  (ARCFACE/arc_main.py:130-176), computed by the fused HIP ArcFace path.
* :class:`NetClassifier` — bias-free ``feature @ W`` with W stored
  [feat_dim, nb_cls] (NESTED/model/model.py:64-76).
* :class:`ClassifierModel` — backbone (num_classes=0) + head, one module so a
  single DDP wrapper covers both (the reference wraps backbone and ARC head
  in two DDP instances, ARCFACE/arc_main.py:238-243).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..ops import functional as Fn
from .layers import Linear


class MLPHead(nn.Module):
    def __init__(self, in_features=2048, hidden=512, out_features=1000, log_softmax=False):
        super().__init__()
        self.fc1 = Linear(in_features, hidden)
        self.fc2 = Linear(hidden, out_features)
        self.log_softmax = log_softmax
        self.out_features = out_features

    def forward(self, f):
        h = self.fc1(f, relu=True)
        y = self.fc2(h)
        if self.log_softmax:
            y = Fn.log_softmax(y, self.out_features)
        return y


class ArcMarginProduct(nn.Module):
    """cos(theta + m) margin on the target class, scaled by s; weight [out, in] (xavier init)."""

    def __init__(self, in_features=256, out_features=2173, s=30.0, m=0.50, easy_margin=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.s, self.m, self.easy_margin = s, m, easy_margin
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        nn.init.xavier_uniform_(self.weight)
        self.cos_m, self.sin_m = math.cos(m), math.sin(m)
        self.th, self.mm = math.cos(math.pi - m), math.sin(math.pi - m) * m

    def forward(self, x, label, return_logits=False):
        """-> (mean CE loss over margin logits, label rank, margin logits or empty)."""
        return Fn.arcface_loss(x, self.weight, label, self.s, self.m, self.easy_margin, return_logits)

    @torch.no_grad()
    def margin_logits(self, x, label):
        """The reference's output tensor (ARCFACE/arc_main.py:157-176) in plain torch math."""
        cos = torch.nn.functional.linear(torch.nn.functional.normalize(x.float()),
                                         torch.nn.functional.normalize(self.weight.float()))
        sine = torch.sqrt((1.0 - cos.pow(2)).clamp(0, 1))
        phi = cos * self.cos_m - sine * self.sin_m
        phi = torch.where(cos > 0, phi, cos) if self.easy_margin else torch.where(cos > self.th, phi, cos - self.mm)
        one_hot = torch.zeros_like(cos).scatter_(1, label.view(-1, 1).long(), 1)
        return (one_hot * phi + (1.0 - one_hot) * cos) * self.s


class NewFC(nn.Module):
    """ARCFACE/arc_main.py:106-113 ``NewFC``: a plain Linear returning the features (unused in the
    reference's training path; provided for API parity) -- on the MFMA GEMM."""

    def __init__(self, in_features, out_features):
        super().__init__()
        self.fc = Linear(in_features, out_features)

    def forward(self, features):
        return self.fc(features)


class ArcFaceNet(nn.Module):
    """ARCFACE/arc_main.py:115-129 ``ArcFaceNet`` (dead code in the reference, kept for API parity):
    log(exp(s cos(theta_y + m)) / (sum_j exp(s cos theta_j) - exp(s cos theta_y) + exp(s cos(theta_y + m))))
    for EVERY column y (the reference's un-labelled formulation), with theta = acos(cos / 10) -- the
    reference divides the cosine by 10 before acos ("prevents underflow"); kept as written.  The
    cosine GEMM runs on the MFMA kernel; the transcendental tail is plain torch (no training path
    uses this head)."""

    def __init__(self, cls_num=10, feature_dim=2):
        super().__init__()
        self.w = nn.Parameter(torch.randn(feature_dim, cls_num))

    def forward(self, features, m=1.0, s=10.0):
        f = torch.nn.functional.normalize(features.float(), dim=1)
        w = torch.nn.functional.normalize(self.w.float(), dim=0)
        cos = Fn.linear(f.to(features.dtype), w.t().contiguous()).float()
        theta = torch.acos(cos / 10)
        num = torch.exp(s * torch.cos(theta + m))
        e = torch.exp(s * torch.cos(theta))
        den = e.sum(dim=1, keepdim=True) - e + num
        return torch.log(num / den)


class NetClassifier(nn.Module):
    def __init__(self, feat_dim, nb_cls):
        super().__init__()
        w = torch.empty(nb_cls, feat_dim)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))  # nn.Linear init, stored transposed like the reference
        self.weight = nn.Parameter(w.t().contiguous())

    def forward(self, feature):
        return Fn.linear(feature, self.weight.t())


class ClassifierModel(nn.Module):
    """backbone.forward_features -> head.  ``head`` may be any module mapping [B, F] -> logits/features."""

    def __init__(self, backbone, head):
        super().__init__()
        self.backbone, self.head = backbone, head

    def forward(self, x):
        return self.head(self.backbone.forward_features(x))
