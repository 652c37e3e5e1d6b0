"""ARCFACE workload (ARCFACE/arc_main.py).

ResNet-50 backbone -> 2048->512->ReLU->256->LogSoftmax "embedding"
(ARCFACE/arc_main.py:223-231, kept for parity: the margin head then
L2-normalises those log-probabilities) -> ArcMarginProduct(256 -> C, s=30,
m=0.5, easy margin) -> CE, trained jointly under DDP with Adam (default) or
SGD(momentum 0.9, wd 5e-4).  The reference wraps backbone and ARC head in two
DDP instances (two reducers); here backbone+head+margin are one module under
one DDP wrapper (one bucketed all-reduce stream, same math).

Eval: the reference applies the margin with the TRUE labels at validation
(ARCFACE/arc_main.py:368); that is the default (``--arc-eval-with-labels``),
``--arc-eval-plain-cosine`` ranks plain cosines instead.
"""
from __future__ import annotations

import torch.nn as nn

from ..engine.loop import ClassificationLoop
from ..engine.runtime import build_data, setup
from ..models import build_model
from ..models.heads import ArcMarginProduct, MLPHead
from ..ops import functional as Fn
from ..optim import StepLR, build_optimizer
from ..parallel.ddp import attach_optimizer, wrap_ddp


class ArcFaceModel(nn.Module):
    def __init__(self, backbone, embed_head, arc):
        super().__init__()
        self.backbone, self.embed, self.arc = backbone, embed_head, arc

    def features(self, x):
        return self.embed(self.backbone.forward_features(x))

    def forward(self, x, labels):
        loss, rank, _ = self.arc(self.features(x), labels)
        return loss, rank


def build_arcface(args):
    backbone = build_model(args.model, num_classes=0)
    if args.pretrained:
        from ..models.pretrained import load_pretrained

        load_pretrained(backbone, args.pretrained)
    embed = MLPHead(backbone.feat_dim, args.hidden, args.embed_dim, log_softmax=True)
    arc = ArcMarginProduct(args.embed_dim, args.num_classes, s=args.arc_s, m=args.arc_m, easy_margin=args.easy_margin)
    return ArcFaceModel(backbone, embed, arc)


def run(args):
    rt = setup(args)
    train_data, val_data, _, _ = build_data(args, rt)
    model = build_arcface(args).to(rt.device)
    net = wrap_ddp(model, rt.local_rank, syncbn=args.syncbn and (rt.world > 1 or args.force_ddp), bucket_cap_mb=args.bucket_cap_mb,
                   first_bucket_mb=args.first_bucket_mb, force=args.force_ddp)
    name = args.optimizer.lower()
    wd = args.weight_decay if name == "sgd" else 0.0  # ARCFACE/arc_main.py:249-253
    opt = build_optimizer(name, model.parameters(), args.lr, args.momentum, wd)
    attach_optimizer(net, opt)
    sched = StepLR(opt, step_size=args.step_size, gamma=args.gamma)

    def fwd_train(batch):
        return net(batch[0], batch[1])

    def fwd_eval(batch):
        x, y = batch[0], batch[1]
        f = model.features(x)
        return Fn.arcface_rows(f, model.arc.weight, y, model.arc.s, model.arc.m, model.arc.easy_margin,
                               with_margin=args.arc_eval_with_labels)

    loop = ClassificationLoop(args, rt, {"model": model}, opt, sched, train_data, val_data, fwd_train, fwd_eval,
                              train_modules=[net])
    return loop.run()
