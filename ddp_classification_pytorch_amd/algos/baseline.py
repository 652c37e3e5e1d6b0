"""BASELINE workload: DDP + SyncBN image classification (BASELINE/main.py).

Backbone (TResNet-M default, or a ResNet with the 2048->512->ReLU->C MLP head
of BASELINE/main.py:137-142), CE loss, SGD(lr 1e-3, momentum 0.9),
StepLR(10, 0.1) per epoch, per-epoch validation (top-1/top-3) and checkpoint.
"""
from __future__ import annotations

import torch

from ..engine.loop import ClassificationLoop
from ..engine.runtime import build_data, setup
from ..models import build_model
from ..models.heads import ClassifierModel, MLPHead
from ..ops import functional as Fn
from ..optim import StepLR, build_optimizer
from ..parallel.ddp import attach_optimizer, wrap_ddp


def build_classifier(args, log_softmax=False):
    """TResNet / VGG carry their own classifier (timm / torchvision heads); the ResNets get the
    reference's MLP head.  ``--pretrained FILE`` loads a local torchvision / timm / reference file
    into the backbone (BASELINE/main.py:135,143-144) and raises if it does not fit the model."""
    from ..models.pretrained import load_pretrained

    if args.model.startswith("tresnet") or args.model.startswith("vgg"):
        model = build_model(args.model, num_classes=args.num_classes)
        if args.pretrained:
            load_pretrained(model, args.pretrained)  # the classifier is skipped when the class count differs
        return model
    backbone = build_model(args.model, num_classes=0)
    if args.pretrained:
        load_pretrained(backbone, args.pretrained)
    head = MLPHead(backbone.feat_dim, args.hidden, args.num_classes, log_softmax=log_softmax)
    return ClassifierModel(backbone, head)


def run(args):
    rt = setup(args)
    train_data, val_data, _, _ = build_data(args, rt)
    model = build_classifier(args).to(rt.device)
    net = wrap_ddp(model, rt.local_rank, syncbn=args.syncbn and (rt.world > 1 or args.force_ddp), bucket_cap_mb=args.bucket_cap_mb,
                   first_bucket_mb=args.first_bucket_mb, force=args.force_ddp)
    opt = build_optimizer(args.optimizer, model.parameters(), args.lr, args.momentum, args.weight_decay,
                          args.nesterov)
    attach_optimizer(net, opt)  # multi-GPU: the step runs per gradient bucket behind its all-reduce
    sched = StepLR(opt, step_size=args.step_size, gamma=args.gamma)
    C = args.num_classes

    def fwd_train(batch):
        x, y = batch[0], batch[1]
        return Fn.cross_entropy(net(x), y, C, smoothing=args.label_smoothing, return_rank=True)

    def fwd_eval(batch):
        x, y = batch[0], batch[1]
        return Fn.cross_entropy_rows(net(x), y, C)

    loop = ClassificationLoop(args, rt, {"model": model}, opt, sched, train_data, val_data, fwd_train, fwd_eval,
                              train_modules=[net])
    return loop.run()
