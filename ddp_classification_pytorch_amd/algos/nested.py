"""NESTED workload: nested dropout over the feature dimension + best-K search
(NESTED/train.py:93-452).

* ``NetFeat`` (frozen BN by default) + bias-free ``NetClassifier``;
* K ~ GaussianDist(mu, nested, feat_dim) per step (host RNG, like the
  reference); the feature is masked to its first K+1 dims by the
  ``prefix_mask`` kernel (the reference multiplies by one of 2048 mask
  tensors it keeps on the GPU), or standard dropout when ``--dropout > 0``;
* two SGD optimizers (feature net, classifier), linear warm-up for
  ``--warmUpIter`` iterations to ``--lr``, then MultiStepLR per optimizer;
* ``TestNested``: per validation batch the top-1/top-3 hit counts for EVERY
  prefix length K come from one ``nested_eval`` kernel (prefix-cumulative
  scores, running label rank) instead of 2048 masked GEMMs and a
  [2048, B, C] tensor; best K = argmax(acc - 1e-5 K); best checkpoint
  ``netBest.pth`` = {'feat', 'cls'};
* ``history.json`` each epoch; the output directory is renamed with the best
  accuracy and K at the end (NESTED/train.py:450-452).
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from ..engine.checkpoint import is_rank0, load_checkpoint
from ..engine.logger import MetricsLogger
from ..engine.loop import _check_transports, valid_count
from ..engine.runtime import build_data, setup
from ..models.heads import NetClassifier
from ..models.nested import NetFeat
from ..ops import functional as Fn
from ..optim import FusedSGD, MultiStepLR
from ..parallel.ddp import attach_optimizer, wrap_ddp
from ..utils.misc import AverageMeter, ProgressBar


def gaussian_dist(mu, std, n):
    """NESTED/train.py:93-97."""
    d = np.array([np.exp(-(((i - mu) / std) ** 2)) for i in range(1, n + 1)])
    return d / np.sum(d)


def _step(net_feat, net_cls, opts, x, y, dist_k, dropout, nb_cls, rng):
    for o in opts:
        o.zero_grad(set_to_none=True)
    feature = net_feat(x)
    if dist_k is not None:
        k = int(rng.choice(len(dist_k), p=dist_k))
        feature = Fn.nested_mask(feature, k)
    elif dropout > 0:
        feature = Fn.dropout(feature, p=dropout, training=True)
    out = net_cls(feature)
    loss, rank = Fn.cross_entropy(out, y, nb_cls, return_rank=True)
    loss.backward()
    for o in opts:
        o.step()
    return loss, rank


@torch.no_grad()
def test_nested(net_feat, net_cls, val_data, feat_dim):
    """Per-K accuracy over the validation set -> (acc[K], acc3[K]) on every rank."""
    net_feat.eval()
    net_cls.eval()
    dev = next(net_cls.parameters()).device
    counts = torch.zeros(feat_dim, 2, dtype=torch.float64, device=dev)
    n = torch.zeros(1, dtype=torch.float64, device=dev)
    left = valid_count(getattr(val_data, "sampler", None), float("inf"))
    for batch in val_data:
        x, y = batch[0], batch[1]
        k = int(min(y.numel(), left))
        left -= k
        if k <= 0:
            continue
        feat = net_feat(x)[:k]
        counts += Fn.nested_eval_counts(feat, net_cls.weight, y[:k]).double()
        n += k
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(counts)
        dist.all_reduce(n)
    acc = (counts[:, 0] / n).cpu()
    acc3 = (counts[:, 1] / n).cpu()
    return acc, acc3


@torch.no_grad()
def test_standard(net_feat, net_cls, val_data, nb_cls):
    net_feat.eval()
    net_cls.eval()
    dev = next(net_cls.parameters()).device
    acc = torch.zeros(4, dtype=torch.float64, device=dev)
    left = valid_count(getattr(val_data, "sampler", None), float("inf"))
    for batch in val_data:
        x, y = batch[0], batch[1]
        k = int(min(y.numel(), left))
        left -= k
        if k <= 0:
            continue
        _, rank = Fn.cross_entropy_rows(net_cls(net_feat(x)), y, nb_cls)
        Fn.metric_accum(acc, rank[:0].float(), 0.0, rank, k)  # [loss 0, top-1, top-3, count]
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(acc)
    a = acc.tolist()[1:]
    return a[0] / max(a[2], 1), a[1] / max(a[2], 1)


def run(args):
    rt = setup(args)
    logger = MetricsLogger(args.out_dir if rt.is_main else None)
    train_data, val_data, _, _ = build_data(args, rt, drop_last_train=True)
    net_feat = NetFeat(args.model, args.dataset, pretrained=args.pretrained).to(rt.device)
    net_cls = NetClassifier(net_feat.feat_dim, args.num_classes).to(rt.device)
    feat_dim, nb_cls = net_feat.feat_dim, args.num_classes
    if args.resume:
        load_checkpoint(args.resume, {"feat": net_feat, "cls": net_cls}, map_location="cpu")
    dist_k = gaussian_dist(args.mu, args.nested, feat_dim) if args.nested > 0 else None
    # torch semantics: a params list that requires no grad is skipped by the fused kernel
    opt_feat = FusedSGD([p for p in net_feat.parameters()], lr=1e-4, momentum=args.momentum,
                        weight_decay=args.weight_decay)
    opt_cls = FusedSGD(net_cls.parameters(), lr=1e-4, momentum=args.momentum, weight_decay=args.weight_decay)
    opts = [opt_feat, opt_cls]
    # DDP over both networks (the reference runs NESTED single-GPU).  Frozen-BN gamma/beta stop
    # requiring grad in train(freeze_bn=True), which must happen before DDP registers the
    # parameters it all-reduces.
    net_feat.train(True, freeze_bn=args.freeze_bn)
    ddp_kw = dict(syncbn=False, bucket_cap_mb=args.bucket_cap_mb, first_bucket_mb=args.first_bucket_mb,
                  force=args.force_ddp)
    feat_net = wrap_ddp(net_feat, rt.local_rank, **ddp_kw)
    cls_net = wrap_ddp(net_cls, rt.local_rank, **ddp_kw)
    attach_optimizer(feat_net, opt_feat)
    attach_optimizer(cls_net, opt_cls)
    rng = np.random.RandomState(args.seed + rt.rank)
    bar = ProgressBar(stream=None) if rt.is_main else None

    def train_mode():
        net_feat.train(True, freeze_bn=args.freeze_bn)
        net_cls.train()

    # ---- linear LR warm-up (NESTED/train.py:276-326)
    n_iter = 0
    while n_iter < args.warmup_iters:
        train_mode()
        for batch in train_data:
            n_iter += 1
            if n_iter >= args.warmup_iters:
                break
            lr = n_iter / float(args.warmup_iters) * args.lr
            for o in opts:
                for g in o.param_groups:
                    g["lr"] = lr
            _step(feat_net, cls_net, opts, batch[0], batch[1], dist_k, args.dropout, nb_cls, rng)
            if args.max_steps_per_epoch and n_iter >= args.max_steps_per_epoch:
                n_iter = args.warmup_iters
                break

    def evaluate(epoch, best):
        if dist_k is not None:
            acc, acc3 = test_nested(net_feat, net_cls, val_data, feat_dim)
            score = acc - 1e-5 * torch.arange(feat_dim, dtype=acc.dtype)
            k = int(torch.argmax(score))
            a1, a3 = float(acc[k]), float(acc3[k])
        else:
            a1, a3 = test_standard(net_feat, net_cls, val_data, nb_cls)
            k = feat_dim - 1
        logger.line(f"Nested ... Epoch {epoch:d}, Acc {a1 * 100:.3f} %, K {k:d} (Best Acc {best['acc'] * 100:.3f} %)")
        if a1 > best["acc"]:
            best.update(acc=a1, k=k)
            if is_rank0():
                torch.save({"feat": net_feat.state_dict(), "cls": net_cls.state_dict()},
                           os.path.join(args.out_dir, "netBest.pth"))
        if dist.is_initialized():
            dist.barrier()
        return a1, a3, k

    best = {"acc": 0.0, "k": 0}
    history = {"trainAcc": [], "trainTop3": [], "valAcc": [], "valTop3": [], "valK": [], "trainLoss": []}
    a1, a3, k = evaluate(0, best)
    for o in opts:
        for g in o.param_groups:
            g["lr"] = args.lr
    scheds = [MultiStepLR(o, milestones=args.milestones, gamma=args.gamma) for o in opts]
    for epoch in range(args.epochs):
        train_mode()
        sampler = getattr(train_data, "sampler", None)
        if sampler is not None:
            sampler.set_epoch(epoch)
        losses, top1, top3 = AverageMeter(), AverageMeter(), AverageMeter()
        n_steps = len(train_data) if not args.max_steps_per_epoch else min(len(train_data), args.max_steps_per_epoch)
        t0 = time.time()
        for i, batch in enumerate(train_data):
            if i >= n_steps:
                break
            loss, rank = _step(feat_net, cls_net, opts, batch[0], batch[1], dist_k, args.dropout, nb_cls, rng)
            if (i + 1) % args.log_interval == 0 or i + 1 == n_steps:
                B = rank.numel()
                losses.update(loss.item(), B)
                top1.update(100.0 * (rank < 1).sum().item() / B, B)
                top3.update(100.0 * (rank < 3).sum().item() / B, B)
                _check_transports()  # a timed-out SyncBN peer exchange ends the run (parallel/peer.py)
                if bar is not None:
                    bar(i, n_steps, f"Loss: {losses.avg:.3f} | Top1: {top1.avg:.3f}% | Top3: {top3.avg:.3f}%")
        a1, a3, k = evaluate(epoch + 1, best)
        history["trainAcc"].append(top1.avg)
        history["trainTop3"].append(top3.avg)
        history["trainLoss"].append(losses.avg)
        history["valAcc"].append(a1)
        history["valTop3"].append(a3)
        history["valK"].append(k)
        logger.log("epoch", epoch=epoch, train_loss=losses.avg, train_top1=top1.avg, val_top1=a1, val_top3=a3,
                   k=k, time=time.time() - t0)
        if is_rank0():
            with open(os.path.join(args.out_dir, "history.json"), "w") as f:
                json.dump(history, f)
        for s in scheds:
            s.step()
    msg = f"Best Performance: {best['acc'] * 100:.3f} at K={best['k']}"
    logger.line(msg)
    if is_rank0() and getattr(args, "rename_out_dir", True):
        final = f"{args.out_dir.rstrip('/')}_Acc{best['acc'] * 100:.3f}_K{best['k']}"
        if not os.path.exists(final):
            os.replace(args.out_dir, final)
    return best
