"""PLC — progressive label correction for feature-dependent label noise
(PLC/utils.py:149-360, PLC/FolderDataset.py).

Vectorised re-implementations of the reference's per-sample Python loops:

* :func:`label_noise` — synthetic feature-dependent noise of type I/II/III
  from a posterior ``eta`` (top-2 classes u, s): with probability
  ``noise_level/factor`` the label becomes u, otherwise s (multi-class), or
  the binary flip model for 2 classes (PLC/utils.py:149-220).
* :func:`eta_approximation` — train ``f`` with SGD(nesterov, wd 5e-4) and
  collect softmax posteriors for every training index at the last epoch
  (PLC/utils.py:223-288).
* :func:`lrt_correction` — likelihood-ratio test: relabel to the argmax when
  f[y]/max f < delta; raise delta by ``delta_increment`` (cap 0.9) when fewer
  than 0.1 % of labels changed (PLC/utils.py:291-318).
* :func:`prob_correction` — probabilistic variant (PLC/utils.py:321-360).
* :func:`run` — end-to-end PLC training on our kernels: warm-up epochs on the
  noisy labels, then per epoch: posterior pass over the training set (by
  dataset index), label correction, ``update_corrupted_label``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ..engine.logger import MetricsLogger
from ..engine.loop import ClassificationLoop
from ..engine.runtime import build_data, setup
from ..ops import functional as Fn
from ..optim import FusedSGD
from ..parallel.ddp import attach_optimizer, wrap_ddp


def label_noise(targets, eta, noise_type=0, factor=1.2, rng=None):
    """-> (noisy labels int64 [n], f_us [n]).  ``eta``: [n, C] posteriors."""
    rng = rng if rng is not None else np.random
    y = np.array(targets, dtype=np.int64).copy()
    eta = torch.as_tensor(eta, dtype=torch.float64)
    classes = len(np.unique(y))
    if classes == 2:
        eu = eta[:, 1].numpy()
        if noise_type == 0:
            f = 2 * eu * (eu - 0.5) ** 2
        elif noise_type == 1:
            f = (eu >= 0.5) * (1 - eu) + (eu < 0.5) * eu
        else:
            f = -2 * (eu - 0.5) ** 2 + 0.5
        keep = rng.binomial(1, np.clip(1 - f, 0, 1))
        y = np.where(y == 1, keep, y)
        return y, f
    top = eta.topk(2, dim=1)
    eu, es = top.values[:, 0].numpy(), top.values[:, 1].numpy()
    u, s = top.indices[:, 0].numpy(), top.indices[:, 1].numpy()
    d = np.abs(eu - es)
    if noise_type == 0:
        f = -0.5 * (eu - es) ** 2 + 0.5
        level = np.maximum(1 - f, 0.5)
    elif noise_type == 1:
        f = 1 - d ** 3
        level = 1 - f
    else:
        f = 1 - d ** 3 / 3 - d ** 2 / 3 - d / 3
        level = 1 - f
    ind = rng.binomial(1, np.clip(level / factor, 0, 1))
    y = ind * u + (1 - ind) * s
    return y.astype(np.int64), f


def lrt_correction(y_tilde, f_x, current_delta=0.3, delta_increment=0.1):
    y = torch.as_tensor(np.array(y_tilde), dtype=torch.int64).clone()
    f = torch.as_tensor(f_x, dtype=torch.float64)
    fm, y_mle = f.max(1)
    lr = f.gather(1, y.view(-1, 1)).squeeze(1) / fm
    change = lr < current_delta
    y[change] = y_mle[change]
    if int(change.sum()) < 0.001 * len(y):
        current_delta = min(current_delta + delta_increment, 0.9)
    return y, current_delta


def prob_correction(y_noise, f_x, random_state=0, current_delta=0.3, delta_increment=0.1, thd=0.1):
    flipper = np.random.RandomState(random_state)
    y = np.array(y_noise, dtype=np.int64).copy()
    p = torch.softmax(torch.as_tensor(f_x, dtype=torch.float64), 1).numpy()
    top = p.argmax(1)
    ptop = p[np.arange(len(y)), top]
    confident = ptop >= thd
    ratio = p[np.arange(len(y)), y] / ptop
    change = confident & (ratio < current_delta)
    y[change] = top[change]
    # not confident: multinomial over the normalised top-1 distribution == top-1 (reference keeps k=1)
    unconf = ~confident
    if unconf.any():
        flipper.multinomial(1, [1.0], int(unconf.sum()))
        y[unconf] = top[unconf]
    if not change.any():
        current_delta += delta_increment
    return y, current_delta


def eta_approximation(model, loader, n, num_classes, device, epochs=1, lr=0.01, log=print, net=None):
    """Train ``model`` (forward through ``net``, its DDP wrapper, when given) and return
    softmax posteriors [n, C] for every dataset index (batches must yield (x, y, index));
    under DDP every rank fills the rows of its own shard and the table is all-reduced."""
    net = net if net is not None else model
    opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, nesterov=True, weight_decay=5e-4)
    eta = torch.zeros(n, num_classes)
    for ep in range(epochs):
        model.train()
        correct = total = 0
        for x, y, idx in loader:
            if y.numel() == 1:
                continue
            logits = net(x)
            loss, rank = Fn.cross_entropy(logits, y, num_classes, return_rank=True)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            correct += int((rank == 0).sum())
            total += y.numel()
            if ep == epochs - 1:
                eta[idx.cpu()] = torch.softmax(logits.detach().float(), 1).cpu()
        log(f"Epoch [{ep + 1}|{epochs}] \t Train Acc {100.0 * correct / max(total, 1):.3f}")
    if dist.is_initialized() and dist.get_world_size() > 1:
        # disjoint shards (plus identical DistributedSampler padding rows): sum and renormalise
        dev = next(model.parameters()).device
        e, c = eta.to(dev), (eta.sum(1) > 0).to(dev, torch.float32)
        dist.all_reduce(e)
        dist.all_reduce(c)
        eta = (e / c.clamp_min(1).unsqueeze(1)).cpu()
    return eta


@torch.no_grad()
def posteriors(model, loader, n, num_classes):
    model.eval()
    dev = next(model.parameters()).device
    out = torch.zeros(n, num_classes, device=dev)
    cnt = torch.zeros(n, device=dev)
    for x, y, idx in loader:
        out[idx] = torch.softmax(model(x).float(), 1)
        cnt[idx] = 1.0
    if dist.is_initialized() and dist.get_world_size() > 1:
        # ranks own disjoint indices except DistributedSampler padding (identical rows): sum and renormalise
        dist.all_reduce(out)
        dist.all_reduce(cnt)
        out = out / cnt.clamp_min(1).unsqueeze(1)
    return out.cpu()


def run(args):
    """Labels live in a device table indexed by dataset index, so corrections are
    visible immediately (persistent loader workers hold stale dataset copies)."""
    from .baseline import build_classifier

    rt = setup(args)
    logger = MetricsLogger(args.out_dir if rt.is_main else None)
    train_data, val_data, train_set, _ = build_data(args, rt)
    model = build_classifier(args).to(rt.device)
    net = wrap_ddp(model, rt.local_rank, syncbn=args.syncbn and (rt.world > 1 or args.force_ddp), bucket_cap_mb=args.bucket_cap_mb,
                   first_bucket_mb=args.first_bucket_mb, force=args.force_ddp)
    opt = FusedSGD(model.parameters(), lr=args.lr, momentum=args.momentum, nesterov=True,
                   weight_decay=args.weight_decay)
    C = args.num_classes
    n = len(train_set)
    base = getattr(train_set, "targets", None)
    if base is None:
        base = getattr(train_set, "labels")
    labels = torch.tensor([int(v) for v in base], dtype=torch.int64, device=rt.device)
    if args.plc_eta_epochs > 0:
        # synthetic feature-dependent noise from a posterior estimate (PLC/utils.py:149-288)
        eta = eta_approximation(model, train_data, n, C, rt.device, epochs=args.plc_eta_epochs, lr=args.lr,
                                log=logger.line, net=net)
        noisy, _ = label_noise(labels.cpu().numpy(), eta, args.plc_noise_type, rng=np.random.RandomState(args.seed))
        noisy = torch.as_tensor(noisy, device=rt.device)
        changed = int((noisy != labels).sum())
        logger.line(f"Corrupted Size {changed} | Noisy Level {100.0 * changed / max(n, 1):.3f}%")
        labels = noisy
    delta = args.plc_delta
    attach_optimizer(net, opt)  # after the posterior-estimation phase, which steps its own optimizer

    def fwd_train(batch):
        x, idx = batch[0], batch[2]
        return Fn.cross_entropy(net(x), labels[idx], C, return_rank=True)

    def fwd_eval(batch):
        return Fn.cross_entropy_rows(model(batch[0]), batch[1], C)

    loop = ClassificationLoop(args, rt, {"model": model}, opt, None, train_data, val_data, fwd_train, fwd_eval,
                              logger=logger, train_modules=[net])
    for epoch in range(args.epochs):
        tr = loop.train_epoch(epoch)
        f_x = posteriors(model, train_data, n, C)
        cur = labels.cpu().numpy()
        if args.plc_correction == "lrt":
            new, delta = lrt_correction(cur, f_x, delta, args.plc_delta_inc)
        else:
            new, delta = prob_correction(cur, f_x, args.seed, delta, args.plc_delta_inc)
        new = torch.as_tensor(np.asarray(new), dtype=torch.int64, device=rt.device)
        changed = int((new != labels).sum())
        labels = new
        if hasattr(train_set, "update_corrupted_label"):
            train_set.update_corrupted_label(labels.tolist())
        va = loop.evaluate()
        logger.line(f"PLC epoch {epoch + 1}: train top1 {100 * tr['top1']:.2f} | val top1 {100 * va['top1']:.2f} "
                    f"| corrected {changed} labels, delta {delta:.2f}")
        logger.log("plc", epoch=epoch, corrected=changed, delta=delta, val_top1=va["top1"])
    return loop.best
