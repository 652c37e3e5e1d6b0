"""Process / device / data setup shared by every workload.

* :func:`setup` — torchrun-compatible process group (RCCL on GPU, gloo on CPU)
  with an explicit timeout (the reference uses the default
  and a hard-wired tcp://127.0.0.1:8989 with rank=local_rank,
  BASELINE/main.py:35-38), device selection, seeding (BASELINE/main.py:43-50),
  output directory.
* :func:`build_data` — train/val loaders for ``--data folder | imagefolder |
  list | synthetic`` with rank-sharded samplers and the on-device prefetcher.
"""
from __future__ import annotations

import os

import torch

from .. import _ext, tuning
from ..data import (CappedImageFolder, DevicePrefetcher, ImageFolder, ListDataset, ShardSampler, SyntheticImages,
                    build_loader, build_transform, norm_stats)
from ..parallel.ddp import graph_safe_nccl_env, init_distributed
from ..utils.misc import set_seed, worker_init_fn


class Runtime:
    def __init__(self, rank, local_rank, world, device):
        self.rank, self.local_rank, self.world, self.device = rank, local_rank, world, device

    @property
    def is_main(self):
        return self.rank == 0


def setup(args) -> Runtime:
    want_cuda = (args.device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda")
    backend = args.dist_backend or ("nccl" if want_cuda else "gloo")
    if getattr(args, "graph", False):
        graph_safe_nccl_env()
    if getattr(args, "syncbn_transport", None):
        os.environ["DCP_SYNCBN_TRANSPORT"] = args.syncbn_transport  # read by convert_sync_batchnorm
    if getattr(args, "syncbn_shared_group", False):
        os.environ["DCP_SYNCBN_SHARED_GROUP"] = "1"  # read by parallel.ddp.bn_process_group
    rank, local, world = init_distributed(backend, force=getattr(args, "force_ddp", False))
    if want_cuda:
        # (one GPU per rank; tests run several gloo ranks on one device: wrap like bench.py)
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        kops = _ext.hip_ops()  # GPU path requires the gfx950 library: fail loudly here, not mid-epoch
        # per-shape conv configuration autotuning (the reference's cudnn.benchmark=True); the
        # DCP_AUTOTUNE environment variable (_ext.py) overrides the flag either way
        env = os.environ.get("DCP_AUTOTUNE")
        tune = getattr(args, "autotune", False) if env is None else env == "1"
        kops.set_tuning(tuning.slot("autotune"), 1 if tune else 0)
    else:
        device = torch.device("cpu")
    set_seed(args.seed + rank)
    if rank == 0:
        os.makedirs(args.out_dir, exist_ok=True)
    return Runtime(rank, local, world, device)


def _datasets(args):
    tr_t = build_transform(args.transform, True, args.image_size)
    va_t = build_transform(args.transform, False, args.image_size)
    if args.data == "synthetic":
        n_tr, n_va = args.synthetic_train_size, args.synthetic_val_size
        size = args.image_size if args.transform != "baseline" or args.image_size != 224 else 224
        learn = getattr(args, "synthetic_learnable", False)
        tr = SyntheticImages(n_tr, size=size, num_classes=args.num_classes, seed=args.seed,
                             return_index=args.workload == "plc", learnable=learn)
        va = SyntheticImages(n_va, size=size, num_classes=args.num_classes, seed=args.seed + 1,
                             return_index=args.workload == "plc", learnable=learn)
        return tr, va
    if args.data == "shards":
        from ..data.shards import ShardDataset

        tr = ShardDataset(args.shard_train or os.path.join(args.folder, "train.dcps"), tr_t)
        va = ShardDataset(args.shard_val or os.path.join(args.folder, "test.dcps"), va_t)
        return tr, va
    if args.data == "list":
        tr = ListDataset(args.folder, "train", tr_t, seed=args.seed)
        va = ListDataset(args.folder, "val", va_t)
        return tr, va
    train_dir = args.train_dir or os.path.join(args.folder, "train")
    val_dir = args.val_dir or os.path.join(args.folder, "test")
    if args.data == "imagefolder":
        return ImageFolder(train_dir, tr_t), ImageFolder(val_dir, va_t)
    tr = CappedImageFolder(train_dir, tr_t, args.imgs_limited, args.num_class_dirs, args.glob_order)
    va = CappedImageFolder(val_dir, va_t, args.imgs_limited, args.num_class_dirs, args.glob_order)
    return tr, va


class WithIndex(torch.utils.data.Dataset):
    """(img, label) -> (img, label, index) (PLC needs dataset indices)."""

    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        item = self.ds[i]
        return (item[0], item[1], i) if len(item) == 2 else item

    def __getattr__(self, name):
        if name == "ds":
            raise AttributeError(name)
        return getattr(self.ds, name)


def _shard_loaders(args, rt, tr, va, tr_s, va_s, mean, std, cpad, s2d, drop_last_train):
    """Native loaders (C++ gather + GPU crop/resize) when the transform preset maps onto them;
    None for presets with rotation/padding (those run the PIL DataLoader over the same shard)."""
    from ..data.shards import ShardLoader, aug_preset

    try:
        tr_aug, tr_size = aug_preset(args.transform, True, args.image_size)
        va_aug, va_size = aug_preset(args.transform, False, args.image_size)
    except ValueError:
        return None
    idx = args.workload == "plc"
    kw = dict(device=rt.device, threads=args.loader_threads, seed=args.seed, mean=mean, std=std, cpad=cpad,
              return_index=idx)
    tr_l = ShardLoader(tr.path, args.batchsize, tr_s, tr_aug, tr_size, drop_last=drop_last_train,
                       s2d=s2d, **kw)
    va_l = ShardLoader(va.path, args.batchsize, va_s, va_aug, va_size, s2d=s2d, **kw)
    return tr_l, va_l


def _device_synthetic(args, rt: Runtime):
    """--data synthetic-device: on-device uint8 batches (a pool of two per split, different per rank),
    normalised by the input kernel every step -- the input bench.py times, so a main.py run measures
    the training loop itself."""
    from ..data import SyntheticLoader

    if args.workload == "plc":
        raise ValueError("--data synthetic-device has no per-sample dataset labels (PLC relabels its dataset)")
    mean, std = norm_stats(args.dataset if "CIFAR" in args.dataset.upper() else "imagenet")
    cpad = 3 if str(args.model).startswith("tresnet") else 8
    s2d = 4 if str(args.model).startswith("tresnet") else str(args.model).startswith(("resnet", "resnext"))
    kw = dict(size=args.image_size, num_classes=args.num_classes, device=rt.device, mean=mean, std=std, cpad=cpad,
              s2d=s2d)
    B = args.batchsize
    tr = SyntheticLoader(B, max(1, args.synthetic_train_size // B), seed=args.seed + 17 * rt.rank, **kw)
    va = SyntheticLoader(B, max(1, args.synthetic_val_size // B), seed=args.seed + 17 * rt.rank + 7, **kw)
    return tr, va, None, None


def build_data(args, rt: Runtime, drop_last_train=False):
    if args.data == "synthetic-device":
        return _device_synthetic(args, rt)
    tr, va = _datasets(args)
    if args.workload == "plc" and args.data != "synthetic" and not isinstance(tr, ListDataset):
        tr, va = WithIndex(tr), WithIndex(va)
    mean, std = norm_stats(args.dataset if "CIFAR" in args.dataset.upper() else "imagenet")
    cpad = 3 if str(args.model).startswith("tresnet") else 8
    # space-to-depth stem inputs written by the input kernel: ImageNet ResNets 2x2, TResNet 4x4
    s2d = 4 if str(args.model).startswith("tresnet") else str(args.model).startswith(("resnet", "resnext"))
    tr_s = ShardSampler(tr, rt.world, rt.rank, shuffle=True, seed=args.seed, drop_last=drop_last_train)
    va_s = ShardSampler(va, rt.world, rt.rank, shuffle=False, seed=args.seed)
    if args.data == "shards":
        native = _shard_loaders(args, rt, tr, va, tr_s, va_s, mean, std, cpad, s2d, drop_last_train)
        if native is not None:
            return native + (tr, va)
    workers = args.workers if args.data != "synthetic" else min(args.workers, 2)
    tr_l = build_loader(tr, args.batchsize, tr_s, workers=workers, drop_last=drop_last_train,
                        worker_init_fn=worker_init_fn)
    va_l = build_loader(va, args.batchsize, va_s, workers=workers, drop_last=False, worker_init_fn=worker_init_fn)
    return (DevicePrefetcher(tr_l, rt.device, mean, std, cpad, s2d), DevicePrefetcher(va_l, rt.device, mean, std, cpad, s2d),
            tr, va)
