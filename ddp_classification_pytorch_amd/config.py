"""One CLI for every workload: a superset of the reference's per-script flags
 with the reference's names accepted as aliases.

    BASELINE  BASELINE/main.py:25-32     --local_rank --world_size --folder --model --batchsize
    ARCFACE   ARCFACE/arc_main.py:34-43  + --optimizer
    CDR       CDR/main.py:32-57          --lr --result_dir --noise_rate --num_gradual --dataset --n_epoch ...
    NESTED    NESTED/train.py:458-486    --train-dir --val-dir --dataset --warmUpIter --lrSchedule --arch ...

Launcher compatibility: ``--local-rank`` / ``--local_rank`` and the torchrun
environment (LOCAL_RANK / RANK / WORLD_SIZE) are all honoured.
Hard-coded reference constants become defaults (NUM_CLASS=2173, LR=1e-3,
NUM_EPOCH=100, image caps 500/400, s=30, m=0.5, easy margin).
"""
from __future__ import annotations

import argparse
import os

WORKLOAD_DEFAULTS = {
    "baseline": dict(model="tresnet_m", batchsize=16, lr=1e-3, epochs=100, optimizer="sgd", momentum=0.9,
                     weight_decay=0.0, imgs_limited=500, step_size=10, gamma=0.1, hidden=512, syncbn=True,
                     transform="baseline", autotune=True),
    "arcface": dict(model="resnet50", batchsize=32, lr=1e-3, epochs=100, optimizer="adam", momentum=0.9,
                    weight_decay=5e-4, imgs_limited=400, step_size=10, gamma=0.1, hidden=512, syncbn=True,
                    transform="arcface", autotune=True),
    "cdr": dict(model="resnet50", batchsize=128, lr=1e-3, epochs=200, optimizer="sgd", momentum=0.9,
                weight_decay=0.0, imgs_limited=500, hidden=512, syncbn=False, transform="cdr",
                milestones=[10, 20], gamma=0.1, autotune=False),
    "nested": dict(model="resnet50", batchsize=128, lr=1e-2, epochs=150, optimizer="sgd", momentum=0.9,
                   weight_decay=5e-4, syncbn=False, transform="nested", milestones=[20, 30, 40, 120], gamma=0.1,
                   autotune=False),
    "plc": dict(model="resnet50", batchsize=64, lr=1e-2, epochs=10, optimizer="sgd", momentum=0.9, weight_decay=5e-4,
                syncbn=False, transform="plc", autotune=False),
}


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X-native DDP image classification (gfx950 HIP kernels + RCCL)")
    a = p.add_argument
    a("--workload", default="baseline", choices=sorted(WORKLOAD_DEFAULTS))
    # launcher / distributed
    a("--local-rank", "--local_rank", dest="local_rank", type=int, default=None)
    a("--world_size", "--world-size", dest="world_size", type=int, default=None)
    a("--dist-backend", default=None, help="nccl (=RCCL) on GPU, gloo on CPU")
    a("--syncbn", dest="syncbn", action="store_true", default=None, help="cross-replica BN (reference default)")
    a("--no-syncbn", dest="syncbn", action="store_false")
    a("--syncbn-transport", default=None, choices=["rccl", "peer"],
      help="SyncBN statistics exchange: rccl collectives (default) or the peer-memory mailboxes (parallel/peer.py)")
    a("--syncbn-shared-group", action="store_true",
      help="SyncBN collectives on the gradient communicator (the default group) instead of their own; the "
           "fallback if two RCCL communicators in flight on one GPU misbehave (DCP_SYNCBN_SHARED_GROUP=1)")
    a("--force-ddp", action="store_true",
      help="one process: still create a (world-1) process group and train through the data-parallel engine "
           "(measures the engine's own cost; tests its HIP-graph capture)")
    a("--bucket-cap-mb", type=float, default=25.0)
    a("--first-bucket-mb", type=float, default=4.0)
    a("--device", default=None, help="cuda (default when available) or cpu")
    a("--graph", dest="graph", action="store_true", default=None,
      help="replay the training step as a HIP graph (launch-bound small batches); with several ranks the "
           "bucket engine's all-reduces and per-bucket optimizer are captured too.  Default ON for the "
           "baseline / arcface / cdr loops on the GPU (DCP_GRAPH=0 or --no-graph: eager)")
    a("--no-graph", "--eager", dest="graph", action="store_false")
    # data
    a("--data", default="folder", choices=["folder", "imagefolder", "list", "synthetic", "synthetic-device", "shards"],
      help="synthetic: random images through the host DataLoader path; synthetic-device: random uint8 batches "
           "generated once on the GPU (the bench.py input, no host pipeline in the step)")
    a("--shard-train", dest="shard_train", default=None, help="--data shards: train shard (default <folder>/train.dcps)")
    a("--shard-val", dest="shard_val", default=None, help="--data shards: val shard (default <folder>/test.dcps)")
    a("--loader-threads", dest="loader_threads", type=int, default=8, help="native shard loader host threads")
    a("--folder", default="/root/commonfile/foodH/", help="root with train/ and test/ class folders")
    a("--train-dir", "--train_dir", dest="train_dir", default=None)
    a("--val-dir", "--val_dir", dest="val_dir", default=None)
    a("--dataset", default=None, help="food | Clothing1M | CIFAR10 | CIFAR100 (selects transforms/classes)")
    a("--imgs-limited", dest="imgs_limited", type=int, default=None, help="per-class image cap")
    a("--num-class-dirs", dest="num_class_dirs", type=int, default=None, help="use only the first N class dirs")
    a("--glob-order", action="store_true", help="reference-compat unsorted class order")
    a("--workers", "--num_workers", dest="workers", type=int, default=4)
    a("--image-size", dest="image_size", type=int, default=None)
    a("--synthetic-train-size", type=int, default=2048)
    a("--synthetic-val-size", type=int, default=512)
    a("--synthetic-learnable", action="store_true",
      help="--data synthetic: images carry their class (per-class colour template + noise) so the loss can fall")
    # model
    a("--model", default=None)
    a("--arch", default=None, help="NESTED alias of --model")
    a("--num-classes", "--num_class", dest="num_classes", type=int, default=2173)
    a("--hidden", type=int, default=None, help="MLP head hidden width")
    a("--pretrained", default=None, help="local torchvision-format weights file")
    # optimisation
    a("--batchsize", "--batch_size", "--batch-size", dest="batchsize", type=int, default=None, help="per-process batch")
    a("--epochs", "--n_epoch", "--nbEpoch", dest="epochs", type=int, default=None)
    a("--lr", type=float, default=None)
    a("--momentum", type=float, default=None)
    a("--weight-decay", "--weight_decay", "--weightDecay", dest="weight_decay", type=float, default=None)
    a("--optimizer", default=None, help="SGD | Adam | AdamW")
    a("--nesterov", action="store_true")
    a("--step-size", dest="step_size", type=int, default=None)
    a("--gamma", type=float, default=None)
    a("--lrSchedule", "--milestones", dest="milestones", type=int, nargs="+", default=None)
    a("--warmup-iters", "--warmUpIter", dest="warmup_iters", type=int, default=0)
    a("--label-smoothing", type=float, default=0.0)
    # run control / persistence
    a("--seed", type=int, default=999)
    a("--out-dir", "--out_dir", "--result_dir", dest="out_dir", default="output")
    a("--resume", "--resumePth", dest="resume", default=None)
    a("--save-every", type=int, default=1)
    a("--log-interval", "--print_freq", dest="log_interval", type=int, default=20)
    a("--max-steps-per-epoch", type=int, default=None, help="truncate epochs (smoke runs)")
    a("--eval-every", type=int, default=1)
    a("--fail-at-step", type=int, default=None, help="fault injection: raise at this global step")
    a("--auto-resume", dest="auto_resume", action="store_true",
      help="resume from <out-dir>/last.pth when it exists (restart after a failure)")
    a("--heartbeat-every", dest="heartbeat_every", type=int, default=0,
      help="every N steps append a line to <out-dir>/heartbeat_rank<r>.txt")
    a("--profile", action="store_true", help="torch.profiler (roctracer) trace of 4 steps into <out-dir>/profile")
    a("--autotune", dest="autotune", action="store_true", default=None,
      help="time the conv kernel configurations per layer shape on first use and keep the fastest "
           "(default for baseline / arcface, whose reference scripts set cudnn.benchmark=True: "
           "BASELINE/main.py:40, ARCFACE/arc_main.py:51)")
    a("--no-autotune", dest="autotune", action="store_false",
      help="fixed heuristic kernel configurations (bit-reproducible run to run)")
    # ARCFACE
    a("--s", "--arc-s", dest="arc_s", type=float, default=30.0)
    a("--m", "--arc-m", dest="arc_m", type=float, default=0.5)
    a("--hard-margin", dest="easy_margin", action="store_false", default=True)
    a("--embed-dim", type=int, default=256)
    a("--arc-eval-with-labels", action="store_true", default=True,
      help="reference behaviour: margin applied with true labels at eval (ARCFACE/arc_main.py:368)")
    a("--arc-eval-plain-cosine", dest="arc_eval_with_labels", action="store_false")
    # CDR (unused reference flags accepted for CLI compatibility)
    a("--noise_rate", "--noise-rate", dest="noise_rate", type=float, default=0.2)
    a("--num_gradual", type=int, default=10)
    a("--noise_type", default="symmetric")
    a("--train_len", type=int, default=None)
    for legacy in ("--n", "--d", "--p", "--c", "--fr_type", "--split_percentage", "--gpu", "--model_type"):
        a(legacy, default=None, help=argparse.SUPPRESS)
    # NESTED
    a("--nested", type=float, default=100.0, help="std of the Gaussian over K (0 = off)")
    a("--mu", type=float, default=0.0)
    a("--dropout", type=float, default=0.0)
    a("--freeze-bn", "--freeze_bn", dest="freeze_bn", action="store_true", default=True)
    a("--no-freeze-bn", dest="freeze_bn", action="store_false")
    # PLC
    a("--plc-noise-type", type=int, default=0, help="0/1/2 = type I/II/III feature-dependent noise")
    a("--plc-delta", type=float, default=0.3)
    a("--plc-delta-inc", type=float, default=0.1)
    a("--plc-eta-epochs", type=int, default=2)
    a("--plc-correction", default="lrt", choices=["lrt", "prob"])
    return p


def resolve(args: argparse.Namespace) -> argparse.Namespace:
    """Fill workload defaults, environment-provided ranks and aliases."""
    d = WORKLOAD_DEFAULTS[args.workload]
    if getattr(args, "autotune", None) is None and os.environ.get("DCP_AUTOTUNE") in ("0", "1"):
        args.autotune = os.environ["DCP_AUTOTUNE"] == "1"  # the env switch, when no flag was given
    for k, v in d.items():
        if getattr(args, k, None) is None:
            setattr(args, k, v)
    if args.arch and not getattr(args, "model_explicit", False):
        args.model = args.arch
    if args.hidden is None:
        args.hidden = 512
    if args.local_rank is None:
        args.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    args.rank = int(os.environ.get("RANK", str(args.local_rank)))
    if args.world_size is None:
        args.world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if args.dataset is None:
        args.dataset = {"nested": "Clothing1M", "plc": "Clothing1M"}.get(args.workload, "food")
    if args.image_size is None:
        args.image_size = 32 if "CIFAR" in args.dataset.upper() else 224
    if "CIFAR" in args.dataset.upper():
        args.num_classes = 10 if args.dataset.upper() == "CIFAR10" else 100
        args.transform = "cifar"
        if not args.model.startswith("cifar_") and args.model.startswith("resnet"):
            args.model = "cifar_" + args.model
    if args.workload == "cdr" and args.num_class_dirs is None and args.data == "folder":
        args.num_class_dirs = 100  # CDR/main.py:73
    if args.graph is None:
        # HIP-graph replay wherever the step grapher is eligible: the ClassificationLoop workloads on a
        # GPU (fixed-shape batches; a short last batch runs eagerly; torch-DDP steps stay eager, see
        # engine/loop.py).  At the reference's per-GPU batches of 16-64 replay is 1.3-1.5x the eager
        # step; NESTED / PLC run their own loops.
        env = os.environ.get("DCP_GRAPH")
        on_gpu = (args.device or "cuda").startswith("cuda") and _cuda_available()
        args.graph = (env == "1") if env in ("0", "1") else (on_gpu and args.workload in ("baseline", "arcface", "cdr"))
    if args.nested > 0 and args.dropout > 0:
        raise ValueError("nested dropout and standard dropout are mutually exclusive (NESTED/train.py:489-490)")
    return args


def _cuda_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def parse_args(argv=None):
    p = build_parser()
    return resolve(p.parse_args(argv))
