#!/usr/bin/env python3
"""Entry point for every workload (one process per GPU).

    # BASELINE (BASELINE/train.sh): 2 GPUs, DDP + SyncBN
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 main.py --workload baseline --folder /data/foodH --model resnet50
    # ARCFACE (ARCFACE/arc_train.sh)
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 main.py --workload arcface --folder /data/foodH
    # CDR (CDR/train.sh), NESTED (NESTED/train.sh), PLC: single process or DDP
    python main.py --workload cdr --folder /data/food --lr 0.1 --batch_size 128
    python main.py --workload nested --train-dir .../train --val-dir .../val --warmUpIter 10000
    # synthetic data (no files needed)
    python main.py --workload baseline --data synthetic --model resnet18 --num-classes 10 --epochs 1

Also accepts the legacy ``python -m torch.distributed.launch`` flags
(``--local-rank`` / ``--local_rank``).
"""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from ddp_classification_pytorch_amd.config import parse_args  # noqa: E402


def main(argv=None):
    args = parse_args(argv)
    if args.workload == "baseline":
        from ddp_classification_pytorch_amd.algos.baseline import run
    elif args.workload == "arcface":
        from ddp_classification_pytorch_amd.algos.arcface import run
    elif args.workload == "cdr":
        from ddp_classification_pytorch_amd.algos.cdr import run
    elif args.workload == "nested":
        from ddp_classification_pytorch_amd.algos.nested import run
    elif args.workload == "plc":
        from ddp_classification_pytorch_amd.algos.plc import run
    else:  # pragma: no cover - argparse restricts choices
        raise ValueError(args.workload)
    try:
        return run(args)
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
