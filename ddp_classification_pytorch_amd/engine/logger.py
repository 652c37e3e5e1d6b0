"""Rank-0 logging: console progress line, JSONL metrics, and the reference's
text artefacts (``output.txt`` per-epoch lines, BASELINE/main.py:254-256;
``history.json``, NESTED/train.py:421,435-445; CDR results txt with
``.bak-<timestamp>`` rotation, CDR/main.py:288-292).  Only rank 0 writes
(the reference appends from every rank).
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch.distributed as dist


def _rank0():
    return not dist.is_initialized() or dist.get_rank() == 0


class MetricsLogger:
    def __init__(self, out_dir=None, jsonl="metrics.jsonl", text="output.txt", echo=True, stream=None):
        self.out_dir = out_dir
        self.echo = echo
        self.stream = stream or sys.stdout
        self.history = {}
        self.t0 = time.time()
        if out_dir and _rank0():
            os.makedirs(out_dir, exist_ok=True)
        self.jsonl = os.path.join(out_dir, jsonl) if out_dir else None
        self.text = os.path.join(out_dir, text) if out_dir else None

    def log(self, kind: str, **fields):
        if not _rank0():
            return
        rec = {"kind": kind, "time": round(time.time() - self.t0, 3)}
        rec.update({k: (float(v) if hasattr(v, "item") else v) for k, v in fields.items()})
        if self.jsonl:
            with open(self.jsonl, "a") as f:
                f.write(json.dumps(rec) + "\n")
        for k, v in rec.items():
            if k in ("kind", "time") or not isinstance(v, (int, float)):
                continue
            self.history.setdefault(f"{kind}/{k}", []).append(v)

    def progress(self, msg: str, end="\r"):
        if _rank0() and self.echo:
            self.stream.write(msg + end)
            self.stream.flush()

    def line(self, msg: str):
        if not _rank0():
            return
        if self.echo:
            print(msg, file=self.stream, flush=True)
        if self.text:
            with open(self.text, "a") as f:
                f.write(msg + "\n")

    def dump_history(self, name="history.json"):
        if _rank0() and self.out_dir:
            with open(os.path.join(self.out_dir, name), "w") as f:
                json.dump(self.history, f)


def rotate_results_file(path: str):
    """CDR/main.py:288-292: move an existing results file aside as .bak-<timestamp>."""
    if _rank0() and os.path.exists(path):
        os.replace(path, f"{path}.bak-{time.strftime('%Y%m%d-%H%M%S')}")
