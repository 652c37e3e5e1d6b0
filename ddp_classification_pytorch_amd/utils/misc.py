"""Small utilities shared by the workloads.

* :func:`set_seed` — python/numpy/torch/HIP seeding (BASELINE/main.py:43-50,
  CDR/main.py:61-62, PLC/utils.py:145-146 ``init_fn_`` worker seeding).
* :class:`AverageMeter`, :func:`accuracy` (precision@k), :func:`format_time`,
  :func:`progress_bar` (NESTED/utils.py:14-132) — the progress bar takes an
  explicit width instead of the hard-coded 30 columns.
* :func:`download_url`, :func:`check_integrity`, :func:`list_dir`,
  :func:`list_files`, :func:`makedir_exist_ok`, :func:`check_folder`
  (PLC/utils.py:14-146).  There is no network here: ``download_url`` only
  verifies an existing file unless a fetcher is available.
"""
from __future__ import annotations

import hashlib
import os
import random
import sys
import time

import numpy as np
import torch


def set_seed(seed: int, deterministic: bool = False):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    if deterministic:
        torch.use_deterministic_algorithms(True, warn_only=True)


def worker_init_fn(worker_id: int, base: int = 77):
    """PLC/utils.py:145-146: numpy seed = 77 + worker id."""
    np.random.seed(base + worker_id)


class AverageMeter:
    """Running average (NESTED/utils.py:14-29)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0.0
        self.avg = 0.0
        self.sum = 0.0
        self.count = 0

    def update(self, val, n=1):
        self.val = float(val)
        self.sum += float(val) * n
        self.count += n
        self.avg = self.sum / max(self.count, 1)


@torch.no_grad()
def accuracy(output: torch.Tensor, target: torch.Tensor, topk=(1,)):
    """precision@k in percent (NESTED/utils.py:32-46)."""
    maxk = min(max(topk), output.shape[1])
    bs = target.size(0)
    _, pred = output.float().topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1).expand_as(pred.t()))
    return [correct[: min(k, maxk)].reshape(-1).float().sum(0) * (100.0 / bs) for k in topk]


def accuracy_from_rank(rank: torch.Tensor, topk=(1, 3)):
    """Top-k hit counts from the fused CE kernel's label rank (#logits > logit[label])."""
    return [(rank < k).sum() for k in topk]


def format_time(seconds: float) -> str:
    """NESTED/utils.py:102-132: the two leading non-zero units, e.g. "1D2h", "3m4s", "5ms"."""
    days = int(seconds / 3600 / 24)
    seconds -= days * 3600 * 24
    hours = int(seconds / 3600)
    seconds -= hours * 3600
    minutes = int(seconds / 60)
    seconds -= minutes * 60
    secondsf = int(seconds)
    millis = int((seconds - secondsf) * 1000)
    out, n = "", 0
    for v, u in ((days, "D"), (hours, "h"), (minutes, "m"), (secondsf, "s"), (millis, "ms")):
        if v > 0 and n < 2:  # at most two units, as the reference (its counter starts at 1)
            out += f"{v}{u}"
            n += 1
    return out or "0ms"


class ProgressBar:
    """ASCII progress bar (NESTED/utils.py:58-99) writing to a stream."""

    def __init__(self, width: int = 30, stream=None):
        self.width = width
        self.stream = stream or sys.stdout
        self.t0 = self.last = time.time()

    def __call__(self, current: int, total: int, msg: str = ""):
        if current == 0:
            self.t0 = time.time()
        now = time.time()
        step, self.last = now - self.last, now
        done = int(self.width * (current + 1) / max(total, 1))
        bar = "=" * max(done - 1, 0) + (">" if done < self.width else "=") + "." * (self.width - done)
        line = f" [{bar}] Step: {format_time(step)} | Tot: {format_time(now - self.t0)}"
        if msg:
            line += " | " + msg
        line += f" {current + 1}/{total}"
        self.stream.write("\r" + line)
        if current + 1 >= total:
            self.stream.write("\n")
        self.stream.flush()


def progress_bar(current, total, msg=None, _bar=[None]):  # noqa: B006 - module-level singleton bar
    if _bar[0] is None:
        _bar[0] = ProgressBar()
    _bar[0](current, total, msg or "")


# ----------------------------------------------------------------------------- PLC/utils.py:14-146
def calculate_md5(fpath: str, chunk_size: int = 1024 * 1024) -> str:
    md5 = hashlib.md5()
    with open(fpath, "rb") as f:
        for chunk in iter(lambda: f.read(chunk_size), b""):
            md5.update(chunk)
    return md5.hexdigest()


def check_md5(fpath: str, md5: str) -> bool:
    return md5 == calculate_md5(fpath)


def check_integrity(fpath: str, md5: str = None) -> bool:
    if not os.path.isfile(fpath):
        return False
    return True if md5 is None else check_md5(fpath, md5)


def makedir_exist_ok(dirpath: str):
    os.makedirs(dirpath, exist_ok=True)


def download_url(url: str, root: str, filename: str = None, md5: str = None) -> str:
    """Return the local path if it exists and verifies; this build never touches the network."""
    root = os.path.expanduser(root)
    filename = filename or os.path.basename(url)
    fpath = os.path.join(root, filename)
    makedir_exist_ok(root)
    if check_integrity(fpath, md5):
        return fpath
    raise RuntimeError(f"{fpath} missing or corrupt and downloads are disabled (no network): place it manually")


def list_dir(root: str, prefix: bool = False):
    root = os.path.expanduser(root)
    dirs = [p for p in os.listdir(root) if os.path.isdir(os.path.join(root, p))]
    return [os.path.join(root, d) for d in dirs] if prefix else dirs


def list_files(root: str, suffix, prefix: bool = False):
    root = os.path.expanduser(root)
    files = [p for p in os.listdir(root) if os.path.isfile(os.path.join(root, p)) and p.endswith(suffix)]
    return [os.path.join(root, d) for d in files] if prefix else files


def check_folder(save_dir: str) -> str:
    makedir_exist_ok(save_dir)
    return save_dir


def rank0_print(*args, **kw):
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_rank() == 0:
        print(*args, **kw, flush=True)
