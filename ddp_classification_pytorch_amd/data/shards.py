"""Pre-decoded image shards + the native (C++ thread pool -> pinned -> GPU augment) batch loader.

Reference input path: ``DataLoader(ImageFolderMy, num_workers=4, pin_memory=True)`` with PIL
decode and RandomResizedCrop / Resize+CenterCrop / ToTensor / Normalize on the host workers
(BASELINE/main.py:58-76,97-131) and ``inputs.cuda(non_blocking=True)`` (:273-274).  JPEG decode
plus augmentation on a few host cores tops out far below the ~14k img/s one MI355X trains
ResNet-50 at (SURVEY.md §7.5 risk 8), so this path splits the work MI355X-first:

1. **offline, once**: :func:`pack_image_folder` decodes every image (PIL, process pool), resizes
   its shorter side to ``short_side`` and appends the raw uint8 HWC pixels to one shard file
   (format below) -- variable image sizes, like the original JPEGs;
2. **per batch, host** (``csrc/host/loader.cpp``, loaded with ctypes): a std::thread pool memcpys
   the batch's records from the memory-mapped shard into a pinned slot, in the order the
   distributed sampler produced, and samples each image's crop box / flip with torchvision's
   RandomResizedCrop algorithm from a counter RNG keyed by (seed, epoch, index);
3. **per batch, device**: one H2D copy of the raw records, then ``dcp::crop_resize`` (bilinear
   crop+resize+flip, csrc/augment.hip) and ``dcp::to_nhwc`` / ``to_nhwc_s2d`` (normalise to bf16
   NHWC) on a side stream; the compute stream waits on an event only.

Shard file (little-endian)::

    Header (48 B)   magic "DCPSHRD1", u32 version=1, u32 channels=3, u64 count,
                    u64 index_off, u64 data_off, u64 max_bytes
    Index           count x {u64 offset (from data_off), u32 h, u32 w, i64 label}
    Data            records, h*w*3 uint8 each (HWC, RGB), then zero padding to 8 bytes

Differences from the PIL pipeline (documented, not hidden): the resample is plain bilinear on
the stored (short_side-resized) image, without PIL's antialiasing filter on downscales, and
Resize+CenterCrop is one resample of the centre box instead of two.  Presets that need
rotation or padding (CDR, CIFAR, PLC) stay on the PIL path.
"""
from __future__ import annotations

import ctypes
import os
import struct
from collections import deque

import numpy as np
import torch

from .. import build_ext
from ..ops import functional as Fn
from .transforms import IMAGENET_MEAN, IMAGENET_STD

MAGIC = b"DCPSHRD1"
_HDR = struct.Struct("<8sIIQQQQ")  # 48 bytes
_IDX = np.dtype([("offset", "<u8"), ("h", "<u4"), ("w", "<u4"), ("label", "<i8")])  # 24 bytes
assert _HDR.size == 48 and _IDX.itemsize == 24


# ----------------------------------------------------------------------------- file format
def write_shard(path: str, samples) -> int:
    """Write ``samples`` (iterable of (uint8 HWC RGB array, int label)) to ``path``; returns count."""
    tmp = path + f".tmp{os.getpid()}"
    index = []
    off = 0
    max_bytes = 0
    with open(tmp, "wb") as f:
        f.write(b"\0" * _HDR.size)
        for img, label in samples:
            a = np.ascontiguousarray(img, dtype=np.uint8)
            if a.ndim != 3 or a.shape[2] != 3 or a.shape[0] == 0 or a.shape[1] == 0:
                raise ValueError(f"shard records are HxWx3 uint8, got {a.shape}")
            f.write(a.tobytes())
            index.append((off, a.shape[0], a.shape[1], int(label)))
            off += a.nbytes
            max_bytes = max(max_bytes, a.nbytes)
        data_off = _HDR.size
        pad = (-(data_off + off)) % 8  # 8-byte aligned index (the records themselves are byte data)
        f.write(b"\0" * pad)
        index_off = data_off + off + pad
        idx = np.array(index, dtype=_IDX) if index else np.zeros(0, dtype=_IDX)
        f.write(idx.tobytes())
        f.seek(0)
        f.write(_HDR.pack(MAGIC, 1, 3, len(index), index_off, data_off, max_bytes))
    os.replace(tmp, path)
    return len(index)


def read_index(path: str):
    """(header dict, structured index array) of a shard file."""
    with open(path, "rb") as f:
        magic, ver, ch, count, index_off, data_off, max_bytes = _HDR.unpack(f.read(_HDR.size))
    if magic != MAGIC or ver != 1 or ch != 3:
        raise ValueError(f"{path}: not a DCPSHRD1 shard")
    idx = np.fromfile(path, dtype=_IDX, count=count, offset=index_off)
    return dict(count=count, index_off=index_off, data_off=data_off, max_bytes=max_bytes), idx


def _decode(args):
    path, label, short_side = args
    from PIL import Image

    with open(path, "rb") as fh:
        img = Image.open(fh).convert("RGB")
    if short_side:
        w, h = img.size
        s = short_side / min(w, h)
        img = img.resize((max(1, round(w * s)), max(1, round(h * s))), Image.BILINEAR)
    return np.asarray(img, dtype=np.uint8), label


def _file_list(dataset):
    if hasattr(dataset, "imgs") and hasattr(dataset, "labels"):  # CappedImageFolder / ImageFolder
        return list(zip(dataset.imgs, dataset.labels))
    if hasattr(dataset, "image_list"):  # ListDataset (paths relative to data_root)
        return [(os.path.join(dataset.data_root, p), l) for p, l in zip(dataset.image_list, dataset.label_list)]
    if hasattr(dataset, "samples"):
        return list(dataset.samples)
    raise TypeError(f"cannot list the image files of {type(dataset).__name__}")


def pack_image_folder(dataset, path: str, short_side: int = 256, workers: int = 4) -> int:
    """Decode every (path, label) of an image-folder dataset (:class:`CappedImageFolder`,
    :class:`ImageFolder`, :class:`ListDataset`) into one shard at ``path``, in dataset order."""
    samples = [(p, int(l), short_side) for p, l in _file_list(dataset)]
    if workers > 1:
        import multiprocessing as mp

        with mp.get_context("spawn").Pool(workers) as pool:
            return write_shard(path, pool.imap(_decode, samples, chunksize=16))
    return write_shard(path, map(_decode, samples))


class ShardDataset(torch.utils.data.Dataset):
    """Map-style view of a shard: ``(PIL image, label)`` (so the regular transform presets and
    DataLoader work on it) or the raw uint8 HWC array with ``raw=True``."""

    def __init__(self, path: str, transform=None, raw: bool = False):
        self.path, self.transform, self.raw = path, transform, raw
        self.hdr, self.index = read_index(path)
        self.targets = self.index["label"].astype(np.int64).tolist()
        self._mm = None

    def __len__(self):
        return int(self.hdr["count"])

    def image(self, i: int) -> np.ndarray:
        if self._mm is None:
            self._mm = np.memmap(self.path, dtype=np.uint8, mode="r")
        e = self.index[i]
        a = self.hdr["data_off"] + int(e["offset"])
        return np.asarray(self._mm[a:a + int(e["h"]) * int(e["w"]) * 3]).reshape(int(e["h"]), int(e["w"]), 3)

    def __getitem__(self, i):
        a = self.image(i)
        if self.raw:
            return a, self.targets[i]
        from PIL import Image

        img = Image.fromarray(a)
        return (self.transform(img) if self.transform else img), self.targets[i]


# ----------------------------------------------------------------------------- native library
class AugSpec(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("resize", ctypes.c_int32), ("crop", ctypes.c_int32),
                ("scale_lo", ctypes.c_float), ("scale_hi", ctypes.c_float),
                ("ratio_lo", ctypes.c_float), ("ratio_hi", ctypes.c_float), ("flip_p", ctypes.c_float)]


MODE_RRC, MODE_CENTER, MODE_WHOLE = 0, 1, 2


def aug_preset(name: str, train: bool, size: int = 224):
    """(AugSpec, output edge) of the reference transform presets (see transforms.build_transform)."""
    name = name.lower()
    if name in ("baseline", "arcface"):
        # BASELINE/main.py:58-76: train RRC(256, scale 0.8-1), no flip; val Resize(256)+CenterCrop(224)
        if train:
            return AugSpec(MODE_RRC, 0, 0, 0.8, 1.0, 3 / 4, 4 / 3, 0.0), (size if size != 224 else 256)
        return AugSpec(MODE_CENTER, 256, size if size in (224, 256) else size, 0, 0, 1, 1, 0.0), 224 if size in (
            224, 256) else size
    if name in ("nested", "clothing1m", "imagenet"):
        # NESTED/train.py:46-65: RRC(224) + flip; val Resize(256)+CenterCrop(224)
        if train:
            return AugSpec(MODE_RRC, 0, 0, 0.08, 1.0, 3 / 4, 4 / 3, 0.5), size
        return AugSpec(MODE_CENTER, 256, size, 0, 0, 1, 1, 0.0), size
    raise ValueError(f"preset {name!r} needs rotation/padding: use the PIL DataLoader path")


_LIB = {"h": None}


def native_lib():
    """ctypes handle of ``_dcp_loader.so`` (built by build_ext.build / build_host)."""
    if _LIB["h"] is None:
        path = build_ext.LOADER_PATH
        if not os.path.exists(path):
            if os.environ.get("DCP_AUTOBUILD", "0") == "1":
                build_ext.build_host(verbose=False)
            else:
                raise RuntimeError(f"native loader not built: {path} (python -m ddp_classification_pytorch_amd.build_ext)")
        lib = ctypes.CDLL(path)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.dcpl_open.restype = vp
        lib.dcpl_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        lib.dcpl_close.argtypes = [vp]
        lib.dcpl_count.restype = i64
        lib.dcpl_count.argtypes = [vp]
        lib.dcpl_pool_create.restype = vp
        lib.dcpl_pool_create.argtypes = [ctypes.c_int]
        lib.dcpl_pool_destroy.argtypes = [vp]
        lib.dcpl_submit.restype = i64
        lib.dcpl_submit.argtypes = [vp, vp, vp, ctypes.c_int, vp, i64, vp, vp, ctypes.POINTER(AugSpec),
                                    ctypes.c_uint64, ctypes.c_uint64]
        lib.dcpl_wait.restype = ctypes.c_int
        lib.dcpl_wait.argtypes = [vp, i64]
        _LIB["h"] = lib
    return _LIB["h"]


class NativeGather:
    """One memory-mapped shard + a host thread pool: ``submit(indices, slot)`` gathers records
    and samples augmentation boxes asynchronously, ``wait(ticket)`` joins."""

    def __init__(self, path: str, threads: int = 8):
        self.lib = native_lib()
        err = ctypes.create_string_buffer(512)
        self.shard = self.lib.dcpl_open(path.encode(), err, len(err))
        if not self.shard:
            raise RuntimeError("dcpl_open: " + err.value.decode())
        self.pool = self.lib.dcpl_pool_create(int(threads))
        self.hdr, _ = read_index(path)

    def __len__(self):
        return int(self.lib.dcpl_count(self.shard))

    def submit(self, indices: torch.Tensor, out: torch.Tensor, meta: torch.Tensor, labels: torch.Tensor,
               aug: AugSpec, seed: int, epoch: int) -> int:
        assert indices.dtype == torch.int64 and indices.is_contiguous() and not indices.is_cuda
        B = indices.numel()
        assert meta.shape == (B, 8) and labels.shape == (B,) and out.dtype == torch.uint8
        t = self.lib.dcpl_submit(self.pool, self.shard, indices.data_ptr(), B, out.data_ptr(), out.numel(),
                                 meta.data_ptr(), labels.data_ptr(), ctypes.byref(aug), int(seed) & (2**64 - 1),
                                 int(epoch))
        if t < 0:
            raise ValueError(f"dcpl_submit rejected the batch (code {t})")
        return t

    def wait(self, ticket: int):
        rc = self.lib.dcpl_wait(self.pool, ticket)
        if rc != 0:
            raise RuntimeError(f"dcpl_wait: gather failed ({rc})")

    def close(self):
        if getattr(self, "pool", None):
            self.lib.dcpl_pool_destroy(self.pool)
            self.pool = None
        if getattr(self, "shard", None):
            self.lib.dcpl_close(self.shard)
            self.shard = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardLoader:
    """Batches of (normalised NHWC activations, labels[, dataset index]) from a shard.

    ``sampler`` supplies the per-epoch index order (e.g. :class:`ShardSampler`, DistributedSampler
    semantics); ``prefetch`` batches are in flight (host gather -> pinned slot -> H2D -> augment)
    while the caller trains on the current one.  A slot is only refilled after the side stream's
    copy out of it has completed (event per slot).  Same yield signature as
    :class:`DevicePrefetcher`, so the training loop is unchanged.
    """

    def __init__(self, path: str, batch_size: int, sampler=None, aug: AugSpec = None, out_size: int = 224,
                 device="cuda", threads: int = 8, prefetch: int = 3, seed: int = 0, drop_last: bool = False,
                 mean=IMAGENET_MEAN, std=IMAGENET_STD, cpad: int = 8, s2d=False, return_index: bool = False):
        self.gather = NativeGather(path, threads)
        self.batch_size, self.sampler, self.out_size = int(batch_size), sampler, int(out_size)
        self.aug = aug if aug is not None else AugSpec(MODE_WHOLE, 0, 0, 1, 1, 1, 1, 0.0)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.prefetch, self.seed, self.drop_last = max(1, int(prefetch)), int(seed), drop_last
        self.cpad, self.s2d, self.return_index = cpad, Fn.s2d_for(s2d, self.out_size, self.out_size), return_index
        self.mean = torch.tensor(mean, dtype=torch.float32, device=self.device)
        self.std = torch.tensor(std, dtype=torch.float32, device=self.device)
        self.epoch = 0
        stride = int(self.gather.hdr["max_bytes"])
        pin = self.cuda
        nslots = self.prefetch + 1
        self.slots = [dict(buf=torch.empty(self.batch_size * stride, dtype=torch.uint8, pin_memory=pin),
                           meta=torch.empty((self.batch_size, 8), dtype=torch.int64, pin_memory=pin),
                           labels=torch.empty(self.batch_size, dtype=torch.int64, pin_memory=pin),
                           idx=None, event=None) for _ in range(nslots)]
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def _order(self):
        if self.sampler is None:
            return list(range(len(self.gather)))
        return list(iter(self.sampler))

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.gather)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _batches(self):
        order = self._order()
        nb = len(self)
        for i in range(nb):
            yield torch.tensor(order[i * self.batch_size:(i + 1) * self.batch_size], dtype=torch.int64)

    def _submit(self, slot, idx):
        if slot["event"] is not None:
            slot["event"].synchronize()  # the previous H2D copy out of this slot has finished
            slot["event"] = None
        B = idx.numel()
        slot["idx"] = idx
        epoch = getattr(self.sampler, "epoch", self.epoch)  # the training loop drives sampler.set_epoch
        slot["ticket"] = self.gather.submit(idx, slot["buf"], slot["meta"][:B], slot["labels"][:B], self.aug,
                                            self.seed, epoch)

    def _convert(self, slot):
        """Join the host gather of ``slot`` and run H2D + augment + normalise (side stream)."""
        self.gather.wait(slot["ticket"])
        idx = slot["idx"]
        B = idx.numel()
        meta = slot["meta"][:B]
        used = int(meta[:, 0].max().item()) + int((meta[:, 1] * meta[:, 2]).max().item()) * 3 if B else 0
        used = min(used, slot["buf"].numel())
        src = slot["buf"][:used].to(self.device, non_blocking=True)
        labels = slot["labels"][:B].to(self.device, non_blocking=True)
        imgs = Fn.crop_resize(src, meta, self.out_size, self.out_size)
        x = Fn.to_device_nhwc(imgs, self.mean, self.std, cpad=self.cpad, nchw=False, in_scale=1.0 / 255.0,
                              s2d=self.s2d)
        out = (x, labels)
        if self.return_index:
            out = out + (idx.to(self.device, non_blocking=True),)
        if self.cuda:
            slot["event"] = torch.cuda.Event()
            slot["event"].record(self.stream)
        else:
            out = tuple(t.clone() for t in out)  # CPU: detach from the reusable slot buffers
        return out

    def __iter__(self):
        batches = self._batches()
        inflight = deque()
        free = deque(self.slots)

        def fill():
            while free and len(inflight) < self.prefetch:
                try:
                    idx = next(batches)
                except StopIteration:
                    return
                s = free.popleft()
                self._submit(s, idx)
                inflight.append(s)

        fill()
        cur_stream = torch.cuda.current_stream(self.device) if self.cuda else None
        try:
            while inflight:
                s = inflight.popleft()
                if self.cuda:
                    with torch.cuda.stream(self.stream):
                        out = self._convert(s)
                    cur_stream.wait_stream(self.stream)
                    for t in out:
                        t.record_stream(cur_stream)
                else:
                    out = self._convert(s)
                free.append(s)
                fill()
                yield out
        finally:
            # an abandoned epoch (break / exception) must not leave host threads writing into
            # slots that the next epoch, or the allocator, hands out again
            for s in inflight:
                try:
                    self.gather.wait(s["ticket"])
                except RuntimeError:
                    pass

    def close(self):
        self.gather.close()

    def __del__(self):
        try:
            self.close()  # joins the host threads while the pinned slots are still alive
        except Exception:
            pass
