"""Image augmentation on the host (PIL), producing uint8 HWC arrays.

The reference applies torchvision transforms ending in ToTensor+Normalize on
CPU workers (BASELINE/main.py:58-76, ARCFACE/arc_main.py:69-87,
CDR/main.py:112-130, NESTED/train.py:28-65).  Here the host pipeline stops at
uint8 HWC (4x fewer bytes over PCIe than fp32 CHW) and normalisation +
NHWC/bf16 conversion runs on the GPU (``ops.functional.to_device_nhwc``).
torchvision is not required.
"""
from __future__ import annotations

import math
import random

import numpy as np
from PIL import Image

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
CIFAR10_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR10_STD = (0.2023, 0.1994, 0.2010)
CIFAR100_MEAN = (0.5071, 0.4867, 0.4408)  # NESTED/train.py:35
CIFAR100_STD = (0.2675, 0.2565, 0.2761)


class Compose:
    def __init__(self, ts):
        self.ts = list(ts)

    def __call__(self, img):
        for t in self.ts:
            img = t(img)
        return img

    def __repr__(self):
        return "Compose(" + ", ".join(type(t).__name__ for t in self.ts) + ")"


def _size(s):
    return (s, s) if isinstance(s, int) else tuple(s)


class Resize:
    """Shorter side -> size (int) or exact (h, w)."""

    def __init__(self, size, interpolation=Image.BILINEAR):
        self.size, self.interp = size, interpolation

    def __call__(self, img):
        w, h = img.size
        if isinstance(self.size, int):
            if w <= h:
                nw, nh = self.size, int(round(self.size * h / w))
            else:
                nh, nw = self.size, int(round(self.size * w / h))
        else:
            nh, nw = self.size
        return img.resize((nw, nh), self.interp)


class CenterCrop:
    def __init__(self, size):
        self.size = _size(size)

    def __call__(self, img):
        w, h = img.size
        th, tw = self.size
        i = int(round((h - th) / 2.0))
        j = int(round((w - tw) / 2.0))
        return img.crop((j, i, j + tw, i + th))


class RandomResizedCrop:
    """torchvision semantics: area scale + log-uniform aspect ratio, 10 tries, center fallback."""

    def __init__(self, size, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3), interpolation=Image.BILINEAR):
        self.size, self.scale, self.ratio, self.interp = _size(size), scale, ratio, interpolation

    def params(self, img):
        w, h = img.size
        area = h * w
        lr = (math.log(self.ratio[0]), math.log(self.ratio[1]))
        for _ in range(10):
            ta = area * random.uniform(*self.scale)
            ar = math.exp(random.uniform(*lr))
            cw = int(round(math.sqrt(ta * ar)))
            ch = int(round(math.sqrt(ta / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                return random.randint(0, h - ch), random.randint(0, w - cw), ch, cw
        in_ratio = w / h
        if in_ratio < min(self.ratio):
            cw, ch = w, int(round(w / min(self.ratio)))
        elif in_ratio > max(self.ratio):
            ch, cw = h, int(round(h * max(self.ratio)))
        else:
            cw, ch = w, h
        return (h - ch) // 2, (w - cw) // 2, ch, cw

    def __call__(self, img):
        i, j, h, w = self.params(img)
        return img.crop((j, i, j + w, i + h)).resize((self.size[1], self.size[0]), self.interp)


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, img):
        return img.transpose(Image.FLIP_LEFT_RIGHT) if random.random() < self.p else img


class RandomRotation:
    def __init__(self, degrees):
        self.degrees = (-degrees, degrees) if isinstance(degrees, (int, float)) else degrees

    def __call__(self, img):
        return img.rotate(random.uniform(*self.degrees), resample=Image.NEAREST)


class RandomCrop:
    """CIFAR-style crop with zero padding (NESTED/train.py:40-45)."""

    def __init__(self, size, padding=0):
        self.size, self.padding = _size(size), padding

    def __call__(self, img):
        if self.padding:
            w, h = img.size
            canvas = Image.new(img.mode, (w + 2 * self.padding, h + 2 * self.padding))
            canvas.paste(img, (self.padding, self.padding))
            img = canvas
        w, h = img.size
        th, tw = self.size
        i, j = random.randint(0, h - th), random.randint(0, w - tw)
        return img.crop((j, i, j + tw, i + th))


class Identity:
    def __call__(self, img):
        return img


class ToUint8HWC:
    def __call__(self, img):
        return np.asarray(img.convert("RGB"), dtype=np.uint8)


def build_transform(name: str, train: bool, size: int = 224):
    """Pipelines of the reference workloads (all end in uint8 HWC)."""
    name = name.lower()
    if name in ("baseline", "arcface"):
        # BASELINE/main.py:58-76: train RRC(256, scale 0.8-1); val Resize(256)+CenterCrop(224)
        if train:
            return Compose([RandomResizedCrop(size if size != 224 else 256, scale=(0.8, 1.0)), ToUint8HWC()])
        return Compose([Resize(256), CenterCrop(224 if size in (224, 256) else size), ToUint8HWC()])
    if name == "cdr":
        # CDR/main.py:112-130
        if train:
            return Compose([RandomResizedCrop(256), RandomRotation(15), RandomHorizontalFlip(), CenterCrop(224),
                            ToUint8HWC()])
        return Compose([Resize(256), CenterCrop(224), ToUint8HWC()])
    if name in ("nested", "clothing1m"):
        # NESTED/train.py:46-65 (Clothing1M branch)
        if train:
            return Compose([RandomResizedCrop(224), RandomHorizontalFlip(), ToUint8HWC()])
        return Compose([Resize(256), CenterCrop(224), ToUint8HWC()])
    if name in ("cifar", "cifar10", "cifar100"):
        if train:
            return Compose([RandomCrop(32, padding=4), RandomHorizontalFlip(), ToUint8HWC()])
        return Compose([ToUint8HWC()])
    if name == "plc":
        # PLC/FolderDataset.py: 256x256 bicubic resize
        return Compose([Resize((256, 256), Image.BICUBIC), RandomHorizontalFlip() if train else Identity(),
                        CenterCrop(224), ToUint8HWC()])
    raise ValueError(f"unknown transform preset {name}")


def norm_stats(name: str):
    name = name.lower()
    if name == "cifar10":
        return CIFAR10_MEAN, CIFAR10_STD
    if name in ("cifar100", "cifar"):
        return CIFAR100_MEAN, CIFAR100_STD
    return IMAGENET_MEAN, IMAGENET_STD
