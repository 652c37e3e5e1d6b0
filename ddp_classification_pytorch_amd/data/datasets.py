"""Datasets of the reference workloads (all return uint8 HWC images).

* :class:`CappedImageFolder` — ``root/<class>/*.jpg`` with a per-class image cap
  and an optional class limit (BASELINE/main.py:97-121 cap 500,
  ARCFACE/arc_main.py:178-204 cap 400, CDR/main.py:69-94 cap 500 + first 100
  classes).  Classes are SORTED by default; ``glob_order=True`` reproduces
  the reference's unsorted ``glob`` order (which can mismatch train/test
  labels across directories).
* :class:`ImageFolder` — torchvision-style (sorted classes, all images;
  NESTED/train.py:71-72).
* :class:`ListDataset` — Clothing1M annotation lists returning
  ``(img, label, index)`` with class-balanced train subsampling and in-place
  relabelling (PLC/FolderDataset.py:9-110).
* :class:`SyntheticImages` — deterministic random uint8 images + labels of a
  given shape (benchmarks / tests; no files needed).
"""
from __future__ import annotations

import glob
import os

import numpy as np
import torch
from PIL import Image

IMG_EXTS = (".jpg", ".jpeg", ".png", ".bmp", ".ppm", ".webp", ".JPEG", ".JPG", ".PNG")


def _load_rgb(path):
    with open(path, "rb") as f:
        return Image.open(f).convert("RGB")


class CappedImageFolder(torch.utils.data.Dataset):
    def __init__(self, root, transform=None, imgs_limited=500, num_classes_limit=None, glob_order=False,
                 exts=(".jpg",)):
        classes = glob.glob(os.path.join(root, "*"))
        classes = [c for c in classes if os.path.isdir(c)]
        if not glob_order:
            classes = sorted(classes)
        if num_classes_limit is not None:
            classes = classes[:num_classes_limit]
        self.classes = [os.path.basename(c) for c in classes]
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        self.transform = transform
        self.imgs, self.labels = [], []
        for i, cdir in enumerate(classes):
            files = []
            for e in exts:
                files += glob.glob(os.path.join(cdir, "*" + e))
            if not glob_order:
                files = sorted(files)
            if imgs_limited is not None and len(files) > imgs_limited:
                files = files[:imgs_limited]
            self.imgs += files
            self.labels += [i] * len(files)
        self.targets = self.labels

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, index):
        img = _load_rgb(self.imgs[index])
        if self.transform is not None:
            img = self.transform(img)
        return img, self.labels[index]


class ImageFolder(CappedImageFolder):
    def __init__(self, root, transform=None):
        super().__init__(root, transform, imgs_limited=None, exts=IMG_EXTS)


class ListDataset(torch.utils.data.Dataset):
    """Clothing1M-style annotation lists (PLC/FolderDataset.py:9-82)."""

    SPLITS = {
        "train": ("annotations/noisy_train_key_list.txt", "annotations/my_train_label.txt"),
        "val": ("annotations/clean_val_key_list.txt", "annotations/my_val_label.txt"),
        "test": ("annotations/clean_test_key_list.txt", "annotations/my_test_label.txt"),
    }

    def __init__(self, data_root, split="train", transform=None, cls_size=18976, seed=None, resize=256):
        self.data_root, self.transform, self.resize = data_root, transform, resize
        fpath, lpath = (os.path.join(data_root, p) for p in self.SPLITS[split])
        with open(fpath) as f:
            images = [ln.strip() for ln in f if ln.strip()]
        with open(lpath) as f:
            labels = [int(ln.strip()) for ln in f if ln.strip()]
        if split == "train":
            rng = np.random.RandomState(seed) if seed is not None else np.random
            images, labels = np.array(images), np.array(labels)
            keep_img, keep_lab = [], []
            for c in np.unique(labels):  # class-balanced subsample, at most cls_size per class
                idx = rng.permutation(np.where(labels == c)[0])[:cls_size]
                keep_img.append(images[idx])
                keep_lab.append(labels[idx])
            images = np.concatenate(keep_img).tolist()
            labels = np.concatenate(keep_lab).tolist()
        self.image_list, self.label_list = images, labels
        self.targets = self.label_list

    def __len__(self):
        return len(self.label_list)

    def __getitem__(self, index):
        img = Image.open(os.path.join(self.data_root, self.image_list[index]))
        if self.resize:
            img = img.resize((self.resize, self.resize), resample=Image.BICUBIC)
        img = img.convert("RGB")  # grey -> 3 channels
        if self.transform is not None:
            img = self.transform(img)
        return img, int(self.label_list[index]), index

    def update_corrupted_label(self, noise_label):
        """In-place relabel (PLC/FolderDataset.py:80-82)."""
        self.label_list[:] = [int(x) for x in noise_label]
        self.targets = self.label_list


def write_label_files(data_root, split_lists: dict, out_dir="annotations"):
    """Generate ``my_*_label.txt`` label files from (key list, key->label map) pairs
    (the data-prep half of PLC/FolderDataset.py:85-184, without hard-coded paths)."""
    os.makedirs(os.path.join(data_root, out_dir), exist_ok=True)
    for split, (keys, key2label) in split_lists.items():
        with open(os.path.join(data_root, out_dir, f"my_{split}_label.txt"), "w") as f:
            for k in keys:
                f.write(f"{int(key2label[k])}\n")


class SyntheticImages(torch.utils.data.Dataset):
    """n random uint8 HWC images of shape (size, size, 3) with labels in [0, num_classes).

    ``learnable``: each image is its class's colour template (a coarse 4 x 4 grid of per-class
    colours, the same for every split) plus noise, so the label is a function of the image and a
    few epochs of training must lower the loss (the workload learning tests); otherwise pixels and
    labels are independent (throughput runs)."""

    def __init__(self, n, size=224, num_classes=1000, seed=0, return_index=False, learnable=False):
        self.n, self.size, self.num_classes, self.seed = n, size, num_classes, seed
        self.return_index = return_index
        self.learnable = bool(learnable)
        g = np.random.RandomState(seed)
        self.labels = g.randint(0, num_classes, size=n).tolist()
        self.targets = self.labels
        if self.learnable:
            t = np.random.RandomState(12345).randint(0, 256, size=(num_classes, 4, 4, 3)).astype(np.float32)
            rep = -(-size // 4)
            self.templates = np.repeat(np.repeat(t, rep, axis=1), rep, axis=2)[:, :size, :size]

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = np.random.RandomState(self.seed * 1000003 + i)
        if self.learnable:
            noise = g.randint(-40, 41, size=(self.size, self.size, 3)).astype(np.float32)
            img = np.clip(self.templates[self.labels[i]] + noise, 0, 255).astype(np.uint8)
        else:
            img = g.randint(0, 256, size=(self.size, self.size, 3), dtype=np.uint8)
        if self.return_index:
            return img, self.labels[i], i
        return img, self.labels[i]


def make_fake_image_folder(root, num_classes=3, per_class=4, size=40, seed=0, ext=".jpg"):
    """Write a tiny ``root/{train,test}/<class>/*.jpg`` tree (tests / smoke runs)."""
    g = np.random.RandomState(seed)
    for split in ("train", "test"):
        for c in range(num_classes):
            d = os.path.join(root, split, f"class_{c:03d}")
            os.makedirs(d, exist_ok=True)
            for k in range(per_class):
                arr = (g.rand(size, size, 3) * 64 + c * 60).clip(0, 255).astype(np.uint8)
                Image.fromarray(arr).save(os.path.join(d, f"img_{k:04d}{ext}"))
    return root
