"""Data layer: sampler semantics vs torch DistributedSampler, capped image
folders, Clothing1M list dataset, transforms, collate / prefetcher."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from ddp_classification_pytorch_amd.data import (CappedImageFolder, DevicePrefetcher, ImageFolder, ListDataset,
                                                  ShardSampler, SyntheticImages, build_loader, build_transform,
                                                  make_fake_image_folder)


class _DS:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n", [1, 7, 10, 33])
@pytest.mark.parametrize("world", [1, 2, 3, 4])
@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("drop_last", [False, True])
def test_shard_sampler_matches_torch(n, world, shuffle, drop_last):
    if drop_last and n < world:
        return
    for rank in range(world):
        ours = ShardSampler(_DS(n), world, rank, shuffle=shuffle, seed=3, drop_last=drop_last)
        ref = torch.utils.data.DistributedSampler(_DS(n), world, rank, shuffle=shuffle, seed=3, drop_last=drop_last)
        for ep in (0, 5):
            ours.set_epoch(ep)
            ref.set_epoch(ep)
            assert list(ours) == list(ref)
            assert len(ours) == len(ref)


def test_capped_folder_caps_and_classes(tmp_path):
    root = make_fake_image_folder(str(tmp_path), num_classes=4, per_class=6, size=20)
    ds = CappedImageFolder(os.path.join(root, "train"), None, imgs_limited=5)
    assert len(ds) == 4 * 5
    assert ds.classes == sorted(ds.classes)
    ds2 = CappedImageFolder(os.path.join(root, "train"), None, imgs_limited=500, num_classes_limit=2)
    assert len(ds2) == 2 * 6 and set(ds2.labels) == {0, 1}
    img, lab = ds[0]
    assert isinstance(img, Image.Image) and lab == 0
    full = ImageFolder(os.path.join(root, "test"), build_transform("cifar", False))
    arr, lab = full[len(full) - 1]
    assert arr.dtype == np.uint8 and arr.shape == (20, 20, 3) and lab == 3


def test_list_dataset(tmp_path):
    root = str(tmp_path)
    os.makedirs(os.path.join(root, "annotations"))
    os.makedirs(os.path.join(root, "images"))
    keys, labels = [], []
    for i in range(12):
        k = f"images/{i}.png"
        mode = "L" if i % 3 == 0 else "RGB"  # grey images are converted to 3 channels
        Image.new(mode, (30, 40), color=i * 10 if mode == "L" else (i * 10, 0, 0)).save(os.path.join(root, k))
        keys.append(k)
        labels.append(i % 3)
    for split, fn in (("train", "noisy_train_key_list.txt"), ("val", "clean_val_key_list.txt")):
        with open(os.path.join(root, "annotations", fn), "w") as f:
            f.write("\n".join(keys) + "\n")
        with open(os.path.join(root, "annotations", f"my_{split}_label.txt"), "w") as f:
            f.write("\n".join(map(str, labels)) + "\n")
    tr = ListDataset(root, "train", build_transform("plc", True), cls_size=3, seed=0)
    assert len(tr) == 9 and sorted(set(tr.label_list)) == [0, 1, 2]
    img, lab, idx = tr[4]
    assert img.shape == (224, 224, 3) and idx == 4
    tr.update_corrupted_label([0] * len(tr))
    assert set(tr.targets) == {0}
    va = ListDataset(root, "val", None)
    assert len(va) == 12


@pytest.mark.parametrize("preset,size", [("baseline", 256), ("cdr", 224), ("nested", 224), ("cifar", 32)])
def test_transforms_output(preset, size):
    img = Image.fromarray(np.random.RandomState(0).randint(0, 255, (300, 260, 3), dtype=np.uint8))
    if preset == "cifar":
        img = img.resize((32, 32))
    out = build_transform(preset, True)(img)
    assert out.dtype == np.uint8 and out.shape == (size, size, 3)
    val = build_transform(preset, False)(img)
    assert val.shape == ((224, 224, 3) if preset != "cifar" else (32, 32, 3))


def test_loader_and_prefetcher_cpu():
    ds = SyntheticImages(10, size=16, num_classes=5, seed=0, return_index=True)
    loader = build_loader(ds, 4, ShardSampler(ds, 1, 0, shuffle=False), workers=0)
    pf = DevicePrefetcher(loader, "cpu", cpad=8)
    batches = list(pf)
    assert len(batches) == 3
    x, y, idx = batches[0]
    assert x.shape == (4, 16, 16, 8) and x.dtype == torch.float32
    assert torch.all(x[..., 3:] == 0)
    assert torch.equal(idx, torch.arange(4))
    img0 = torch.from_numpy(ds[0][0]).float() / 255.0
    expect = (img0[..., 0] - 0.485) / 0.229
    assert torch.allclose(x[0, ..., 0], expect, atol=1e-5)
