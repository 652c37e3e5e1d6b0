"""Native shard loader (csrc/host/loader.cpp via ctypes + crop_resize reference math): file
round trip, sampler order, torchvision RandomResizedCrop box semantics, determinism across
thread counts, and the CPU end-to-end batch path."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ddp_classification_pytorch_amd.data import ShardSampler, make_fake_image_folder
from ddp_classification_pytorch_amd.data.datasets import CappedImageFolder
from ddp_classification_pytorch_amd.data.shards import (MODE_CENTER, MODE_RRC, MODE_WHOLE, AugSpec, NativeGather,
                                                        ShardDataset, ShardLoader, aug_preset, pack_image_folder,
                                                        read_index, write_shard)
from ddp_classification_pytorch_amd.ops import _ref


def _images(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        h, w = int(rng.integers(20, 70)), int(rng.integers(20, 70))
        out.append((rng.integers(0, 256, (h, w, 3), dtype=np.uint8), i % 5))
    return out


@pytest.fixture
def shard(tmp_path):
    imgs = _images(37)
    p = str(tmp_path / "s.dcps")
    assert write_shard(p, imgs) == 37
    return p, imgs


def test_write_read_roundtrip(shard):
    p, imgs = shard
    hdr, idx = read_index(p)
    assert hdr["count"] == 37 and hdr["max_bytes"] == max(a.nbytes for a, _ in imgs)
    ds = ShardDataset(p, raw=True)
    for i in (0, 5, 36):
        a, lab = ds[i]
        np.testing.assert_array_equal(a, imgs[i][0])
        assert lab == imgs[i][1]
    img, lab = ShardDataset(p)[3]  # PIL view for the transform presets
    assert img.size == (imgs[3][0].shape[1], imgs[3][0].shape[0])


def _gather(p, order, aug, threads=4, seed=1, epoch=0):
    g = NativeGather(p, threads)
    B = len(order)
    buf = torch.empty(B * int(g.hdr["max_bytes"]), dtype=torch.uint8)
    meta = torch.empty((B, 8), dtype=torch.int64)
    labels = torch.empty(B, dtype=torch.int64)
    t = g.submit(torch.tensor(order, dtype=torch.int64), buf, meta, labels, aug, seed, epoch)
    g.wait(t)
    g.close()
    return buf, meta, labels


def test_native_gather_bytes_and_labels(shard):
    p, imgs = shard
    order = [5, 0, 36, 5, 12]
    buf, meta, labels = _gather(p, order, AugSpec(MODE_WHOLE, 0, 0, 1, 1, 1, 1, 0.0))
    for b, i in enumerate(order):
        a = imgs[i][0]
        off, H, W = (int(v) for v in meta[b, :3])
        assert (H, W) == a.shape[:2]
        np.testing.assert_array_equal(buf[off:off + a.nbytes].numpy().reshape(a.shape), a)
        assert labels[b].item() == imgs[i][1]
        assert meta[b, 3:7].tolist() == [0, 0, H, W]


def test_rrc_boxes_follow_torchvision_bounds(shard):
    p, imgs = shard
    order = list(range(37)) * 4
    aug = AugSpec(MODE_RRC, 0, 0, 0.08, 1.0, 3 / 4, 4 / 3, 0.5)
    _, meta, _ = _gather(p, order, aug)
    flips = meta[:, 7].float().mean().item()
    assert 0.2 < flips < 0.8
    for b, i in enumerate(order):
        H, W, y0, x0, h, w = (int(v) for v in meta[b, 1:7])
        assert 0 <= y0 and y0 + h <= H and 0 <= x0 and x0 + w <= W and h > 0 and w > 0
        area = h * w / (H * W)
        # sampled boxes respect the scale range up to rounding; fallbacks are centred
        fallback = (y0 == (H - h) // 2 and x0 == (W - w) // 2)
        assert fallback or 0.08 * 0.5 <= area <= 1.0


def test_center_box_matches_resize_centercrop():
    # Resize(256) + CenterCrop(224) on a 300x400 image == centre box of 224*300/256 = 262.5 -> 262
    aug, out = aug_preset("baseline", train=False)
    assert aug.mode == MODE_CENTER and out == 224


def test_gather_deterministic_across_threads(shard):
    p, _ = shard
    order = list(range(37))
    aug = AugSpec(MODE_RRC, 0, 0, 0.08, 1.0, 3 / 4, 4 / 3, 0.5)
    m1 = _gather(p, order, aug, threads=1, seed=7, epoch=3)[1]
    m8 = _gather(p, order, aug, threads=8, seed=7, epoch=3)[1]
    assert torch.equal(m1, m8)
    m_ep = _gather(p, order, aug, threads=8, seed=7, epoch=4)[1]
    assert not torch.equal(m1[:, 3:], m_ep[:, 3:])
    # the box depends on the dataset index, not the batch position
    rev = _gather(p, order[::-1], aug, threads=3, seed=7, epoch=3)[1]
    assert torch.equal(rev.flip(0)[:, 1:], m1[:, 1:])


def test_crop_resize_ref_identity_and_flip():
    img = torch.randint(0, 256, (10, 12, 3), dtype=torch.uint8)
    src = img.reshape(-1)
    meta = torch.tensor([[0, 10, 12, 0, 0, 10, 12, 0], [0, 10, 12, 0, 0, 10, 12, 1]])
    out = _ref.crop_resize(src, meta, 10, 12)
    assert torch.equal(out[0], img)
    assert torch.equal(out[1], img.flip(1))


def test_crop_resize_ref_matches_interpolate():
    img = torch.randint(0, 256, (40, 50, 3), dtype=torch.uint8)
    meta = torch.tensor([[0, 40, 50, 3, 7, 30, 33, 0]])
    out = _ref.crop_resize(img.reshape(-1), meta, 24, 20)
    crop = img[3:33, 7:40].permute(2, 0, 1)[None].float()
    ref = F.interpolate(crop, size=(24, 20), mode="bilinear", align_corners=False)[0].permute(1, 2, 0)
    assert (out.float() - ref).abs().max().item() <= 0.5 + 1e-3


def test_shard_loader_cpu_epoch(shard):
    p, imgs = shard
    sampler = ShardSampler(list(range(37)), num_replicas=2, rank=1, shuffle=True, seed=4)
    aug, _ = aug_preset("nested", train=True, size=16)
    ld = ShardLoader(p, batch_size=8, sampler=sampler, aug=aug, out_size=16, device="cpu", threads=3, prefetch=2,
                     return_index=True)
    ld.set_epoch(2)
    seen = []
    for x, y, idx in ld:
        assert x.shape[1:] == (16, 16, 8) and x.dtype == torch.float32
        assert x[..., 3:].abs().max().item() == 0  # padded channels
        for lab, i in zip(y.tolist(), idx.tolist()):
            assert lab == imgs[i][1]
        seen += idx.tolist()
    assert seen == list(sampler) and len(seen) == 19 and len(ld) == 3
    ld.close()


def test_pack_image_folder(tmp_path):
    root = make_fake_image_folder(str(tmp_path / "imgs"), num_classes=2, per_class=3, size=40)
    ds = CappedImageFolder(root + "/train")
    p = str(tmp_path / "f.dcps")
    assert pack_image_folder(ds, p, short_side=32, workers=1) == 6
    sd = ShardDataset(p, raw=True)
    for i in range(6):
        a, lab = sd[i]
        assert min(a.shape[:2]) == 32 and lab == ds.labels[i]


def test_corrupt_shard_rejected(tmp_path):
    p = str(tmp_path / "bad.dcps")
    with open(p, "wb") as f:
        f.write(b"NOTASHARD" * 10)
    with pytest.raises(RuntimeError, match="bad magic"):
        NativeGather(p)


def test_main_with_shards_end_to_end(tmp_path):
    """pack the reference folder layout, then train one epoch through --data shards (CPU)."""
    import main as entry
    from tools import pack_shards

    root = make_fake_image_folder(str(tmp_path / "food"), num_classes=3, per_class=4, size=48)
    pack_shards.main(["--folder", root, "--short-side", "40", "--workers", "1"])
    out = str(tmp_path / "run")
    entry.main(["--workload", "baseline", "--model", "resnet18", "--data", "shards", "--folder", root,
                "--image-size", "32", "--num-classes", "3", "--batchsize", "4", "--epochs", "1", "--out-dir", out,
                "--device", "cpu", "--log-interval", "100", "--loader-threads", "2"])
    assert os.path.exists(os.path.join(out, "last.pth"))


def test_shard_loader_abandoned_epoch_then_new_epoch(shard):
    """Breaking out of an epoch joins the in-flight gathers; the next epoch starts clean."""
    p, imgs = shard
    sampler = ShardSampler(list(range(37)), num_replicas=1, rank=0, shuffle=True, seed=1)
    ld = ShardLoader(p, batch_size=4, sampler=sampler, aug=None, out_size=16, device="cpu", threads=4, prefetch=3,
                     return_index=True)
    for i, _ in enumerate(ld):
        if i == 1:
            break
    ld.set_epoch(1)
    seen = [j for _, _, idx in ld for j in idx.tolist()]
    assert seen == list(sampler)
    ld.close()
