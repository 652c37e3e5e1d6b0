"""GPU half of the native shard loader: the crop_resize HIP kernel against the fp32 reference
math (ops/_ref.py:crop_resize) and a ShardLoader epoch on cuda:0 against the CPU path."""
import numpy as np
import pytest
import torch

from ddp_classification_pytorch_amd.data import ShardSampler
from ddp_classification_pytorch_amd.data.shards import ShardLoader, aug_preset, write_shard
from ddp_classification_pytorch_amd.ops import _ref
from ddp_classification_pytorch_amd.ops import functional as Fn

pytestmark = pytest.mark.gpu


def _batch(B, seed=0):
    g = torch.Generator().manual_seed(seed)
    recs, metas, off = [], [], 0
    for b in range(B):
        H, W = int(torch.randint(8, 90, (1,), generator=g)), int(torch.randint(8, 90, (1,), generator=g))
        h = int(torch.randint(1, H + 1, (1,), generator=g))
        w = int(torch.randint(1, W + 1, (1,), generator=g))
        y0 = int(torch.randint(0, H - h + 1, (1,), generator=g))
        x0 = int(torch.randint(0, W - w + 1, (1,), generator=g))
        recs.append(torch.randint(0, 256, (H * W * 3,), dtype=torch.uint8, generator=g))
        metas.append([off, H, W, y0, x0, h, w, b % 2])
        off += H * W * 3
    return torch.cat(recs), torch.tensor(metas, dtype=torch.int64)


@pytest.mark.parametrize("Ho,Wo", [(37, 53), (64, 64), (224, 224)])
def test_crop_resize_kernel_matches_reference(Ho, Wo):
    src, meta = _batch(9)
    ref = _ref.crop_resize(src, meta, Ho, Wo)
    out = Fn.crop_resize(src.cuda(), meta, Ho, Wo).cpu()
    d = (out.int() - ref.int()).abs()
    assert d.max().item() <= 1
    assert (d == 0).float().mean().item() > 0.999


def test_crop_resize_rejects_out_of_bounds_box():
    src, meta = _batch(2)
    bad = meta.clone()
    bad[1, 5] = bad[1, 1] + 1  # crop taller than the record
    with pytest.raises(RuntimeError, match="outside"):
        Fn.crop_resize(src.cuda(), bad, 16, 16)


def test_shard_loader_gpu_matches_cpu(tmp_path):
    rng = np.random.default_rng(1)
    imgs = [(rng.integers(0, 256, (int(rng.integers(40, 80)), int(rng.integers(40, 80)), 3), dtype=np.uint8), i % 7)
            for i in range(45)]
    p = str(tmp_path / "g.dcps")
    write_shard(p, imgs)
    aug, _ = aug_preset("nested", train=True, size=32)
    outs = {}
    for dev in ("cpu", "cuda"):
        sampler = ShardSampler(list(range(45)), num_replicas=1, rank=0, shuffle=True, seed=2)
        ld = ShardLoader(p, batch_size=16, sampler=sampler, aug=aug, out_size=32, device=dev, threads=4,
                         prefetch=2, s2d=True)
        ld.set_epoch(1)
        outs[dev] = [(x.float().cpu(), y.cpu()) for x, y in ld]
        ld.close()
    assert len(outs["cpu"]) == len(outs["cuda"]) == 3
    for (xc, yc), (xg, yg) in zip(outs["cpu"], outs["cuda"]):
        assert torch.equal(yc, yg)
        assert xg.shape == xc.shape
        # one uint8 level of resample rounding + bf16 normalisation
        assert (xg - xc).abs().max().item() < 0.06
