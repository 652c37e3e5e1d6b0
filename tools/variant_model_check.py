#!/usr/bin/env python3
"""Which BatchNorm layer's statistics change when one autotuner candidate is forced model-wide:
one training-mode forward of ResNet-50 (batch 16, 64 px) under the heuristic and under each
candidate; per BN layer, the relative change of the running-statistic update.

    python tools/variant_model_check.py [--cfgs 8,9] [--model resnet50]
"""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext, tuning  # noqa: E402
from ddp_classification_pytorch_amd.models import build_model  # noqa: E402
from ddp_classification_pytorch_amd.models.layers import BatchNorm2d  # noqa: E402
from ddp_classification_pytorch_amd.ops import functional as Fn  # noqa: E402
from tests.test_autotune_variants_gpu import TG, TG_SLOTS  # noqa: E402


def run(K, base, imgs, cfg, perturb=0.0):
    tuning.apply(K, "", reset=True)
    for sl, v in zip(TG_SLOTS, cfg):
        K.set_tuning(tuning.slot(sl), int(v))
    m = copy.deepcopy(base)
    if perturb:
        g = torch.Generator(device=imgs.device).manual_seed(5)
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(1.0 + perturb * torch.randn(p.shape, device=p.device, generator=g))
    x = Fn.to_device_nhwc(imgs, cpad=8, nchw=True)
    with torch.no_grad():
        out = m(x)
    torch.cuda.synchronize()
    tuning.apply(K, "", reset=True)
    return out, {n: (b.running_mean.clone(), b.running_var.clone()) for n, b in m.named_modules()
                 if isinstance(b, BatchNorm2d)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default=",".join(str(i) for i in range(1, len(TG))) + ",p24,p30")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=64)
    a = ap.parse_args()
    K = _ext.hip_ops()
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    base = build_model(a.model, num_classes=100).to(dev)
    imgs = torch.randn(a.batch, 3, a.size, a.size, device=dev)
    o0, s0 = run(K, base, imgs, TG[0])
    for cs in a.cfgs.split(","):
        # "p<e>": the heuristic with every weight perturbed by 2^-e relative (fp32 rounding yardstick)
        ci = 0 if cs.startswith("p") else int(cs)
        o, s = run(K, base, imgs, TG[ci], perturb=2.0 ** -int(cs[1:]) if cs.startswith("p") else 0.0)
        worst = []
        for n, (rm, rv) in s.items():
            rm0, rv0 = s0[n]
            # the update's size: running = 0.9 old + 0.1 batch -> compare the batch parts
            d = max(((rm - rm0).norm() / (rm0.norm() + 1e-12)).item(), ((rv - rv0).norm() / (rv0 - 0.9).norm()).item())
            worst.append((d, n))
        worst.sort(reverse=True)
        first = next(((d, n) for n, (d2, _) in zip(s.keys(), [(0, 0)] * len(s)) for d, nn in [(max(
            ((s[n][0] - s0[n][0]).norm() / (s0[n][0].norm() + 1e-12)).item(), 0.0), n)] if d > 1e-5), None)
        print(f"cfg {cs} {TG[ci]}: out relerr {((o - o0).float().norm() / o0.float().norm()).item():.2e}; "
              f"first BN with a changed mean: {first}; worst: " +
              ", ".join(f"{n} {d:.1e}" for d, n in worst[:4]), flush=True)


if __name__ == "__main__":
    main()
