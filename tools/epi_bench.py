#!/usr/bin/env python3
"""Timing of the dgrad + fused BN-backward epilogue (conv_dgrad_bn) on the ResNet-50 b512
1x1 shapes, against the plain dgrad of the same shape, under kernel tuning configs:
    python tools/epi_bench.py ",2=3"        (2=3: k-loop ablated -> epilogue cost alone)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402
from ddp_classification_pytorch_amd.tuning import slot as tslot  # noqa: E402
from tools.ew_bench import timeit  # noqa: E402

# (H, C = BN channels / dgrad output, Co = conv output channels / dgrad input, res+add)
SHAPES = [(56, 256, 64, True), (28, 512, 128, True), (14, 1024, 256, True), (56, 64, 256, False),
          (28, 128, 512, False)]


def main():
    K = _ext.hip_ops()
    cfgs = (sys.argv[1] if len(sys.argv) > 1 else "").split(",")
    N = 512
    for H, C, Co, full in SHAPES:
        w = torch.randn(Co, 1, 1, C, device="cuda") / C ** 0.5
        _, wt = K.weight_prep(w, 0, True)
        dy = torch.randn(N, H, H, Co, device="cuda").bfloat16()
        y = torch.randn(N, H, H, C, device="cuda").bfloat16()
        add = torch.randn(N, H, H, C, device="cuda").bfloat16() if full else None
        r = torch.randn(N, H, H, C, device="cuda").bfloat16() if full else None
        v = [torch.rand(C, device="cuda") + 0.5 for _ in range(4)]
        mask = K.bn_act_mask(y, r, v[0], v[1], 1, 0.0)[1] if full else None
        S = N * H * H * C * 2
        for cfg in cfgs:
            for i in range(16):
                K.set_tuning(i, 0)
            for kv in filter(None, cfg.split(";")):
                i, val = kv.split("=")
                K.set_tuning(tslot(i), int(val))
            t_bn = min(timeit(lambda: K.conv_dgrad_bn(dy, wt, 0, add, y, None if full else r, *v, 1, mask))
                       for _ in range(3))
            t_pl = min(timeit(lambda: K.conv_dgrad(dy, wt, H, H, 1, 0, add)) for _ in range(3))
            nb = dy.numel() * 2 + S * (3 if full else 2) + (S // 16 if full else 0)
            print(f"H{H} C{C} Co{Co} {'res+add' if full else 'plain  '} cfg={cfg or 'default':10s} "
                  f"dgrad_bn {t_bn:7.1f}us ({nb / t_bn / 1e6:4.2f} TB/s)  plain dgrad {t_pl:7.1f}us", flush=True)
    for i in range(16):
        K.set_tuning(i, 0)


if __name__ == "__main__":
    main()
