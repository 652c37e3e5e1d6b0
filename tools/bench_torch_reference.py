#!/usr/bin/env python3
"""Comparison point: the reference's software stack on the same MI355X.

The reference trains torchvision ResNet-50 with plain PyTorch (cuDNN on
CUDA; MIOpen + hipBLASLt on ROCm), fp32, DDP.  torchvision is not installed
here, so this builds the standard ResNet-50 v1.5 from torch.nn modules and
runs the same synthetic step as bench.py in the most favourable stock-PyTorch
configuration (channels_last + bf16 autocast + foreach SGD) — i.e. what a
user of the reference gets on MI355X without this framework.

    python tools/bench_torch_reference.py --batch 256 --steps 20
"""
import argparse
import json
import time

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    def __init__(self, cin, planes, stride, down):
        super().__init__()
        self.c1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.b1 = nn.BatchNorm2d(planes)
        self.c2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(planes)
        self.c3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.b3 = nn.BatchNorm2d(planes * 4)
        self.down = nn.Sequential(nn.Conv2d(cin, planes * 4, 1, stride, bias=False),
                                  nn.BatchNorm2d(planes * 4)) if down else None
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        r = x if self.down is None else self.down(x)
        y = self.relu(self.b1(self.c1(x)))
        y = self.relu(self.b2(self.c2(y)))
        return self.relu(self.b3(self.c3(y)) + r)


class ResNet50(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                                  nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for planes, n, s in [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]:
            for i in range(n):
                layers.append(Bottleneck(cin, planes, s if i == 0 else 1, i == 0))
                cin = planes * 4
        self.layers = nn.Sequential(*layers)
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        return self.fc(torch.flatten(self.pool(self.layers(self.stem(x))), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--fp32", action="store_true", help="reference-exact fp32 (no autocast)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    model = ResNet50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    lossf = nn.CrossEntropyLoss()
    imgs = torch.randint(0, 256, (a.batch, 3, 224, 224), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 1000, (a.batch,), device=dev)
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev).view(1, 3, 1, 1) * 255
    std = torch.tensor([0.229, 0.224, 0.225], device=dev).view(1, 3, 1, 1) * 255

    def step():
        x = ((imgs.float() - mean) / std).contiguous(memory_format=torch.channels_last)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=not a.fp32):
            loss = lossf(model(x), labels)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for i in range(a.warmup):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        # MIOpen's find pass at a new batch can run minutes: keep the log moving
        print(f"warmup step {i}: {time.perf_counter() - t0:.1f}s", flush=True)
    t = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(json.dumps({"stack": "stock PyTorch-ROCm (MIOpen/hipBLASLt) " + ("fp32" if a.fp32 else "bf16 autocast"),
                      "images_per_s": round(a.batch * a.steps / dt, 1), "ms_per_step": round(dt / a.steps * 1e3, 2),
                      "batch": a.batch, "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
