"""Pretrained-weight loading from LOCAL files (no network).

The reference downloads torchvision / timm / model-zoo weights
(BASELINE/main.py:135,144; NESTED/model/imagenet_resnet.py:16-22,179-224).
Here a torchvision-format ResNet ``state_dict`` file (``.pth`` loaded with
``weights_only=True``, or ``.safetensors``) is mapped onto our NHWC modules:
conv weights are permuted [Co,Ci,KH,KW] -> [Co,KH,KW,Ci] by
``Conv2d._load_from_state_dict``; ``fc.*`` is skipped when the class count
differs.  Returns the (missing, unexpected) key lists.
"""
from __future__ import annotations

import os

import torch


def read_state_dict(path: str):
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        return load_file(path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    for k in ("state_dict", "model", "net"):
        if isinstance(sd, dict) and k in sd and isinstance(sd[k], dict):
            sd = sd[k]
    return {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}


def load_pretrained(model: torch.nn.Module, path: str, strict: bool = False):
    if not os.path.exists(path):
        raise FileNotFoundError(f"pretrained weights not found: {path} (downloads are disabled)")
    sd = read_state_dict(path)
    own = model.state_dict()
    filtered = {}
    for k, v in sd.items():
        if k not in own:
            continue
        tgt = own[k]
        if v.shape == tgt.shape or (v.dim() == 4 and v.permute(0, 2, 3, 1).shape == tgt.shape):
            filtered[k] = v
        elif v.dim() == 4 and tgt.dim() == 4 and v.shape[1] < tgt.shape[3]:
            filtered[k] = torch.nn.functional.pad(v.permute(0, 2, 3, 1), (0, tgt.shape[3] - v.shape[1]))
    res = model.load_state_dict(filtered, strict=strict)
    return res.missing_keys, res.unexpected_keys
