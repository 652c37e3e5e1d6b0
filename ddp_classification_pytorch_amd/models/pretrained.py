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
import re

import torch

# reference CIFAR ResNet (NESTED/model/cifar_resnet.py:11-131) -> torchvision-style names
_CIFAR_RES_FN = {"0": "conv1", "1": "bn1", "3": "conv2", "4": "bn2", "6": "conv3", "7": "bn3"}


def remap_reference_keys(sd: dict) -> dict:
    """Map the reference's own parameter names onto ours (checkpoint interop, ``--resumePth``):

    * NESTED ``NetFeat`` (NESTED/model/model.py:12-42) keeps its backbone in a Sequential
      ``feat_net``: CIFAR ``feat_net.0`` = conv1 (Sequential conv, BN), ``feat_net.1..4`` =
      conv2_x..conv5_x; ImageNet ``feat_net.0/1`` = conv1 / bn1, ``feat_net.4..7`` = layer1..4;
    * CIFAR ResNet names (NESTED/model/cifar_resnet.py:84-95): ``conv1.{0,1}`` -> conv1 / bn1,
      ``convK_x.i.residual_function.{0,1,3,4,6,7}`` -> ``layer{K-1}.i.{conv1,bn1,conv2,bn2,conv3,bn3}``,
      ``shortcut.{0,1}`` -> ``downsample.{0,1}``;
    * a ``module.`` (DataParallel / DDP) prefix is dropped;
    * 4-D conv weights go from the torch layout [Co,Ci,KH,KW] to ours [Co,KH,KW,Ci] here, explicitly:
      Conv2d's shape-based permute cannot tell the two apart when Ci == KH == KW (the CIFAR stem's
      3x3 conv over 3 channels).
    Keys already in our naming pass through unchanged."""
    out = {}
    cifar_feat = any(re.match(r"(module\.)?feat_net\.\d+\.\d+\.(residual_function|shortcut)", k) for k in sd)
    for k, v in sd.items():
        if k.startswith("module."):
            k = k[len("module."):]
        m = re.match(r"feat_net\.(\d+)\.(.*)", k)
        if m:
            i, rest = int(m.group(1)), m.group(2)
            if cifar_feat:
                k = ("conv1" if i == 0 else f"conv{i + 1}_x") + "." + rest
            else:
                names = {0: "conv1", 1: "bn1", 4: "layer1", 5: "layer2", 6: "layer3", 7: "layer4"}
                if i not in names:
                    continue
                k = names[i] + "." + rest
        m = re.match(r"conv1\.([01])\.(.*)", k)
        if m:
            k = ("conv1." if m.group(1) == "0" else "bn1.") + m.group(2)
        m = re.match(r"conv([2-5])_x\.(\d+)\.(residual_function|shortcut)\.(\d+)\.(.*)", k)
        if m:
            stage, blk, part, idx, rest = m.groups()
            if part == "residual_function":
                if idx not in _CIFAR_RES_FN:
                    continue
                sub = _CIFAR_RES_FN[idx]
            else:
                sub = f"downsample.{idx}"
            k = f"layer{int(stage) - 1}.{blk}.{sub}.{rest}"
        if v.dim() == 4 and k.endswith("weight"):
            v = v.permute(0, 2, 3, 1).contiguous()
        out[k] = v
    return out


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
    sd = remap_reference_keys(read_state_dict(path))
    own = model.state_dict()
    filtered = {}
    for k, v in sd.items():
        if k not in own:
            continue
        tgt = own[k]
        if v.shape == tgt.shape:
            filtered[k] = v
        elif v.dim() == 4 and tgt.dim() == 4 and v.shape[:3] == tgt.shape[:3] and v.shape[3] < tgt.shape[3]:
            filtered[k] = torch.nn.functional.pad(v, (0, tgt.shape[3] - v.shape[3]))  # zero-padded input channels
    res = model.load_state_dict(filtered, strict=strict)
    return res.missing_keys, res.unexpected_keys
