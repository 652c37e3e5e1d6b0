"""Pretrained-weight loading from LOCAL files (no network).

The reference downloads its weights (BASELINE/main.py:135 torchvision ``resnet50(pretrained=True)``,
BASELINE/main.py:143-144 timm ``tresnet_m_miil_in21k`` -- the BASELINE default model --
NESTED/model/vgg.py:17 torchvision ``vgg19_bn``, NESTED/model/imagenet_resnet.py:16-22,179-224
model-zoo ResNets).  Here a local ``.pth`` (``weights_only=True``) or ``.safetensors`` file in any
of those formats is mapped onto our NHWC modules:

* **ResNet / ResNeXt** (torchvision, the reference's own ResNets and NetFeat checkpoints): names
  map 1:1 (reference ``feat_net.*`` / CIFAR ``convK_x`` names through :func:`remap_reference_keys`);
* **TResNet-M** (timm): both the original inplace_abn checkpoints (``body.conv1.0`` conv,
  ``body.conv1.1`` InplaceABN, ``conv1.0.0`` under an anti-alias Sequential, ``downsample.1.0``
  behind the AvgPool) and the later timm format (``conv1.conv`` / ``conv1.bn`` BatchNorm, whose
  weight is inplace_abn's effective ``|gamma| + eps``); SE ``fc1``/``fc2`` 1x1 convs become our
  Linear weights; ``head.fc`` -> ``fc``;
* **VGG19-bn** (torchvision ``features.N`` / ``classifier.{0,3,6}``, also the reference NetFeat's
  ``feat_net.`` / ``forward1.0`` / ``forward2.0`` names): conv/BN indices map onto ``convs.k``,
  and fc1's columns are permuted from torch's (C, H, W) flatten order to our NHWC (H, W, C) order.

Conv weights go from the torch layout [Co, Ci, KH, KW] to ours [Co, KH, KW, Ci] when the FILE is
in torch layout: decided per file from the 4-D tensors whose shape tells the two apart, and then
applied to the ambiguous ones too (Ci == KH == KW, e.g. a 3x3 conv over 3 channels).  A state_dict
saved by this framework passes through unpermuted.

:func:`load_pretrained` fails loudly: it raises when fewer than ``min_match`` (90 %) of the target's
tensors received a value (a wrong file, a wrong family, an unknown naming), instead of training
from random weights without a word.  It returns (missing, unexpected, matched fraction).
"""
from __future__ import annotations

import os
import re

import torch

# reference CIFAR ResNet (NESTED/model/cifar_resnet.py:11-131) -> torchvision-style names
_CIFAR_RES_FN = {"0": "conv1", "1": "bn1", "3": "conv2", "4": "bn2", "6": "conv3", "7": "bn3"}
IABN_EPS = 1e-5


def remap_reference_keys(sd: dict, torch_layout: bool = True) -> dict:
    """Map the reference's own parameter names onto ours (checkpoint interop, ``--resumePth``):

    * NESTED ``NetFeat`` (NESTED/model/model.py:12-42) keeps its backbone in a Sequential
      ``feat_net``: CIFAR ``feat_net.0`` = conv1 (Sequential conv, BN), ``feat_net.1..4`` =
      conv2_x..conv5_x; ImageNet ``feat_net.0/1`` = conv1 / bn1, ``feat_net.4..7`` = layer1..4;
    * CIFAR ResNet names (NESTED/model/cifar_resnet.py:84-95): ``conv1.{0,1}`` -> conv1 / bn1,
      ``convK_x.i.residual_function.{0,1,3,4,6,7}`` -> ``layer{K-1}.i.{conv1,bn1,conv2,bn2,conv3,bn3}``,
      ``shortcut.{0,1}`` -> ``downsample.{0,1}``;
    * a ``module.`` (DataParallel / DDP) prefix is dropped;
    * ``torch_layout``: the file holds 4-D conv weights in the torch layout [Co,Ci,KH,KW] (every
      reference / torchvision file does): they are permuted to ours [Co,KH,KW,Ci] here, explicitly,
      since Conv2d's shape-based permute cannot tell the two apart when Ci == KH == KW (the CIFAR
      stem's 3x3 conv over 3 channels).  A file of our own layout passes ``torch_layout=False``.
    Keys already in our naming keep their names."""
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
        if torch_layout and v.dim() == 4 and k.endswith("weight"):
            v = v.permute(0, 2, 3, 1).contiguous()
        out[k] = v
    return out


# ----------------------------------------------------------------------------- timm TResNet
def _tresnet_key(k: str):
    """timm TResNet name -> (our name, kind) or None; kind is 'conv', 'bn', 'lin' or 'other'."""
    k = k[len("module."):] if k.startswith("module.") else k
    if k.startswith("head.fc."):
        return "fc." + k[len("head.fc."):], "lin"
    if k.startswith("fc."):
        return k, "lin"
    if not k.startswith("body."):
        return None
    k = k[len("body."):]
    m = re.match(r"conv1\.(?:0\.|conv\.)(weight)$", k)
    if m:
        return "stem.conv.weight", "conv"
    m = re.match(r"conv1\.(?:1\.|bn\.)(.*)$", k)
    if m:
        return "stem.bn." + m.group(1), "bn"
    m = re.match(r"(layer\d\.\d+)\.(.*)$", k)
    if not m:
        return None
    blk, rest = m.groups()
    m = re.match(r"se\.(fc[12])\.(weight|bias)$", rest)
    if m:
        return f"{blk}.se.{m.group(1)}.{m.group(2)}", "lin"
    # downsample: [AvgPool,] conv2d_iabn  ->  downsample.{0|1}.{0,1}  or  downsample.{0|1}.{conv,bn}
    m = re.match(r"downsample\.\d+\.(0|1|conv|bn)\.(.*)$", rest)
    if m:
        part = "conv" if m.group(1) in ("0", "conv") else "bn"
        return f"{blk}.downsample.conv.{part}.{m.group(2)}", part
    # convN: conv2d_iabn = (conv, iabn) -> convN.{0,1}; with anti-alias Sequential(conv2d_iabn, aa)
    # -> convN.0.{0,1}; later timm: convN.{conv,bn}
    m = re.match(r"(conv\d)\.(?:0\.)?(0|1|conv|bn)\.(.*)$", rest)
    if m:
        conv, part, tail = m.groups()
        part = "conv" if part in ("0", "conv") else "bn"
        if part == "conv" and tail != "weight":
            return None
        return f"{blk}.{conv}.{part}.{tail}", part
    return None


def convert_timm_tresnet(model: torch.nn.Module, sd: dict) -> dict:
    """timm TResNet state_dict -> ours (names; SE 1x1 convs -> Linear; BN weight semantics).

    The inplace_abn checkpoints store the raw gamma of every BN (the effective weight is
    |gamma| + eps everywhere); later timm stores the BatchNorm weight |gamma| + eps.  Our layers with
    ``inplace_abn`` set apply |w| + eps themselves; the others are plain BN.  So: plain layer <-
    |gamma| + eps (old format) or the weight as is (new format); inplace_abn layer <- gamma (old) or
    weight - eps (new, exact since that weight is >= eps)."""
    from .layers import BatchNorm2d

    new_format = any(".bn." in k or k.endswith("conv1.conv.weight") for k in sd)
    iabn = {n for n, m in model.named_modules() if isinstance(m, BatchNorm2d) and m.inplace_abn}
    out = {}
    for k, v in sd.items():
        r = _tresnet_key(k)
        if r is None:
            continue
        name, kind = r
        if kind == "lin" and v.dim() == 4:  # SE fc1 / fc2: 1x1 convs [out, in, 1, 1]
            v = v.reshape(v.shape[0], v.shape[1])
        if kind == "bn" and name.endswith(".weight"):
            mod = name[: -len(".weight")]
            if mod in iabn:
                v = v - IABN_EPS if new_format else v
            else:
                v = v if new_format else v.abs() + IABN_EPS
        out[name] = v
    return out


# ----------------------------------------------------------------------------- torchvision VGG
def convert_torchvision_vgg(model: torch.nn.Module, sd: dict) -> dict:
    """torchvision vgg19_bn (or the reference NESTED NetFeat wrapping it) -> our VGG.

    ``features``: for every conv of the config, the conv index and the BN right after it;
    ``classifier.0 / .3 / .6`` (NetFeat: ``forward1.0`` / ``forward2.0``) -> fc1 / fc2 / fc3, fc1's
    columns permuted from the (C, 7, 7) flatten to our (7, 7, C) one."""
    plan = getattr(model, "plan", None)
    if plan is None and hasattr(model, "net"):
        model, plan = model.net, model.net.plan
    idx, conv_at = 0, {}
    for k, item in enumerate(plan):
        if item == "M":
            idx += 1
        else:
            conv_at[idx] = sum(1 for x in plan[:k] if x != "M")
            idx += 3  # conv, BN, ReLU
    prefix = "net." if hasattr(model, "net") else ""
    out, conv_bias = {}, {}
    for k, v in sd.items():
        k = k[len("module."):] if k.startswith("module.") else k
        k = k[len("feat_net."):] if k.startswith("feat_net.") else k
        m = re.match(r"features\.(\d+)\.(.*)$", k)
        if m:
            i, rest = int(m.group(1)), m.group(2)
            if i in conv_at and rest == "bias":
                conv_bias[conv_at[i]] = v  # our convs feeding BN carry no bias: folded below
            elif i in conv_at:
                out[f"{prefix}convs.{conv_at[i]}.conv.{rest}"] = v
            elif i - 1 in conv_at:
                out[f"{prefix}convs.{conv_at[i - 1]}.bn.{rest}"] = v
            continue
        m = re.match(r"(?:classifier\.(\d)|forward1\.(0)|forward2\.(0))\.(weight|bias)$", k)
        if m:
            ci = m.group(1)
            fc = {"0": "fc1", "3": "fc2", "6": "fc3"}.get(ci) if ci is not None else ("fc1" if m.group(2) else "fc2")
            if fc == "fc1" and m.group(4) == "weight" and v.dim() == 2 and v.shape[1] % 49 == 0:
                C = v.shape[1] // 49
                v = v.reshape(v.shape[0], C, 7, 7).permute(0, 2, 3, 1).reshape(v.shape[0], -1)
            out[f"{prefix}{fc}.{m.group(4)}"] = v
    # BN(conv(x) + b) == BN'(conv(x)) with running_mean' = running_mean - b (batch statistics:
    # the bias cancels exactly; running statistics: it moves the mean by b)
    for c, b in conv_bias.items():
        rm = out.get(f"{prefix}convs.{c}.bn.running_mean")
        if rm is not None:
            out[f"{prefix}convs.{c}.bn.running_mean"] = rm - b
    return out


# ----------------------------------------------------------------------------- loading
def read_state_dict(path: str):
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        return load_file(path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and sd.get("format") == "dcp-ckpt-v1":  # our own checkpoint: its model
        models = sd.get("models", {})
        sd = models.get("model", next(iter(models.values()), {}))
        return {k: v for k, v in sd.items()}
    for k in ("state_dict", "model", "net"):
        if isinstance(sd, dict) and k in sd and isinstance(sd[k], dict):
            sd = sd[k]
    return {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}


def file_is_torch_layout(sd: dict, own: dict) -> bool:
    """Does this file hold 4-D conv weights as [Co, Ci, KH, KW]?  Voted by the tensors whose
    target shape tells the two layouts apart; a file with none (only ambiguous convs) is treated
    as torch layout, which every external source uses."""
    torch_votes = ours_votes = 0
    for k, v in sd.items():
        t = own.get(k)
        if t is None or v.dim() != 4 or t.dim() != 4:
            continue
        direct = tuple(v.shape) == tuple(t.shape)
        perm = tuple(v.permute(0, 2, 3, 1).shape) == tuple(t.shape)
        if perm and not direct:
            torch_votes += 1
        elif direct and not perm:
            ours_votes += 1
    return torch_votes >= ours_votes


def _family(model):
    names = {type(m).__name__ for m in model.modules()}
    if "TResNet" in names:
        return "tresnet"
    if "VGG" in names:
        return "vgg"
    return "resnet"


def convert_state_dict(model: torch.nn.Module, sd: dict) -> dict:
    """Any supported external / reference / own state_dict -> names and layouts of ``model``."""
    fam = _family(model)
    if fam == "tresnet" and any(k.startswith(("body.", "module.body.")) for k in sd):
        sd = convert_timm_tresnet(model, sd)
    elif fam == "vgg" and any(re.match(r"(module\.)?(feat_net\.)?(features|classifier|forward[12])\.", k)
                              for k in sd):
        sd = convert_torchvision_vgg(model, sd)
    own = model.state_dict()
    named = remap_reference_keys(sd, torch_layout=False)
    torch_layout = file_is_torch_layout(named, own)
    if torch_layout:
        named = {k: (v.permute(0, 2, 3, 1).contiguous() if v.dim() == 4 and k.endswith("weight") else v)
                 for k, v in named.items()}
    return named


def load_pretrained(model: torch.nn.Module, path: str, strict: bool = False, min_match: float = 0.9):
    """Load a local weights file into ``model``; raises when fewer than ``min_match`` of the model's
    tensors (``num_batches_tracked`` counters aside) received a value.  Tensors whose shape differs
    (a classifier over another class count) are skipped; an input-channel dimension smaller than
    ours is zero-padded (the stem's 3 -> 8 channels).  Returns (missing, unexpected, fraction)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"pretrained weights not found: {path} (downloads are disabled)")
    sd = convert_state_dict(model, read_state_dict(path))
    own = model.state_dict()
    filtered = {}
    for k, v in sd.items():
        if k not in own:
            continue
        tgt = own[k]
        if v.shape == tgt.shape:
            filtered[k] = v.to(tgt.dtype)
        elif v.dim() == 4 and tgt.dim() == 4 and v.shape[:3] == tgt.shape[:3] and v.shape[3] < tgt.shape[3]:
            filtered[k] = torch.nn.functional.pad(v, (0, tgt.shape[3] - v.shape[3])).to(tgt.dtype)
    counted = [k for k in own if not k.endswith("num_batches_tracked")]
    frac = sum(1 for k in counted if k in filtered) / max(1, len(counted))
    if frac < min_match:
        unmatched = [k for k in counted if k not in filtered][:8]
        raise RuntimeError(f"load_pretrained({path}): only {100 * frac:.1f}% of the {type(model).__name__}'s "
                           f"{len(counted)} tensors matched the file (need {100 * min_match:.0f}%); first unmatched: "
                           f"{unmatched}")
    res = model.load_state_dict(filtered, strict=strict)
    return res.missing_keys, res.unexpected_keys, frac
