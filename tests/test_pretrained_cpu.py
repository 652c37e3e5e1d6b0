"""Pretrained loading for the reference's model families from synthesized local files (no network,
no timm / torchvision installed): timm TResNet-M in both checkpoint formats (the BASELINE default
``tresnet_m_miil_in21k``, BASELINE/main.py:143-144), torchvision VGG19-bn (NESTED/model/vgg.py:17,
including the reference NetFeat's names), torchvision ResNets; plus the loud failure on a file that
does not fit, and our own (already NHWC) state_dicts passing through unpermuted."""
import pytest
import torch

from ddp_classification_pytorch_amd.models import build_model
from ddp_classification_pytorch_amd.models.layers import BatchNorm2d
from ddp_classification_pytorch_amd.models.pretrained import IABN_EPS, load_pretrained


def _randomize(model, seed=0):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, BatchNorm2d):
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)  # positive: |w| == w
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
    return model


def _tv(w):  # our conv layout [Co, KH, KW, Ci] -> torch [Co, Ci, KH, KW]
    return w.detach().permute(0, 3, 1, 2).contiguous()


def _timm_tresnet_sd(model, new_format):
    """The state_dict timm's TResNet would hold for these weights: old format = the original
    inplace_abn model (every BN an InplaceABN storing raw gamma, convs in nn.Sequential (conv, iabn),
    anti-aliased convs wrapped once more); new format = ConvNormAct (conv / bn, BN weight = |gamma| + eps)."""
    sd = {}

    def put(prefix, cbn, aa=False):
        bn = cbn.bn
        eff = bn.weight.detach().abs() + IABN_EPS if bn.inplace_abn else bn.weight.detach()
        if new_format:
            c, b = prefix + "conv.", prefix + "bn."
            sd[b + "num_batches_tracked"] = torch.tensor(3)
            w = eff
        else:
            c, b = (prefix + "0.0.", prefix + "0.1.") if aa else (prefix + "0.", prefix + "1.")
            w = bn.weight.detach() if bn.inplace_abn else eff - IABN_EPS  # raw gamma with |g| + eps == eff
        sd[c + "weight"] = _tv(cbn.conv.weight)
        sd[b + "weight"] = w.clone()
        for n in ("bias", "running_mean", "running_var"):
            sd[b + n] = getattr(bn, n).detach().clone()

    put("body.conv1.", model.stem)
    for li in range(1, 5):
        for bi, blk in enumerate(getattr(model, f"layer{li}")):
            p = f"body.layer{li}.{bi}."
            basic = type(blk).__name__ == "TBasicBlock"
            put(p + "conv1.", blk.conv1, aa=basic and blk.aa is not None)
            put(p + "conv2.", blk.conv2, aa=(not basic) and blk.aa is not None)
            if not basic:
                put(p + "conv3.", blk.conv3)
            if blk.se is not None:
                for fc in ("fc1", "fc2"):
                    lin = getattr(blk.se, fc)
                    sd[p + f"se.{fc}.weight"] = lin.weight.detach()[:, :, None, None].clone()
                    sd[p + f"se.{fc}.bias"] = lin.bias.detach().clone()
            if blk.downsample is not None:
                put(p + "downsample.1.", blk.downsample.conv)
    sd["head.fc.weight"] = model.fc.weight.detach().clone()
    sd["head.fc.bias"] = model.fc.bias.detach().clone()
    return sd


@pytest.mark.parametrize("new_format", [False, True])
def test_timm_tresnet_checkpoint_loads(tmp_path, new_format):
    torch.manual_seed(0)
    src = _randomize(build_model("tresnet_m", num_classes=11))
    f = tmp_path / "tresnet.pth"
    torch.save({"state_dict": _timm_tresnet_sd(src, new_format)}, f)
    torch.manual_seed(5)
    dst = build_model("tresnet_m", num_classes=11)
    missing, unexpected, frac = load_pretrained(dst, str(f))
    assert frac == 1.0, missing
    want = src.state_dict()
    for k, v in dst.state_dict().items():
        if k.endswith("num_batches_tracked"):
            continue
        assert torch.allclose(v, want[k], atol=2e-7), k
    # a different class count: the head is skipped, everything else loads
    other = build_model("tresnet_m", num_classes=7)
    _, _, frac7 = load_pretrained(other, str(f))
    assert 0.98 < frac7 < 1.0


def test_torchvision_vgg_checkpoint_loads(tmp_path):
    torch.manual_seed(0)
    src = _randomize(build_model("vgg19_bn", num_classes=10))
    sd, idx, k = {}, 0, 0
    g = torch.Generator().manual_seed(3)
    biases = {}
    for item in src.plan:
        if item == "M":
            idx += 1
            continue
        cbn = src.convs[k]
        b = torch.randn(cbn.conv.out_channels, generator=g) * 0.1  # torchvision convs have a bias
        biases[k] = b
        sd[f"features.{idx}.weight"] = _tv(cbn.conv.weight)
        sd[f"features.{idx}.bias"] = b
        for n in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
            t = getattr(cbn.bn, n).detach().clone()
            sd[f"features.{idx + 1}.{n}"] = t + b if n == "running_mean" else t
        idx, k = idx + 3, k + 1
    fc1 = src.fc1.weight.detach()  # ours: columns in (h, w, c) order -> torchvision's (c, h, w)
    sd["classifier.0.weight"] = fc1.reshape(4096, 7, 7, 512).permute(0, 3, 1, 2).reshape(4096, -1).clone()
    sd["classifier.0.bias"] = src.fc1.bias.detach().clone()
    sd["classifier.3.weight"] = src.fc2.weight.detach().clone()
    sd["classifier.3.bias"] = src.fc2.bias.detach().clone()
    sd["classifier.6.weight"] = torch.randn(1000, 4096)  # ImageNet head: skipped (10 classes here)
    sd["classifier.6.bias"] = torch.randn(1000)
    f = tmp_path / "vgg19_bn.pth"
    torch.save(sd, f)
    dst = build_model("vgg19_bn", num_classes=10)
    _, _, frac = load_pretrained(dst, str(f))
    assert frac > 0.95
    want = src.state_dict()
    for k2, v in dst.state_dict().items():
        if k2.startswith("fc3") or k2.endswith("num_batches_tracked"):
            continue
        assert torch.allclose(v, want[k2], atol=1e-6), k2
    # the reference NetFeat's names (feat_net.features / forward1.0 / forward2.0) load the same
    from ddp_classification_pytorch_amd.models.vgg import VGGNetFeat

    ref = {("feat_net." + kk): v for kk, v in sd.items() if not kk.startswith("classifier.6")}
    ref["forward1.0.weight"] = ref.pop("feat_net.classifier.0.weight")
    ref["forward1.0.bias"] = ref.pop("feat_net.classifier.0.bias")
    ref["forward2.0.weight"] = ref.pop("feat_net.classifier.3.weight")
    ref["forward2.0.bias"] = ref.pop("feat_net.classifier.3.bias")
    f2 = tmp_path / "netfeat.pth"
    torch.save(ref, f2)
    nf = VGGNetFeat(pretrained=str(f2))
    assert torch.equal(nf.net.fc1.weight, dst.fc1.weight) and torch.equal(nf.net.convs[3].conv.weight,
                                                                          dst.convs[3].conv.weight)


def test_torchvision_vgg_fc1_permutation_matches_flatten():
    """fc1 over our NHWC flatten == torchvision's fc1 over the NCHW flatten of the same map."""
    from ddp_classification_pytorch_amd.models.pretrained import convert_torchvision_vgg

    m = build_model("vgg19_bn", num_classes=0)
    w = torch.randn(16, 512 * 49)
    ours = convert_torchvision_vgg(m, {"classifier.0.weight": w})["fc1.weight"]
    fmap = torch.randn(2, 512, 7, 7)
    assert torch.allclose(fmap.flatten(1) @ w.t(), fmap.permute(0, 2, 3, 1).flatten(1) @ ours.t(), rtol=1e-4, atol=1e-3)


def test_wrong_file_fails_loudly(tmp_path):
    """A file of another family (here a ResNet-18 for a TResNet) must not train from random
    weights silently."""
    sd = build_model("resnet18", num_classes=0).state_dict()
    f = tmp_path / "r18.pth"
    torch.save(sd, f)
    with pytest.raises(RuntimeError, match="tensors matched"):
        load_pretrained(build_model("tresnet_m", num_classes=10), str(f))
    with pytest.raises(RuntimeError, match="tensors matched"):
        load_pretrained(build_model("resnet50", num_classes=0), str(f))


def test_own_layout_state_dict_is_not_permuted(tmp_path):
    """A state_dict saved by this framework (convs already [Co, KH, KW, Ci]) and one of our
    checkpoints both load unchanged (the permute is decided per file, not per key)."""
    torch.manual_seed(0)
    src = build_model("resnet18", num_classes=0)
    f = tmp_path / "own.pth"
    torch.save(src.state_dict(), f)
    dst = build_model("resnet18", num_classes=0)
    _, _, frac = load_pretrained(dst, str(f))
    assert frac == 1.0
    for k, v in src.state_dict().items():
        assert torch.equal(dst.state_dict()[k], v), k
    ck = tmp_path / "last.pth"
    torch.save({"format": "dcp-ckpt-v1", "models": {"model": src.state_dict()}}, ck)
    dst2 = build_model("resnet18", num_classes=0)
    load_pretrained(dst2, str(ck))
    assert torch.equal(dst2.layer2[0].conv1.weight, src.layer2[0].conv1.weight)
