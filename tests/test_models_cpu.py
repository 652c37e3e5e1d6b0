"""Model zoo: parameter counts (SURVEY.md §2.5.1 / torchvision / timm), shapes,
reference smoke test (NESTED/model/model.py:79-90), checkpoint formats."""
import pytest
import torch

from ddp_classification_pytorch_amd.models import build_model
from ddp_classification_pytorch_amd.models.heads import ArcMarginProduct, MLPHead, NetClassifier
from ddp_classification_pytorch_amd.models.nested import NetFeat
from ddp_classification_pytorch_amd.ops import functional as Fn


def nparams(m):
    return sum(p.numel() for p in m.parameters())


@pytest.mark.parametrize("name,classes,expected", [
    ("resnet18", 1000, 11_689_512),
    ("resnet50", 1000, 25_557_032),
    ("resnet101", 1000, 44_549_160),
    ("resnet152", 1000, 60_192_808),
    ("resnet34", 1000, 21_797_672),
    ("cifar_resnet18", 100, 11_220_132),
    ("resnext50_32x4d", 1000, 25_028_904),
    ("tresnet_m", 1000, 31_389_032),  # timm tresnet_m
    ("vgg19_bn", 1000, 143_678_248 - 5_504),  # torchvision minus the conv biases BN makes redundant
])
def test_param_counts(name, classes, expected):
    assert nparams(build_model(name, num_classes=classes)) == expected


def test_baseline_head_param_count():
    # ResNet-50 + BASELINE MLP head (2048->512->2173) = 25,671,869 ... minus fc(2048->1000)
    bb = build_model("resnet50", num_classes=0)
    head = MLPHead(2048, 512, 2173)
    assert nparams(bb) + nparams(head) == 23_508_032 + 2048 * 512 + 512 + 512 * 2173 + 2173


@pytest.mark.parametrize("name,size,cpad", [("resnet18", 64, 8), ("resnext50_32x4d", 64, 8), ("tresnet_m", 64, 3),
                                            ("cifar_resnet18", 32, 8)])
def test_forward_backward_shapes(name, size, cpad):
    torch.manual_seed(0)
    m = build_model(name, num_classes=7)
    x = Fn.to_device_nhwc(torch.randn(2, 3, size, size), cpad=cpad)
    y = m(x)
    assert y.shape == (2, 7)
    Fn.cross_entropy(y, torch.tensor([0, 6])).backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters() if p.requires_grad)


def test_reference_nested_smoke():
    """NESTED/model/model.py:79-90: CIFAR NetFeat(resnet18) -> [3,512]; NetClassifier(512,10) -> [3,10]."""
    feat = NetFeat("resnet18", "CIFAR100")
    cls = NetClassifier(feat.feat_dim, 10)
    x = Fn.to_device_nhwc(torch.randn(3, 3, 32, 32), cpad=8)
    f = feat(x)
    assert f.shape == (3, 512)
    assert cls(f).shape == (3, 10)
    assert cls.weight.shape == (512, 10)  # reference layout [feat_dim, nb_cls]


def test_netfeat_freeze_bn():
    feat = NetFeat("resnet18", "Clothing1M")
    feat.train(True, freeze_bn=True)
    bns = [m for m in feat.modules() if m.__class__.__name__ == "BatchNorm2d"]
    assert bns and all(not b.training and not b.weight.requires_grad for b in bns)
    rm = bns[0].running_mean.clone()
    feat(Fn.to_device_nhwc(torch.randn(2, 3, 64, 64), cpad=8))
    assert torch.equal(rm, bns[0].running_mean)  # frozen: running stats untouched


def test_torchvision_layout_state_dict_loads():
    m = build_model("resnet18", num_classes=10)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    # convert our NHWC conv weights to torchvision [Co,Ci,KH,KW] and back through load_state_dict
    tv = {k: (v.permute(0, 3, 1, 2).contiguous() if v.dim() == 4 else v) for k, v in sd.items()}
    m2 = build_model("resnet18", num_classes=10)
    m2.load_state_dict(tv)
    for k, v in m2.state_dict().items():
        assert torch.equal(v, sd[k]), k


def test_arc_margin_reference_formula():
    torch.manual_seed(0)
    arc = ArcMarginProduct(16, 9, s=30, m=0.5, easy_margin=True)
    x = torch.randn(5, 16)
    y = torch.randint(0, 9, (5,))
    logits = arc.margin_logits(x, y)
    loss, rank, out = arc(x, y, return_logits=True)
    assert torch.allclose(out, logits, atol=1e-4)
    assert abs(loss.item() - torch.nn.functional.cross_entropy(logits, y).item()) < 1e-4


def test_resnext_train_and_eval_forward():
    """grouped-conv blocks in both BN modes (training statistics / running statistics)."""
    import torch

    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn

    m = build_model("resnext50_32x4d", num_classes=5)
    x = Fn.to_device_nhwc(torch.randn(2, 3, 64, 64), cpad=8, nchw=True)
    assert m(x).shape == (2, 5)
    m.eval()
    with torch.no_grad():
        assert m(x).shape == (2, 5)


def test_vgg_netfeat_mask_dropout_and_adaptive_pool():
    """NESTED/model/vgg.py NetFeat semantics: any input size (adaptive 7x7 pool), mask1 applied to the
    fc1 activations, no dropout unless vgg_dropout > 0, frozen BN via train(mode, freeze_bn)."""
    import torch.nn.functional as F

    from ddp_classification_pytorch_amd.models.vgg import VGGNetFeat
    from ddp_classification_pytorch_amd.ops import functional as Fn

    torch.manual_seed(0)
    net = VGGNetFeat()
    net.train(True, freeze_bn=True)
    x = Fn.to_device_nhwc(torch.randn(2, 3, 64, 64), cpad=8, nchw=True)
    f1 = net(x)
    assert f1.shape == (2, 4096)
    assert torch.equal(net(x), f1)  # no dropout at vgg_dropout = 0 (deterministic in train mode)
    mask = torch.zeros(1, 4096)
    mask[:, :100] = 1
    f2 = net(x, mask1=mask)
    # reference: relu(fc2(relu(fc1(h)) * mask1))
    h = net.net.forward_conv(x)
    a = F.relu(F.linear(h, net.net.fc1.weight, net.net.fc1.bias)) * mask
    ref = F.relu(F.linear(a, net.net.fc2.weight, net.net.fc2.bias))
    assert torch.allclose(f2, ref, rtol=1e-4, atol=1e-5)
    net_d = VGGNetFeat(vgg_dropout=0.5)
    net_d.load_state_dict(net.state_dict())
    net_d.train(True, freeze_bn=True)
    assert not torch.equal(net_d(x), net_d(x))  # fresh dropout masks per call
    net_d.eval()
    assert torch.allclose(net_d(x), net(x))


def test_adaptive_avg_pool_and_dropout_cpu():
    from ddp_classification_pytorch_amd.ops import functional as Fn

    x = torch.randn(2, 5, 6, 16, requires_grad=True)
    y = Fn.adaptive_avg_pool2d(x, 7, 7)
    ref = torch.nn.functional.adaptive_avg_pool2d(x.detach().permute(0, 3, 1, 2), (7, 7)).permute(0, 2, 3, 1)
    assert torch.allclose(y, ref, atol=1e-6)
    y.sum().backward()
    xr = x.detach().clone().requires_grad_(True)
    torch.nn.functional.adaptive_avg_pool2d(xr.permute(0, 3, 1, 2), (7, 7)).sum().backward()
    assert torch.allclose(x.grad, xr.grad, atol=1e-6)
    z = torch.ones(1000, 64, requires_grad=True)
    d = Fn.dropout(z, 0.25)
    kept = (d != 0).float().mean().item()
    assert 0.72 < kept < 0.78 and torch.allclose(d[d != 0], torch.full_like(d[d != 0], 1 / 0.75))
    d.sum().backward()
    assert torch.equal((z.grad != 0), (d != 0))  # backward regenerates the same mask


def _reference_format_cifar_feat_sd(ours):
    """The NESTED NetFeat state_dict a reference run would save for the CIFAR ResNet-18, written
    from our module's tensors under the reference's names (NESTED/model/model.py:17-25: feat_net =
    Sequential(conv1, conv2_x..conv5_x); NESTED/model/cifar_resnet.py:24-42,84-95: conv1 =
    Sequential(conv, bn, relu), residual_function = (conv, bn, relu, conv, bn), shortcut = (conv,
    bn)) in the torch conv layout [Co, Ci, KH, KW]."""
    sd = {}

    def put(prefix, conv=None, bn=None):
        if conv is not None:
            sd[prefix + "weight"] = conv.weight.detach().permute(0, 3, 1, 2).clone()
        if bn is not None:
            for n in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
                sd[prefix + n] = getattr(bn, n).detach().clone()

    net = ours.net
    put("feat_net.0.0.", conv=net.conv1)
    put("feat_net.0.1.", bn=net.bn1)
    for li, layer in enumerate((net.layer1, net.layer2, net.layer3, net.layer4)):
        for bi, blk in enumerate(layer):
            p = f"feat_net.{li + 1}.{bi}."
            put(p + "residual_function.0.", conv=blk.conv1)
            put(p + "residual_function.1.", bn=blk.bn1)
            put(p + "residual_function.3.", conv=blk.conv2)
            put(p + "residual_function.4.", bn=blk.bn2)
            if blk.downsample is not None:
                put(p + "shortcut.0.", conv=blk.downsample[0])
                put(p + "shortcut.1.", bn=blk.downsample[1])
    return sd


def test_reference_cifar_netfeat_checkpoint_loads():
    """A NESTED-reference checkpoint {'feat': NetFeat (feat_net.*), 'cls': ...} of the CIFAR ResNet-18
    (reference names conv1.0/1, convK_x.i.residual_function.j, shortcut; torch conv layout, including
    the ambiguous 3x3x3 stem) resumes into a fresh NetFeat and computes the same features."""
    import os
    import tempfile

    from ddp_classification_pytorch_amd.engine.checkpoint import load_checkpoint
    from ddp_classification_pytorch_amd.models.heads import NetClassifier
    from ddp_classification_pytorch_amd.models.nested import NetFeat
    from ddp_classification_pytorch_amd.ops import functional as Fn

    torch.manual_seed(0)
    src = NetFeat("resnet18", "CIFAR100")
    g = torch.Generator().manual_seed(1)
    for m in src.modules():
        if hasattr(m, "running_mean"):
            m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
            m.running_var.copy_(torch.rand(m.num_features, generator=g) * 0.5 + 0.75)
    src.eval()
    sd = _reference_format_cifar_feat_sd(src)
    assert "feat_net.1.0.residual_function.0.weight" in sd and sd["feat_net.0.0.weight"].shape == (64, 3, 3, 3)
    cls_w = torch.randn(512, 100)
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "netBest.pth")
        torch.save({"feat": sd, "cls": {"weight": cls_w}}, f)
        torch.manual_seed(7)
        ours, cls = NetFeat("resnet18", "CIFAR100"), NetClassifier(512, 100)
        load_checkpoint(f, {"feat": ours, "cls": cls}, restore_rng=False)
    ours.eval()
    x = Fn.to_device_nhwc(torch.randn(2, 3, 32, 32), cpad=8, nchw=True)
    with torch.no_grad():
        want, got = src(x), ours(x)
    assert torch.allclose(got, want, rtol=1e-5, atol=1e-6), (got - want).abs().max()
    assert torch.equal(cls.weight.detach(), cls_w)


def test_torchvision_format_weights_load(tmp_path):
    """load_pretrained: a torchvision-layout ResNet state_dict file ([Co,Ci,KH,KW] convs, 'module.'
    prefix, different fc width skipped) lands on our NHWC modules."""
    from ddp_classification_pytorch_amd.models.pretrained import load_pretrained

    torch.manual_seed(0)
    src = build_model("resnet18", num_classes=0)
    sd = {"module." + k: (v.permute(0, 3, 1, 2).contiguous() if v.dim() == 4 else v)
          for k, v in src.state_dict().items()}
    sd["module.fc.weight"] = torch.randn(1000, 512)
    f = tmp_path / "tv.pth"
    torch.save(sd, f)
    torch.manual_seed(3)
    dst = build_model("resnet18", num_classes=0)
    missing, unexpected, _ = load_pretrained(dst, str(f))
    for k, v in src.state_dict().items():
        assert torch.equal(dst.state_dict()[k], v), k
