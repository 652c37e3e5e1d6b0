"""Space-to-depth stem (CPU reference math): the 7x7/2 ImageNet stem computed as a 4x4/1
conv over the 2x2 space-to-depth input must equal the plain 7x7/2 conv -- forward output
and the weight gradient mapped back onto the 7x7 master (models/resnet.py)."""
import pytest
import torch
import torch.nn.functional as F

from ddp_classification_pytorch_amd.models import build_model, input_layout
from ddp_classification_pytorch_amd.ops import _ref
from ddp_classification_pytorch_amd.ops import functional as Fn


@pytest.mark.parametrize("H,W", [(32, 32), (18, 26), (224, 224)])
def test_s2d_stem_equals_7x7_stride2(H, W):
    torch.manual_seed(0)
    img = torch.randn(2, 3, H, W)
    w = torch.randn(64, 7, 7, 3, requires_grad=True)
    # plain 7x7 / stride 2 / pad 3 conv
    ref = F.conv2d(img, w.permute(0, 3, 1, 2), stride=2, padding=3).permute(0, 2, 3, 1)
    # s2d input straight from the image and from the 8-channel NHWC layout
    x16 = Fn.to_device_nhwc(img, cpad=8, s2d=True)
    assert torch.equal(x16, Fn.nhwc_to_s2d(Fn.to_device_nhwc(img, cpad=8)))
    buf = torch.zeros(64, 4, 4, 16)
    y, _ = Fn.stem_conv_s2d(x16, w, buf)
    assert y.shape == ref.shape
    assert torch.allclose(y, ref, atol=1e-4, rtol=1e-4)
    g = torch.randn_like(ref)
    (gw_ref,) = torch.autograd.grad((ref * g).sum(), w)
    (gw,) = torch.autograd.grad((y * g).sum(), w)
    assert ((gw - gw_ref).norm() / gw_ref.norm()).item() < 1e-5


def test_geo_conv_reference_asymmetric_pad():
    """conv_fwd_geo / conv_wgrad_geo: top/left pad p, output grid given explicitly."""
    torch.manual_seed(0)
    x = torch.randn(2, 9, 9, 16)
    w = torch.randn(8, 4, 4, 16)
    y, _ = _ref.conv_fwd_geo(x, w, 1, 2, 9, 9, False)
    full = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), padding=2)[:, :, :9, :9]
    assert torch.allclose(y, full.permute(0, 2, 3, 1), atol=1e-5)
    dy = torch.randn(2, 9, 9, 8)
    dw = _ref.conv_wgrad_geo(dy, x, 4, 4, 1, 2)
    wr = w.clone().requires_grad_(True)
    out = F.conv2d(x.permute(0, 3, 1, 2), wr.permute(0, 3, 1, 2), padding=2)[:, :, :9, :9]
    (out * dy.permute(0, 3, 1, 2)).sum().backward()
    assert torch.allclose(dw, wr.grad, atol=1e-3)


def test_resnet_s2d_stem_matches_plain_stem():
    torch.manual_seed(0)
    m1 = build_model("resnet18", num_classes=10)
    m0 = build_model("resnet18", num_classes=10, stem_s2d=False)
    m0.load_state_dict(m1.state_dict())
    assert input_layout(m1) == {"cpad": 8, "s2d": True} and input_layout(m0)["s2d"] is False
    img = torch.rand(4, 3, 64, 64)
    labels = torch.randint(0, 10, (4,))
    out = []
    for m, s2d in ((m1, True), (m0, False)):
        x = Fn.to_device_nhwc(img, cpad=8, s2d=s2d)
        loss = Fn.cross_entropy(m(x), labels)
        loss.backward()
        out.append((loss.item(), m.conv1.weight.grad.clone()))
    assert abs(out[0][0] - out[1][0]) < 1e-4
    assert ((out[0][1] - out[1][1]).norm() / out[1][1].norm()).item() < 1e-3


def test_tresnet_s2d4_input_matches_model_space_to_depth():
    """TResNet's SpaceToDepth(4) stem input written by the input kernel (``input_layout`` s2d=4:
    [N, H/4, W/4, 48], channel (py*4 + px)*3 + c, timm's order) == the model's own
    space_to_depth of the plain 3-channel NHWC input, and the model gives the same output."""
    torch.manual_seed(0)
    m = build_model("tresnet_m", num_classes=10).eval()
    lay = input_layout(m)
    assert lay == {"cpad": 3, "s2d": 4}
    img = torch.randint(0, 256, (2, 3, 64, 96), dtype=torch.uint8)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    x3 = Fn.to_device_nhwc(img, mean, std, cpad=3, in_scale=1 / 255.0)
    x48 = Fn.to_device_nhwc(img, mean, std, in_scale=1 / 255.0, **lay)
    assert x48.shape == (2, 16, 24, 48)
    assert torch.equal(x48, _ref.space_to_depth(x3, 4, False))
    with torch.no_grad():
        assert torch.allclose(m(x48), m(x3), atol=1e-5)
    assert Fn.s2d_for(4, 224, 224) == 4 and Fn.s2d_for(4, 226, 224) == 0 and Fn.s2d_for(True, 6, 8) == 2
