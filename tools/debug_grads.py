"""Localise gradient mismatches between our GPU model and an fp64 mirror."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from ddp_classification_pytorch_amd.models import build_model  # noqa: E402
from ddp_classification_pytorch_amd.ops import functional as Fn  # noqa: E402
from tests.model_mirror import _bn, _conv  # noqa: E402


def relerr(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main(name="resnet18", size=64, batch=8):
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m1 = build_model(name, num_classes=100).to(dev)
    m2 = copy.deepcopy(m1).double()
    imgs = torch.randn(batch, 3, size, size, device=dev)
    lab = torch.randint(0, 100, (batch,), device=dev)
    acts1, acts2 = [], []
    x = Fn.to_device_nhwc(imgs, cpad=8)
    y, s = m1.conv1(x, stats=True)
    y = m1.bn1(y, s)
    y.retain_grad(); acts1.append(("stem", y))
    y = Fn.max_pool2d(y)
    y.retain_grad(); acts1.append(("pool", y))
    for li, L in enumerate([m1.layer1, m1.layer2, m1.layer3, m1.layer4]):
        for bi, b in enumerate(L):
            y = b(y)
            y.retain_grad(); acts1.append((f"l{li+1}.{bi}", y))
    f = Fn.global_avg_pool(y)
    f.retain_grad(); acts1.append(("gap", f))
    out = m1.fc(f)
    Fn.cross_entropy(out, lab).backward()

    y2 = F.relu(_bn(_conv(imgs.double(), m2.conv1), m2.bn1, True))
    y2.retain_grad(); acts2.append(y2)
    y2 = F.max_pool2d(y2, 3, 2, 1)
    y2.retain_grad(); acts2.append(y2)
    for L in [m2.layer1, m2.layer2, m2.layer3, m2.layer4]:
        for b2 in L:
            xin = y2
            r = xin if b2.downsample is None else _bn(_conv(xin, b2.downsample[0]), b2.downsample[1], True)
            z = F.relu(_bn(_conv(xin, b2.conv1), b2.bn1, True))
            if hasattr(b2, "conv3"):
                z = F.relu(_bn(_conv(z, b2.conv2), b2.bn2, True))
                z = _bn(_conv(z, b2.conv3), b2.bn3, True)
            else:
                z = _bn(_conv(z, b2.conv2), b2.bn2, True)
            y2 = F.relu(z + r)
            y2.retain_grad(); acts2.append(y2)
    f2 = y2.mean((2, 3))
    f2.retain_grad(); acts2.append(f2)
    out2 = F.linear(f2, m2.fc.weight, m2.fc.bias)
    F.cross_entropy(out2, lab).backward()
    print("logits", relerr(out, out2))
    for (n, a), b in zip(acts1, acts2):
        p = (lambda t: t.permute(0, 2, 3, 1)) if b.dim() == 4 else (lambda t: t)
        print(f"{n:8s} act {relerr(a, p(b)):.2e} grad {relerr(a.grad, p(b.grad)):.2e}")
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        print(f"{n:32s} {relerr(p1.grad, p2.grad):.2e}")


def torch_bf16_error(name="resnet18", size=64, batch=8):
    """How far stock-PyTorch bf16 autocast (MIOpen) lands from fp64 on the same net/input."""
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    from tests.model_mirror import mirror_forward
    m1 = build_model(name, num_classes=100).to(dev)
    m2 = copy.deepcopy(m1).double()
    m3 = copy.deepcopy(m1)
    imgs = torch.randn(batch, 3, size, size, device=dev)
    lab = torch.randint(0, 100, (batch,), device=dev)
    F.cross_entropy(mirror_forward(m2, imgs.double()), lab).backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = mirror_forward(m3, imgs)
    F.cross_entropy(out.float(), lab).backward()
    x = Fn.to_device_nhwc(imgs, cpad=8)
    Fn.cross_entropy(m1(x), lab).backward()
    g = lambda m: torch.cat([p.grad.double().flatten() for p in m.parameters()])
    print(f"{name}: torch-bf16 vs fp64 {relerr(g(m3), g(m2)):.3e}   ours vs fp64 {relerr(g(m1), g(m2)):.3e}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "cmp":
        for n, sz, b in [("resnet18", 64, 8), ("resnet18", 112, 32), ("resnet50", 112, 16), ("resnet50", 224, 32)]:
            torch_bf16_error(n, sz, b)
    else:
        main(*(sys.argv[1:2] or ["resnet18"]))
