"""Large per-GPU batch (288 GB HBM sizing, BASELINE.json config 5): a conv whose output has
more than 2^32 elements.  The epilogue row offsets are 64-bit (csrc/conv_igemm.hip); with
32-bit offsets the images past element 2^32 would wrap onto the first ones.

ResNet-50 stage-1 expansion conv 64 -> 256 at 56x56 with N = 5,400 images: 4.34e9 outputs
(8.7 GB bf16).  Images on both sides of the 2^32 boundary are compared with an fp32 matmul."""
import pytest
import torch

from ddp_classification_pytorch_amd import _ext

pytestmark = pytest.mark.gpu


def test_conv_output_past_2pow32_elements():
    K = _ext.hip_ops()
    N, H, W, Ci, Co = 5400, 56, 56, 64, 256
    assert N * H * W * Co > 2**32
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, W, Ci, device=dev, generator=g, dtype=torch.float32).bfloat16()
    w = (torch.randn(Co, 1, 1, Ci, device=dev, generator=g) / 8.0).bfloat16()
    y, slabs = K.conv_fwd(x, w, 1, 0, True)
    torch.cuda.synchronize()
    assert y.shape == (N, H, W, Co)
    boundary = 2**32 // (H * W * Co)  # the image holding element 2^32
    for n in (0, boundary - 1, boundary, boundary + 1, N - 1):
        ref = x[n].float().reshape(-1, Ci) @ w.float().reshape(Co, Ci).t()
        got = y[n].float().reshape(-1, Co)
        err = ((got - ref).norm() / ref.norm()).item()
        assert err < 1e-2, (n, err)
    # per-channel statistics from the epilogue cover every row (n = N*H*W)
    st = K.bn_stats(y, slabs)
    assert int(st[0, 0, 0].item()) == N * H * W
    del x, y, slabs
    torch.cuda.empty_cache()


def test_stem_maxpool_past_2pow31_elements():
    """The stem's 3x3/2 max pool at R101 b3072 (BASELINE.json config 5 swept to 3072): the input
    holds 2.47e9 elements, past the old 2^31 flat-index guard; element offsets are 64-bit now."""
    import torch.nn.functional as F

    K = _ext.hip_ops()
    N, H, W, C = 3072, 112, 112, 64
    assert N * H * W * C > 2**31
    dev = torch.device("cuda")
    x = torch.empty(N, H, W, C, device=dev, dtype=torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(1)
    for i in range(0, N, 512):  # fill in chunks: an fp32 temporary of the whole would be 9.9 GB
        x[i:i + 512] = torch.randn(min(512, N - i), H, W, C, device=dev, generator=g).bfloat16()
    y, idx = K.maxpool_fwd(x, 3, 2, 1)
    dy = torch.ones_like(y)
    dx = K.maxpool_bwd(dy, idx, H, W, 3, 2, 1)
    torch.cuda.synchronize()
    for n in (0, 2**31 // (H * W * C), N - 1):
        xn = x[n:n + 1].permute(0, 3, 1, 2).float()
        ref = F.max_pool2d(xn, 3, 2, 1).permute(0, 2, 3, 1)
        assert torch.equal(y[n:n + 1].float(), ref), n
        # every window's argmax receives its 1.0: the gradient mass equals the window count
        assert dx[n].float().sum().item() == float(y[n].numel()), n
    del x, y, idx, dy, dx
    torch.cuda.empty_cache()


def test_resnet50_headline_batch_4096_copies():
    """The headline's per-GPU batch (bench.py r50: 4,096 images, ~156 GB): one training step of
    ResNet-50 on 4 copies of the same 1,024 images.  Every copy sees the same batch statistics, so
    the copies' logits agree with each other and with the 1,024-image step (up to summation order),
    and so do the loss and the weight gradients -- an index that wrapped past 2^31 / 2^32 elements
    anywhere in the step (stem activations: 3.3e9 elements, 6.6 GB) would break one of the copies."""
    from ddp_classification_pytorch_amd.models import build_model, input_layout
    from ddp_classification_pytorch_amd.ops import functional as Fn

    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = build_model("resnet50", num_classes=1000).to(dev)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    g = torch.Generator(device=dev).manual_seed(2)
    imgs = torch.randint(0, 256, (1024, 3, 224, 224), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 1000, (1024,), device=dev, generator=g)

    def step(reps):
        model.zero_grad(set_to_none=True)
        x = Fn.to_device_nhwc(imgs.repeat(reps, 1, 1, 1), mean, std, in_scale=1 / 255.0, **input_layout(model))
        out = model(x)
        loss = Fn.cross_entropy(out, labels.repeat(reps))
        loss.backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
        return out.float()[:, :1000].clone(), float(loss), grads

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()

    out1, loss1, g1 = step(1)
    out2, loss2, g2 = step(2)
    out4, loss4, g4 = step(4)
    assert out4.shape[0] == 4096 and torch.isfinite(out4).all()
    # the wrap detector: the four copies inside the 4,096-image step agree with each other
    within = max(rel(out4[1024 * k:1024 * (k + 1)], out4[:1024]) for k in range(1, 4))
    within2 = rel(out2[1024:], out2[:1024])
    # across batch sizes the kernel plans differ (split-K / stream-K by grid size) and so does the
    # fp32 summation order of the BN statistics: bf16 rounding then moves the logits of a
    # random-init net by a few per cent; the 2,048-image step (no tensor near 2^31 elements) is
    # the yardstick for that drift
    d2, d4 = rel(out2[:1024], out1), rel(out4[:1024], out1)
    gw2 = max(rel(g2[n], g1[n]) for n in g1 if g1[n].norm() > 0)
    gw4 = max(rel(g4[n], g1[n]) for n in g1 if g1[n].norm() > 0)
    worst = max((n for n in g1 if g1[n].norm() > 0), key=lambda n: rel(g4[n], g1[n]))
    gall = lambda g: torch.cat([g[n].reshape(-1) for n in sorted(g1)])  # noqa: E731
    G1, G2, G4 = gall(g1), gall(g2), gall(g4)
    print(f"worst parameter {worst}: |g| {g1[worst].norm().item():.3e} (largest |g| "
          f"{max(v.norm().item() for v in g1.values()):.3e}); whole-gradient rel diff vs b1024: "
          f"b2048 {rel(G2, G1):.3e}, b4096 {rel(G4, G1):.3e}; b4096 vs b2048 {rel(G4, G2):.3e}")
    print(f"copies within b4096 {within:.2e}, b2048 {within2:.2e}; logits vs b1024: b2048 {d2:.3e}, "
          f"b4096 {d4:.3e}; worst weight-gradient rel diff vs b1024: b2048 {gw2:.3e}, b4096 {gw4:.3e}; "
          f"loss {loss1:.5f} / {loss2:.5f} / {loss4:.5f}")
    # yardsticks at batch 1,024: the same step again (deterministic kernels: identical) and with every
    # weight perturbed by ~2^-22 relative (an fp32-rounding-sized change; the net at init is chaotic
    # in its gradients, so this alone moves them by as much as a different kernel plan does)
    out1b, _, g1b = step(1)
    with torch.no_grad():
        for p_ in model.parameters():
            p_.mul_(1 + 2.0 ** -22 * torch.randn_like(p_))
    _, _, g1p = step(1)
    rerun, perturbed = rel(gall(g1b), G1), rel(gall(g1p), G1)
    print(f"b1024 rerun: logits {rel(out1b, out1):.3e}, gradient {rerun:.3e}; b1024 with 2^-22 weight "
          f"noise: gradient {perturbed:.3e}")
    assert rerun == 0.0
    assert within < 1e-2 and within2 < 1e-2, (within, within2)
    assert d4 < max(2.0 * d2, 2e-2), (d4, d2)
    assert abs(loss4 - loss1) <= 1e-2 * abs(loss1)
    assert g4.keys() == g1.keys()
    assert gw4 < max(2.0 * gw2, 5e-2), (gw4, gw2)
    assert rel(G4, G1) < 2.0 * max(perturbed, 1e-2), (rel(G4, G1), perturbed)
    del model, out1, out2, out4, g1, g2, g4
    torch.cuda.empty_cache()
