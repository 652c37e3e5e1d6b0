"""Backward fusion protocol (CPU reference math): the stride-1 conv consuming a BN output
runs that BN's backward reduction in its dgrad epilogue (BNSource), and a block input's
secondary consumers hand their gradient to the primary conv (GradJoin).  Gradients must
equal the unfused path, and every backward order of the join must stay correct."""
import pytest
import torch

from ddp_classification_pytorch_amd.models import build_model
from ddp_classification_pytorch_amd.ops import _ref
from ddp_classification_pytorch_amd.ops import functional as Fn


@pytest.fixture(autouse=True)
def _plain_fusion_on():
    """Exercise the plain BN+ReLU epilogue fusion on every layer (by default only on small ones)."""
    saved = Fn._PLAIN_FUSE_MAX[0]
    Fn.set_plain_bn_backward_fusion(True)
    yield
    Fn.set_plain_bn_backward_fusion(False, saved)


def _grads(name, fuse, size=32, seed=0):
    Fn.set_bn_backward_fusion(fuse)
    try:
        torch.manual_seed(seed)
        m = build_model(name, num_classes=10)
        g = torch.Generator().manual_seed(1)
        imgs = torch.rand(4, 3, size, size, generator=g, dtype=torch.float32)
        labels = torch.randint(0, 10, (4,), generator=g)
        x = Fn.to_device_nhwc(imgs, cpad=8, nchw=True)
        loss = Fn.cross_entropy(m(x), labels)
        loss.backward()
        return loss.item(), torch.cat([p.grad.flatten() for p in m.parameters()])
    finally:
        Fn.set_bn_backward_fusion(True)


@pytest.mark.parametrize("name", ["resnet18", "resnet50", "resnext50_32x4d"])
def test_fused_bn_backward_matches_unfused(name, monkeypatch):
    calls = []
    orig = _ref.conv_dgrad_bn

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(_ref, "conv_dgrad_bn", counting)
    l1, g1 = _grads(name, True)
    n_fused = len(calls)
    l0, g0 = _grads(name, False)
    assert len(calls) == n_fused  # nothing fused with the switch off
    assert n_fused > 0
    assert abs(l1 - l0) < 1e-6
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-5


@pytest.mark.parametrize("prologue", [True, False])
def test_resnet50_fuses_expected_layers(monkeypatch, prologue):
    calls = []
    orig = _ref.conv_dgrad_bn
    monkeypatch.setattr(_ref, "conv_dgrad_bn", lambda *a, **k: calls.append(1) or orig(*a, **k))
    Fn.set_bn_prologue(prologue)
    try:
        _grads("resnet50", True)
    finally:
        Fn.set_bn_prologue(False)
    # conv2 of the 13 stride-1 blocks, conv1 of the 15 blocks after the first, and conv3 of all 16
    # unless bn2 runs as conv3's prologue (its backward is then the prologue op's own)
    assert len(calls) == 13 + 15 + (0 if prologue else 16)


@pytest.mark.parametrize("name", ["resnet50", "resnext50_32x4d"])
def test_bn_prologue_matches_separate_bn(name, monkeypatch):
    """bn2 + ReLU inside conv3's GEMMs (K5 prologue) == BN-apply pass then conv: same loss and
    gradients, and the prologue ops run for every bottleneck."""
    calls = []
    orig = _ref.conv_fwd_pro
    monkeypatch.setattr(_ref, "conv_fwd_pro", lambda *a, **k: calls.append(1) or orig(*a, **k))
    saved = Fn._PLAIN_FUSE_MAX[0]
    Fn.set_plain_bn_backward_fusion(False, 0)
    try:
        Fn.set_bn_prologue(True)
        l1, g1 = _grads(name, True)
        assert len(calls) == 16
        Fn.set_bn_prologue(False)
        l0, g0 = _grads(name, True)
        assert len(calls) == 16
    finally:
        Fn.set_bn_prologue(False)
        Fn.set_plain_bn_backward_fusion(False, saved)
    assert abs(l1 - l0) < 1e-6
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-5


class _Probe(torch.autograd.Function):
    """Identity whose backward deposits into a GradJoin (a secondary consumer)."""

    @staticmethod
    def forward(ctx, x, join):
        ctx.join = join
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return ctx.join.deposit(g * 3.0), None


@pytest.mark.parametrize("late", [False, True])
def test_gradjoin_any_order(late):
    """Deposit before the claim: summed by the primary.  Deposit after the claim: handed
    back to autograd unchanged."""
    x = torch.randn(8, requires_grad=True)
    j = Fn.GradJoin(1)
    if late:
        j.claim()  # the primary already ran
        out = (_Probe.apply(x, j)).sum()
        out.backward()
        assert torch.allclose(x.grad, torch.full_like(x, 3.0))
    else:
        assert j.deposit(torch.ones(8)) is None
        add, complete = j.claim()
        assert complete and torch.equal(add, torch.ones(8))
        assert j.deposit(torch.ones(8)) is not None  # after the claim: returned unchanged


def test_unfused_fallback_when_conv_output_shared():
    """A BN output consumed by a fusing conv AND another op: the BN backward receives the
    autograd sum (not the fused buffer) and must take the unfused path -- still exact."""
    torch.manual_seed(0)
    from ddp_classification_pytorch_amd.models.layers import BatchNorm2d, Conv2d

    def run(fuse):
        Fn.set_bn_backward_fusion(fuse)
        try:
            torch.manual_seed(0)
            conv0, bn, conv1 = Conv2d(8, 16, 3, 1, 1), BatchNorm2d(16), Conv2d(16, 16, 1)
            x = torch.randn(2, 6, 6, 8)
            y, s = conv0(x)
            z = bn(y, s, act="relu")
            out, _ = conv1(z)
            loss = (out * out).sum() + (z * 0.5).sum()  # second consumer of z
            loss.backward()
            return torch.cat([p.grad.flatten() for p in (conv0.weight, bn.weight, bn.bias, conv1.weight)])
        finally:
            Fn.set_bn_backward_fusion(True)

    g1, g0 = run(True), run(False)
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-5


def test_ref_mask_path_matches_residual_path():
    """CPU reference: the activation-mask form of the fused BN-backward dgrad equals the
    residual-recompute form (the GPU kernels are checked the same way in test_kernels_gpu)."""
    import torch

    from ddp_classification_pytorch_amd.ops import _ref

    torch.manual_seed(0)
    N, H, Ci, Co = 2, 6, 16, 8
    y, r = torch.randn(N, H, H, Ci) * 2, torch.randn(N, H, H, Ci)
    scale, shift = torch.rand(Ci) + 0.5, torch.randn(Ci) * 0.3
    mean, invstd = torch.randn(Ci) * 0.2, torch.rand(Ci) + 0.5
    z, mask = _ref.bn_act_mask(y, r, scale, shift, 1, 0.0)
    assert mask.shape == (N, H, H, Ci // 8)
    assert torch.equal(_ref.unpack_mask(mask), (y * scale + shift + r > 0).float())
    wt = torch.randn(Ci, 1, 1, Co)
    dy, add = torch.randn(N, H, H, Co), torch.randn(N, H, H, Ci)
    g0, s0 = _ref.conv_dgrad_bn(dy, wt, 0, add, y, r, scale, shift, mean, invstd, 1)
    g1, s1 = _ref.conv_dgrad_bn(dy, wt, 0, add, y, None, scale, shift, mean, invstd, 1, mask)
    assert torch.allclose(g0, g1) and torch.allclose(s0, s1)


@pytest.mark.parametrize("name,size,cpad", [("resnet50", 64, 8), ("resnet18", 32, 8), ("tresnet_m", 64, 3)])
def test_shortcut_bn_fusion_matches_unfused(name, size, cpad):
    """A projection shortcut's BN applied inside the block's last BN pass (Fn.batch_norm_add_bn_act)
    gives the same loss, parameter gradients and running statistics as the separate BN."""
    import copy

    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn

    torch.manual_seed(3)
    m1 = build_model(name, num_classes=10)
    m2 = copy.deepcopy(m1)
    imgs = torch.randn(3, 3, size, size)
    labels = torch.randint(0, 10, (3,))
    out = []
    for m, fuse in ((m1, True), (m2, False)):
        Fn.set_shortcut_bn_fusion(fuse)
        try:
            x = Fn.to_device_nhwc(imgs, cpad=cpad, nchw=True)
            loss = Fn.cross_entropy(m(x), labels)
            loss.backward()
        finally:
            Fn.set_shortcut_bn_fusion(True)
        out.append(loss.detach())
    assert torch.allclose(out[0], out[1], rtol=1e-5, atol=1e-6)
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p1.grad, p2.grad, rtol=1e-3, atol=1e-5), n
    for (n, b1), b2 in zip(m1.named_buffers(), m2.buffers()):
        if b1.dtype.is_floating_point:
            assert torch.allclose(b1, b2, rtol=1e-5, atol=1e-6), n


@pytest.mark.parametrize("name,size,cpad", [("tresnet_m", 64, 3), ("resnet50", 64, 8)])
def test_gradjoin_matches_autograd_sum(name, size, cpad, monkeypatch):
    """The GradJoin hand-off (secondary consumers deposit, the block's first conv adds in its dgrad
    epilogue) gives the same gradients as letting autograd sum the block-input gradients."""
    import copy

    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn

    torch.manual_seed(4)
    m1 = build_model(name, num_classes=10)
    m2 = copy.deepcopy(m1)
    imgs = torch.randn(2, 3, size, size)
    labels = torch.randint(0, 10, (2,))

    def run(m):
        loss = Fn.cross_entropy(m(Fn.to_device_nhwc(imgs, cpad=cpad, nchw=True)), labels)
        loss.backward()
        return loss.detach()

    l1 = run(m1)
    with monkeypatch.context() as mp:  # every deposit refused: autograd adds the gradients
        mp.setattr(Fn.GradJoin, "deposit", lambda self, g: g)
        l2 = run(m2)
    assert torch.allclose(l1, l2, rtol=1e-6, atol=1e-7)
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p1.grad, p2.grad, rtol=1e-3, atol=1e-5), n


def test_resnext_grouped_dgrad_fuses_bn_backward(monkeypatch):
    """ResNeXt's stride-1 grouped 3x3 convs fuse bn1's backward reduction into their dgrad
    (grouped_conv_dgrad_bn) and the gradients equal the unfused path."""
    calls = []
    orig = _ref.grouped_conv_dgrad_bn
    monkeypatch.setattr(_ref, "grouped_conv_dgrad_bn", lambda *a, **k: calls.append(1) or orig(*a, **k))
    l1, g1 = _grads("resnext50_32x4d", True)
    assert len(calls) == 13  # the stride-1 grouped convs (16 blocks minus 3 stride-2 ones)
    l0, g0 = _grads("resnext50_32x4d", False)
    assert len(calls) == 13
    assert abs(l1 - l0) < 1e-6
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-5


def test_tresnet_leaky_bn_backward_fusion(monkeypatch):
    """TResNet's leaky-ReLU BNs (InplaceABN) fuse their backward reduction into the consuming
    conv's dgrad (raw gradient returned, masked sums): gradients equal the unfused path."""
    calls = []
    orig = _ref.conv_dgrad_bn

    def counting(*a, **k):
        if a[10] == 2:
            calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(_ref, "conv_dgrad_bn", counting)
    Fn.set_leaky_bn_backward_fusion(True)  # opt-in (measured slower on the GPU)
    out = []
    for fuse in (True, False):
        Fn.set_bn_backward_fusion(fuse)
        try:
            torch.manual_seed(5)
            m = build_model("tresnet_m", num_classes=10)
            for mod in m.modules():  # the leaky fusion covers the non-InplaceABN storage mode
                if hasattr(mod, "inplace_abn"):
                    mod.inplace_abn = False
            g = torch.Generator().manual_seed(2)
            imgs = torch.rand(2, 3, 64, 64, generator=g)
            labels = torch.randint(0, 10, (2,), generator=g)
            loss = Fn.cross_entropy(m(Fn.to_device_nhwc(imgs, cpad=3, nchw=True)), labels)
            loss.backward()
            out.append((loss.item(), torch.cat([p.grad.flatten() for p in m.parameters()])))
        finally:
            Fn.set_bn_backward_fusion(True)
        if fuse:
            n_leaky = len(calls)
    Fn.set_leaky_bn_backward_fusion(False)
    assert n_leaky > 10
    (l1, g1), (l0, g0) = out
    assert abs(l1 - l0) < 1e-6
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-5



@pytest.mark.parametrize("max_elems,expect", [(0, 15), (8192, 15 + 10 + 13), (1 << 25, 15 + 13 + 16)])
def test_plain_fusion_size_rule(monkeypatch, max_elems, expect):
    """Plain BN + ReLU layers fuse their backward reduction into the consuming stride-1 conv's dgrad
    only up to ``max_elems`` activation elements.  Threshold 0: only the BN + residual + ReLU layers
    (ResNet-50: conv1 of the 15 blocks after the first).  32px ResNet-50 at batch 4, threshold 8192:
    stage 1's plain BN outputs (16,384 elements) stay unfused; in stages 2-4 conv2 of the 3 + 5 + 2
    stride-1 blocks and conv3 of all 4 + 6 + 3 blocks fuse.  Gradients equal the unfused path."""
    saved = Fn._PLAIN_FUSE_MAX[0]
    Fn.set_plain_bn_backward_fusion(False, max_elems)
    calls = []
    orig = _ref.conv_dgrad_bn
    monkeypatch.setattr(_ref, "conv_dgrad_bn", lambda *a, **k: calls.append(1) or orig(*a, **k))
    try:
        l1, g1 = _grads("resnet50", True)
        n = len(calls)
        l0, g0 = _grads("resnet50", False)
    finally:
        Fn.set_plain_bn_backward_fusion(False, saved)
    assert n == expect
    assert abs(l1 - l0) < 1e-6
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-5


@pytest.mark.parametrize("train", [True, False])
def test_tresnet_inplace_abn_matches_stored_input_backward(train):
    """InplaceABN (only the activation output saved; backward inverts leaky ReLU and the affine
    in place of reading the BN input) == the same net with the BN input saved: loss and every
    gradient (|gamma| + eps effective weight in both), training and frozen-statistics modes."""
    out = []
    for iabn in (True, False):
        torch.manual_seed(5)
        m = build_model("tresnet_m", num_classes=10)
        n = 0
        for mod in m.modules():
            if getattr(mod, "inplace_abn", False):
                n += 1
                if not iabn:  # same effective weight, BN-input storage
                    mod.inplace_abn = False
                    with torch.no_grad():
                        mod.weight.copy_(mod.weight.abs() + mod.iabn_eps)
        assert n == 1 + 3 + 4 + 2 * 11 + 2 * 3  # stem, basic conv1, bottleneck conv1 + conv2
        if not train:
            for mod in m.modules():
                if hasattr(mod, "inplace_abn"):
                    mod.frozen = True
        g = torch.Generator().manual_seed(2)
        imgs = torch.rand(2, 3, 64, 64, generator=g)
        labels = torch.randint(0, 10, (2,), generator=g)
        loss = Fn.cross_entropy(m(Fn.to_device_nhwc(imgs, cpad=3, nchw=True)), labels)
        loss.backward()
        out.append((loss.item(), torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None])))
    (l1, g1), (l0, g0) = out
    assert abs(l1 - l0) < 1e-5
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-4


def test_eval_coefficient_cache_sees_untracked_bn_updates():
    """On the GPU the BN statistics kernels rewrite running_mean / running_var and the fused
    optimizers rewrite gamma / beta without bumping ``_version``.  The eval-coefficient cache must
    still refresh: after a training-stats forward (``_nbt_pending``) and after an optimizer step
    (weight generation).  ``.data`` writes reproduce the version-less update on the CPU."""
    from ddp_classification_pytorch_amd.models.layers import BatchNorm2d

    bn = BatchNorm2d(8)
    bn.eval()
    c0 = [t.clone() for t in Fn.bn_eval_coefficients(bn)]
    bn.running_mean.data.add_(1.0)  # a statistics kernel: no version bump
    bn._nbt_pending += 1            # ... during a training forward, which counts itself
    c1 = Fn.bn_eval_coefficients(bn)
    assert not torch.allclose(c0[0], c1[0])
    assert torch.allclose(c1[0], bn.running_mean)
    bn.flush_batches_tracked()      # pending -> num_batches_tracked: the key must stay fresh
    c1b = Fn.bn_eval_coefficients(bn)
    assert torch.allclose(c1b[0], bn.running_mean)
    bn.weight.data.mul_(2.0)        # a fused optimizer step: pointer-table update, no version bump
    Fn.bump_weight_generation()     # ... which every optimizer step does
    c2 = Fn.bn_eval_coefficients(bn)
    assert torch.allclose(c2[2], c1b[2] * 2.0)
    # frozen BN (gamma / beta without grad): nothing changes, the cached tensors are reused
    bn.weight.requires_grad_(False)
    bn.bias.requires_grad_(False)
    c3 = Fn.bn_eval_coefficients(bn)
    Fn.bump_weight_generation()
    assert Fn.bn_eval_coefficients(bn)[2] is c3[2]


@pytest.mark.parametrize("train", [True, False])
def test_iabn_fold_matches_separate_gamma_launches(train):
    """InplaceABN with the raw weight handed to the BN kernels (|gamma| + eps in the finalize,
    sign(gamma) on the weight gradient in the backward's elementwise pass; DCP_IABN_FOLD default)
    == the separate iabn_gamma / sign_mul ops: loss, every gradient and the running statistics, with
    some gammas negative (the sign path).  Frozen statistics (train=False) keep the separate ops."""
    out = []
    for fold in (True, False):
        Fn.set_iabn_fold(fold)
        try:
            torch.manual_seed(7)
            m = build_model("tresnet_m", num_classes=10)
            with torch.no_grad():
                for mod in m.modules():
                    if getattr(mod, "inplace_abn", False):
                        mod.weight.mul_(torch.where(torch.rand_like(mod.weight) < 0.3, -1.0, 1.0))
                        if not train:
                            mod.frozen = True
            g = torch.Generator().manual_seed(3)
            imgs = torch.rand(2, 3, 64, 64, generator=g)
            labels = torch.randint(0, 10, (2,), generator=g)
            loss = Fn.cross_entropy(m(Fn.to_device_nhwc(imgs, cpad=3, nchw=True)), labels)
            loss.backward()
            rs = torch.cat([b.flatten() for n, b in m.named_buffers() if "running" in n])
            out.append((loss.item(), torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None]), rs))
        finally:
            Fn.set_iabn_fold(True)
    (l1, g1, r1), (l0, g0, r0) = out
    assert abs(l1 - l0) < 1e-6
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-6
    assert torch.allclose(r1, r0, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("model", ["resnet18", "tresnet_m"])
def test_bn_fin_act_path_matches_two_launches(model):
    """The one-launch BN finalize + apply wiring (DCP_BN_FIN_ACT=1, _BNAct.forward -> bn_fin_act) ==
    the default two-op path on the CPU reference: loss, gradients, running statistics."""
    out = []
    for fused in (True, False):
        Fn.set_bn_fin_act(fused)
        try:
            torch.manual_seed(5)
            m = build_model(model, num_classes=10)
            g = torch.Generator().manual_seed(2)
            imgs = torch.rand(2, 3, 64, 64, generator=g)
            labels = torch.randint(0, 10, (2,), generator=g)
            from ddp_classification_pytorch_amd.models import input_layout
            loss = Fn.cross_entropy(m(Fn.to_device_nhwc(imgs, nchw=True, **input_layout(m))), labels)
            loss.backward()
            rs = torch.cat([b.flatten() for n, b in m.named_buffers() if "running" in n])
            out.append((loss.item(), torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None]), rs))
        finally:
            Fn.set_bn_fin_act(False)
    (l1, g1, r1), (l0, g0, r0) = out
    assert l1 == l0
    assert torch.equal(g1, g0)
    assert torch.equal(r1, r0)


def test_se_gate_fused_matches_gemm_chain():
    """TResNet-M's squeeze-excitation gates as one fused op per direction (Fn.se_gate) == the
    Linear / GEMM chain on the CPU reference: loss and every gradient; the fused op really runs."""
    from ddp_classification_pytorch_amd.models import input_layout
    calls = [0]
    orig = _ref.se_gate_fwd

    def counting(*a, **k):
        calls[0] += 1
        return orig(*a, **k)

    out = []
    _ref.se_gate_fwd = counting
    try:
        for fused in (True, False):
            Fn.set_se_fused(fused)
            torch.manual_seed(5)
            m = build_model("tresnet_m", num_classes=10)
            g = torch.Generator().manual_seed(2)
            imgs = torch.rand(2, 3, 64, 64, generator=g)
            labels = torch.randint(0, 10, (2,), generator=g)
            loss = Fn.cross_entropy(m(Fn.to_device_nhwc(imgs, nchw=True, **input_layout(m))), labels)
            loss.backward()
            out.append((loss.item(), torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None])))
    finally:
        _ref.se_gate_fwd = orig
        Fn.set_se_fused(True)
    assert calls[0] > 0
    (l1, g1), (l0, g0) = out
    assert abs(l1 - l0) < 1e-6
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-6
