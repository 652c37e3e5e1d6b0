"""Numerics of every gfx950 HIP primitive against the plain-PyTorch fp32
reference (ops/_ref.py) on identical bf16-rounded inputs."""
import math

import pytest
import torch

from ddp_classification_pytorch_amd import _ext
from ddp_classification_pytorch_amd.tuning import slot as tslot
from ddp_classification_pytorch_amd.ops import _ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def K():
    return _ext.hip_ops()


def relerr(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape) * scale).bfloat16()


# ResNet-50 conv shapes at small batch, plus edge cases
CONV_SHAPES = [
    # N, H, W, Ci, Co, k, stride, pad
    (2, 56, 56, 64, 64, 1, 1, 0),
    (2, 56, 56, 64, 64, 3, 1, 1),
    (2, 56, 56, 64, 256, 1, 1, 0),
    (2, 56, 56, 256, 64, 1, 1, 0),
    (2, 56, 56, 256, 128, 1, 1, 0),
    (2, 56, 56, 128, 128, 3, 2, 1),
    (2, 28, 28, 128, 512, 1, 1, 0),
    (2, 56, 56, 256, 512, 1, 2, 0),
    (2, 28, 28, 512, 128, 1, 1, 0),
    (2, 28, 28, 128, 128, 3, 1, 1),
    (2, 14, 14, 256, 256, 3, 1, 1),
    (2, 28, 28, 512, 1024, 1, 2, 0),
    (2, 14, 14, 512, 512, 3, 2, 1),
    (2, 7, 7, 512, 2048, 1, 1, 0),
    (2, 7, 7, 2048, 512, 1, 1, 0),
    (2, 7, 7, 512, 512, 3, 1, 1),
    (2, 64, 64, 8, 64, 7, 2, 3),     # stem (3 channels padded to 8)
    (3, 9, 11, 64, 72, 3, 1, 1),     # ragged M and Co
    (1, 13, 13, 32, 40, 3, 2, 1),    # odd spatial, stride 2, Cs % 64 != 0
    (2, 32, 32, 8, 64, 3, 1, 1),     # CIFAR stem
    (8, 2, 2, 512, 512, 3, 1, 1),    # tiny spatial (ResNet-18 layer4 at 64px)
    (8, 4, 4, 256, 512, 3, 2, 1),
    (8, 2, 2, 512, 512, 1, 1, 0),
    (8, 4, 4, 256, 512, 1, 2, 0),
    (16, 16, 16, 64, 64, 3, 1, 1),   # layer1 3x3 at 64 px: one direct-kernel strip per image
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_fwd_stats(K, shape):
    N, H, W, Ci, Co, k, s, p = shape
    x = rnd(N, H, W, Ci)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci))
    y, slabs = K.conv_fwd(x.to(DEV), w.to(DEV), s, p, True)
    yr, _ = _ref.conv_fwd(x.float(), w.float(), s, p, False)
    assert y.shape == yr.shape
    assert relerr(y, yr) < 1e-2
    st = K.bn_stats(y, slabs)  # (n, mean, M2) from the conv-epilogue tile statistics
    sr = _ref.bn_stats(y.float().cpu(), None)
    assert torch.equal(st[0, 0].cpu(), sr[0, 0])
    assert relerr(st[0, 1], sr[0, 1]) < 1e-4
    assert relerr(st[0, 2], sr[0, 2]) < 1e-4


@pytest.mark.parametrize("shape", [c for c in CONV_SHAPES if c[3] % 8 == 0 and c[3] > 8])
def test_conv_dgrad(K, shape):
    N, H, W, Ci, Co, k, s, p = shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = rnd(N, Ho, Wo, Co)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Co))
    wb, wt = K.weight_prep(w.float().to(DEV), 0, True)
    dx = K.conv_dgrad(dy.to(DEV), wt, H, W, s, p)
    dxr = _ref.conv_dgrad(dy.float(), w.float().permute(3, 1, 2, 0), H, W, s, p)
    assert dx.shape == dxr.shape
    assert relerr(dx, dxr) < 1e-2


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_wgrad(K, shape):
    N, H, W, Ci, Co, k, s, p = shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = rnd(N, Ho, Wo, Co)
    x = rnd(N, H, W, Ci)
    dw = K.conv_wgrad(dy.to(DEV), x.to(DEV), k, k, s, p)
    dwr = _ref.conv_wgrad(dy.float(), x.float(), k, k, s, p)
    assert dw.shape == dwr.shape
    assert relerr(dw, dwr) < 5e-3


def test_weight_prep(K):
    w = torch.randn(70, 3, 3, 24)
    wb, wt = K.weight_prep(w.to(DEV), 128, True)
    rb, rt = _ref.weight_prep(w, 128, True)
    assert wb.shape == rb.shape and wt.shape == rt.shape
    assert relerr(wb, rb) < 5e-3 and relerr(wt, rt) < 5e-3


@pytest.mark.parametrize("shape,co_pad,ci", [((70, 3, 3, 24), 128, 0), ((64, 1, 1, 256), 64, 0),
                                             ((64, 4, 4, 6), 64, 8), ((1000, 2048), 1024, 0)])
def test_mt_weight_prep_layouts(shape, co_pad, ci):
    """The per-step whole-model weight refresh (misc.hip mt_weight_prep: 4-wide path when every row
    is a multiple of 4 channels, scalar path otherwise -- the 6 -> 8 channel case) against the fp32
    weight: the bf16 copy [Co_pad][T][Ci] and the transposed copy [Ci][T][Co_pad], zero padded."""
    from ddp_classification_pytorch_amd.ops.functional import _MTWeightCache
    torch.manual_seed(0)
    w = torch.randn(*shape, device=DEV)
    wb, wt = _MTWeightCache().get(w, co_pad, True, ci)
    torch.cuda.synchronize()
    Co, Ci_src = shape[0], shape[-1]
    T = math.prod(shape[1:-1])
    Ci = ci or Ci_src
    ref = torch.zeros(co_pad, T, Ci)
    ref[:Co, :, :Ci_src] = w.cpu().reshape(Co, T, Ci_src).bfloat16().float()
    assert torch.equal(wb.float().cpu().reshape(co_pad, T, Ci), ref)
    assert torch.equal(wt.float().cpu().reshape(Ci, T, co_pad), ref.permute(2, 1, 0))


@pytest.mark.parametrize("B,K_,N,relu,bias", [(256, 2048, 512, True, True), (32, 512, 2176, False, True),
                                               (5, 256, 64, False, False)])
def test_linear(K, B, K_, N, relu, bias):
    x = rnd(B, K_)
    w = torch.randn(N, K_) / math.sqrt(K_)
    b = torch.randn(N) if bias else None
    wb, wt = K.weight_prep(w.to(DEV), N, True)
    y = K.linear_fwd(x.to(DEV), wb, b.to(DEV) if bias else None, int(relu))
    yr = _ref.linear_fwd(x.float(), w.bfloat16().float(), b, int(relu))
    assert relerr(y, yr) < 1e-2
    dy = rnd(B, N)
    dx = K.linear_fwd(dy.to(DEV), wt, None, 0)
    assert relerr(dx, dy.float() @ w.bfloat16().float()) < 1e-2
    dw = K.linear_wgrad(dy.to(DEV), x.to(DEV))
    assert relerr(dw, dy.float().t() @ x.float()) < 5e-3


def test_linear_unpadded_bias(K):
    """A 1000-way head on the 1024-wide padded GEMM with its 1000-entry bias: the columns past the
    bias get none (the epilogue reads only nbias entries); Fn.linear's bias gradient has 1000."""
    from ddp_classification_pytorch_amd.ops import functional as Fn
    x = rnd(64, 512)
    w = torch.randn(1000, 512) / math.sqrt(512)
    b = torch.randn(1000)
    wb, _ = K.weight_prep(w.to(DEV), 1024, True)
    y = K.linear_fwd(x.to(DEV), wb, b.to(DEV), 0)
    assert y.shape == (64, 1024)
    yr = x.float() @ w.bfloat16().float().t() + b
    assert relerr(y[:, :1000], yr) < 1e-2
    # padded weight rows are zero and no bias is added there
    assert y[:, 1000:].float().abs().max().item() == 0.0
    wd, bd = w.clone().to(DEV).requires_grad_(True), b.clone().to(DEV).requires_grad_(True)
    out = Fn.linear(x.to(DEV), wd, bd)
    assert out.shape == (64, 1000)
    g = rnd(64, 1000).to(DEV)
    out.backward(g)
    assert bd.grad.shape == (1000,) and relerr(bd.grad, g.float().sum(0)) < 1e-2


@pytest.mark.parametrize("act,res,shape", [(1, False, (4, 14, 14, 256)), (1, True, (4, 14, 14, 256)),
                                           (0, False, (4, 14, 14, 256)), (2, True, (4, 14, 14, 256)),
                                           (1, True, (8, 2, 2, 512)), (1, False, (8, 2, 2, 512)),
                                           (1, True, (3, 5, 7, 64))])
def test_bn_train_fwd_bwd(K, act, res, shape):
    N, H, W, C = shape
    x = rnd(N, H, W, C, scale=2.0) + 0.5
    r = rnd(N, H, W, C) if res else None
    g = torch.rand(C) + 0.5
    b = torch.randn(C) * 0.1
    rm, rv = torch.zeros(C), torch.ones(C)
    rmd, rvd = rm.to(DEV), rv.to(DEV)
    cnt = N * H * W
    tot = K.bn_stats(x.to(DEV), None)
    mean, invstd, scale, shift = K.bn_finalize(tot, g.to(DEV), b.to(DEV), rmd, rvd, 0.1, 1e-5)
    totr = _ref.bn_stats(x.float(), None)
    meanr, invr, scr, shr = _ref.bn_finalize(totr, g, b, rm, rv, 0.1, 1e-5)
    assert relerr(mean, meanr) < 1e-4 and relerr(invstd, invr) < 1e-4
    assert relerr(rmd, rm) < 1e-4 and relerr(rvd, rv) < 1e-4
    y = K.bn_act(x.to(DEV), r.to(DEV) if res else None, scale, shift, act, 0.01)
    yr = _ref.bn_act(x.float(), r.float() if res else None, scr, shr, act, 0.01)
    assert relerr(y, yr) < 1e-2
    dy = rnd(N, H, W, C)
    sums = K.bn_bwd_reduce(dy.to(DEV), x.to(DEV), r.to(DEV) if res else None, scale, shift, mean, invstd, act, 0.01)
    sumsr = _ref.bn_bwd_reduce(dy.float(), x.float(), r.float() if res else None, scr, shr, meanr, invr, act, 0.01)
    assert relerr(sums, sumsr) < 1e-3
    dx, dres = K.bn_bwd_elemt(dy.to(DEV), x.to(DEV), r.to(DEV) if res else None, scale, shift, mean, invstd, sums,
                              float(cnt), act, 0.01, res)
    dxr, dresr = _ref.bn_bwd_elemt(dy.float(), x.float(), r.float() if res else None, scr, shr, meanr, invr, sumsr,
                                   float(cnt), act, 0.01, res)
    assert relerr(dx, dxr) < 2e-2
    if res:
        assert relerr(dres, dresr) < 1e-2


def test_bn_matches_torch_batchnorm(K):
    # end-to-end against torch.nn.functional.batch_norm + relu autograd (fp32)
    N, H, W, C = 8, 7, 7, 64
    x = rnd(N, H, W, C) * 3 + 1
    g, b = torch.rand(C) + 0.5, torch.randn(C)
    xt = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    gt, bt = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yt = torch.relu(torch.nn.functional.batch_norm(xt, None, None, gt, bt, training=True, eps=1e-5))
    dy = torch.randn_like(yt)
    yt.backward(dy)
    from ddp_classification_pytorch_amd.ops import functional as Fn
    xd = x.to(DEV).requires_grad_(True)
    gd, bd = g.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    y = Fn.batch_norm_act(xd, None, gd, bd, torch.zeros(C, device=DEV), torch.ones(C, device=DEV), True, 0.1, 1e-5)
    y.backward(dy.permute(0, 2, 3, 1).contiguous().bfloat16().to(DEV))
    assert relerr(y, yt.detach().permute(0, 2, 3, 1)) < 1e-2
    assert relerr(xd.grad, xt.grad.permute(0, 2, 3, 1)) < 3e-2
    assert relerr(gd.grad, gt.grad) < 1e-2
    assert relerr(bd.grad, bt.grad) < 1e-2


@pytest.mark.parametrize("shape", [(3, 56, 56, 64), (2, 7, 7, 2048), (5, 28, 28, 256), (1, 3, 5, 8)])
def test_hw_reductions_split(K, shape):
    """global average pool and the SE channel-scale backward as two-level reductions over the
    rows (hw_splits row splits per image, 256 / (C/8) rows per pass) vs the fp32 reference"""
    torch.manual_seed(0)
    N, H, W, C = shape
    x = rnd(N, H, W, C)
    assert relerr(K.gap_fwd(x.to(DEV)), _ref.gap_fwd(x.float())) < 1e-2
    g, dy, r = rnd(N, C), rnd(N, H, W, C), rnd(N, H, W, C)
    for res, relu in [(None, False), (r, True)]:
        rd = res.to(DEV) if res is not None else None
        rf = res.float() if res is not None else None
        got = K.chan_scale_bwd(dy.to(DEV), x.to(DEV), g.to(DEV), rd, relu, res is not None)
        want = _ref.chan_scale_bwd(dy.float(), x.float(), g.float(), rf, relu, res is not None)
        # (dg comes back in the gate's dtype, bf16: one rounding of the fp32 sum)
        assert relerr(got[0], want[0]) < 1e-2 and relerr(got[1], want[1]) < 4e-3
        assert got[1].dtype == torch.bfloat16
        if res is not None:
            assert relerr(got[2], want[2]) < 1e-2


def test_pools(K):
    x = rnd(2, 17, 15, 64)
    y, idx = K.maxpool_fwd(x.to(DEV), 3, 2, 1)
    yr, idxr = _ref.maxpool_fwd(x.float(), 3, 2, 1)
    assert relerr(y, yr) < 1e-6
    dy = rnd(*y.shape)
    dx = K.maxpool_bwd(dy.to(DEV), idx, 17, 15, 3, 2, 1)
    dxr = _ref.maxpool_bwd(dy.float(), idx.cpu(), 17, 15, 3, 2, 1)
    assert relerr(dx, dxr) < 1e-2
    g = K.gap_fwd(x.to(DEV))
    assert relerr(g, _ref.gap_fwd(x.float())) < 1e-2
    dg = rnd(2, 64)
    assert relerr(K.gap_bwd(dg.to(DEV), 17, 15), _ref.gap_bwd(dg.float(), 17, 15)) < 1e-2
    s = K.space_to_depth(rnd(2, 16, 8, 8).to(DEV), 4, False)
    x2 = rnd(2, 16, 8, 8)
    assert torch.equal(K.space_to_depth(x2.to(DEV), 4, False).cpu(), _ref.space_to_depth(x2, 4, False))
    assert torch.equal(K.space_to_depth(K.space_to_depth(x2.to(DEV), 4, False), 4, True).cpu(), x2)


@pytest.mark.parametrize("ld,C,bf", [(2176, 2173, True), (10, 10, False), (64, 33, True)])
def test_xent(K, ld, C, bf):
    B = 16
    full = torch.randn(B, ld) * 3
    logits = full.bfloat16() if bf else full
    lab = torch.randint(0, C, (B,))
    loss, rank = K.xent_fwd(logits.to(DEV)[:, :C], lab.to(DEV), C, 0.0)
    lr_, rr = _ref.xent_fwd(logits[:, :C], lab, C, 0.0)
    assert relerr(loss, lr_) < 1e-4
    assert torch.equal(rank.cpu(), rr)
    go = torch.tensor(1.0, device=DEV)
    d = K.xent_bwd(logits.to(DEV)[:, :C], lab.to(DEV), C, go, 1.0 / B, 0.0, False)
    xt = logits[:, :C].float().clone().requires_grad_(True)
    torch.nn.functional.cross_entropy(xt, lab).backward()
    assert relerr(d, xt.grad) < 1e-4


def test_log_softmax(K):
    x = torch.randn(8, 256)
    y = K.log_softmax_fwd(x.to(DEV), 256)
    assert relerr(y, torch.log_softmax(x, 1)) < 1e-5
    dy = torch.randn(8, 256)
    xt = x.clone().requires_grad_(True)
    torch.log_softmax(xt, 1).backward(dy)
    dx = K.log_softmax_bwd(y, dy.to(DEV), 256, False)
    assert relerr(dx, xt.grad) < 1e-4


def test_arcface_fused_vs_reference_module():
    """Fused ArcFace fwd/bwd vs an fp32 autograd rendering of ArcMarginProduct + CE."""
    from ddp_classification_pytorch_amd.ops import functional as Fn
    torch.manual_seed(0)
    B, D, C = 32, 256, 1000
    x = torch.randn(B, D)
    W = torch.randn(C, D) * 0.05
    lab = torch.randint(0, C, (B,))
    s, m = 30.0, 0.5
    xt, Wt = x.clone().requires_grad_(True), W.clone().requires_grad_(True)
    cos = torch.nn.functional.linear(torch.nn.functional.normalize(xt), torch.nn.functional.normalize(Wt))
    sine = torch.sqrt((1.0 - cos.pow(2)).clamp(0, 1))
    phi = cos * math.cos(m) - sine * math.sin(m)
    phi = torch.where(cos > 0, phi, cos)
    oh = torch.zeros_like(cos).scatter_(1, lab.view(-1, 1), 1)
    out = (oh * phi + (1 - oh) * cos) * s
    lt = torch.nn.functional.cross_entropy(out, lab)
    lt.backward()
    xd, Wd = x.to(DEV).requires_grad_(True), W.to(DEV).requires_grad_(True)
    loss, rank, _ = Fn.arcface_loss(xd, Wd, lab.to(DEV), s, m, True)
    loss.backward()
    assert abs(loss.item() - lt.item()) / lt.item() < 2e-2
    assert relerr(xd.grad, xt.grad) < 5e-2
    assert relerr(Wd.grad, Wt.grad) < 5e-2


def test_fused_sgd_adam_match_torch():
    from ddp_classification_pytorch_amd.optim import FusedAdam, FusedSGD
    torch.manual_seed(0)
    shapes = [(64, 3, 3, 32), (5000,), (17, 9)]
    for mk, tk, kw in [(FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=5e-4, nesterov=True)),
                       (FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9)),
                       (FusedAdam, torch.optim.Adam, dict(lr=1e-3, weight_decay=1e-4))]:
        ps = [torch.randn(*s) for s in shapes]
        a = [p.clone().to(DEV).requires_grad_(True) for p in ps]
        b = [p.clone().requires_grad_(True) for p in ps]
        oa, ob = mk(a, **kw), tk(b, **kw)
        for _ in range(3):
            gs = [torch.randn(*s) for s in shapes]
            for p, g in zip(a, gs):
                p.grad = g.to(DEV)
            for p, g in zip(b, gs):
                p.grad = g.clone()
            oa.step()
            ob.step()
        for p, q in zip(a, b):
            assert relerr(p.detach(), q.detach()) < 1e-5


def test_fused_sgd_misaligned_grad_views():
    """The fused SGD step's 16-byte path needs 16-byte-aligned parameter, gradient and momentum
    slices; gradients that are views into one flat buffer at odd offsets (a bucket layout after a
    10-element bias) take the 4-byte loop.  Both must match torch.optim.SGD."""
    from ddp_classification_pytorch_amd.optim import FusedSGD
    torch.manual_seed(0)
    shapes = [(10,), (64, 3, 3, 32), (5000,), (4100,)]
    for kw in (dict(lr=0.1, momentum=0.9, weight_decay=5e-4, nesterov=True), dict(lr=0.05, momentum=0.0)):
        ps = [torch.randn(*sh) for sh in shapes]
        a = [p.clone().to(DEV).requires_grad_(True) for p in ps]
        b = [p.clone().requires_grad_(True) for p in ps]
        oa, ob = FusedSGD(a, **kw), torch.optim.SGD(b, **kw)
        n = sum(p.numel() for p in ps)
        for _ in range(3):
            flat = torch.randn(n + 1, device=DEV)
            off = 1  # every view starts 4 bytes past a 16-byte boundary (plus the running offsets)
            for p, q in zip(a, b):
                g = flat[off:off + p.numel()].view(p.shape)
                p.grad = g
                q.grad = g.detach().cpu().clone()
                off += p.numel()
            oa.step()
            ob.step()
        for p, q in zip(a, b):
            assert relerr(p.detach(), q.detach()) < 1e-5


def test_cdr_threshold_mask():
    from ddp_classification_pytorch_amd.algos.cdr import cdr_mask_gradients
    torch.manual_seed(0)
    params = [torch.randn(64, 3, 3, 16), torch.randn(1000, 20), torch.randn(37)]
    gd = [torch.randn_like(p) for p in params]
    pd = [p.to(DEV).requires_grad_(True) for p in params]
    for p, g in zip(pd, gd):
        p.grad = g.to(DEV)
    thr = cdr_mask_gradients(pd, nonzero_ratio=0.8, clip=0.8)
    # reference: CDR/main.py:186-204 over the 2-D/4-D tensors
    sel = [(p, g) for p, g in zip(params, gd) if p.dim() in (2, 4)]
    metric = torch.cat([(g * p).abs().view(-1) for p, g in sel])
    nz = int(0.8 * metric.numel())
    ref_thr = torch.topk(metric, nz)[0][-1]
    assert abs(float(thr) - float(ref_thr)) <= 1e-6 * float(ref_thr)
    for (p, g), q in zip(sel, [q for q in pd if q.dim() in (2, 4)]):
        mask = ((p * g).abs() >= ref_thr).float() * 0.8
        assert relerr(q.grad, mask * g) < 1e-6
    assert torch.equal(pd[2].grad.cpu(), gd[2])


def test_nested_eval_counts(K):
    torch.manual_seed(0)
    B, D, C = 16, 48, 37
    f = torch.randn(B, D)
    W = torch.randn(D, C)
    lab = torch.randint(0, C, (B,))
    cnt = K.nested_eval(f.to(DEV), W.to(DEV), lab.to(DEV))
    ref = _ref.nested_eval(f, W, lab)
    assert torch.equal(cnt.cpu(), ref)
    assert torch.equal(K.nested_eval_scalar(f.to(DEV), W.to(DEV), lab.to(DEV)).cpu(), ref)


@pytest.mark.parametrize("B,D,C", [(128, 2048, 2173), (37, 300, 70), (8, 65, 257), (130, 129, 4500)])
def test_nested_eval_fast_matches_scalar(K, B, D, C):
    """K19: the rank-ballot TestNested path counts exactly what the one-workgroup-per-sample kernel
    counts (identical fp32 fma chains), on the reference's shape (val batch 128, 2048 features,
    2173 classes), ragged sample / dimension / class counts, and C past the scalar kernel's 4096
    limit against the fp32 CPU reference; ReLU-like features with exact zeros included."""
    torch.manual_seed(1)
    f = torch.relu(torch.randn(B, D)).to(DEV)
    W = (torch.randn(D, C) * 0.05).to(DEV)
    lab = torch.randint(0, C, (B,)).to(DEV)
    fast = K.nested_eval(f, W, lab)
    if C <= 4096:
        assert torch.equal(fast, K.nested_eval_scalar(f, W, lab))
    else:
        ref = _ref.nested_eval(f.cpu()[:, :64], W.cpu()[:64], lab.cpu())
        assert (fast.cpu()[:64] - ref).abs().max().item() <= 1  # fma vs mul+add rounding: near-ties only
    assert fast[:, 0].le(fast[:, 1]).all() and fast.max().item() <= B


@pytest.mark.parametrize("Ci,Co,k,s", [(256, 64, 1, 1), (64, 128, 3, 1), (128, 64, 3, 2)])
def test_conv_dgrad_fused_add(K, Ci, Co, k, s):
    """dgrad epilogue that adds the identity-path gradient (ResidualLink)."""
    N, H = 2, 14
    p = k // 2
    Ho = (H + 2 * p - k) // s + 1
    w = torch.randn(Co, k, k, Ci) / (k * k * Ci) ** 0.5
    _, wt = K.weight_prep(w.to(DEV), 0, True)
    dy = rnd(N, Ho, Ho, Co)
    add = rnd(N, H, H, Ci)
    dx = K.conv_dgrad(dy.to(DEV), wt, H, H, s, p, add.to(DEV))
    ref = _ref.conv_dgrad(dy.float(), w.bfloat16().float().permute(3, 1, 2, 0), H, H, s, p).float() + add.float()
    assert relerr(dx, ref) < 1e-2


@pytest.mark.parametrize("N,H,Ci,Co,k,add,res,act", [
    (2, 14, 256, 64, 1, True, True, 1),     # conv1 of an identity block: join add + residual BN3
    (2, 14, 64, 64, 3, False, False, 1),    # conv2 (3x3 s1) consuming BN1 (BN=64 tile)
    (2, 14, 128, 512, 1, False, False, 1),  # conv3 consuming BN2, 128-channel tiles
    (3, 9, 72, 40, 3, True, False, 0),      # ragged M / channels, identity activation
    (8, 7, 512, 2048, 1, False, True, 1),   # layer4: M = 392 (not a multiple of 128)
    (4, 56, 256, 64, 1, True, True, 1),     # batch-4 layer1: 98 tiles -> the one-launch row reduction
    (40, 56, 64, 64, 3, False, False, 1),   # 980 tiles: the row reduction's 8-deep loop and tail
])
def test_conv_dgrad_bn_fused(K, N, H, Ci, Co, k, add, res, act):
    """dgrad epilogue fused with the BN(+ReLU)(+residual) backward reduction: the masked
    gradient and the per-channel (sum g', sum g' xhat) against the fp32 reference."""
    torch.manual_seed(0)
    p = k // 2
    w = torch.randn(Co, k, k, Ci) / (k * k * Ci) ** 0.5
    _, wt = K.weight_prep(w.to(DEV), 0, True)
    dy = rnd(N, H, H, Co)
    y = rnd(N, H, H, Ci, scale=2.0) + 0.5
    a = rnd(N, H, H, Ci) if add else None
    r = rnd(N, H, H, Ci) if res else None
    scale = torch.rand(Ci) + 0.5
    shift = torch.randn(Ci) * 0.3
    mean = torch.randn(Ci) * 0.2 + 0.5
    invstd = torch.rand(Ci) + 0.5
    d = lambda t: None if t is None else t.to(DEV)
    g, sums = K.conv_dgrad_bn(dy.to(DEV), wt, p, d(a), y.to(DEV), d(r), scale.to(DEV), shift.to(DEV),
                              mean.to(DEV), invstd.to(DEV), act)
    wtr = _ref.weight_prep(w.bfloat16().float(), 0, True)[1]
    rg, rsums = _ref.conv_dgrad_bn(dy.float(), wtr, p, None if a is None else a.float(), y.float(),
                                   None if r is None else r.float(), scale, shift, mean, invstd, act)
    assert relerr(g, rg) < 1e-2
    # masks can flip where the reference's z sits on 0; the sums are judged loosely but tightly
    # enough to catch a missing row, channel or tile
    assert relerr(sums[0], rsums[0]) < 2e-2
    assert relerr(sums[1], rsums[1]) < 2e-2


@pytest.mark.parametrize("N,H,W,C,G,KH,stride,pad", [
    (2, 14, 14, 128, 32, 3, 1, 1),   # CG=4  (super-group 16, 4 groups block-diagonal)
    (3, 13, 11, 256, 32, 3, 2, 1),   # CG=8, odd spatial, stride 2, M not a multiple of 256
    (2, 28, 28, 512, 32, 3, 2, 1),   # CG=16
    (4, 7, 7, 1024, 32, 3, 1, 1),    # CG=32 (super-group 32), blocks span many images
    (3, 14, 14, 1024, 32, 3, 2, 1),  # CG=32 stride 2: the largest halo (>64 KB LDS)
    (2, 9, 9, 64, 16, 1, 1, 0),      # 1x1 grouped
    (2, 10, 10, 128, 2, 3, 1, 1),    # CG=64: direct-kernel fallback
])
def test_grouped_conv_shapes(K, N, H, W, C, G, KH, stride, pad):
    x = rnd(N, H, W, C)
    w = rnd(C, KH, KH, C // G, scale=0.3)
    y = K.grouped_conv_fwd(x.to(DEV), w.to(DEV), G, stride, pad)
    assert relerr(y, _ref.grouped_conv_fwd(x.float(), w.float(), G, stride, pad)) < 1e-2
    dy = rnd(*y.shape)
    dx = K.grouped_conv_dgrad(dy.to(DEV), w.to(DEV), H, W, G, stride, pad)
    assert relerr(dx, _ref.grouped_conv_dgrad(dy.float(), w.float(), H, W, G, stride, pad)) < 1e-2
    dw = K.grouped_conv_wgrad(dy.to(DEV), x.to(DEV), KH, KH, G, stride, pad)
    assert relerr(dw, _ref.grouped_conv_wgrad(dy.float(), x.float(), KH, KH, G, stride, pad)) < 5e-3
    # split partials + a fixed-order reduce on every path (the direct fallback included): bitwise
    # reproducible
    assert torch.equal(dw, K.grouped_conv_wgrad(dy.to(DEV), x.to(DEV), KH, KH, G, stride, pad))


@pytest.mark.parametrize("sg", [16, 32])
def test_grouped_wgrad_supergroups(K, sg):
    """grouped-conv weight gradient with 16- and 32-channel super-groups (g_tune[16])"""
    torch.manual_seed(0)
    x, dy = rnd(2, 14, 14, 128), rnd(2, 14, 14, 128)
    try:
        K.set_tuning(tslot("gconv_sg"), sg)
        dw = K.grouped_conv_wgrad(dy.to(DEV), x.to(DEV), 3, 3, 32, 1, 1)
        torch.cuda.synchronize()
    finally:
        K.set_tuning(tslot("gconv_sg"), 0)
    assert relerr(dw, _ref.grouped_conv_wgrad(dy.float(), x.float(), 3, 3, 32, 1, 1)) < 5e-3


def test_grouped_and_dw_and_se(K):
    x = rnd(2, 14, 14, 128)
    w = rnd(128, 3, 3, 4, scale=0.3)
    y = K.grouped_conv_fwd(x.to(DEV), w.to(DEV), 32, 2, 1)
    assert relerr(y, _ref.grouped_conv_fwd(x.float(), w.float(), 32, 2, 1)) < 1e-2
    dy = rnd(*y.shape)
    dx = K.grouped_conv_dgrad(dy.to(DEV), w.to(DEV), 14, 14, 32, 2, 1)
    assert relerr(dx, _ref.grouped_conv_dgrad(dy.float(), w.float(), 14, 14, 32, 2, 1)) < 1e-2
    dw = K.grouped_conv_wgrad(dy.to(DEV), x.to(DEV), 3, 3, 32, 2, 1)
    assert relerr(dw, _ref.grouped_conv_wgrad(dy.float(), x.float(), 3, 3, 32, 2, 1)) < 5e-3
    filt = torch.tensor([1.0, 2.0, 1.0])
    filt = (filt[:, None] * filt[None, :]) / 16
    z = K.dwconv_fwd(x.to(DEV), filt.to(DEV), 3, 2, 1, True)
    assert relerr(z, _ref.dwconv_fwd(x.float(), filt, 3, 2, 1, True)) < 1e-2
    dz = rnd(*z.shape)
    assert relerr(K.dwconv_bwd(dz.to(DEV), filt.to(DEV), 14, 14, 3, 2, 1, True),
                  _ref.dwconv_bwd(dz.float(), filt, 14, 14, 3, 2, 1, True)) < 1e-2
    g = rnd(2, 128)
    r = rnd(*x.shape)
    for res, relu in [(None, False), (r, True)]:
        rd = res.to(DEV) if res is not None else None
        rf = res.float() if res is not None else None
        assert relerr(K.chan_scale_fwd(x.to(DEV), g.to(DEV), rd, relu),
                      _ref.chan_scale_fwd(x.float(), g.float(), rf, relu)) < 1e-2
        dyy = rnd(*x.shape)
        got = K.chan_scale_bwd(dyy.to(DEV), x.to(DEV), g.to(DEV), rd, relu, res is not None)
        want = _ref.chan_scale_bwd(dyy.float(), x.float(), g.float(), rf, relu, res is not None)
        assert relerr(got[0], want[0]) < 1e-2 and relerr(got[1], want[1]) < 1e-2
        if res is not None:
            assert relerr(got[2], want[2]) < 1e-2
    # sigmoid linear + its backward
    xs, ws = rnd(8, 64), torch.randn(64, 64) / 8
    wb, _ = K.weight_prep(ws.to(DEV), 64, False)
    ys = K.linear_fwd(xs.to(DEV), wb, None, 2)
    assert relerr(ys, torch.sigmoid(xs.float() @ ws.bfloat16().float().t())) < 1e-2
    dys = rnd(8, 64)
    assert relerr(K.act_bwd(dys.to(DEV), ys, 2), _ref.act_bwd(dys.float(), ys.float().cpu(), 2)) < 2e-2


def test_to_nhwc(K):
    img = torch.randint(0, 256, (2, 3, 20, 24), dtype=torch.uint8)
    mean = torch.tensor([0.485, 0.456, 0.406])
    std = torch.tensor([0.229, 0.224, 0.225])
    y = K.to_nhwc(img.to(DEV), True, 8, 1 / 255.0, mean.to(DEV), std.to(DEV))
    yr = _ref.to_nhwc(img, True, 8, 1 / 255.0, mean, std)
    assert y.shape == (2, 20, 24, 8)
    assert relerr(y, yr) < 1e-2
    # NHWC uint8 source (the data-loader path) and fp32 source
    imh = img.permute(0, 2, 3, 1).contiguous()
    assert relerr(K.to_nhwc(imh.to(DEV), False, 8, 1 / 255.0, mean.to(DEV), std.to(DEV)), yr) < 1e-2
    imf = torch.randn(2, 3, 20, 24)
    assert relerr(K.to_nhwc(imf.to(DEV), True, 8, 1.0, None, None), _ref.to_nhwc(imf, True, 8, 1.0, None, None)) < 1e-2


@pytest.mark.parametrize("nchw", [True, False])
def test_to_nhwc_s2d(K, nchw):
    img = torch.randint(0, 256, (3, 3, 20, 24), dtype=torch.uint8)
    if not nchw:
        img = img.permute(0, 2, 3, 1).contiguous()
    mean = torch.tensor([0.485, 0.456, 0.406])
    std = torch.tensor([0.229, 0.224, 0.225])
    y = K.to_nhwc_s2d(img.to(DEV), nchw, 1 / 255.0, mean.to(DEV), std.to(DEV))
    yr = _ref.to_nhwc_s2d(img, nchw, 1 / 255.0, mean, std)
    assert y.shape == (3, 10, 12, 16)
    assert relerr(y, yr) < 1e-2
    assert (y.view(-1, 4, 4)[:, :, 3] == 0).all()  # the pad channel of every phase


@pytest.mark.parametrize("nchw", [True, False])
def test_to_nhwc_s2d4_tresnet(K, nchw):
    """TResNet's SpaceToDepth(4) input in one pass from the images: [N, H/4, W/4, 48] ==
    space_to_depth(to_nhwc(images), 4) of the fp32 reference."""
    img = torch.randint(0, 256, (3, 3, 20, 24), dtype=torch.uint8)
    if not nchw:
        img = img.permute(0, 2, 3, 1).contiguous()
    mean = torch.tensor([0.485, 0.456, 0.406])
    std = torch.tensor([0.229, 0.224, 0.225])
    y = K.to_nhwc_s2d(img.to(DEV), nchw, 1 / 255.0, mean.to(DEV), std.to(DEV), 4)
    yr = _ref.space_to_depth(_ref.to_nhwc(img, nchw, 3, 1 / 255.0, mean, std), 4, False)
    assert y.shape == (3, 5, 6, 48)
    assert relerr(y, yr) < 1e-2


@pytest.mark.parametrize("N,H,Ci,Co,k,pad", [(4, 112, 16, 64, 4, 2), (2, 9, 16, 72, 4, 2), (3, 15, 64, 64, 3, 1)])
def test_conv_geo(K, N, H, Ci, Co, k, pad):
    """explicit-grid conv (the s2d stem: 4x4 taps, top/left pad 2, output grid = input grid)"""
    torch.manual_seed(0)
    x = rnd(N, H, H, Ci)
    w = rnd(Co, k, k, Ci, scale=(k * k * Ci) ** -0.5)
    y, slabs = K.conv_fwd_geo(x.to(DEV), w.to(DEV), 1, pad, H, H, True)
    yr, _ = _ref.conv_fwd_geo(x.float(), w.float(), 1, pad, H, H, False)
    assert relerr(y, yr) < 1e-2
    assert slabs.shape == ((N * H * H + 127) // 128, 2, Co)
    dy = rnd(N, H, H, Co)
    dw = K.conv_wgrad_geo(dy.to(DEV), x.to(DEV), k, k, 1, pad)
    assert relerr(dw, _ref.conv_wgrad_geo(dy.float(), x.float(), k, k, 1, pad)) < 1e-2


@pytest.mark.parametrize("N,H,W", [(4, 112, 112), (3, 30, 48), (2, 8, 16), (2, 9, 9), (3, 56, 56)])
def test_stem_fwd(K, N, H, W):
    """dedicated s2d stem kernel (stem.hip; (2, 9, 9) takes the implicit-GEMM fallback, W = 56 the
    half-tile rows of the 112 px input): output
    vs the fp32 conv, its BN partials (taken from the fp32 accumulators) vs statistics of the
    fp32 conv, and BN finalize from the partials vs from the stored bf16 activations"""
    torch.manual_seed(0)
    x = rnd(N, H, W, 16)
    w = rnd(64, 4, 4, 16, scale=256 ** -0.5)
    y, part = K.stem_fwd(x.to(DEV), w.to(DEV), True)
    yr, _ = _ref.conv_fwd_geo(x.float(), w.float(), 1, 2, H, W, False)
    assert y.shape == (N, H, W, 64)
    assert relerr(y, yr) < 1e-2
    rows = yr.double().reshape(-1, 64).to(DEV)
    if part.shape[1] == 3:
        assert part.shape == (N * ((H + 15) // 16), 3, 64)
        n = part[:, 0].double()
        assert torch.all(n.sum(0) == N * H * W)
        mu = (n * part[:, 1].double()).sum(0) / n.sum(0)
        m2 = part[:, 2].double().sum(0) + (n * (part[:, 1].double() - mu) ** 2).sum(0)
        assert torch.allclose(mu, rows.mean(0), atol=1e-5, rtol=1e-4)
        assert torch.allclose(m2 / rows.shape[0], rows.var(0, unbiased=False), atol=1e-6, rtol=1e-4)
    g, b = torch.rand(64, device=DEV) + 0.5, torch.randn(64, device=DEV)
    a = K.bn_stats_finalize(y, part, g, b, None, None, 0.1, 1e-5)
    r = K.bn_stats_finalize(y, None, g, b, None, None, 0.1, 1e-5)
    for u, v in zip(a, r):  # partials: fp32 accumulators; reference: the bf16-rounded y
        assert torch.allclose(u, v, atol=3e-3, rtol=5e-3)
    st = K.bn_stats(y, part)
    assert torch.allclose(st, K.bn_stats(y, None), atol=1e-3, rtol=5e-3)  # bf16 rounding of y
    y2, empty = K.stem_fwd(x.to(DEV), w.to(DEV), False)
    assert torch.equal(y2, y) and empty.numel() == 0


def test_s2d_stem_gpu_matches_plain_stem():
    """The s2d stem (4x4/1 over the space-to-depth input) vs the plain 7x7/2 conv on the HIP
    kernels: same output and, for the same upstream gradient, the same 7x7 weight gradient."""
    from ddp_classification_pytorch_amd.ops import functional as Fn

    torch.manual_seed(0)
    img = torch.randint(0, 256, (8, 3, 64, 64), dtype=torch.uint8, device=DEV)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    x8 = Fn.to_device_nhwc(img, mean, std, in_scale=1 / 255.0)
    x16 = Fn.to_device_nhwc(img, mean, std, in_scale=1 / 255.0, s2d=True)
    assert torch.equal(x16, Fn.nhwc_to_s2d(x8))
    w = (torch.randn(64, 7, 7, 3, device=DEV) * 0.05).requires_grad_(True)
    y1, _ = Fn.stem_conv_s2d(x16, w, torch.zeros(64, 4, 4, 16, device=DEV))
    y0, _ = Fn.conv2d(x8, w, 2, 3)
    assert y1.shape == y0.shape
    assert relerr(y1, y0) < 1e-2
    g = torch.randn_like(y0.float()).bfloat16()
    (g1,) = torch.autograd.grad(y1, w, g)
    (g0,) = torch.autograd.grad(y0, w, g)
    assert relerr(g1, g0) < 1e-2


@pytest.mark.parametrize("size,batch", [(64, 4), (96, 3), (224, 2), (112, 3)])  # 112: W = 56, half tiles
def test_fused_stem_matches_unfused(size, batch):
    """The one-op stem (stem conv + BN + ReLU + max pool, one-pass fused backward in stem.hip)
    against the unfused chain (stem conv, BN+ReLU+pool, two-pass BN/pool backward, implicit-GEMM
    weight gradient) on a ResNet-18: loss, stem / BN1 gradients and a deep layer's gradient."""
    import copy
    from ddp_classification_pytorch_amd.models import build_model, input_layout
    from ddp_classification_pytorch_amd.models import resnet as R
    from ddp_classification_pytorch_amd.ops import functional as Fn

    torch.manual_seed(0)
    m1 = build_model("resnet18", num_classes=10).to(DEV)
    m0 = copy.deepcopy(m1)
    img = torch.randint(0, 256, (batch, 3, size, size), dtype=torch.uint8, device=DEV)
    lab = torch.randint(0, 10, (batch,), device=DEV)
    mean, std = torch.tensor((0.485, 0.456, 0.406), device=DEV), torch.tensor((0.229, 0.224, 0.225), device=DEV)
    x = Fn.to_device_nhwc(img, mean, std, nchw=True, in_scale=1 / 255.0, **input_layout(m1))
    assert Fn.stem_bn_pool_fusable(x)
    losses = []
    prev = R._FUSED_STEM[0]
    for m, fused in ((m1, True), (m0, False)):
        R._FUSED_STEM[0] = fused
        try:
            loss = Fn.cross_entropy(m(x), lab)
            loss.backward()
        finally:
            R._FUSED_STEM[0] = prev
        losses.append(float(loss))
    assert abs(losses[0] - losses[1]) < 1e-3 * max(1.0, abs(losses[1]))
    assert relerr(m1.conv1.weight.grad, m0.conv1.weight.grad) < 2e-2
    assert relerr(m1.bn1.weight.grad, m0.bn1.weight.grad) < 2e-2
    assert relerr(m1.bn1.bias.grad, m0.bn1.bias.grad) < 2e-2
    assert relerr(m1.layer4[1].conv2.weight.grad, m0.layer4[1].conv2.weight.grad) < 2e-2
    assert torch.allclose(m1.bn1.running_mean, m0.bn1.running_mean, atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("shape,stride", [((8, 2, 2, 512), 1), ((8, 4, 4, 256), 2), ((4, 8, 8, 64), 1)])
def test_basic_block_vs_fp64(shape, stride):
    import copy
    import torch.nn.functional as F
    from ddp_classification_pytorch_amd.models.layers import BatchNorm2d, Conv2d
    from ddp_classification_pytorch_amd.models.resnet import BasicBlock
    from tests.model_mirror import _bn, _conv
    torch.manual_seed(0)
    N, H, W, C = shape
    planes = C if stride == 1 else 2 * C
    ds = None
    if stride != 1:
        ds = torch.nn.Sequential(Conv2d(C, planes, 1, stride, 0), BatchNorm2d(planes))
    b1 = BasicBlock(C, planes, stride, ds).to(DEV)
    b2 = copy.deepcopy(b1).double()
    x = torch.relu(torch.randn(N, H, W, C, device=DEV))
    x1 = x.bfloat16().requires_grad_(True)
    y1 = b1(x1)
    x2 = x1.detach().double().permute(0, 3, 1, 2).clone().requires_grad_(True)
    r = x2 if ds is None else _bn(_conv(x2, b2.downsample[0]), b2.downsample[1], True)
    z = F.relu(_bn(_conv(x2, b2.conv1), b2.bn1, True))
    z = _bn(_conv(z, b2.conv2), b2.bn2, True)
    y2 = F.relu(z + r)
    assert relerr(y1, y2.permute(0, 2, 3, 1)) < 3e-2
    g = torch.randn(y1.shape, device=DEV)
    y1.backward(g.bfloat16())
    y2.backward(g.double().permute(0, 3, 1, 2))
    # bf16 activations/gradients through two BN backwards: ~5 % from fp64 is the bf16 floor here
    assert relerr(x1.grad, x2.grad.permute(0, 2, 3, 1)) < 1e-1
    for (n, p1), (_, p2) in zip(b1.named_parameters(), b2.named_parameters()):
        assert relerr(p1.grad, p2.grad) < 1e-1, n


def test_bn_stats_large_mean_stable(K):
    """mean/std = 300: a (sum, sumsq) formulation in fp32 loses ~1e-2 of the variance."""
    torch.manual_seed(0)
    x = (300.0 + 1.0 * torch.randn(64, 30, 30, 64)).bfloat16()
    st = K.bn_stats(x.to(DEV), None)
    sr = _ref.bn_stats(x.float(), None)
    assert relerr(st[0, 2], sr[0, 2]) < 1e-3
    # and merged across "ranks"
    two = torch.cat([K.bn_stats(x[:32].contiguous().to(DEV), None), K.bn_stats(x[32:].contiguous().to(DEV), None)])
    mean, invstd, _, _ = K.bn_finalize(two, None, None, None, None, 0.1, 0.0)
    var = sr[0, 2] / sr[0, 0]
    assert relerr(invstd, 1 / var.sqrt()) < 1e-3


@pytest.mark.parametrize("shape", [(4, 32, 32, 64), (3, 17, 15, 64), (2, 12, 10, 128)])
def test_bn_act_maxpool_fused(K, shape):
    """stem BN + ReLU + 3x3/2 max pool fused: forward pooled values / argmax and both backward
    passes against the unfused reference chain."""
    N, H, W, C = shape
    torch.manual_seed(0)
    x = rnd(N, H, W, C, scale=2.0) + 0.3
    scale, shift = torch.rand(C) + 0.5, torch.randn(C) * 0.3
    mean, invstd = torch.randn(C) * 0.2, torch.rand(C) + 0.5
    d = lambda t: t.to(DEV)
    y, idx = K.bn_act_maxpool(d(x), d(scale), d(shift), 1, 3, 2, 1)
    yr, idxr = _ref.bn_act_maxpool(x.float(), scale, shift, 1, 3, 2, 1)
    assert relerr(y, yr) < 1e-2
    assert (idx.cpu() == idxr).float().mean().item() > 0.99  # ties on the bf16 grid may pick another max
    dy = rnd(*y.shape)
    sums = K.maxpool_bn_bwd_reduce(d(dy), idx, d(x), d(scale), d(shift), d(mean), d(invstd), 1, 3, 2, 1)
    sr = _ref.maxpool_bn_bwd_reduce(dy.float(), idx.cpu(), x.float(), scale, shift, mean, invstd, 1, 3, 2, 1)
    assert relerr(sums, sr) < 5e-3  # the kernel rounds the gathered pool gradient to bf16, as the unfused chain
    cnt = float(N * H * W)
    dx = K.maxpool_bn_bwd_elemt(d(dy), idx, d(x), d(scale), d(shift), d(mean), d(invstd), 1, sums, cnt, 3, 2, 1)
    dxr = _ref.maxpool_bn_bwd_elemt(dy.float(), idx.cpu(), x.float(), scale, shift, mean, invstd, 1, sr, cnt, 3, 2, 1)
    assert relerr(dx, dxr) < 2e-2


@pytest.mark.parametrize("N,H", [(4, 14), (48, 56)])
@pytest.mark.parametrize("slab", [False, True])
def test_bn_stats_finalize_fused_matches(K, slab, N, H):
    """Local-BN one-launch path == bn_finalize(bn_stats(.)) (the SyncBN path at world size 1) to
    rounding, running stats too, on the one-level slab merge (<= 1024 slabs of 128 rows) and the
    two-level merges (48 x 56 x 56 rows: 1176 slabs / 256 raw partials).  The statistics also match
    the fp64 reference."""
    torch.manual_seed(0)
    x = rnd(N, H, H, 64).to(DEV)
    slabs = None
    if slab:
        w = rnd(128, 1, 1, 64, scale=0.125)
        x, slabs = K.conv_fwd(x, w.to(DEV), 1, 0, True)
        st, sr = K.bn_stats(x, slabs), _ref.bn_stats(x.float().cpu(), None)
        assert torch.equal(st[0, 0].cpu(), sr[0, 0])
        assert relerr(st[0, 1], sr[0, 1]) < 1e-4 and relerr(st[0, 2], sr[0, 2]) < 1e-4
    C = x.shape[-1]
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    rm1, rv1 = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5
    rm2, rv2 = rm1.clone(), rv1.clone()
    ref = K.bn_finalize(K.bn_stats(x, slabs), g, b, rm1, rv1, 0.1, 1e-5)
    out = K.bn_stats_finalize(x, slabs, g, b, rm2, rv2, 0.1, 1e-5)
    # the same merge order in both; the two kernels' float contraction may differ in the last bit
    for r, o in zip(ref, out):
        assert torch.allclose(r, o, rtol=1e-5, atol=1e-8)
    assert torch.allclose(rm1, rm2, rtol=1e-5, atol=1e-8) and torch.allclose(rv1, rv2, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("cfg", [(("tg_stages", 3), ("tg_kdepth", 32)), (("tg_stages", 4), ("tg_kdepth", 32)),
                                 (("tg_stages", 3),)])
@pytest.mark.parametrize("shape", [(2, 14, 14, 256, 256, 3, 1, 1), (2, 28, 28, 128, 512, 1, 1, 0),
                                   (3, 9, 11, 64, 72, 3, 1, 1), (2, 56, 56, 64, 256, 1, 1, 0)])
def test_conv_pipeline_variants(K, cfg, shape):
    """Every tap-GEMM pipeline variant (k-tile depth 32/64, 2-4 LDS stages) against the
    fp32 reference: forward with statistics, data gradient, fused BN-backward data gradient."""
    N, H, W, Ci, Co, k, s, p = shape
    x = rnd(N, H, W, Ci)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci))
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = rnd(N, Ho, Wo, Co)
    wb, wt = K.weight_prep(w.float().to(DEV), 0, True)
    try:
        for i, v in cfg:
            K.set_tuning(tslot(i), v)
        y, slabs = K.conv_fwd(x.to(DEV), wb, s, p, True)
        dx = K.conv_dgrad(dy.to(DEV), wt, H, W, s, p)
        torch.cuda.synchronize()
    finally:
        for i, _ in cfg:
            K.set_tuning(tslot(i), 0)
    yr, _ = _ref.conv_fwd(x.float(), w.float(), s, p, False)
    assert relerr(y, yr) < 1e-2
    st = K.bn_stats(y, slabs)
    sr = _ref.bn_stats(y.float().cpu(), None)
    assert relerr(st[0, 1], sr[0, 1]) < 1e-4 and relerr(st[0, 2], sr[0, 2]) < 1e-4
    dxr = _ref.conv_dgrad(dy.float(), w.float().permute(3, 1, 2, 0), H, W, s, p)
    assert relerr(dx, dxr) < 1e-2


@pytest.mark.parametrize("cfg", [(("tg_stages", 3), ("tg_kdepth", 32)), (("tg_stages", 4), ("tg_kdepth", 32))])
def test_conv_dgrad_bn_pipeline_variants(K, cfg):
    """The fused BN-backward dgrad epilogue behind the 32-deep ring variants equals the
    default pipeline's result (same fp32 reference tolerance)."""
    torch.manual_seed(1)
    N, H, Ci, Co, k = 2, 14, 256, 128, 3
    w = torch.randn(Co, k, k, Ci) / (k * k * Ci) ** 0.5
    _, wt = K.weight_prep(w.to(DEV), 0, True)
    args = [rnd(N, H, H, Co).to(DEV), wt, 1, rnd(N, H, H, Ci).to(DEV), (rnd(N, H, H, Ci, scale=2.0) + 0.5).to(DEV),
            rnd(N, H, H, Ci).to(DEV), (torch.rand(Ci) + 0.5).to(DEV), (torch.randn(Ci) * 0.3).to(DEV),
            (torch.randn(Ci) * 0.2 + 0.5).to(DEV), (torch.rand(Ci) + 0.5).to(DEV), 1]
    g0, s0 = K.conv_dgrad_bn(*args)
    try:
        for i, v in cfg:
            K.set_tuning(tslot(i), v)
        g1, s1 = K.conv_dgrad_bn(*args)
        torch.cuda.synchronize()
    finally:
        for i, _ in cfg:
            K.set_tuning(tslot(i), 0)
    assert relerr(g1, g0) < 1e-2
    assert relerr(s1[0], s0[0]) < 2e-2 and relerr(s1[1], s0[1]) < 2e-2


def test_bn_act_mask_and_masked_dgrad_bn(K):
    """bn_act_mask's activation bits against the reference, and the fused BN-backward dgrad
    reading those bits instead of the residual gives the same result as recomputing z."""
    torch.manual_seed(2)
    N, H, Ci, Co = 2, 14, 256, 64
    y = rnd(N, H, H, Ci, scale=2.0)
    r = rnd(N, H, H, Ci)
    scale, shift = torch.rand(Ci) + 0.5, torch.randn(Ci) * 0.3
    mean, invstd = torch.randn(Ci) * 0.2, torch.rand(Ci) + 0.5
    z, mask = K.bn_act_mask(y.to(DEV), r.to(DEV), scale.to(DEV), shift.to(DEV), 1, 0.0)
    zr, mr = _ref.bn_act_mask(y, r, scale, shift, 1, 0.0)
    assert mask.shape == (N, H, H, Ci // 8) and mask.dtype == torch.uint8
    assert torch.equal(mask.cpu(), mr)
    assert relerr(z, zr) < 1e-2
    w = torch.randn(Co, 1, 1, Ci) / Ci ** 0.5
    _, wt = K.weight_prep(w.to(DEV), 0, True)
    dy, add = rnd(N, H, H, Co).to(DEV), rnd(N, H, H, Ci).to(DEV)
    d = lambda t: t.to(DEV)
    g0, s0 = K.conv_dgrad_bn(dy, wt, 0, add, d(y), d(r), d(scale), d(shift), d(mean), d(invstd), 1)
    g1, s1 = K.conv_dgrad_bn(dy, wt, 0, add, d(y), None, d(scale), d(shift), d(mean), d(invstd), 1, mask)
    assert torch.equal(g0, g1)
    # the two epilogue variants are separate instantiations: FMA contraction of the sums may differ
    assert relerr(s1, s0) < 1e-5


@pytest.mark.parametrize("cfg", [(("wg_rows", 32),), (("wg_rows", 32), ("wg_splits_per_cu", 4)), (("wg_cols", 4),),
                                 (("wg_cols", 3),), (("wg_rows", 32), ("wg_cols", 3)), (("wg_split_cap", 8),),
                                 (("wg_split_cap", 8), ("wg3x3", 1))])
@pytest.mark.parametrize("shape", [(2, 56, 56, 64, 64, 3, 1, 1), (2, 28, 28, 128, 512, 1, 1, 0),
                                   (2, 14, 14, 256, 128, 3, 2, 1), (3, 9, 11, 64, 72, 3, 1, 1),
                                   (8, 56, 56, 64, 64, 1, 1, 0)])  # > 64 splits: one-launch row reduction
def test_conv_wgrad_variants(K, cfg, shape):
    """Weight gradient with 32-row k-tiles, another split plan, the narrow (Co <= 64) kernel's
    256- / 192-column tiles (g_tune[14] = 4 / 3) and a capped split count (g_tune[27]; direct 3x3
    and implicit GEMM), against the fp32 reference."""
    N, H, W, Ci, Co, k, s, p = shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy, x = rnd(N, Ho, Wo, Co), rnd(N, H, W, Ci)
    try:
        for i, v in cfg:
            K.set_tuning(tslot(i), v)
        dw = K.conv_wgrad(dy.to(DEV), x.to(DEV), k, k, s, p)
        torch.cuda.synchronize()
    finally:
        for i, _ in cfg:
            K.set_tuning(tslot(i), 0)
    assert relerr(dw, _ref.conv_wgrad(dy.float(), x.float(), k, k, s, p)) < 5e-3


@pytest.mark.parametrize("N,H,W,Ci,Co", [(2, 56, 56, 64, 64), (2, 28, 28, 128, 128), (3, 14, 14, 256, 128),
                                        (2, 7, 7, 128, 64), (2, 13, 17, 64, 192), (1, 9, 112, 64, 64)])
def test_wgrad3x3_direct(K, N, H, W, Ci, Co):
    """Direct 3x3 / stride-1 weight gradient (wgrad3x3.hip: strip-staged windows, partial strips,
    several channel blocks) against the fp32 reference and the implicit-GEMM path (g_tune[15] = 1)."""
    torch.manual_seed(0)
    dy, x = rnd(N, H, W, Co), rnd(N, H, W, Ci)
    dw = K.conv_wgrad(dy.to(DEV), x.to(DEV), 3, 3, 1, 1)
    assert relerr(dw, _ref.conv_wgrad(dy.float(), x.float(), 3, 3, 1, 1)) < 5e-3
    try:
        K.set_tuning(tslot("wg3x3"), 1)
        dw_gemm = K.conv_wgrad(dy.to(DEV), x.to(DEV), 3, 3, 1, 1)
        torch.cuda.synchronize()
    finally:
        K.set_tuning(tslot("wg3x3"), 0)
    assert relerr(dw, dw_gemm) < 2e-3


@pytest.mark.parametrize("N,H,Ci,Co,k,pad", [(2, 32, 16, 64, 4, 2), (2, 16, 8, 64, 3, 1)])
def test_narrow_channel_conv_bk32(K, N, H, Ci, Co, k, pad):
    """Narrow-channel (per-lane tap lookup) convolution with 32-deep k-tiles (g_tune[13] = 32):
    the space-to-depth stem geometry and a CIFAR-style stem, against the fp32 reference."""
    x = rnd(N, H, H, Ci)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci))
    wb, _ = K.weight_prep(w.float().to(DEV), 0, False)
    try:
        K.set_tuning(tslot("narrow_kdepth"), 32)
        y, slabs = K.conv_fwd_geo(x.to(DEV), wb, 1, pad, H, H, True)
        torch.cuda.synchronize()
    finally:
        K.set_tuning(tslot("narrow_kdepth"), 0)
    yr, _ = _ref.conv_fwd_geo(x.float(), w.float(), 1, pad, H, H, False)
    assert relerr(y, yr) < 1e-2
    st = K.bn_stats(y, slabs)
    sr = _ref.bn_stats(y.float().cpu(), None)
    assert relerr(st[0, 1], sr[0, 1]) < 1e-4 and relerr(st[0, 2], sr[0, 2]) < 1e-4


@pytest.mark.parametrize("shape", [(2, 14, 14, 256), (3, 7, 9, 64), (1, 5, 5, 2048)])
def test_bn2_act_mask_shortcut_bn(K, shape):
    """BN + ReLU with a projection-shortcut residual normalised on the fly (bn2_act_mask) against
    the reference, and equal to bn_act_mask over the materialised shortcut activation."""
    torch.manual_seed(5)
    C = shape[-1]
    x, r = rnd(*shape, scale=2.0), rnd(*shape, scale=3.0)
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.3
    rsc, rsh = torch.rand(C) + 0.2, torch.randn(C) * 0.5
    d = lambda t: t.to(DEV)
    y, m = K.bn2_act_mask(d(x), d(r), d(sc), d(sh), d(rsc), d(rsh), 1, 0.0)
    yr, mr = _ref.bn2_act_mask(x, r, sc, sh, rsc, rsh, 1, 0.0)
    assert relerr(y, yr) < 1e-2
    assert (m.cpu() != mr).float().mean().item() < 1e-3  # bits may differ only where z rounds across 0
    rv = K.bn_act(d(r), None, d(rsc), d(rsh), 0, 0.0)
    y2, _ = K.bn_act_mask(d(x), rv, d(sc), d(sh), 1, 0.0)
    assert relerr(y, y2) < 1e-2


def test_bn2_bwd_elemt_matches_two_passes(K):
    torch.manual_seed(6)
    N, H, C = 2, 14, 256
    g, x, r = rnd(N, H, H, C), rnd(N, H, H, C, scale=2.0), rnd(N, H, H, C, scale=3.0)
    d = lambda t: t.to(DEV)
    pr = [torch.rand(C) + 0.5, torch.randn(C) * 0.2, torch.rand(C) + 0.5, torch.randn(2, C) * 5]
    qr = [torch.rand(C) + 0.2, torch.randn(C) * 0.4, torch.rand(C) + 0.3, torch.randn(2, C) * 7]
    count = float(N * H * H)
    dx, dr = K.bn2_bwd_elemt(d(g), d(x), d(r), *[d(t) for t in pr], *[d(t) for t in qr], count)
    rx, rr = _ref.bn2_bwd_elemt(g, x, r, *pr, *qr, count)
    assert relerr(dx, rx) < 1e-2 and relerr(dr, rr) < 1e-2
    z = torch.zeros(C)
    dx1, _ = K.bn_bwd_elemt(d(g), d(x), None, d(pr[0]), d(z), d(pr[1]), d(pr[2]), d(pr[3]), count, 0, 0.0, False)
    assert relerr(dx, dx1) < 1e-3


@pytest.mark.parametrize("de", [0, 1])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("N,H,W", [(2, 56, 56), (3, 7, 9), (1, 13, 30), (2, 28, 28), (1, 1, 5), (1, 4, 126),
                                   (2, 64, 64), (16, 16, 16)])
def test_conv3x3_direct_c64(K, N, H, W, variant, de):
    """The direct 64->64 3x3 kernel (conv3x3.hip) against the reference conv and against the
    implicit GEMM it replaces (g_tune[18] = 1 forces the latter); BN partials vs bn_stats.
    de = 1: the register-direct store epilogue (default; g_tune[30] = 2: the LDS-staged one)."""
    torch.manual_seed(7)
    x = rnd(N, H, W, 64, scale=2.0).abs()  # post-ReLU-like input: non-zero channel means
    w = rnd(64, 3, 3, 64, scale=1.0 / 24)
    K.set_tuning(tslot("c3_variant"), variant)  # 0: 8 waves, double-buffered; 1: 4 waves, single; 2: 4 waves, double;
    # 3 / 4: variant 0 with s_setprio for the upper wave half / the upper half's subtiles reversed
    K.set_tuning(tslot("c3_epilogue"), 0 if de else 2)
    try:
        y, part = K.conv_fwd(x.to(DEV), w.to(DEV), 1, 1, True)
        y3, none = K.conv_fwd(x.to(DEV), w.to(DEV), 1, 1, False)
    finally:
        K.set_tuning(tslot("c3_variant"), 0)
        K.set_tuning(tslot("c3_epilogue"), 0)
    if W <= 100 and variant != 2:  # wider rows / the smaller windows of variant 2: implicit GEMM (slabs)
        assert part.shape[1:] == (3, 64)  # (n, mean, M2) partials of the direct kernel
    yr, _ = _ref.conv_fwd(x.float(), w.float(), 1, 1, False)
    assert relerr(y, yr) < 1e-2
    K.set_tuning(tslot("c3_off"), 1)
    try:
        y2, _ = K.conv_fwd(x.to(DEV), w.to(DEV), 1, 1, True)
    finally:
        K.set_tuning(tslot("c3_off"), 0)
    assert relerr(y, y2) < 5e-3
    st = K.bn_stats(y, part)
    sr = _ref.bn_stats(y.float().cpu(), None)
    assert torch.equal(st[0, 0].cpu(), sr[0, 0])
    assert relerr(st[0, 1], sr[0, 1]) < 1e-4
    assert relerr(st[0, 2], sr[0, 2]) < 1e-4
    assert none.numel() == 0 and torch.equal(y3, y)


def test_gap_bwd_with_add(K):
    torch.manual_seed(9)
    dy, add = rnd(3, 96), rnd(3, 5, 7, 96)
    out = K.gap_bwd(dy.to(DEV), 5, 7, add.to(DEV))
    ref = _ref.gap_bwd(dy, 5, 7, add)
    assert relerr(out, ref) < 1e-2
    assert relerr(K.gap_bwd(dy.to(DEV), 5, 7), _ref.gap_bwd(dy, 5, 7)) < 1e-2


@pytest.mark.parametrize("N,H,C,s", [(2, 56, 128, 1), (3, 14, 512, 1), (2, 28, 256, 2), (1, 7, 1024, 1)])
def test_grouped_conv_fwd_stats(K, N, H, C, s):
    """ResNeXt 32x4d grouped 3x3 forward with the BN partials from the MFMA epilogue."""
    torch.manual_seed(11)
    G = 32
    x = rnd(N, H, H, C, scale=2.0).abs()
    w = rnd(C, 3, 3, C // G, scale=1.0 / math.sqrt(9 * C // G))
    y0 = K.grouped_conv_fwd(x.to(DEV), w.to(DEV), G, s, 1)
    y, part = K.grouped_conv_fwd_stats(x.to(DEV), w.to(DEV), G, s, 1)
    assert torch.equal(y, y0)
    assert part.dim() == 3 and part.shape[1:] == (3, C)
    st = K.bn_stats(y, part)
    sr = _ref.bn_stats(y.float().cpu(), None)
    assert torch.equal(st[0, 0].cpu(), sr[0, 0])
    assert relerr(st[0, 1], sr[0, 1]) < 1e-4
    assert relerr(st[0, 2], sr[0, 2]) < 1e-4


@pytest.mark.parametrize("N,H,C", [(2, 56, 128), (3, 14, 512), (1, 7, 1024)])
def test_grouped_conv_dgrad_bn(K, N, H, C):
    """Grouped dgrad with the ReLU-BN backward reduction in its epilogue vs the reference."""
    torch.manual_seed(12)
    G = 32
    dy = rnd(N, H, H, C)
    w = rnd(C, 3, 3, C // G, scale=1.0 / math.sqrt(9 * C // G))
    z = rnd(N, H, H, C, scale=2.0)
    scale, shift = torch.rand(C) + 0.5, torch.randn(C) * 0.3
    mean, invstd = torch.randn(C) * 0.2, torch.rand(C) + 0.5
    d = lambda t: t.to(DEV)
    g, sums = K.grouped_conv_dgrad_bn(d(dy), d(w), H, H, G, 1, 1, d(z), d(scale), d(shift), d(mean), d(invstd))
    gr, sr = _ref.grouped_conv_dgrad_bn(dy, w, H, H, G, 1, 1, z, scale, shift, mean, invstd)
    assert relerr(g, gr) < 1e-2
    assert sums.shape == (2, C)
    assert relerr(sums, sr) < 2e-2
    dx = K.grouped_conv_dgrad(d(dy), d(w), H, H, G, 1, 1)
    zr = z.float() * scale + shift
    ref = torch.where(zr > 0, dx.cpu(), torch.zeros_like(dx.cpu()))
    assert (g.cpu() != ref).float().mean().item() < 1e-3  # masks may differ only where z*scale+shift ~ 0


@pytest.mark.parametrize("N,H,C,s", [(2, 56, 128, 1), (3, 13, 256, 2), (2, 14, 512, 1), (3, 7, 1024, 1),
                                     (2, 14, 1024, 2)])
@pytest.mark.parametrize("spw", [2, 3, 8, 83, 34])  # 10 * spw + ring buffers: 8 x 3 ring, 3 x 3 ring
def test_grouped_conv_multi_supergroup_matches(K, N, H, C, s, spw):
    """Forward (+BN partials) and data gradient (plain and BN-fused) with several super-groups per
    workgroup (g_tune gconv_spw; an LDS ring of halo + weight-fragment (+ z) stages) against one
    super-group per workgroup: the same MFMA sums in the same order, so bitwise-equal outputs."""
    torch.manual_seed(21)
    G = 32
    Ho = (H + 2 - 3) // s + 1
    d = lambda t: t.to(DEV)
    x = rnd(N, H, H, C, scale=2.0)
    w = rnd(C, 3, 3, C // G, scale=1.0 / math.sqrt(9 * C // G))
    dy = rnd(N, Ho, Ho, C)
    co = [torch.rand(C) + 0.5, torch.randn(C) * 0.3, torch.randn(C) * 0.2, torch.rand(C) + 0.5]
    out = {}
    try:
        for v in (1, spw):
            K.set_tuning(tslot("gconv_spw"), v)
            y, part = K.grouped_conv_fwd_stats(d(x), d(w), G, s, 1)
            dx = K.grouped_conv_dgrad(d(dy), d(w), H, H, G, s, 1)
            g, sums = K.grouped_conv_dgrad_bn(d(dy), d(w), H, H, G, s, 1, d(x), *[d(c) for c in co])
            torch.cuda.synchronize()
            out[v] = (y.cpu(), part.cpu(), dx.cpu(), g.cpu(), sums.cpu())
    finally:
        K.set_tuning(tslot("gconv_spw"), 0)
    y1, p1, dx1, g1, s1 = out[1]
    y2, p2, dx2, g2, s2 = out[spw]
    assert torch.equal(y1, y2) and torch.equal(dx1, dx2) and torch.equal(g1, g2)
    assert torch.allclose(p1, p2, rtol=1e-5, atol=1e-5)
    assert torch.allclose(s1, s2, rtol=1e-5, atol=1e-4)
    assert relerr(y2, _ref.grouped_conv_fwd(x.float(), w.float(), G, s, 1)) < 1e-2
    assert relerr(dx2, _ref.grouped_conv_dgrad(dy.float(), w.float(), H, H, G, s, 1)) < 1e-2


@pytest.mark.parametrize("M,C", [(1024, 1000), (7, 16), (3000, 2048), (1, 8), (513, 4096)])
def test_colsum(K, M, C):
    x = rnd(M, C)
    out = K.colsum(x.to(DEV))
    assert relerr(out, x.float().sum(0)) < 1e-5


@pytest.mark.parametrize("k,add", [(3, False), (1, True), (3, True)])
def test_conv_dgrad_bn_leaky(K, k, add):
    """Leaky-ReLU BN fused into the dgrad epilogue: raw gradient stored, masked sums."""
    torch.manual_seed(13)
    N, H, Ci, Co = 2, 14, 64, 128
    pad = k // 2
    dy = rnd(N, H, H, Co)
    w = torch.randn(Co, k, k, Ci) / math.sqrt(k * k * Co)
    _, wt = K.weight_prep(w.to(DEV), 0, True)
    y = rnd(N, H, H, Ci, scale=2.0)
    a = rnd(N, H, H, Ci) if add else None
    scale, shift = torch.rand(Ci) + 0.5, torch.randn(Ci) * 0.3
    mean, invstd = torch.randn(Ci) * 0.2, torch.rand(Ci) + 0.5
    d = lambda t: t.to(DEV) if t is not None else None
    g, s = K.conv_dgrad_bn(d(dy), wt, pad, d(a), d(y), None, d(scale), d(shift), d(mean), d(invstd), 2, None, 1e-3)
    wtr = _ref.weight_prep(w.bfloat16().float(), 0, True)[1]
    gr, sr = _ref.conv_dgrad_bn(dy.float(), wtr, pad, None if a is None else a.float(), y.float(), None, scale, shift,
                                mean, invstd, 2, None, 1e-3)
    assert relerr(g, gr) < 1e-2
    assert relerr(s, sr) < 2e-2


@pytest.mark.parametrize("shape", [(2, 56, 56, 64, 256, 1, 1, 0), (2, 28, 28, 128, 128, 3, 1, 1),
                                   (2, 56, 56, 128, 128, 3, 2, 1), (2, 28, 28, 256, 512, 1, 2, 0),
                                   (3, 9, 11, 64, 72, 3, 1, 1), (2, 7, 7, 512, 2048, 1, 1, 0)])
@pytest.mark.parametrize("act,res", [(1, False), (1, True), (0, False), (2, False)])
def test_conv_fwd_affine_folded_bn(K, shape, act, res):
    """Eval-mode BN folded into the conv store epilogue == conv -> bf16 -> BN apply (+res) -> act."""
    N, H, W, Ci, Co, k, s, p = shape
    x = rnd(N, H, W, Ci)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci))
    scale = torch.rand(Co) + 0.5
    shift = torch.randn(Co) * 0.2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    r = rnd(N, Ho, Wo, Co) if res else None
    y = K.conv_fwd_affine(x.to(DEV), w.to(DEV), s, p, scale.to(DEV), shift.to(DEV), act, 0.1,
                          r.to(DEV) if res else None)
    c, _ = K.conv_fwd(x.to(DEV), w.to(DEV), s, p, False)  # the unfused chain's bf16 conv output
    yr = _ref.bn_act(c.cpu().float(), r.float() if res else None, scale, shift, act, 0.1)
    assert y.shape == yr.shape
    assert relerr(y, yr) < 5e-3


@pytest.mark.parametrize("act,want_g", [(1, True), (1, False), (0, False), (2, True)])
def test_act_scale_bwd(K, act, want_g):
    M, C = 3000, 256
    dy, y = rnd(M, C), rnd(M, C)
    scale = torch.rand(C) + 0.5
    dc, g = K.act_scale_bwd(dy.to(DEV), y.to(DEV), scale.to(DEV), act, 0.1, want_g)
    dcr, gr = _ref.act_scale_bwd(dy.float(), y.float(), scale, act, 0.1, want_g)
    assert relerr(dc, dcr) < 5e-3
    if want_g:
        assert relerr(g, gr) < 5e-3


@pytest.mark.parametrize("act", [2, 0])
def test_bn_backward_inplace_abn_from_output(K, act):
    """InplaceABN backward kernels (inv): reading only the output y = act(x*scale + shift) with
    beta / 1/gamma in the mean / invstd slots == the standard backward reading the input x."""
    M, C = 4096, 128
    x = rnd(M, C)
    gamma = torch.rand(C) + 0.5
    beta = torch.randn(C) * 0.3
    mean = torch.randn(C) * 0.1
    invstd = torch.rand(C) + 0.5
    scale = gamma * invstd
    shift = beta - mean * scale
    slope = 0.01
    y = _ref.bn_act(x.float(), None, scale, shift, act, slope).bfloat16()
    dy = rnd(M, C)
    d = lambda t: t.to(DEV)  # noqa: E731
    got = K.bn_bwd_reduce(d(dy), d(y), None, d(scale), d(shift), d(beta), d(1.0 / gamma), act, slope, True)
    ref = _ref.bn_bwd_reduce(dy.float(), x.float(), None, scale, shift, mean, invstd, act, slope)
    assert relerr(got, ref) < 2e-2  # y is bf16: the recovered xhat carries its rounding
    dx, _ = K.bn_bwd_elemt(d(dy), d(y), None, d(scale), d(shift), d(beta), d(1.0 / gamma), d(ref), float(M), act,
                           slope, False, True)
    dxr, _ = _ref.bn_bwd_elemt(dy.float(), x.float(), None, scale, shift, mean, invstd, ref, float(M), act, slope,
                               False)
    assert relerr(dx, dxr) < 2e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_philox_dropout(K, dtype):
    """Philox dropout: keep fraction ~ 1 - p, kept values scaled by 1/(1-p), backward regenerates the
    forward's mask, and every call (the device counter advances) draws a new mask."""
    from ddp_classification_pytorch_amd.ops import functional as Fn

    x = torch.ones(257, 1031, device=DEV, dtype=dtype, requires_grad=True)
    y = Fn.dropout(x, 0.3)
    keep = (y != 0)
    frac = keep.float().mean().item()
    assert abs(frac - 0.7) < 0.01, frac
    assert torch.allclose(y[keep].float(), torch.full_like(y[keep].float(), 1 / 0.7), rtol=1e-2)
    y.backward(torch.ones_like(y))
    assert torch.equal(x.grad != 0, keep)
    y2 = Fn.dropout(x, 0.3)
    assert not torch.equal(y2 != 0, keep)


def test_adaptive_avg_pool_kernels(K):
    x = rnd(2, 10, 13, 64)
    y = K.adaptive_avg_pool(x.to(DEV), 7, 7)
    yr = _ref.adaptive_avg_pool(x.float(), 7, 7)
    assert relerr(y, yr) < 5e-3
    dy = rnd(2, 7, 7, 64)
    dx = K.adaptive_avg_pool_bwd(dy.to(DEV), 10, 13)
    dxr = _ref.adaptive_avg_pool_bwd(dy.float(), 10, 13)
    assert relerr(dx, dxr) < 5e-3


@pytest.mark.parametrize("shape", [(2, 14, 14, 256, 256, 3, 1, 1), (3, 28, 28, 128, 512, 1, 1, 0),
                                   (2, 7, 7, 512, 2048, 1, 1, 0), (2, 28, 28, 256, 512, 1, 2, 0),
                                   (3, 9, 11, 128, 128, 3, 1, 1), (1, 13, 13, 256, 384, 3, 2, 1),
                                   (2, 7, 7, 1024, 256, 1, 1, 0), (5, 3, 3, 64, 320, 3, 1, 1)])
@pytest.mark.parametrize("mode", [1, 3])
@pytest.mark.parametrize("cvar", [0, 1, 2, 3])
@pytest.mark.parametrize("stages,persist", [(0, 0), (5, 0), (0, 1)])
def test_big_tile_tap_gemm_matches(K, shape, mode, cvar, stages, persist):
    """The 8-wave 256 x 256 (tg_big = 1; 256 x 128 below 256 channels) and 4-wave 256 x 128
    (tg_big = 3) big-tile tap GEMMs under every schedule: the 8-wave tile's default ping-pong
    (tg_big_cvar = 0 / 3), fragments read across the barrier in lockstep (1; the 4-wave tile's
    default) or after it (2), == the fp32 reference and the 128-row kernel: forward with BN statistics (ragged
    M: quadrants past M write no slab) and the data gradient (stride 1 and the stride-2 parity
    classes), channel counts that are not a multiple of the tile; the 256 x 256 tile also with its
    5-slot (160 KB) LDS-DMA ring (tg_big_stages = 5), and both tiles as persistent workgroups
    looping over tiles (tg_big_persist = 1)."""
    if stages and mode != 1:
        pytest.skip("the 5-slot ring is the 256 x 256 tile's")
    N, H, W, Ci, Co, k, s, p = shape
    torch.manual_seed(0)
    x = rnd(N, H, W, Ci).to(DEV)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci)).to(DEV)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = rnd(N, Ho, Wo, Co).to(DEV)
    wb, wt = K.weight_prep(w.float(), 0, True)
    outs = []
    try:
        for m in (2, mode):
            K.set_tuning(tslot("tg_big"), m)
            K.set_tuning(tslot("tg_big_cvar"), cvar if m != 2 else 0)
            K.set_tuning(tslot("tg_big_stages"), stages if m != 2 else 0)
            K.set_tuning(tslot("tg_big_persist"), persist if m != 2 else 0)
            y, slabs = K.conv_fwd(x, wb, s, p, True)
            st = K.bn_stats(y, slabs)
            dx = K.conv_dgrad(dy, wt, H, W, s, p)
            torch.cuda.synchronize()
            outs.append((y.float().cpu(), st.cpu(), dx.float().cpu()))
    finally:
        K.set_tuning(tslot("tg_big"), 0)
        K.set_tuning(tslot("tg_big_cvar"), 0)
        K.set_tuning(tslot("tg_big_stages"), 0)
        K.set_tuning(tslot("tg_big_persist"), 0)
    (y0, s0, d0), (y1, s1, d1) = outs
    assert relerr(y1, y0) < 1e-2 and relerr(d1, d0) < 1e-2
    assert torch.equal(s1[0, 0], s0[0, 0]) and relerr(s1[0, 1:], s0[0, 1:]) < 1e-3
    yr, _ = _ref.conv_fwd(x.float().cpu(), w.float().cpu(), s, p, False)
    assert relerr(y1, yr) < 1e-2
    sr = _ref.bn_stats(y1, None)
    assert relerr(s1[0, 1], sr[0, 1]) < 1e-4 and relerr(s1[0, 2], sr[0, 2]) < 1e-4
    dxr = _ref.conv_dgrad(dy.float().cpu(), w.float().cpu().permute(3, 1, 2, 0), H, W, s, p)
    assert relerr(d1, dxr) < 1e-2


@pytest.mark.parametrize("shape", [
    (2, 56, 56, 64, 256),    # stage-1 conv3: one 64-deep k-tile, 128-wide tiles
    (3, 28, 28, 128, 512),   # stage 2: 32-deep k-tiles
    (2, 14, 14, 256, 1024),  # stage 3 (weight gradient: the 256x256 tile kernel)
    (4, 7, 7, 512, 2048),    # stage 4
    (3, 13, 11, 128, 256),   # M not a multiple of 128
    (2, 9, 9, 64, 64),       # 64-wide tiles
])
def test_conv_bn_prologue(K, shape):
    """K5: BN + ReLU applied to the 1x1 conv's operands in registers == the fp32 reference of
    conv(bf16(relu(x * scale + shift))) -- forward output, its BN statistics slabs and the weight
    gradient (the input recomputed in the B fragments)."""
    N, H, W, C, Co = shape
    torch.manual_seed(0)
    x = rnd(N, H, W, C)
    w = rnd(Co, 1, 1, C, scale=1.0 / math.sqrt(C))
    scale = torch.rand(C) + 0.5
    shift = torch.randn(C) * 0.5
    y, slabs = K.conv_fwd_pro(x.to(DEV), w.to(DEV), scale.to(DEV), shift.to(DEV), True)
    yr, _ = _ref.conv_fwd_pro(x.float(), w.float(), scale, shift, False)
    assert y.shape == (N, H, W, Co)
    assert relerr(y, yr) < 5e-3
    st = K.bn_stats(y, slabs)
    rst = _ref.bn_stats(y.cpu().float(), None)
    assert relerr(st[0, 1], rst[0, 1]) < 1e-3 and relerr(st[0, 2], rst[0, 2]) < 1e-3
    dy = rnd(N, H, W, Co)
    dw = K.conv_wgrad_pro(dy.to(DEV), x.to(DEV), scale.to(DEV), shift.to(DEV))
    dwr = _ref.conv_wgrad_pro(dy.float(), x.float(), scale, shift)
    assert dw.shape == (Co, 1, 1, C)
    assert relerr(dw, dwr) < 5e-3


def test_iabn_gamma_and_sign_mul(K):
    """InplaceABN effective weight |g| + eps with its reciprocal, and the gradient d * sign(g)."""
    g = torch.randn(1000)
    g[::7] = 0.0
    d = torch.randn(1000)
    ge, rg = K.iabn_gamma(g.to(DEV), 1e-5)
    rge, rrg = _ref.iabn_gamma(g, 1e-5)
    assert torch.allclose(ge.cpu(), rge) and torch.allclose(rg.cpu(), rrg, rtol=1e-6)
    assert torch.equal(K.sign_mul(d.to(DEV), g.to(DEV)).cpu(), _ref.sign_mul(d, g))


@pytest.mark.parametrize("C", [64, 1024, 2048])
def test_iabn_folded_finalize_and_weight_gradient(K, C):
    """The InplaceABN effective weight folded into the BN kernels: the finalize with iabn_eps ==
    the finalize of |g| + eps (and writes 1 / (|g| + eps)), and bn_bwd_elemt's graw output ==
    sums[1] * sign(g) (zeros included), while its dx is unchanged."""
    M = 3000
    torch.manual_seed(C)
    x = rnd(M, C).to(DEV)
    g = torch.randn(C)
    g[::5] = 0.0
    b = torch.randn(C) * 0.1
    eff = g.abs() + 1e-5
    rg = torch.empty(C, device=DEV)
    outs = []
    for gamma, ie, out in ((g, 1e-5, rg), (eff, -1.0, None)):
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        outs.append(K.bn_stats_finalize(x, None, gamma.to(DEV), b.to(DEV), rm, rv, 0.1, 1e-5, ie, out) + (rm, rv))
    for a, c in zip(*outs):
        assert torch.equal(a, c)
    assert torch.allclose(rg.cpu(), 1.0 / eff, rtol=1e-6)
    mean, invstd, scale, shift = outs[1][:4]
    y = K.bn_act(x, None, scale, shift, 2, 0.01)
    dy = rnd(M, C).to(DEV)
    sums = K.bn_bwd_reduce(dy, y, None, scale, shift, b.to(DEV), rg, 2, 0.01, True)
    dx1, dg = K.bn_bwd_elemt(dy, y, None, scale, shift, b.to(DEV), rg, sums, float(M), 2, 0.01, False, True, g.to(DEV))
    dx0, _ = K.bn_bwd_elemt(dy, y, None, scale, shift, b.to(DEV), rg, sums, float(M), 2, 0.01, False, True)
    assert torch.equal(dx1, dx0)
    assert torch.equal(dg.cpu(), _ref.sign_mul(sums[1].cpu(), g))


def test_tresnet_iabn_fold_matches_separate_launches_gpu():
    """TResNet-M on the GPU: the folded InplaceABN weight path (default) == the separate
    iabn_gamma / sign_mul launches -- loss, gradients, running statistics (some gammas negative)."""
    from ddp_classification_pytorch_amd.models import build_model, input_layout
    from ddp_classification_pytorch_amd.ops import functional as Fn

    out = []
    for fold in (True, False):
        Fn.set_iabn_fold(fold)
        try:
            torch.manual_seed(7)
            m = build_model("tresnet_m", num_classes=10).to(DEV)
            with torch.no_grad():
                for mod in m.modules():
                    if getattr(mod, "inplace_abn", False):
                        mod.weight.mul_(torch.where(torch.rand_like(mod.weight) < 0.3, -1.0, 1.0))
            gen = torch.Generator().manual_seed(3)
            imgs = torch.randint(0, 256, (4, 3, 64, 64), dtype=torch.uint8, generator=gen).to(DEV)
            labels = torch.randint(0, 10, (4,), generator=gen).to(DEV)
            x = Fn.to_device_nhwc(imgs, (0.5, 0.5, 0.5), (0.25, 0.25, 0.25), in_scale=1 / 255.0, **input_layout(m))
            loss = Fn.cross_entropy(m(x), labels)
            loss.backward()
            torch.cuda.synchronize()
            rs = torch.cat([b.flatten() for n, b in m.named_buffers() if "running" in n]).cpu()
            out.append((loss.item(), torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None]).cpu(),
                        rs))
        finally:
            Fn.set_iabn_fold(True)
    (l1, g1, r1), (l0, g0, r0) = out
    assert abs(l1 - l0) < 1e-6
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-6
    assert torch.equal(r1, r0)


def test_conv_autotune_same_results(K):
    """g_tune[25] = 1 (DCP_AUTOTUNE): the first call of each conv problem times the candidate
    configurations and keeps one; forward and data gradient are bitwise the untuned results (every
    candidate accumulates in the same k order), the BN statistics equal them to fp32 rounding (a
    64-channel tile sums a slab's rows in another order), the weight gradient too (another split-K
    plan), and later calls reuse the choice."""
    torch.manual_seed(0)
    shapes = [(5, 14, 14, 256, 256, 3, 1, 1), (3, 28, 28, 128, 512, 1, 1, 0), (3, 28, 28, 256, 512, 1, 2, 0)]
    for N, H, W, Ci, Co, k, s, p in shapes:
        x = rnd(N, H, W, Ci).to(DEV)
        w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci)).to(DEV)
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        dy = rnd(N, Ho, Wo, Co).to(DEV)
        wb, wt = K.weight_prep(w.float(), 0, True)
        K.set_tuning(tslot("autotune"), 0)  # (a workload run earlier in this process may have left it on)
        y0, s0 = K.conv_fwd(x, wb, s, p, True)
        d0 = K.conv_dgrad(dy, wt, H, W, s, p)
        g0 = K.conv_wgrad(dy, x, k, k, s, p)
        n0 = K.autotune_entries()
        try:
            K.set_tuning(tslot("autotune"), 1)
            y1, s1 = K.conv_fwd(x, wb, s, p, True)
            d1 = K.conv_dgrad(dy, wt, H, W, s, p)
            g1 = K.conv_wgrad(dy, x, k, k, s, p)
            n1 = K.autotune_entries()
            y2, _ = K.conv_fwd(x, wb, s, p, True)
            assert K.autotune_entries() == n1 > n0
        finally:
            K.set_tuning(tslot("autotune"), 0)
        torch.cuda.synchronize()
        assert torch.equal(y1, y0) and torch.equal(y2, y0), (N, H, Ci, Co, k, s)
        assert torch.equal(d1, d0), (N, H, Ci, Co, k, s)
        st0, st1 = K.bn_stats(y0, s0), K.bn_stats(y1, s1)
        assert relerr(st1[0, 1:], st0[0, 1:]) < 1e-5
        assert relerr(g1, g0) < 1e-5  # another split count sums the rows in another order


@pytest.mark.parametrize("shape", [(2, 14, 14, 64, 256, 1, 1, 0), (3, 9, 11, 128, 320, 1, 1, 0),
                                   (2, 7, 7, 256, 1024, 1, 1, 0), (2, 14, 14, 128, 256, 3, 1, 1),
                                   (2, 28, 28, 256, 512, 1, 2, 0)])
def test_conv_fwd_256_channel_tiles(K, shape):
    """256-channel tap-GEMM tiles (g_tune[0] = 256: 64 x 128 outputs per wave, statistics
    epilogue) == the fp32 reference and the 128-channel tiles, ragged M and channel counts that are
    not a multiple of 256 included; dgrad is unaffected (falls back to 128).  Split-K off in both
    arms: the 256-channel tile does not split (the autotuner drops it where the heuristic does)."""
    N, H, W, Ci, Co, k, s, p = shape
    torch.manual_seed(0)
    x = rnd(N, H, W, Ci).to(DEV)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci)).to(DEV)
    wb, _ = K.weight_prep(w.float(), 0, True)
    outs = []
    try:
        K.set_tuning(tslot("tg_split_k"), 2)
        for bn in (0, 256):
            K.set_tuning(tslot("tg_tile_n"), bn)
            y, slabs = K.conv_fwd(x, wb, s, p, True)
            st = K.bn_stats(y, slabs)
            torch.cuda.synchronize()
            outs.append((y.float().cpu(), st.cpu()))
    finally:
        K.set_tuning(tslot("tg_tile_n"), 0)
        K.set_tuning(tslot("tg_split_k"), 0)
    (y0, s0), (y1, s1) = outs
    assert torch.equal(y1, y0)  # same k order: bit-identical outputs
    assert torch.equal(s1[0, 0], s0[0, 0]) and relerr(s1[0, 1:], s0[0, 1:]) < 1e-4
    yr, _ = _ref.conv_fwd(x.float().cpu(), w.float().cpu(), s, p, False)
    assert relerr(y1, yr) < 1e-2


@pytest.mark.parametrize("N,H,C,Co,mask", [(2, 14, 256, 64, True), (3, 7, 512, 128, False), (2, 9, 64, 64, True)])
def test_conv_dgrad_bn_strided_add(K, N, H, C, Co, mask):
    """conv_dgrad_bn with a compact stride-2 add source (a projection block's downsample gradient,
    StridedGrad) == the same call with that source expanded to full size (zeros off the even
    pixels), odd H included."""
    torch.manual_seed(0)
    dy = rnd(N, H, H, Co).to(DEV)
    w = rnd(Co, 1, 1, C, scale=1.0 / math.sqrt(C)).to(DEV)
    _, wt = K.weight_prep(w.float(), 0, True)
    y = rnd(N, H, H, C).to(DEV)
    res = rnd(N, H, H, C).to(DEV)
    scale, shift = (torch.rand(C) + 0.5).to(DEV), torch.randn(C).to(DEV)
    mean, invstd = torch.randn(C).to(DEV), (torch.rand(C) + 0.5).to(DEV)
    hc = (H + 1) // 2
    compact = rnd(N, hc, hc, C).to(DEV)
    full = torch.zeros(N, H, H, C, dtype=compact.dtype, device=DEV)
    full[:, ::2, ::2] = compact
    m = None
    if mask:
        _, m = K.bn_act_mask(y, res, scale, shift, 1, 0.0)
    r = None if mask else res
    d0, s0 = K.conv_dgrad_bn(dy, wt, 0, full, y, r, scale, shift, mean, invstd, 1, m, 0.0)
    d1, s1 = K.conv_dgrad_bn(dy, wt, 0, compact, y, r, scale, shift, mean, invstd, 1, m, 0.0)
    assert torch.equal(d0, d1) and torch.equal(s0, s1)


def test_resnet50_strided_deposit_same_gradients(K):
    """ResNet-50 training step with the downsample convs' input gradients deposited compact
    (StridedGrad, default) == with them as full-size tensors: loss and every parameter gradient."""
    from ddp_classification_pytorch_amd.models import build_model, input_layout
    from ddp_classification_pytorch_amd.ops import functional as Fn

    g = torch.Generator().manual_seed(3)
    imgs = torch.randint(0, 256, (4, 3, 64, 64), dtype=torch.uint8, generator=g).to(DEV)
    labels = torch.randint(0, 10, (4,), generator=g).to(DEV)
    res = {}
    try:
        for on in (False, True):
            Fn.set_strided_deposit(on)
            torch.manual_seed(0)
            m = build_model("resnet50", num_classes=10).to(DEV)
            x = Fn.to_device_nhwc(imgs, (0.5, 0.5, 0.5), (0.25, 0.25, 0.25), nchw=True, in_scale=1 / 255.0,
                                  **input_layout(m))
            loss = Fn.cross_entropy(m(x), labels)
            loss.backward()
            res[on] = (loss.item(), {n: p.grad.detach().float().cpu() for n, p in m.named_parameters()})
    finally:
        Fn.set_strided_deposit(True)
    assert res[False][0] == res[True][0]
    for n, g0 in res[False][1].items():
        assert relerr(res[True][1][n], g0) < 1e-5, n


@pytest.mark.parametrize("shape", [(24, 56, 56, 128, 256, 3, 1, 1), (40, 28, 28, 512, 256, 1, 1, 0),
                                   (16, 30, 30, 256, 512, 3, 2, 1), (9, 20, 20, 64, 320, 3, 1, 1)])
def test_big_tile_persistent_identical(K, shape):
    """Persistent big-tile workgroups (tg_big_persist = 1: one per CU, several tiles each -- these
    grids have 1.1-5 tiles per CU) == one workgroup per tile, bit for bit: forward + BN statistics
    and the data gradient (stride-2 parity classes included)."""
    N, H, W, Ci, Co, k, s, p = shape
    torch.manual_seed(0)
    x = rnd(N, H, W, Ci).to(DEV)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci)).to(DEV)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = rnd(N, Ho, Wo, Co).to(DEV)
    wb, wt = K.weight_prep(w.float(), 0, True)
    outs = []
    try:
        K.set_tuning(tslot("tg_big"), 1)
        for persist in (0, 1):
            K.set_tuning(tslot("tg_big_persist"), persist)
            y, slabs = K.conv_fwd(x, wb, s, p, True)
            dx = K.conv_dgrad(dy, wt, H, W, s, p)
            torch.cuda.synchronize()
            outs.append((y, slabs.clone(), dx))
    finally:
        K.set_tuning(tslot("tg_big"), 0)
        K.set_tuning(tslot("tg_big_persist"), 0)
    (y0, s0, d0), (y1, s1, d1) = outs
    assert torch.equal(y0, y1) and torch.equal(s0, s1) and torch.equal(d0, d1)


@pytest.mark.parametrize("shape", [(2, 56, 56, 128, 128, 3), (3, 14, 14, 512, 256, 3), (2, 13, 13, 64, 256, 1)])
def test_conv_dgrad_stride2_parity_streams(K, shape):
    """Stride-2 data gradient with its four parity classes on concurrent streams
    (dgrad_parity_streams = 1) == the serial classes, eagerly and replayed from a HIP graph."""
    N, H, W, Ci, Co, k = shape
    p = k // 2
    Ho, Wo = (H + 2 * p - k) // 2 + 1, (W + 2 * p - k) // 2 + 1
    torch.manual_seed(0)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci)).to(DEV)
    _, wt = K.weight_prep(w.float(), 0, True)
    dy = rnd(N, Ho, Wo, Co).to(DEV)
    ref = K.conv_dgrad(dy, wt, H, W, 2, p)
    try:
        K.set_tuning(tslot("dgrad_parity_streams"), 1)
        got = K.conv_dgrad(dy, wt, H, W, 2, p)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            K.conv_dgrad(dy, wt, H, W, 2, p)  # warm-up outside the capture
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = K.conv_dgrad(dy, wt, H, W, 2, p)
        dy.mul_(-1.0)
        g.replay()
        torch.cuda.synchronize()
    finally:
        K.set_tuning(tslot("dgrad_parity_streams"), 0)
    assert torch.equal(out, K.conv_dgrad(dy, wt, H, W, 2, p))


@pytest.mark.parametrize("N,H,W", [(2, 56, 56), (3, 9, 11), (1, 20, 33)])
def test_conv3x3_bn_prologue(K, N, H, W):
    """K5 on the 64-channel 3x3 consumer: conv3x3_fwd_pro / conv3x3_wgrad_pro apply relu(x * scale
    + shift) once per staged window element == the fp32 reference of conv(bf16(relu(BN(x)))) with
    zero padding of the BN output; forward statistics partials vs bn_stats; == the unfused
    bn_act -> conv_fwd / conv_wgrad kernels."""
    torch.manual_seed(0)
    C = 64
    x = rnd(N, H, W, C).to(DEV)
    w = rnd(C, 3, 3, C, scale=1.0 / math.sqrt(9 * C)).to(DEV)
    wb, _ = K.weight_prep(w.float(), 0, True)
    scale, shift = (torch.rand(C) + 0.5).to(DEV), (torch.randn(C) * 0.5).to(DEV)
    assert K.conv3x3_pro_fits(N, H, W, C, C)
    y, part = K.conv3x3_fwd_pro(x, wb, scale, shift, True)
    a = K.bn_act(x, None, scale, shift, 1, 0.0)
    y0, _ = K.conv_fwd(a, wb, 1, 1, False)
    assert torch.equal(y, y0)
    yr, _ = _ref.conv3x3_fwd_pro(x.float().cpu(), w.float().cpu(), scale.cpu(), shift.cpu(), False)
    assert relerr(y, yr) < 1e-2
    st, sr = K.bn_stats(y, part), _ref.bn_stats(y.float().cpu(), None)
    assert relerr(st[0, 1], sr[0, 1]) < 1e-4 and relerr(st[0, 2], sr[0, 2]) < 1e-4
    dy = rnd(N, H, W, C).to(DEV)
    dw = K.conv3x3_wgrad_pro(dy, x, scale, shift)
    dw0 = K.conv_wgrad(dy, a, 3, 3, 1, 1)
    assert dw.shape == dw0.shape and relerr(dw, dw0) < 1e-5
    dwr = _ref.conv3x3_wgrad_pro(dy.float().cpu(), x.float().cpu(), scale.cpu(), shift.cpu())
    assert relerr(dw, dwr) < 5e-3


def test_resnet50_bn_prologue3x3_same_training_step(K):
    """ResNet-50 with layer1's bn1 + ReLU inside conv2's staged windows (default) vs the separate
    BN-apply pass: the same loss and BN running statistics, and every parameter gradient as close
    to the fp32 CPU reference model's (``ops/_ref.py``) as the unfused path's is."""
    import copy

    from ddp_classification_pytorch_amd.models import build_model, input_layout
    from ddp_classification_pytorch_amd.ops import functional as Fn

    g = torch.Generator().manual_seed(5)
    imgs = torch.randint(0, 256, (4, 3, 96, 96), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (4,), generator=g)
    torch.manual_seed(0)
    base = build_model("resnet50", num_classes=10)

    def step(m, dev):
        x = Fn.to_device_nhwc(imgs.to(dev), (0.5, 0.5, 0.5), (0.25, 0.25, 0.25), nchw=True, in_scale=1 / 255.0,
                              **input_layout(m))
        loss = Fn.cross_entropy(m(x), labels.to(dev))
        loss.backward()
        return loss.item(), {n: p.grad.detach().float().cpu() for n, p in m.named_parameters()}

    ref = step(copy.deepcopy(base), "cpu")
    res = {}
    try:
        for on in (False, True):
            Fn.set_bn_prologue3x3(on)
            m = copy.deepcopy(base).to(DEV)
            loss, grads = step(m, DEV)
            torch.cuda.synchronize()
            res[on] = (loss, grads, m.layer1[0].bn1.running_mean.detach().cpu().clone(),
                       int(m.layer1[0].bn1.num_batches_tracked))
    finally:
        Fn.set_bn_prologue3x3(True)
    assert abs(res[False][0] - res[True][0]) < 1e-4 * max(1.0, abs(res[False][0]))
    assert torch.allclose(res[True][2], res[False][2], rtol=1e-5, atol=1e-6)
    assert res[True][3] == res[False][3]
    # the fused path rounds bn1's incoming gradient to bf16 once more (the direct kernel's dgrad
    # output feeds a separate BN-backward pass; the unfused tap GEMM applies it in its epilogue),
    # so the two bf16 paths differ by rounding noise, amplified in the cancelling bias sums of the
    # early BNs.  What must hold: the fused path is no further from the fp32 model than that noise.
    for n, g0 in ref[1].items():
        e_off, e_on = relerr(res[False][1][n], g0), relerr(res[True][1][n], g0)
        assert e_on <= 1.5 * e_off + 2e-2, (n, e_on, e_off)


@pytest.mark.parametrize("shape", [(4, 28, 28, 256, 256, 3, 1, 1), (6, 27, 25, 128, 384, 3, 2, 1),
                                   (6, 14, 14, 512, 512, 3, 1, 1), (5, 28, 28, 256, 512, 1, 2, 0)])
@pytest.mark.parametrize("mode", [1, 3])
@pytest.mark.parametrize("sk", [3, 5, 7])
def test_big_tile_stream_k_matches(K, shape, mode, sk):
    """Stream-K big tiles (tg_big_sk >= 3: the tiles' k-steps split evenly over exactly `sk`
    workgroups, so tiles are cut between workgroups at arbitrary k-steps, the tail piece published
    as an fp32 partial and added by the workgroup that finishes the tile) == the same tile without
    stream-K and the fp32 reference: forward with BN statistics and the data gradient (stride-2
    shapes: the parity classes, each with its own k-step count)."""
    N, H, W, Ci, Co, k, s, p = shape
    torch.manual_seed(1)
    x = rnd(N, H, W, Ci).to(DEV)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci)).to(DEV)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = rnd(N, Ho, Wo, Co).to(DEV)
    wb, wt = K.weight_prep(w.float(), 0, True)
    outs = []
    try:
        K.set_tuning(tslot("tg_big"), mode)
        for v in (2, sk):
            K.set_tuning(tslot("tg_big_sk"), v)
            y, slabs = K.conv_fwd(x, wb, s, p, True)
            st = K.bn_stats(y, slabs)
            dx = K.conv_dgrad(dy, wt, H, W, s, p)
            torch.cuda.synchronize()
            outs.append((y.float().cpu(), st.cpu(), dx.float().cpu()))
    finally:
        K.set_tuning(tslot("tg_big"), 0)
        K.set_tuning(tslot("tg_big_sk"), 0)
    (y0, s0, d0), (y1, s1, d1) = outs
    # a split tile sums two fp32 partial chains: equal up to fp32 rounding before the bf16 store
    assert relerr(y1, y0) < 4e-3 and relerr(d1, d0) < 4e-3
    assert relerr(s1[0, 1:], s0[0, 1:]) < 1e-3
    yr, _ = _ref.conv_fwd(x.float().cpu(), w.float().cpu(), s, p, False)
    assert relerr(y1, yr) < 1e-2
    sr = _ref.bn_stats(y1, None)
    assert relerr(s1[0, 1], sr[0, 1]) < 1e-4 and relerr(s1[0, 2], sr[0, 2]) < 1e-4
    dxr = _ref.conv_dgrad(dy.float().cpu(), w.float().cpu().permute(3, 1, 2, 0), H, W, s, p)
    assert relerr(d1, dxr) < 1e-2


# weight-stationary persistent 1x1 kernel (conv_ws.hip): K in {64, 128, 256}, Co % 128 == 0; M with
# partial 256-row tiles and partial 128-row slabs, several tiles per workgroup (the cross-tile ring
# and the stores that drain under the next tile), both epilogues (plain / BN statistics)
WS_SHAPES = [
    # N, H, W, Ci, Co
    (2, 56, 56, 64, 256),
    (2, 28, 28, 128, 512),
    (3, 14, 14, 256, 1024),
    (5, 7, 7, 256, 2048),
    (1, 9, 11, 64, 128),      # M = 99: one partial tile, the second slab empty
    (7, 13, 17, 128, 256),    # M = 1547: ragged last tile
    (64, 14, 14, 256, 1024),  # 49 tiles x 8 column blocks: several tiles per workgroup
]


# ... and the store-decoupled loader / consumer kernel (conv1x1_ps.hip, tg_ps) on the same shapes
@pytest.mark.parametrize("kernel", ["tg_ws", "tg_ps", "tg_ps=3"])
@pytest.mark.parametrize("shape", WS_SHAPES)
def test_conv1x1_weight_stationary(K, shape, kernel):
    N, H, W, Ci, Co = shape
    torch.manual_seed(Ci + Co + N)
    x = rnd(N, H, W, Ci)
    w = rnd(Co, 1, 1, Ci, scale=1.0 / math.sqrt(Ci))
    name, _, val = kernel.partition("=")
    try:
        K.set_tuning(tslot(name), int(val or 1))
        y, slabs = K.conv_fwd(x.to(DEV), w.to(DEV), 1, 0, True)
        y0, _ = K.conv_fwd(x.to(DEV), w.to(DEV), 1, 0, False)
        torch.cuda.synchronize()
    finally:
        K.set_tuning(tslot(name), 0)
    ytap, _ = K.conv_fwd(x.to(DEV), w.to(DEV), 1, 0, True)  # the tap GEMM: same k order, same bits
    yr, _ = _ref.conv_fwd(x.float(), w.float(), 1, 0, False)
    assert relerr(y, yr) < 1e-2
    assert torch.equal(y, ytap) and torch.equal(y0, ytap)
    st = K.bn_stats(y, slabs)
    sr = _ref.bn_stats(y.float().cpu(), None)
    assert torch.equal(st[0, 0].cpu(), sr[0, 0])
    assert relerr(st[0, 1], sr[0, 1]) < 1e-4
    assert relerr(st[0, 2], sr[0, 2]) < 1e-4


def _bn_two_launch(K, z, slabs, r, g, b, rm, rv, act, want_mask, ieps=-1.0, rgo=None):
    mean, invstd, scale, shift = K.bn_stats_finalize(z, slabs, g, b, rm, rv, 0.1, 1e-5, ieps, rgo)
    if want_mask:
        y, mask = K.bn_act_mask(z, r, scale, shift, act, 0.01)
    else:
        y, mask = K.bn_act(z, r, scale, shift, act, 0.01), None
    return y, mask, mean, invstd, scale, shift


@pytest.mark.parametrize("N,H,Ci,Co,act,res,want_mask,part", [
    (2, 56, 64, 256, 1, True, True, False),      # 49 slabs, residual + mask bits
    (32, 56, 64, 256, 1, False, False, False),   # 784 slabs (batch-32 layer1), 400+ workgroups
    (4, 7, 256, 2048, 1, True, True, False),     # 2048 channels: 32 finalize workgroups
    (2, 14, 64, 512, 2, False, False, False),    # leaky ReLU
    (2, 14, 64, 128, 0, True, False, True),      # (n, mean, M2) partials instead of slabs
    (1, 3, 64, 24, 1, False, False, False),      # 9 rows, 24 channels (3-chunk rows)
])
def test_bn_fin_act_matches_two_launches(K, N, H, Ci, Co, act, res, want_mask, part):
    """bn_fin_act (finalize + BN/act in ONE launch, workgroups synchronised through write-through
    coefficients and counters) == bn_stats_finalize followed by bn_act / bn_act_mask, bit for bit,
    running statistics included; no spin timeout."""
    torch.manual_seed(N * 1000 + Co)
    x = rnd(N, H, H, Ci).to(DEV)
    w = rnd(Co, 1, 1, Ci, scale=0.1).to(DEV)
    z, slabs = K.conv_fwd(x, w, 1, 0, True)
    if part:
        slabs = K.bn_stats(z, slabs)
    r = rnd(*z.shape).to(DEV) if res else None
    g = torch.randn(Co, device=DEV)
    b = torch.randn(Co, device=DEV) * 0.1
    rm0, rv0 = torch.randn(Co, device=DEV), torch.rand(Co, device=DEV) + 0.5
    rm1, rv1 = rm0.clone(), rv0.clone()
    got = K.bn_fin_act(z, slabs, r, g, b, rm0, rv0, 0.1, 1e-5, act, 0.01, want_mask)
    ref = _bn_two_launch(K, z, slabs, r, g, b, rm1, rv1, act, want_mask)
    for name, a, c in zip(("y", "mask", "mean", "invstd", "scale", "shift"), got, ref):
        if c is None:
            assert a.numel() == 0, name
        else:
            assert torch.equal(a, c), name
    assert torch.equal(rm0, rm1) and torch.equal(rv0, rv1)
    assert K.bn_fin_act_timeouts(z) == 0


def test_bn_fin_act_iabn_and_graph_replay(K):
    """The fused BN with InplaceABN's folded weight (|g| + eps, 1 / it written), and the same launch
    captured in a HIP graph and replayed: every replay re-arms the counters and reproduces the
    eager outputs (the running statistics advance once per replay, like the eager chain)."""
    torch.manual_seed(5)
    C = 512
    x = rnd(8, 14, 14, 64).to(DEV)
    w = rnd(C, 1, 1, 64, scale=0.1).to(DEV)
    z, slabs = K.conv_fwd(x, w, 1, 0, True)
    g = torch.randn(C, device=DEV)
    b = torch.randn(C, device=DEV) * 0.1
    rg0, rg1 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    rm0, rv0 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm1, rv1 = rm0.clone(), rv0.clone()
    got = K.bn_fin_act(z, slabs, None, g, b, rm0, rv0, 0.1, 1e-5, 2, 0.01, False, 1e-5, rg0)
    ref = _bn_two_launch(K, z, slabs, None, g, b, rm1, rv1, 2, False, 1e-5, rg1)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[4], ref[4]) and torch.equal(rg0, rg1)
    assert torch.equal(rm0, rm1) and torch.equal(rv0, rv1)

    rmg, rvg = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    K.bn_fin_act(z, slabs, None, g, b, rmg.clone(), rvg.clone(), 0.1, 1e-5, 1, 0.01, True)  # warm-up
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = K.bn_fin_act(z, slabs, None, g, b, rmg, rvg, 0.1, 1e-5, 1, 0.01, True)
    rme, rve = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    for _ in range(5):
        graph.replay()
        eager = K.bn_fin_act(z, slabs, None, g, b, rme, rve, 0.1, 1e-5, 1, 0.01, True)
        torch.cuda.synchronize()
        for a, c in zip(out, eager):
            assert torch.equal(a, c)
        assert torch.equal(rmg, rme) and torch.equal(rvg, rve)
    assert K.bn_fin_act_timeouts(z) == 0


@pytest.mark.parametrize("model", ["resnet50", "tresnet_m"])
def test_model_bn_fin_act_matches_two_launches_gpu(model):
    """A training step with the one-launch BN finalize + apply (DCP_BN_FIN_ACT=1) == the two-launch
    default, bit for bit: loss, every gradient, running statistics (ResNet-50: ReLU + residual masks;
    TResNet-M: InplaceABN leaky BNs with the folded weight)."""
    from ddp_classification_pytorch_amd.models import build_model, input_layout
    from ddp_classification_pytorch_amd.ops import functional as Fn

    out = []
    for fused in (True, False):
        Fn.set_bn_fin_act(fused)
        try:
            torch.manual_seed(11)
            m = build_model(model, num_classes=10).to(DEV)
            gen = torch.Generator().manual_seed(4)
            imgs = torch.randint(0, 256, (4, 3, 64, 64), dtype=torch.uint8, generator=gen).to(DEV)
            labels = torch.randint(0, 10, (4,), generator=gen).to(DEV)
            x = Fn.to_device_nhwc(imgs, (0.5, 0.5, 0.5), (0.25, 0.25, 0.25), in_scale=1 / 255.0, **input_layout(m))
            loss = Fn.cross_entropy(m(x), labels)
            loss.backward()
            torch.cuda.synchronize()
            rs = torch.cat([b.flatten() for n, b in m.named_buffers() if "running" in n]).cpu()
            out.append((loss.item(), torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None]).cpu(),
                        rs))
        finally:
            Fn.set_bn_fin_act(False)
    (l1, g1, r1), (l0, g0, r0) = out
    assert l1 == l0
    assert torch.equal(g1, g0)
    assert torch.equal(r1, r0)


@pytest.mark.parametrize("N,C,R,bias", [(16, 64, 64, True), (16, 128, 64, True), (16, 256, 128, True),
                                        (32, 256, 128, False), (3, 96, 32, True), (20, 64, 128, True)])
def test_se_gate_kernels_vs_fp32_reference(K, N, C, R, bias):
    """The one-workgroup squeeze-excitation gate (forward: relu(p W1^T + b1) -> sigmoid(. W2^T + b2);
    backward: every weight / bias gradient and dp) against the fp32 reference of the same op with the
    same bf16 rounding points."""
    torch.manual_seed(N + C + R)
    p = rnd(N, C).to(DEV)
    w1, w2 = rnd(R, C, scale=0.2).to(DEV), rnd(C, R, scale=0.2).to(DEV)
    b1 = (torch.randn(R) * 0.1).to(DEV) if bias else None
    b2 = (torch.randn(C) * 0.1).to(DEV) if bias else None
    h, g = K.se_gate_fwd(p, w1, b1, w2, b2, R)
    rh, rg = _ref.se_gate_fwd(p.cpu(), w1.cpu(), None if b1 is None else b1.cpu(), w2.cpu(),
                              None if b2 is None else b2.cpu(), R)
    assert relerr(h, rh) < 1e-2 and relerr(g, rg) < 1e-2
    dg = rnd(N, C).to(DEV)
    w1t, w2t = w1.t().contiguous(), w2.t().contiguous()
    got = K.se_gate_bwd(dg, g, h, p, w1t, w2t)
    ref = _ref.se_gate_bwd(dg.cpu(), g.cpu(), h.cpu(), p.cpu(), w1t.cpu(), w2t.cpu())
    for name, a, b in zip(("dp", "dw1", "db1", "dw2", "db2"), got, ref):
        assert a.shape == b.shape, name
        assert relerr(a, b) < 2e-2, (name, relerr(a, b))


def test_tresnet_se_gate_fused_matches_gemm_chain_gpu():
    """TResNet-M training step on the GPU with the fused squeeze-excitation gates (default at small
    batch) vs the GEMM chain: loss and gradients agree to bf16 summation-order rounding."""
    from ddp_classification_pytorch_amd.models import build_model, input_layout
    from ddp_classification_pytorch_amd.ops import functional as Fn

    out = []
    for fused in (True, False):
        Fn.set_se_fused(fused)
        try:
            torch.manual_seed(7)
            m = build_model("tresnet_m", num_classes=10).to(DEV)
            with torch.no_grad():  # the zero-initialised last BN of each block would zero every SE gradient
                for mod in m.modules():
                    w = getattr(mod, "weight", None)
                    if "BatchNorm" in type(mod).__name__ and w is not None and not bool(w.any()):
                        w.fill_(0.5)
            gen = torch.Generator().manual_seed(3)
            imgs = torch.randint(0, 256, (4, 3, 64, 64), dtype=torch.uint8, generator=gen).to(DEV)
            labels = torch.randint(0, 10, (4,), generator=gen).to(DEV)
            x = Fn.to_device_nhwc(imgs, (0.5, 0.5, 0.5), (0.25, 0.25, 0.25), in_scale=1 / 255.0, **input_layout(m))
            loss = Fn.cross_entropy(m(x), labels)
            loss.backward()
            torch.cuda.synchronize()
            out.append((loss.item(), {n: q.grad.float().cpu() for n, q in m.named_parameters() if q.grad is not None}))
        finally:
            Fn.set_se_fused(True)
    (l1, g1), (l0, g0) = out
    assert abs(l1 - l0) < 2e-2 * max(1.0, abs(l0))
    tot1 = torch.cat([g1[k].flatten() for k in g0])
    tot0 = torch.cat([g0[k].flatten() for k in g0])
    assert ((tot1 - tot0).norm() / tot0.norm()).item() < 5e-2
    se = [k for k in g0 if ".se." in k]
    assert se and any(g0[k].abs().sum() > 0 for k in se)
    for k in se:
        assert relerr(g1[k], g0[k]) < 0.1, k


@pytest.mark.parametrize("N,H,Ci,Co,k,s,p", [(2, 7, 512, 512, 3, 1, 1), (4, 7, 2048, 512, 1, 1, 0),
                                             (3, 14, 1024, 256, 1, 1, 0), (2, 14, 256, 256, 3, 2, 1)])
def test_split_k_short_grids(K, N, H, Ci, Co, k, s, p):
    """Split-K of the 128-row tap GEMM (short grids with deep k-loops: small batches): forward with BN
    statistics and data gradient vs the fp32 reference, vs the unsplit kernels (tg_split_k = 2), and
    bitwise equal whatever the slice count's k depth (32- vs 64-deep k-tiles cut at the same 64-deep
    units)."""
    from ddp_classification_pytorch_amd import tuning

    torch.manual_seed(N * 100 + Ci)
    x = rnd(N, H, H, Ci).to(DEV)
    w = rnd(Co, k, k, Ci, scale=1.0 / math.sqrt(k * k * Ci))
    Ho = (H + 2 * p - k) // s + 1
    dy = rnd(N, Ho, Ho, Co).to(DEV)
    wb, wt = K.weight_prep(w.float().to(DEV), 0, True)
    outs = {}
    for name, spec in (("split", ""), ("off", "tg_split_k=2"), ("split4", "tg_split_k=4"),
                       ("split_bk32", "tg_kdepth=32,tg_stages=2")):
        tuning.apply(K, spec, reset=True)
        try:
            y, sl = K.conv_fwd(x, wb, s, p, True)
            d = K.conv_dgrad(dy, wt, H, H, s, p) if s == 1 else None
            torch.cuda.synchronize()
            outs[name] = (y, K.bn_stats(y, sl), d)
        finally:
            tuning.apply(K, "", reset=True)
    ry, _ = _ref.conv_fwd(x.cpu(), w.bfloat16(), s, p, True)
    for name, (y, st, d) in outs.items():
        assert relerr(y, ry) < 1e-2, name
        assert relerr(st[0, 1:], outs["off"][1][0, 1:]) < 1e-3, name
        if d is not None:
            assert relerr(d, outs["off"][2]) < 1e-2, name
    assert torch.equal(outs["split"][0], outs["split_bk32"][0])

