"""The fused ArcFace head (csrc/arcface.hip) against an fp32 autograd rendering of
the reference's ArcMarginProduct + CrossEntropyLoss (ARCFACE/arc_main.py:130-176, 245): loss,
label rank, dX and dW for the easy and the hard margin, batch / class counts that are not tile
multiples, fp32 and bf16 features, D = 128 / 256 / 512; agreement with the unfused kernel path;
and a 100k-class step whose memory stays O((B + C) D) (no [B, C] cosine or gradient tensor)."""
import math
import os

import pytest
import torch

from ddp_classification_pytorch_amd.ops import functional as Fn

pytestmark = pytest.mark.gpu
DEV = "cuda"


def relerr(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def ref_head(x, W, lab, s, m, easy):
    """fp32 autograd ArcMarginProduct + mean CE; returns (loss, rank, dx, dW)."""
    xt, Wt = x.float().clone().requires_grad_(True), W.float().clone().requires_grad_(True)
    cos = torch.nn.functional.linear(torch.nn.functional.normalize(xt), torch.nn.functional.normalize(Wt))
    sine = torch.sqrt((1.0 - cos.pow(2)).clamp(0, 1))
    phi = cos * math.cos(m) - sine * math.sin(m)
    if easy:
        phi = torch.where(cos > 0, phi, cos)
    else:
        phi = torch.where(cos > math.cos(math.pi - m), phi, cos - math.sin(math.pi - m) * m)
    oh = torch.zeros_like(cos).scatter_(1, lab.view(-1, 1), 1)
    out = (oh * phi + (1 - oh) * cos) * s
    loss = torch.nn.functional.cross_entropy(out, lab)
    loss.backward()
    tgt = out.gather(1, lab.view(-1, 1))
    rank = (out > tgt).sum(1)
    return loss.detach(), rank, xt.grad, Wt.grad


def _check_ranks(got, want, C):
    """Label ranks agree up to near-ties: at random init the C logits s * cos are packed within a
    few units, so bf16 operands move a label's rank by a handful of classes -- the mean move stays
    under 1 % of C, and the top-1 decision (rank 0) agrees on nearly every row."""
    got, want = got.cpu().long(), want.cpu().long()
    assert (got - want).abs().float().mean().item() <= 0.01 * C, (got[:16], want[:16])
    assert ((got == 0) == (want == 0)).float().mean().item() >= 0.95


def run_head(x, W, lab, s, m, easy, fused=True):
    old = os.environ.get("DCP_ARCFACE_FUSED")
    os.environ["DCP_ARCFACE_FUSED"] = "1" if fused else "0"
    try:
        xd, Wd = x.to(DEV).requires_grad_(True), W.to(DEV).requires_grad_(True)
        loss, rank, _ = Fn.arcface_loss(xd, Wd, lab.to(DEV), s, m, easy)
        loss.backward()
        torch.cuda.synchronize()
        return loss.detach(), rank, xd.grad, Wd.grad
    finally:
        if old is None:
            os.environ.pop("DCP_ARCFACE_FUSED", None)
        else:
            os.environ["DCP_ARCFACE_FUSED"] = old


@pytest.mark.parametrize("B,C,D,easy,xdtype", [
    (32, 1000, 256, True, torch.float32),
    (100, 1000, 256, False, torch.float32),   # hard margin, batch not a tile multiple
    (64, 2173, 256, True, torch.bfloat16),    # the reference's class count, bf16 features
    (257, 4097, 128, True, torch.float32),
    (48, 700, 512, False, torch.float32),     # D > 256: the unfused path (fallback)
    (200, 130, 200, True, torch.float32),     # D padded to 256
])
def test_fused_head_matches_fp32_reference(B, C, D, easy, xdtype):
    torch.manual_seed(B + C)
    s, m = 30.0, 0.5
    x = torch.randn(B, D).to(xdtype)
    W = torch.randn(C, D) * 0.05
    lab = torch.randint(0, C, (B,))
    # a few rows whose feature equals their class weight (cos ~ 1: the margin's sin -> 0 guard)
    x[:3] = W[lab[:3]].to(xdtype)
    lr, rr, dxr, dwr = ref_head(x, W, lab, s, m, easy)
    lf, rf, dxf, dwf = run_head(x, W, lab, s, m, easy, fused=True)
    assert abs(lf.item() - lr.item()) / max(abs(lr.item()), 1e-6) < 1e-2, (lf.item(), lr.item())
    _check_ranks(rf.cpu(), rr, C)
    # the margin's guard: finite everywhere, also where the fp32 reference's sqrt(1 - cos^2) has an
    # infinite derivative (cos = 1: those rows and their classes' dW rows are NaN in the reference)
    assert torch.isfinite(dxf).all() and torch.isfinite(dwf).all()
    assert dxf.dtype == xdtype and dxf.shape == (B, D) and dwf.shape == (C, D)
    rx, rw = torch.isfinite(dxr).all(1), torch.isfinite(dwr).all(1)
    assert rx.sum() >= B - 3 and rw.sum() >= C - 3
    assert relerr(dxf[rx.to(DEV)], dxr[rx]) < 3e-2, relerr(dxf[rx.to(DEV)], dxr[rx])
    assert relerr(dwf[rw.to(DEV)], dwr[rw]) < 3e-2, relerr(dwf[rw.to(DEV)], dwr[rw])


@pytest.mark.parametrize("easy", [True, False])
def test_fused_head_matches_unfused_kernels(easy):
    """The fused head and the unfused kernel path (bf16 cosine matrix, separate GEMMs) agree to the
    bf16 noise floor: same loss, ranks, dX, dW."""
    torch.manual_seed(1)
    B, C, D = 256, 10000, 256
    x = torch.randn(B, D)
    W = torch.randn(C, D) * 0.05
    lab = torch.randint(0, C, (B,))
    lf, rf, dxf, dwf = run_head(x, W, lab, 30.0, 0.5, easy, fused=True)
    lu, ru, dxu, dwu = run_head(x, W, lab, 30.0, 0.5, easy, fused=False)
    assert abs(lf.item() - lu.item()) / abs(lu.item()) < 5e-3
    _check_ranks(rf, ru, C)
    assert relerr(dxf, dxu) < 3e-2 and relerr(dwf, dwu) < 3e-2, (relerr(dxf, dxu), relerr(dwf, dwu))


def test_fused_head_invalid_labels_and_graph_capture():
    """Rows with an out-of-range label contribute nothing (loss 0, no gradient), and the head is
    HIP-graph capturable (replay = eager)."""
    torch.manual_seed(2)
    B, C, D = 70, 500, 256
    x = torch.randn(B, D, device=DEV)
    W = (torch.randn(C, D) * 0.05).to(DEV)
    lab = torch.randint(0, C, (B,), device=DEV)
    lab[5] = -1
    lab[6] = C + 3
    xd, Wd = x.clone().requires_grad_(True), W.clone().requires_grad_(True)
    loss, rank, _ = Fn.arcface_loss(xd, Wd, lab, 30.0, 0.5, True)
    loss.backward()
    assert torch.isfinite(loss) and xd.grad[5].abs().max().item() == 0.0 and xd.grad[6].abs().max().item() == 0.0
    g_ref = (loss.detach().clone(), xd.grad.clone(), Wd.grad.clone())
    xs, Ws = x.clone().requires_grad_(True), W.clone().requires_grad_(True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            xs.grad = Ws.grad = None
            l2, _, _ = Fn.arcface_loss(xs, Ws, lab, 30.0, 0.5, True)
            l2.backward()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    xs.grad = Ws.grad = None
    with torch.cuda.graph(graph):
        l3, _, _ = Fn.arcface_loss(xs, Ws, lab, 30.0, 0.5, True)
        l3.backward()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(l3, g_ref[0]) and torch.equal(xs.grad, g_ref[1]) and torch.equal(Ws.grad, g_ref[2])


def test_fused_head_100k_classes_memory():
    """100k classes at batch 1024: the fused step's peak extra memory is O((B + C) D) -- far below
    the unfused path's, which materialises the [B, C] cosines and their gradient."""
    torch.manual_seed(3)
    B, C, D = 1024, 100000, 256
    x = torch.randn(B, D, device=DEV)
    W = (torch.randn(C, D) * 0.05).to(DEV)
    lab = torch.randint(0, C, (B,), device=DEV)
    peaks = {}
    for fused in (True, False):
        os.environ["DCP_ARCFACE_FUSED"] = "1" if fused else "0"
        try:
            xd, Wd = x.clone().requires_grad_(True), W.clone().requires_grad_(True)
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats()
            base = torch.cuda.memory_allocated()
            loss, _, _ = Fn.arcface_loss(xd, Wd, lab, 30.0, 0.5, True)
            loss.backward()
            torch.cuda.synchronize()
            peaks[fused] = torch.cuda.max_memory_allocated() - base
            assert torch.isfinite(loss) and torch.isfinite(Wd.grad).all()
            del xd, Wd, loss
        finally:
            os.environ.pop("DCP_ARCFACE_FUSED", None)
    bc = B * C * 2  # one bf16 [B, C] tensor
    cd = C * D * 4  # one fp32 [C, D] tensor
    # normalised W + its transpose (bf16) + dW (fp32) + small: well under one [B, C] bf16 tensor extra
    assert peaks[True] < 3 * cd + bc // 4, (peaks, bc, cd)
    assert peaks[False] - peaks[True] > bc, (peaks, bc)
