"""Every workload end-to-end on the GPU through the HIP kernels (synthetic data,
tiny epochs), plus memorisation checks that the bf16 kernel path trains."""
import math
import os

import pytest
import torch

import main as entry

pytestmark = pytest.mark.gpu

SYN = ["--data", "synthetic", "--batchsize", "16", "--synthetic-train-size", "64", "--synthetic-val-size", "24",
       "--workers", "0", "--log-interval", "100", "--device", "cuda", "--image-size", "64", "--num-classes", "10",
       "--dataset", "food"]


@pytest.mark.parametrize("workload,model", [("baseline", "resnet50"), ("baseline", "tresnet_m"),
                                            ("baseline", "resnext50_32x4d"), ("arcface", "resnet50"),
                                            ("cdr", "resnet18"), ("plc", "resnet18"), ("nested", "resnet18")])
def test_workload_gpu(tmp_path, workload, model):
    out = str(tmp_path / "o")
    args = ["--workload", workload, "--model", model, "--epochs", "1", "--out-dir", out] + SYN
    if workload == "nested":
        args += ["--warmUpIter", "2", "--arch", model]
    entry.main(args)
    if workload != "nested":
        assert os.path.exists(os.path.join(out, "metrics.jsonl"))


def test_tresnet_memorises_batch():
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn
    from ddp_classification_pytorch_amd.optim import FusedSGD

    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m = build_model("tresnet_m", num_classes=10).to(dev)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9)
    x = Fn.to_device_nhwc(torch.randint(0, 256, (16, 3, 64, 64), dtype=torch.uint8, device=dev),
                          (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), cpad=3, in_scale=1 / 255.0)
    y = torch.randint(0, 10, (16,), device=dev)
    losses = []
    for _ in range(25):
        loss = Fn.cross_entropy(m(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0], losses


def test_tresnet_inplace_abn_saves_activation_memory():
    """InplaceABN storage keeps one activation less per leaky BN layer: the peak memory of a
    TResNet-M training step drops against the same net storing the BN inputs."""
    import torch

    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn

    dev = torch.device("cuda", 0)
    peaks = {}
    for iabn in (True, False):
        torch.manual_seed(0)
        m = build_model("tresnet_m", num_classes=100).to(dev)
        for mod in m.modules():
            if hasattr(mod, "inplace_abn") and not iabn:
                mod.inplace_abn = False
        imgs = torch.randint(0, 256, (64, 3, 224, 224), dtype=torch.uint8, device=dev)
        labels = torch.randint(0, 100, (64,), device=dev)
        x = Fn.to_device_nhwc(imgs, (0.5, 0.5, 0.5), (0.25, 0.25, 0.25), cpad=3, nchw=True, in_scale=1 / 255.0)
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(dev)
        base = torch.cuda.memory_allocated(dev)
        loss = Fn.cross_entropy(m(x), labels)
        loss.backward()
        torch.cuda.synchronize()
        peaks[iabn] = torch.cuda.max_memory_allocated(dev) - base
        assert torch.isfinite(loss).item()
        del m, loss, x
        torch.cuda.empty_cache()
    assert peaks[True] < 0.9 * peaks[False], peaks


def test_bn_prologue_step_matches_separate_bn():
    """ResNet-50 training step with bn2 + ReLU inside conv3's GEMMs (DCP_BN_PROLOGUE, K5) against
    the separate BN-apply pass: same loss and gradients up to bf16 accumulation order, and less
    peak memory in a warm process (the normalised activations are not kept for backward)."""
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn

    dev = torch.device("cuda", 0)
    res = {}
    try:
        # each variant twice, the second one measured: lazily grown per-process workspaces
        # (allocated inside the first step that needs them) are then outside the measurement
        for pro in (False, True, False, True):
            Fn.set_bn_prologue(pro)
            torch.manual_seed(0)
            m = build_model("resnet50", num_classes=100).to(dev)
            imgs = torch.randint(0, 256, (32, 3, 112, 112), dtype=torch.uint8, device=dev,
                                 generator=torch.Generator(device=dev).manual_seed(1))
            labels = torch.arange(32, device=dev) % 100
            x = Fn.to_device_nhwc(imgs, (0.5, 0.5, 0.5), (0.25, 0.25, 0.25), nchw=True, in_scale=1 / 255.0)
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats(dev)
            base = torch.cuda.memory_allocated(dev)
            loss = Fn.cross_entropy(m(x), labels)
            loss.backward()
            torch.cuda.synchronize()
            peak = torch.cuda.max_memory_allocated(dev) - base
            res[pro] = (loss.item(), torch.cat([p.grad.flatten().float() for p in m.parameters()]), peak)
            del m, loss, x
            torch.cuda.empty_cache()
    finally:
        Fn.set_bn_prologue(False)
    (l0, g0, p0), (l1, g1, p1) = res[False], res[True]
    assert abs(l1 - l0) < 1e-2 * abs(l0), (l0, l1)
    assert ((g1 - g0).norm() / g0.norm()).item() < 2e-2
    assert p1 < p0, (p0, p1)


# The autotuner stays on (the workloads' default): its kernel choice depends on the box's timings,
# and 16-step trainings at batch 16 amplify the fp32 summation-order differences of another choice
# (e.g. a BN-statistics epilogue's) into visibly different loss curves -- one ResNet-50 curve rose
# in its third epoch (profiles/r4/learning_test_sensitivity.txt).  So the criterion is smoothed
# (the better of the last two epochs) and ResNet-50 runs 5 epochs, where every recorded variant
# ended at <= 0.58x of its first epoch.
LEARN = ["--data", "synthetic", "--synthetic-learnable", "--batchsize", "16", "--synthetic-train-size", "64",
         "--synthetic-val-size", "16", "--workers", "0", "--log-interval", "4", "--device", "cuda", "--image-size",
         "64", "--num-classes", "10", "--dataset", "food"]


def _epoch_losses(out, workload, tmp_path):
    import glob
    import json

    if workload == "nested":
        hist = glob.glob(str(tmp_path / "o_Acc*" / "history.json"))[0]
        return json.load(open(hist))["trainLoss"]
    return [json.loads(l)["loss"] for l in open(os.path.join(out, "metrics.jsonl")) if '"train_iter"' in l]


@pytest.mark.parametrize("workload,model,extra", [
    ("baseline", "resnet50", ["--lr", "0.05", "--epochs", "5"]),  # 3 epochs ends at 0.66-0.70x: too close
    ("baseline", "tresnet_m", ["--lr", "0.05", "--epochs", "3"]),
    ("arcface", "resnet18", ["--epochs", "4", "--m", "0.2"]),  # Adam 1e-3, s=30 (a 0.5 margin needs more steps)
    ("cdr", "resnet50", ["--lr", "0.05", "--epochs", "5"]),  # CDR keeps only the top |g*w| gradients: slower
    # the synthetic labels are clean, and the eval-mode posteriors of a 4-step model (BN running
    # statistics far from converged) would "correct" most of them: delta 0 runs the correction
    # pass without changing labels
    ("plc", "resnet18", ["--lr", "0.05", "--epochs", "3", "--plc-eta-epochs", "0", "--plc-delta", "0",
                         "--plc-delta-inc", "0"]),
    ("nested", "resnet18", ["--lr", "0.05", "--epochs", "3", "--warmUpIter", "2", "--no-freeze-bn"]),
])
def test_workload_learns(tmp_path, workload, model, extra):
    """Each workload through main.py on the GPU kernels actually trains: 64 synthetic images whose
    pixels carry their class, the per-epoch train loss of the better of the last two epochs at most 70 % of
    the first's
    (BASELINE/main.py:258-314, ARCFACE/arc_main.py:302-414, CDR/main.py:218-253, NESTED/train.py:227-270)."""
    out = str(tmp_path / "o")
    args = ["--workload", workload, "--model", model, "--out-dir", out] + LEARN + extra
    if workload == "nested":
        args += ["--arch", model]
    entry.main(args)
    losses = _epoch_losses(out, workload, tmp_path)
    assert len(losses) >= 3 and all(math.isfinite(v) for v in losses), losses
    assert min(losses[-2:]) <= 0.7 * losses[0], losses
