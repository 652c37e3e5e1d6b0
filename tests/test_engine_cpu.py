"""Engine / CLI: argument aliases, every workload end-to-end on synthetic data
(CPU), checkpoint -> failure -> resume equivalence, log artefacts."""
import json
import os

import pytest
import torch

import main as entry
from ddp_classification_pytorch_amd.config import parse_args
from ddp_classification_pytorch_amd.engine.loop import InjectedFailure

SYN = ["--data", "synthetic", "--dataset", "CIFAR10", "--batchsize", "8", "--synthetic-train-size", "32",
       "--synthetic-val-size", "12", "--workers", "0", "--log-interval", "100", "--device", "cpu"]


def test_cli_aliases():
    a = parse_args(["--local_rank", "0", "--world_size", "1", "--batch_size", "7", "--n_epoch", "3",
                    "--workload", "cdr", "--result_dir", "x"])
    assert a.batchsize == 7 and a.epochs == 3 and a.out_dir == "x" and a.local_rank == 0
    b = parse_args(["--local-rank=0", "--workload", "nested", "--warmUpIter", "5", "--lrSchedule", "1", "2",
                    "--nbEpoch", "4", "--arch", "resnet18"])
    assert b.warmup_iters == 5 and b.milestones == [1, 2] and b.epochs == 4 and b.model == "resnet18"
    c = parse_args(["--workload", "baseline"])
    assert c.model == "tresnet_m" and c.batchsize == 16 and c.num_classes == 2173 and c.lr == 1e-3
    d = parse_args(["--workload", "arcface"])
    assert d.optimizer == "adam" and d.imgs_limited == 400 and d.arc_s == 30 and d.arc_m == 0.5
    with pytest.raises(ValueError):
        parse_args(["--workload", "nested", "--dropout", "0.3"])  # nested>0 && dropout>0 (NESTED/train.py:489)


@pytest.mark.parametrize("workload,model", [("baseline", "resnet18"), ("arcface", "resnet18"), ("cdr", "resnet18"),
                                            ("plc", "resnet18"), ("nested", "resnet18"),
                                            ("baseline", "tresnet_m")])
def test_workload_runs(tmp_path, workload, model):
    out = str(tmp_path / workload)
    args = ["--workload", workload, "--model", model, "--epochs", "1", "--out-dir", out] + SYN
    if workload == "nested":
        args += ["--warmUpIter", "2", "--arch", model]
    if model == "tresnet_m":
        args = [a if a != "CIFAR10" else "food" for a in args] + ["--image-size", "64", "--num-classes", "5"]
    entry.main(args)
    if workload == "nested":
        assert any(p.startswith(workload + "_Acc") for p in os.listdir(tmp_path))
    else:
        assert os.path.exists(os.path.join(out, "last.pth")) or workload == "plc"
        assert os.path.exists(os.path.join(out, "metrics.jsonl"))


def test_failure_and_resume_is_equivalent(tmp_path):
    base = ["--workload", "baseline", "--model", "cifar_resnet18", "--epochs", "2", "--optimizer", "SGD",
            "--lr", "0.05"] + SYN
    # uninterrupted reference run
    torch.manual_seed(0)
    entry.main(base + ["--out-dir", str(tmp_path / "ref")])
    ref = torch.load(tmp_path / "ref" / "last.pth", weights_only=True)
    # run that dies in epoch 2, then resumes from the epoch-1 checkpoint
    with pytest.raises(InjectedFailure):
        entry.main(base + ["--out-dir", str(tmp_path / "ft"), "--fail-at-step", "6"])
    entry.main(base + ["--out-dir", str(tmp_path / "ft"), "--resume", str(tmp_path / "ft" / "last.pth")])
    got = torch.load(tmp_path / "ft" / "last.pth", weights_only=True)
    assert got["epoch"] == ref["epoch"] == 1
    for k, v in ref["models"]["model"].items():
        if v.dtype.is_floating_point:
            assert torch.allclose(v, got["models"]["model"][k], atol=1e-5), k
    lines = open(tmp_path / "ft" / "output.txt").read()
    assert "resumed from" in lines and "VAL Epoch 2" in lines
    recs = [json.loads(x) for x in open(tmp_path / "ref" / "metrics.jsonl")]
    assert {r["kind"] for r in recs} >= {"train_epoch", "val"}


def test_warmup_heartbeat_profile_and_auto_resume(tmp_path):
    """--warmup-iters ramps the LR per iteration from 1e-6 (BASELINE WarmUp, BASELINE/main.py:170-197),
    --heartbeat-every writes a per-rank liveness file, --profile writes a torch.profiler table,
    and --auto-resume continues from last.pth after a failure."""
    out = tmp_path / "run"
    base = ["--workload", "baseline", "--model", "cifar_resnet18", "--epochs", "2", "--optimizer", "SGD",
            "--lr", "0.05"] + SYN
    base = [a if a != "100" else "1" for a in base]  # log every step
    with pytest.raises(InjectedFailure):
        entry.main(base + ["--out-dir", str(out), "--warmup-iters", "3", "--heartbeat-every", "2", "--profile",
                           "--fail-at-step", "6"])
    recs = [json.loads(x) for x in open(out / "metrics.jsonl") if '"train_iter"' in x]
    lrs = [r["lr"] for r in recs]
    assert lrs[:4] == pytest.approx([1e-6 + (0.05 - 1e-6) * n / 3 for n in (1, 2, 3)] + [0.05])
    hb = open(out / "heartbeat_rank0.txt").read().split("\n")
    assert "step 2" in hb[0] and "step 4" in hb[1]
    assert os.path.exists(out / "profile" / "steps.txt")
    entry.main(base + ["--out-dir", str(out), "--auto-resume"])
    text = open(out / "output.txt").read()
    assert "resumed from" in text and "VAL Epoch 2" in text


def test_autotune_defaults_follow_reference_cudnn_benchmark():
    """--autotune (per-shape conv configuration timing, the cudnn.benchmark of these kernels)
    defaults on where the reference sets torch.backends.cudnn.benchmark=True (BASELINE/main.py:40,
    ARCFACE/arc_main.py:51) and off elsewhere; both directions can be forced."""
    from ddp_classification_pytorch_amd.config import parse_args

    assert parse_args(["--workload", "baseline"]).autotune is True
    assert parse_args(["--workload", "arcface"]).autotune is True
    for w in ("cdr", "nested", "plc"):
        assert parse_args(["--workload", w]).autotune is False
    assert parse_args(["--workload", "baseline", "--no-autotune"]).autotune is False
    assert parse_args(["--workload", "cdr", "--autotune"]).autotune is True


def test_resume_mid_warmup_is_equivalent(tmp_path):
    """A checkpoint written while the LR ramp is still running (warm-up longer than an epoch)
    restores a partial-ramp LR into the optimizer; the resumed run must still ramp to --lr and
    end where the uninterrupted run ends."""
    base = ["--workload", "baseline", "--model", "cifar_resnet18", "--epochs", "3", "--optimizer", "SGD",
            "--lr", "0.05", "--warmup-iters", "7"] + SYN
    torch.manual_seed(0)
    entry.main(base + ["--out-dir", str(tmp_path / "ref")])
    ref = torch.load(tmp_path / "ref" / "last.pth", weights_only=True)
    with pytest.raises(InjectedFailure):
        entry.main(base + ["--out-dir", str(tmp_path / "ft"), "--fail-at-step", "5"])  # epoch 2, step 5 of 7
    mid = torch.load(tmp_path / "ft" / "last.pth", weights_only=True)
    assert mid["warmup"]["n"] == 4 and mid["optimizers"]["opt"]["param_groups"][0]["lr"] < 0.05
    entry.main(base + ["--out-dir", str(tmp_path / "ft"), "--resume", str(tmp_path / "ft" / "last.pth")])
    got = torch.load(tmp_path / "ft" / "last.pth", weights_only=True)
    assert got["optimizers"]["opt"]["param_groups"][0]["lr"] == pytest.approx(
        ref["optimizers"]["opt"]["param_groups"][0]["lr"])
    for k, v in ref["models"]["model"].items():
        if v.dtype.is_floating_point:
            assert torch.allclose(v, got["models"]["model"][k], atol=1e-5), k


def test_autotune_env_switch_applies_without_flag(monkeypatch):
    from ddp_classification_pytorch_amd.config import parse_args

    monkeypatch.setenv("DCP_AUTOTUNE", "1")
    assert parse_args(["--workload", "cdr"]).autotune is True
    monkeypatch.setenv("DCP_AUTOTUNE", "0")
    assert parse_args(["--workload", "baseline"]).autotune is False
    assert parse_args(["--workload", "baseline", "--autotune"]).autotune is True  # the flag wins


@pytest.mark.parametrize("workload", ["baseline", "cdr"])
def test_workload_learns_cpu(tmp_path, workload):
    """Plumbing half of the GPU learning tests: class-carrying synthetic images, 3 epochs, the
    train loss falls by at least 30 %."""
    out = tmp_path / "o"
    entry.main(["--workload", workload, "--model", "resnet18", "--data", "synthetic", "--synthetic-learnable",
                "--device", "cpu", "--batchsize", "16", "--synthetic-train-size", "64", "--synthetic-val-size", "16",
                "--epochs", "3", "--out-dir", str(out), "--image-size", "64", "--num-classes", "10", "--dataset", "food",
                "--workers", "0", "--log-interval", "4", "--lr", "0.05"])
    losses = [json.loads(x)["loss"] for x in open(out / "metrics.jsonl") if '"train_iter"' in x]
    assert len(losses) == 3 and losses[-1] <= 0.7 * losses[0], losses


def test_device_synthetic_data_runs(tmp_path):
    """--data synthetic-device (bench.py's on-device input) through main.py."""
    out = tmp_path / "o"
    entry.main(["--workload", "baseline", "--model", "resnet18", "--data", "synthetic-device", "--device", "cpu",
                "--batchsize", "8", "--synthetic-train-size", "16", "--synthetic-val-size", "8", "--epochs", "1",
                "--out-dir", str(out), "--dataset", "CIFAR10", "--log-interval", "1"])
    recs = [json.loads(x) for x in open(out / "metrics.jsonl") if '"train_iter"' in x]
    assert len(recs) == 2 and all(r["img_per_s"] > 0 for r in recs)
