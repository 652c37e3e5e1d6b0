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
