"""HIP-graph capture of a full training step (engine/graph.py): replaying the captured step
reproduces the eager step sequence (deterministic kernels: same losses and weights)."""
import copy

import pytest
import torch

from ddp_classification_pytorch_amd.engine.graph import GraphedStep
from ddp_classification_pytorch_amd.models import build_model, input_layout
from ddp_classification_pytorch_amd.ops import functional as Fn
from ddp_classification_pytorch_amd.optim import FusedSGD

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,size", [("resnet18", 64), ("resnet50", 64)])
def test_graphed_step_matches_eager(name, size):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    base = build_model(name, num_classes=10).to(dev)
    imgs = torch.randint(0, 256, (8, 3, size, size), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 10, (8,), device=dev)
    mean = torch.tensor((0.485, 0.456, 0.406), device=dev)
    std = torch.tensor((0.229, 0.224, 0.225), device=dev)

    def make(model):
        opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        lay = input_layout(model)

        def step():
            x = Fn.to_device_nhwc(imgs, mean, std, nchw=True, in_scale=1 / 255.0, **lay)
            loss = Fn.cross_entropy(model(x), labels)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            return loss

        return step

    m_eager, m_graph = base, copy.deepcopy(base)
    eager = make(m_eager)
    ref = [eager().item() for _ in range(5)][2:]
    graphed = GraphedStep(make(m_graph), warmup=2)
    got = [graphed().item() for _ in range(3)]
    assert all(abs(a - b) <= 1e-4 * max(1.0, abs(a)) for a, b in zip(ref, got)), (ref, got)
    for (n, p1), p2 in zip(m_eager.named_parameters(), m_graph.parameters()):
        assert torch.allclose(p1, p2, rtol=1e-4, atol=1e-5), n


@pytest.mark.parametrize("name", ["resnet50", "resnext50_32x4d"])
def test_wgrad_side_stream_matches(name):
    """DCP_WGRAD_STREAM: conv weight gradients on a second HIP stream beside the data gradients
    give bitwise the same gradients (deterministic kernels), eagerly and when the step is
    captured into a HIP graph (the side stream forks from and rejoins the capturing stream)."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    base = build_model(name, num_classes=10).to(dev)
    imgs = torch.randint(0, 256, (4, 3, 64, 64), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 10, (4,), device=dev)
    mean = torch.tensor((0.485, 0.456, 0.406), device=dev)
    std = torch.tensor((0.229, 0.224, 0.225), device=dev)
    lay = input_layout(base)

    def grads(model):
        for p in model.parameters():
            p.grad = None
        x = Fn.to_device_nhwc(imgs, mean, std, nchw=True, in_scale=1 / 255.0, **lay)
        Fn.cross_entropy(model(x), labels).backward()
        torch.cuda.synchronize()
        return [p.grad.clone() for p in model.parameters()]

    try:
        Fn.set_wgrad_stream(False)
        ref = grads(base)
        Fn.set_wgrad_stream(True)
        got = grads(base)
        for (n, _), a, b in zip(base.named_parameters(), ref, got):
            assert torch.equal(a, b), n
        if name == "resnet50":
            m_eager, m_graph = base, copy.deepcopy(base)

            def make(model):
                opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9)

                def step():
                    x = Fn.to_device_nhwc(imgs, mean, std, nchw=True, in_scale=1 / 255.0, **lay)
                    loss = Fn.cross_entropy(model(x), labels)
                    opt.zero_grad(set_to_none=True)
                    loss.backward()
                    opt.step()
                    return loss

                return step

            Fn.set_wgrad_stream(False)
            eager = make(m_eager)
            ref_l = [eager().item() for _ in range(4)][2:]
            Fn.set_wgrad_stream(True)
            graphed = GraphedStep(make(m_graph), warmup=2)
            got_l = [graphed().item() for _ in range(2)]
            assert all(abs(a - b) <= 1e-4 * max(1.0, abs(a)) for a, b in zip(ref_l, got_l)), (ref_l, got_l)
    finally:
        Fn.set_wgrad_stream(False)


@pytest.mark.parametrize("n,dtype", [(1, torch.int64), (448, torch.int64), (1000, torch.int64), (7, torch.int32),
                                     (2000, torch.int32)])
def test_table_to_device_through_kernel_args(n, dtype):
    rows = torch.randint(-2**30, 2**30, (n,), dtype=dtype).tolist()
    out = Fn.table_to_device(rows, dtype, "cuda")
    assert out.dtype == dtype and out.shape == (n,)
    assert torch.equal(out.cpu(), torch.tensor(rows, dtype=dtype))
    two = Fn.table_to_device([[1, 2], [3, 4], [5, 6]], dtype, "cuda")
    assert two.shape == (3, 2) and two.cpu().tolist() == [[1, 2], [3, 4], [5, 6]]


@pytest.mark.parametrize("workload,extra", [
    ("baseline", ["--optimizer", "SGD", "--lr", "0.05"]),
    ("baseline", ["--optimizer", "SGD", "--lr", "0.05", "--warmup-iters", "4"]),  # eager ramp, then capture
    ("arcface", ["--optimizer", "Adam", "--lr", "1e-3"]),  # device step counter (bias correction)
    ("cdr", ["--lr", "0.05"]),                              # radix-select tables from fill kernels
])
def test_training_loop_graph_matches_eager(tmp_path, workload, extra):
    """main.py --graph (StepGrapher: eager warm-up, capture, replays, recapture per epoch, eager
    short last batch) trains to the same weights as the eager loop, and the host-side counters
    (BN num_batches_tracked, Adam's per-parameter step) advance on every replay."""
    import main as entry

    common = ["--workload", workload, "--model", "resnet18", "--data", "synthetic", "--dataset", "CIFAR10",
              "--batchsize", "16", "--synthetic-train-size", "120", "--synthetic-val-size", "32", "--epochs", "2",
              "--workers", "0", "--log-interval", "100", "--num-classes", "10"] + extra
    outs = {}
    for tag, flag in (("eager", ["--no-graph"]), ("graph", ["--graph"])):
        torch.manual_seed(0)
        entry.main(common + ["--out-dir", str(tmp_path / tag)] + flag)
        outs[tag] = torch.load(tmp_path / tag / "last.pth", weights_only=True)
    for name, me in outs["eager"]["models"].items():
        mg = outs["graph"]["models"][name]
        for k, v in me.items():
            if v.dtype.is_floating_point:
                assert torch.allclose(v, mg[k], rtol=2e-3, atol=2e-4), (name, k)
            else:
                assert torch.equal(v, mg[k]), (name, k)  # num_batches_tracked
    oe, og = outs["eager"]["optimizers"]["opt"]["state"], outs["graph"]["optimizers"]["opt"]["state"]
    for i, st in oe.items():
        if "step" in st:
            assert int(st["step"]) == int(og[i]["step"]) > 8, (i, st["step"], og[i]["step"])


def test_gpu_failure_and_resume(tmp_path):
    """Resume on the GPU (RNG ByteTensors must stay on the host): a run killed in epoch 2
    and resumed from last.pth matches the uninterrupted run."""
    import main as entry
    from ddp_classification_pytorch_amd.engine.loop import InjectedFailure

    base = ["--workload", "arcface", "--model", "resnet18", "--data", "synthetic", "--dataset", "CIFAR10",
            "--batchsize", "16", "--synthetic-train-size", "64", "--synthetic-val-size", "16", "--epochs", "2",
            "--workers", "0", "--log-interval", "100", "--num-classes", "10", "--optimizer", "Adam"]
    torch.manual_seed(0)
    entry.main(base + ["--out-dir", str(tmp_path / "ref")])
    with pytest.raises(InjectedFailure):
        torch.manual_seed(0)
        entry.main(base + ["--out-dir", str(tmp_path / "ft"), "--fail-at-step", "6"])
    entry.main(base + ["--out-dir", str(tmp_path / "ft"), "--auto-resume"])
    ref = torch.load(tmp_path / "ref" / "last.pth", weights_only=True)
    got = torch.load(tmp_path / "ft" / "last.pth", weights_only=True)
    assert got["epoch"] == ref["epoch"] == 1 and got["global_step"] == ref["global_step"]
    for name, m in ref["models"].items():
        for k, v in m.items():
            if v.dtype.is_floating_point:
                assert torch.allclose(v, got["models"][name][k], rtol=1e-3, atol=1e-4), (name, k)
