"""Multi-process data parallelism on CPU (gloo, world_size 2):
* DDP + SyncBN over two half-batches == one process over the full batch
  (loss, BN running stats, every gradient);
* exact distributed metrics (one packed all_reduce);
* the full training entry point under 2 ranks (checkpoint written once)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _ddp_syncbn_worker(rank, world, port, out_dir, shared=False):
    if shared:
        os.environ["DCP_SYNCBN_SHARED_GROUP"] = "1"
    _init(rank, world, port)
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn
    from ddp_classification_pytorch_amd.parallel.ddp import wrap_ddp

    torch.manual_seed(0)
    model = build_model("cifar_resnet18", num_classes=10)
    imgs = torch.randn(8, 3, 32, 32, generator=torch.Generator().manual_seed(1))
    labels = torch.randint(0, 10, (8,), generator=torch.Generator().manual_seed(2))
    net = wrap_ddp(model, None, syncbn=True, bucket_cap_mb=1)
    sl = slice(rank * 4, rank * 4 + 4)
    x = Fn.to_device_nhwc(imgs[sl], cpad=8)
    loss = Fn.cross_entropy(net(x), labels[sl])
    loss.backward()
    lt = loss.detach().clone()
    dist.all_reduce(lt)
    from ddp_classification_pytorch_amd.parallel.ddp import bn_process_group

    assert (bn_process_group() is dist.group.WORLD) == shared
    if rank == 0:
        torch.save({"loss": lt / world, "grads": {n: p.grad.clone() for n, p in model.named_parameters()},
                    "rm": model.bn1.running_mean.clone(), "rv": model.bn1.running_var.clone(),
                    "bufs": {n: b.clone() for n, b in model.named_buffers() if "running" in n}},
                   os.path.join(out_dir, "ddp.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("shared", [False, True])
def test_ddp_syncbn_equals_single_process_full_batch(shared):
    """2-rank DDP + SyncBN == one process on the full batch; ``shared``: the BN statistics on the
    gradient communicator (--syncbn-shared-group, the fallback for stacks where two communicators
    in flight on one GPU misbehave) gives the same result."""
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ddp_syncbn_worker, args=(2, _free_port(), d, shared), nprocs=2, join=True)
        got = torch.load(os.path.join(d, "ddp.pt"), weights_only=True)
    imgs = torch.randn(8, 3, 32, 32, generator=torch.Generator().manual_seed(1))
    labels = torch.randint(0, 10, (8,), generator=torch.Generator().manual_seed(2))

    def single(x):
        torch.manual_seed(0)
        model = build_model("cifar_resnet18", num_classes=10)
        loss = Fn.cross_entropy(model(Fn.to_device_nhwc(x, cpad=8)), labels)
        loss.backward()
        return model, loss

    model, loss = single(imgs)
    # Numerical floor of this net: ReLU kinks make its gradient move ~2e-3 under a 1e-7
    # relative input perturbation, which is the size of fp32 reordering differences
    # between two-rank (Chan-merged) and one-rank BN statistics.
    model_p, _ = single(imgs * (1 + 1e-7 * torch.randn(imgs.shape, generator=torch.Generator().manual_seed(5))))
    flat = lambda m: torch.cat([p.grad.flatten() for p in m.parameters()])  # noqa: E731
    g_ref, g_perm = flat(model), flat(model_p)
    g_ddp = torch.cat([got["grads"][n].flatten() for n, _ in model.named_parameters()])
    floor = ((g_perm - g_ref).norm() / g_ref.norm()).item()
    err = ((g_ddp - g_ref).norm() / g_ref.norm()).item()
    # the mean of two half-batch means == the full-batch mean for equal halves
    assert abs(float(got["loss"]) - loss.item()) < 1e-5
    assert torch.allclose(got["rm"], model.bn1.running_mean, atol=1e-6)
    assert torch.allclose(got["rv"], model.bn1.running_var, atol=1e-5)
    # every BN, including the projection shortcuts normalised inside the block's last BN pass
    for n, b in model.named_buffers():
        if "running" in n:
            assert torch.allclose(got["bufs"][n], b, atol=1e-5), n
    assert err <= 3 * floor + 1e-5, (err, floor)


def _bn_group_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.models.layers import BatchNorm2d
    from ddp_classification_pytorch_amd.ops import functional as Fn
    from ddp_classification_pytorch_amd.parallel import ddp as pddp

    torch.manual_seed(0)
    model = build_model("cifar_resnet18", num_classes=10)
    net = pddp.wrap_ddp(model, None, syncbn=True, bucket_cap_mb=1)
    groups = {m.process_group for m in model.modules() if isinstance(m, BatchNorm2d)}
    calls = []
    real_ag, real_ar = dist.all_gather_into_tensor, dist.all_reduce

    def ag(out, inp, group=None, **kw):
        calls.append(("gather", group))
        return real_ag(out, inp, group=group, **kw)

    def ar(t, op=dist.ReduceOp.SUM, group=None, **kw):
        calls.append(("reduce", group))
        return real_ar(t, op=op, group=group, **kw)

    dist.all_gather_into_tensor, dist.all_reduce = ag, ar
    try:
        x = Fn.to_device_nhwc(torch.randn(4, 3, 32, 32, generator=torch.Generator().manual_seed(rank)), cpad=8)
        loss = Fn.cross_entropy(net(x), torch.randint(0, 10, (4,), generator=torch.Generator().manual_seed(3)))
        n_fwd = len(calls)
        loss.backward()
    finally:
        dist.all_gather_into_tensor, dist.all_reduce = real_ag, real_ar
    bn = pddp.bn_process_group()
    # the gradient buckets of the bucket engine go to the default group (group=None)
    grad_calls = [c for c in calls if c[1] is None]
    bn_calls = [c for c in calls if c[1] is not None]
    n_fwd_bn = sum(1 for c in calls[:n_fwd] if c[1] is not None)
    if rank == 0:
        torch.save({"one_group": len(groups) == 1, "is_bn": groups == {bn}, "not_world": bn is not dist.group.WORLD,
                    "all_on_bn": all(g is bn for _, g in bn_calls), "n_fwd": n_fwd_bn,
                    "n_bwd": len(bn_calls) - n_fwd_bn, "kinds_fwd": sorted({k for k, _ in calls[:n_fwd]}),
                    "grad_calls": len(grad_calls), "buckets": len(net.reducer.buckets),
                    "n_bn": sum(isinstance(m, BatchNorm2d) for m in model.modules())},
                   os.path.join(out_dir, "g.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_uses_dedicated_group_and_coalesces():
    """SyncBN collectives run on their own process group (never queued behind the Reducer's
    buckets on the default group), one all-gather per BN forward and one all-reduce per BN
    backward, a projection block's two BNs sharing one of each."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_bn_group_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = torch.load(os.path.join(d, "g.pt"), weights_only=True)
    assert got["one_group"] and got["is_bn"] and got["not_world"] and got["all_on_bn"]
    assert got["kinds_fwd"] == ["gather"]
    n_bn, n_proj = got["n_bn"], 3  # CIFAR ResNet-18: 20 BNs, 3 projection shortcuts
    assert n_bn == 20
    assert got["n_fwd"] == n_bn - n_proj, got
    assert got["n_bwd"] == n_bn - n_proj, got
    assert got["grad_calls"] == got["buckets"]  # one all-reduce per gradient bucket, default group


def _metrics_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    from ddp_classification_pytorch_amd.parallel.ddp import all_reduce_metrics, reduce_loss

    vec = torch.tensor([float(rank + 1), 2.0 * rank, 1.0, 10.0], dtype=torch.float64)
    all_reduce_metrics(vec)
    rl = reduce_loss(torch.tensor(float(rank + 1)), world)
    if rank == 0:
        torch.save({"vec": vec, "rl": rl}, os.path.join(out_dir, "m.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_exact_metric_allreduce_and_reduce_loss():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_metrics_worker, args=(3, _free_port(), d), nprocs=3, join=True)
        got = torch.load(os.path.join(d, "m.pt"), weights_only=True)
    assert got["vec"].tolist() == [6.0, 6.0, 3.0, 30.0]
    assert float(got["rl"]) == pytest.approx(2.0)  # (1+2+3)/3 on rank 0 (BASELINE/main.py:52-56)


def _entry_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import main as entry

    entry.main(["--workload", "baseline", "--model", "cifar_resnet18", "--data", "synthetic", "--dataset", "CIFAR10",
                "--batchsize", "4", "--synthetic-train-size", "24", "--synthetic-val-size", "10", "--workers", "0",
                "--epochs", "1", "--device", "cpu", "--syncbn", "--out-dir", out_dir, "--log-interval", "100"])


def test_entry_point_two_ranks_gloo():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_entry_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        assert os.path.exists(os.path.join(d, "last.pth"))
        txt = open(os.path.join(d, "output.txt")).read()
        assert "(n=10)" in txt  # exact val count: sampler padding excluded


def _workload_worker(rank, world, port, out_dir, workload):
    """Run a workload under 2 gloo ranks and record, per rank, the final parameters of every
    module it put under DDP (CDR / NESTED / PLC all-reduce their gradients)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import main as entry
    from ddp_classification_pytorch_amd.algos import arcface, baseline, nested, plc
    from ddp_classification_pytorch_amd.parallel import ddp as pddp

    wrapped = []
    orig = pddp.wrap_ddp

    def recording_wrap(model, *a, **kw):
        out = orig(model, *a, **kw)
        wrapped.append((model, out))
        return out

    pddp.wrap_ddp = nested.wrap_ddp = plc.wrap_ddp = arcface.wrap_ddp = baseline.wrap_ddp = recording_wrap
    common = ["--model", "resnet18", "--data", "synthetic", "--dataset", "CIFAR10", "--batchsize", "4",
              "--synthetic-train-size", "16", "--synthetic-val-size", "8", "--workers", "0", "--epochs", "1",
              "--device", "cpu", "--out-dir", os.path.join(out_dir, f"run{rank}"), "--log-interval", "100"]
    extra = {"cdr": [], "nested": ["--nested", "20", "--warmup-iters", "2"], "plc": ["--plc-eta-epochs", "1"],
             "arcface": ["--num-classes", "10"], "baseline": ["--lr", "0.05"]}
    entry.main(["--workload", workload] + common + extra[workload])
    from ddp_classification_pytorch_amd.parallel.reducer import GradSyncDDP

    assert wrapped and all(isinstance(d, (torch.nn.parallel.DistributedDataParallel, GradSyncDDP)) for _, d in wrapped)
    torch.save([{n: p.detach().clone() for n, p in m.named_parameters()} for m, _ in wrapped],
               os.path.join(out_dir, f"params{rank}.pt"))


@pytest.mark.parametrize("workload", ["cdr", "nested", "plc", "arcface", "baseline"])
def test_noisy_label_workloads_stay_in_sync_under_ddp(workload):
    """Ranks start from rank 0's weights (DDP broadcast) and apply all-reduced gradients, so
    after training on different shards (and different seed+rank RNG streams) every rank
    holds the same model."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_workload_worker, args=(2, _free_port(), d, workload), nprocs=2, join=True)
        p0 = torch.load(os.path.join(d, "params0.pt"), weights_only=True)
        p1 = torch.load(os.path.join(d, "params1.pt"), weights_only=True)
    assert len(p0) == len(p1) >= 1
    for a, b in zip(p0, p1):
        assert a.keys() == b.keys()
        for n in a:
            assert torch.allclose(a[n], b[n], atol=1e-6, rtol=1e-5), n


def _syncbn_count_worker(rank, world, port, out_dir, unequal):
    _init(rank, world, port)
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn
    from ddp_classification_pytorch_amd.parallel.ddp import convert_sync_batchnorm

    Fn._SYNCBN_CHECK[0] = True
    torch.manual_seed(0)
    model = convert_sync_batchnorm(build_model("cifar_resnet18", num_classes=10))
    n = 4 + (rank if unequal else 0)
    x = Fn.to_device_nhwc(torch.randn(n, 3, 32, 32, generator=torch.Generator().manual_seed(rank)), cpad=8)
    err = None
    try:
        model(x)
    except RuntimeError as e:
        err = str(e)
    torch.save({"err": err}, os.path.join(out_dir, f"c{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("unequal", [False, True])
def test_syncbn_equal_count_check(unequal):
    """SyncBN's backward normalises by per-rank count x world (equal batches, which the padded
    sharded sampler guarantees); DCP_SYNCBN_CHECK=1 turns a violation into an error."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_syncbn_count_worker, args=(2, _free_port(), d, unequal), nprocs=2, join=True)
        errs = [torch.load(os.path.join(d, f"c{r}.pt"), weights_only=True)["err"] for r in range(2)]
    if unequal:
        assert all(e is not None and "unequal per-rank batch counts" in e for e in errs)
    else:
        assert errs == [None, None]
