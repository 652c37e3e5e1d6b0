"""Multi-rank data parallelism through the HIP kernels on ONE GPU (the round-end
driver runs the real 1/2/4/8-GPU RCCL benchmark; RCCL refuses two ranks on one
device, so these tests use gloo for the collectives while every op runs on cuda:0):

* ``bench.py --gpus 2`` (self-launched ranks, no torchrun on the command line) prints one JSON
  line with n_gpus == 2 and the SyncBN phase's number;
* RCCL itself: a world_size-1 ``nccl`` process group (eager communicator init) under a forced
  DDP wrapper, one ResNet-18 training step whose gradients pass through the RCCL Reducer;
* DDP over 2 ranks x 4 images == one process over the same 8 images (loss and
  every gradient, within the bf16 noise floor), local BN and SyncBN."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_one_gpu():
    env = dict(os.environ, DCP_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "8", "--image-size", "64"]
    out = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["config"]["global_batch"] == 16
    assert rec["value"] > 0 and rec["syncbn_value"] > 0 and rec["dist_backend"] == "gloo"
    assert len(rec["per_rank_ms"]) == 2
    # the peer-memory SyncBN phase ran and agrees with the RCCL/gloo transport on the same inputs
    assert "diagnostic_errors" not in rec, rec.get("diagnostic_errors")
    assert rec["syncbn_peer_value"] > 0
    assert rec["syncbn_peer_max_rel_diff"] <= 1e-6, rec["syncbn_peer_rel_diff_parts"]


@pytest.mark.parametrize("graph", [False, True])
def test_bench_force_ddp_rccl_world1(graph):
    """bench.py --force-ddp: a world-1 RCCL group through the bucket engine, eager and HIP-graph
    replay, with the SyncBN phase, the bucket telemetry (eager) and the collective probe in the
    JSON line."""
    # DCP_SYNCBN_WORLD1: keep the SyncBN collectives at world 1 (torch -- and so the default -- skips them)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               DCP_SYNCBN_WORLD1="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--force-ddp", "--steps", "3", "--warmup", "2",
           "--batch", "8", "--image-size", "64"] + (["--graph"] if graph else [])
    out = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["dist_backend"] == "nccl" and rec["world_size"] == 1 and rec["value"] > 0
    assert rec["syncbn_value"] > 0 and rec["config"]["hip_graph"] == graph
    probe = rec["comm_probe"]
    assert probe["world"] == 1 and set(probe["allreduce_ms"]) == {"4MB", "25MB", "100MB"}
    assert probe["syncbn_allgather_us"] > 0 and probe["syncbn_allreduce_us"] > 0
    if not graph:
        assert rec["comm"]["engine"] == "dcp" and rec["comm"]["buckets"] >= 1


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--batch", "4", "--image-size", "64"]
    out = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "--gpus 2" in out.stderr


def _rccl_worker(rank, world, port, out_dir, engine="torch"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DCP_SYNCBN_WORLD1="1")
    sys.path.insert(0, ROOT)
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn
    from ddp_classification_pytorch_amd.optim import FusedSGD
    from ddp_classification_pytorch_amd.parallel.ddp import bn_process_group, wrap_ddp

    import datetime

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=120))
    torch.manual_seed(0)
    model = build_model("resnet18", num_classes=10).to(dev)
    net = wrap_ddp(model, 0, syncbn=True, bucket_cap_mb=1, force=True, engine=engine)
    assert isinstance(net, torch.nn.parallel.DistributedDataParallel) == (engine == "torch")
    bn_group = bn_process_group()
    assert bn_group is not None and bn_group is not dist.group.WORLD
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (8, 3, 64, 64), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (8,), generator=g)
    x = Fn.to_device_nhwc(imgs.to(dev), (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), cpad=8, in_scale=1 / 255.0)
    loss = Fn.cross_entropy(net(x), labels.to(dev))
    loss.backward()
    grads = {n: p.grad.detach().cpu().clone() for n, p in model.named_parameters()}
    opt.step()
    t = torch.ones(4, device=dev)
    dist.all_reduce(t)  # the default (Reducer) communicator
    dist.all_reduce(t, group=bn_group)  # the SyncBN communicator
    torch.cuda.synchronize()
    torch.save({"loss": loss.item(), "grads": grads, "t": t.cpu(), "backend": dist.get_backend(),
                "rccl": str(torch.cuda.nccl.version())}, os.path.join(out_dir, "rccl.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("engine", ["torch", "dcp"])
def test_rccl_world1_ddp_step(engine):
    """RCCL executes: world-1 ``nccl`` group, forced DDP + SyncBN (torch's Reducer or the bucket
    engine), gradients equal a plain step."""
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rccl_worker, args=(1, _free_port(), d, engine), nprocs=1, join=True)
        got = torch.load(os.path.join(d, "rccl.pt"), weights_only=True)
    assert got["backend"] == "nccl" and torch.equal(got["t"], torch.ones(4))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_model("resnet18", num_classes=10).to(dev)
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (8, 3, 64, 64), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (8,), generator=g)
    x = Fn.to_device_nhwc(imgs.to(dev), (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), cpad=8, in_scale=1 / 255.0)
    loss = Fn.cross_entropy(model(x), labels.to(dev))
    loss.backward()
    assert abs(loss.item() - got["loss"]) < 1e-3 * max(1.0, abs(loss.item()))
    for n, p in model.named_parameters():
        ref = p.grad.detach().cpu().float()
        err = (got["grads"][n].float() - ref).norm() / max(ref.norm().item(), 1e-12)
        assert err < 2e-2, (n, float(err))


def _worker(rank, world, port, syncbn, out_dir, transport="rccl"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      DCP_SYNCBN_TRANSPORT=transport)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn
    from ddp_classification_pytorch_amd.parallel.ddp import wrap_ddp

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_model("resnet18", num_classes=10).to(dev)
    net = wrap_ddp(model, 0, syncbn=syncbn, bucket_cap_mb=1)
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (8, 3, 64, 64), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (8,), generator=g)
    sl = slice(rank * 4, rank * 4 + 4)
    x = Fn.to_device_nhwc(imgs[sl].to(dev), (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), cpad=8,
                          in_scale=1 / 255.0)
    loss = Fn.cross_entropy(net(x), labels[sl].to(dev))
    loss.backward()
    lt = loss.detach().clone().cpu()
    dist.all_reduce(lt)
    if rank == 0:
        torch.save({"loss": lt / world, "grads": {n: p.grad.detach().cpu() for n, p in model.named_parameters()}},
                   os.path.join(out_dir, "ddp.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("syncbn,transport", [(False, "rccl"), (True, "rccl"), (True, "peer")])
def test_ddp_two_ranks_matches_full_batch(syncbn, transport):
    """(transport "peer": the SyncBN statistics through the IPC-mapped mailboxes of
    parallel/peer.py, the two ranks' processes sharing the one GPU)"""
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn

    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), syncbn, d, transport), nprocs=2, join=True)
        got = torch.load(os.path.join(d, "ddp.pt"), weights_only=True)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (8, 3, 64, 64), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (8,), generator=g).to(dev)

    def run(sl, perm=False):
        torch.manual_seed(0)
        m = build_model("resnet18", num_classes=10).to(dev)
        loss = 0.0
        for s in sl:
            idx = torch.arange(8)[s]
            if perm:
                idx = idx.flip(0)  # same samples, reversed order: only the summation order changes
            x = Fn.to_device_nhwc(imgs[idx].to(dev), (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), cpad=8,
                                  in_scale=1 / 255.0)
            loss = loss + Fn.cross_entropy(m(x), labels[idx.to(dev)])
        loss = loss / len(sl)
        loss.backward()
        return loss.item(), torch.cat([p.grad.flatten().float().cpu() for p in m.parameters()])

    sl = [slice(0, 8)] if syncbn else [slice(0, 4), slice(4, 8)]  # global-batch vs per-rank BN statistics
    ref_loss, ref = run(sl)
    _, ref_perm = run(sl, perm=True)
    g_ddp = torch.cat([got["grads"][n].flatten().float() for n, _ in build_model("resnet18", 10).named_parameters()])
    # numerical floor of this tiny-batch bf16 net: the same batch in another summation order
    floor = ((ref_perm - ref).norm() / ref.norm()).item()
    err = ((g_ddp - ref).norm() / ref.norm()).item()
    assert abs(float(got["loss"]) - ref_loss) < 2e-2 * max(1.0, abs(ref_loss))
    assert err <= 3 * floor + 1e-2, (err, floor)


def _rccl_graph_worker(rank, world, port, out_dir, grad_comm, optim="sgd", comm_stream="auto"):
    """World-1 RCCL group, bucket engine + SyncBN (its own communicator) + the optimizer fused per
    bucket: 5 eager steps vs 2 eager warm-up steps + 3 HIP-graph replays of the captured step, from
    the same initial state -- the captured all-reduces, SyncBN collectives and per-bucket optimizer
    launches must replay to the same parameters.  ``comm_stream="1"`` forces the side
    communication stream that world > 1 uses (DCP_COMM_STREAM): the captured fork / join, the
    all-reduce and the per-bucket SGD / Adam on that stream, the autograd gradients held to the
    join."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DCP_COMM_STREAM=comm_stream, DCP_SYNCBN_WORLD1="1")
    sys.path.insert(0, ROOT)
    import datetime

    from ddp_classification_pytorch_amd.engine.graph import GraphedStep
    from ddp_classification_pytorch_amd.models import build_model, input_layout
    from ddp_classification_pytorch_amd.ops import functional as Fn
    from ddp_classification_pytorch_amd.optim import FusedAdam, FusedSGD
    from ddp_classification_pytorch_amd.parallel import reducer as R
    from ddp_classification_pytorch_amd.parallel.ddp import attach_optimizer, graph_safe_nccl_env, wrap_ddp

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    graph_safe_nccl_env()
    dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=120))
    side = R._comm_stream(dev, 1) != torch.cuda.current_stream(dev)
    assert side == (comm_stream == "1"), (side, comm_stream)
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (16, 3, 64, 64), dtype=torch.uint8, generator=g).to(dev)
    labels = torch.randint(0, 10, (16,), generator=g).to(dev)
    out = {}
    for mode in ("eager", "graph"):
        torch.manual_seed(0)
        model = build_model("resnet18", num_classes=10).to(dev)
        net = wrap_ddp(model, 0, syncbn=True, bucket_cap_mb=2, first_bucket_mb=0.5, force=True, engine="dcp",
                       comm_dtype=torch.bfloat16 if grad_comm == "bf16" else torch.float32)
        opt = (FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4) if optim == "sgd"
               else FusedAdam(model.parameters(), lr=1e-3, weight_decay=1e-4))
        attach_optimizer(net, opt)
        x = Fn.to_device_nhwc(imgs, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), in_scale=1 / 255.0,
                              **input_layout(model))

        def step():
            loss = Fn.cross_entropy(net(x), labels)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            return loss.detach()

        if mode == "eager":
            for _ in range(5):
                loss = step()
        else:
            gs = GraphedStep(step, warmup=2, distributed=True)
            for _ in range(3):
                loss = gs()
        torch.cuda.synchronize()
        out[mode] = {"params": {n: p.detach().cpu().clone() for n, p in model.named_parameters()},
                     "rm": model.layer2[0].bn1.running_mean.detach().cpu().clone(), "loss": float(loss),
                     "buckets": len(net.reducer.buckets)}
    torch.save(out, os.path.join(out_dir, "graph.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("grad_comm,optim,comm_stream", [
    ("fp32", "sgd", "auto"), ("bf16", "sgd", "auto"),  # world 1: bucket work on the compute stream
    ("fp32", "sgd", "1"), ("bf16", "sgd", "1"), ("fp32", "adam", "1"),  # the side stream N ranks use
])
def test_rccl_world1_bucket_engine_graph_replay_matches_eager(grad_comm, optim, comm_stream):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rccl_graph_worker, args=(1, _free_port(), d, grad_comm, optim, comm_stream), nprocs=1, join=True)
        got = torch.load(os.path.join(d, "graph.pt"), weights_only=True)
    e, g = got["eager"], got["graph"]
    assert e["buckets"] >= 3
    assert abs(e["loss"] - g["loss"]) < 1e-3 * max(1.0, abs(e["loss"]))
    for n, v in e["params"].items():
        err = (g["params"][n] - v).norm() / max(v.norm().item(), 1e-12)
        assert err < 1e-4, (n, float(err))
    assert torch.allclose(e["rm"], g["rm"], rtol=1e-4, atol=1e-5)


def test_main_graph_force_ddp_side_stream_matches_eager(tmp_path):
    """main.py --graph through the bucket engine on a world-1 RCCL group with the side
    communication stream forced (DCP_COMM_STREAM=1, the N-rank configuration): 2 epochs, the step
    recaptured at the epoch boundary, SyncBN collectives and per-bucket SGD inside the graph --
    the weights equal the eager run's.  The autotuner is on in both runs; they share one tuning
    cache (DCP_TUNE_CACHE: the eager run records its per-shape choices at exit, the graph run
    replays them), so both run the same kernels -- round 5 had to switch the tuner off here because
    two independently tuned runs could pick kernels that sum BN slabs in another order."""
    common = ["--workload", "baseline", "--model", "resnet18", "--data", "synthetic", "--dataset", "CIFAR10",
              "--batchsize", "16", "--synthetic-train-size", "96", "--synthetic-val-size", "32", "--epochs", "2",
              "--workers", "0", "--log-interval", "100", "--num-classes", "10", "--optimizer", "SGD",
              "--lr", "0.05", "--force-ddp", "--syncbn", "--autotune"]
    cache = str(tmp_path / "tune_cache.txt")
    outs = {}
    for tag, flag in (("eager", ["--no-graph"]), ("graph", ["--graph"])):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(_free_port()), DCP_COMM_STREAM="1", DCP_TUNE_CACHE=cache, DCP_SYNCBN_WORLD1="1")
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            env.pop(k, None)
        cmd = [sys.executable, os.path.join(ROOT, "main.py")] + common + ["--out-dir", str(tmp_path / tag)] + flag
        r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        outs[tag] = torch.load(tmp_path / tag / "last.pth", weights_only=True)
        assert os.path.exists(cache)  # written by the first run, replayed by the second
    for name, me in outs["eager"]["models"].items():
        mg = outs["graph"]["models"][name]
        for k, v in me.items():
            if v.dtype.is_floating_point:
                assert torch.allclose(v, mg[k], rtol=2e-3, atol=2e-4), (name, k)
            else:
                assert torch.equal(v, mg[k]), (name, k)


def _gloo_engine_worker(rank, world, port, engine, out_dir):
    """2 gloo ranks on one GPU, 3 SGD steps through ``engine``: the dcp engine runs its buckets on
    the side communication stream (world > 1) with the optimizer fused per bucket behind each
    all-reduce while the rest of backward still runs; torch's DDP steps after backward."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    from ddp_classification_pytorch_amd.models import build_model
    from ddp_classification_pytorch_amd.ops import functional as Fn
    from ddp_classification_pytorch_amd.optim import FusedSGD
    from ddp_classification_pytorch_amd.parallel import reducer as R
    from ddp_classification_pytorch_amd.parallel.ddp import attach_optimizer, wrap_ddp

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_model("resnet18", num_classes=10).to(dev)
    net = wrap_ddp(model, 0, syncbn=False, bucket_cap_mb=1, first_bucket_mb=0.25, engine=engine)
    opt = attach_optimizer(net, FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4))
    if engine == "dcp":
        assert R._comm_stream(dev, world) != torch.cuda.current_stream(dev)
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (3, 8, 3, 64, 64), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 10, (3, 8), generator=g)
    sl = slice(rank * 4, rank * 4 + 4)
    for it in range(3):
        x = Fn.to_device_nhwc(imgs[it, sl].to(dev), (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), cpad=8,
                              in_scale=1 / 255.0)
        loss = Fn.cross_entropy(net(x), labels[it, sl].to(dev))
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    params = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
    torch.save({"params": params, "buckets": len(net.reducer.buckets) if engine == "dcp" else 0},
               os.path.join(out_dir, f"{engine}{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_engine_two_ranks_side_stream_matches_torch_ddp():
    """the bucket engine's world > 1 path (side stream, per-bucket optimizer during
    backward, gradients held to the join) trains 2 ranks to the same weights as torch's DDP, and
    both ranks stay identical."""
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for engine in ("dcp", "torch"):
            mp.spawn(_gloo_engine_worker, args=(2, _free_port(), engine, d), nprocs=2, join=True)
            res[engine] = [torch.load(os.path.join(d, f"{engine}{r}.pt"), weights_only=True) for r in range(2)]
    assert res["dcp"][0]["buckets"] >= 3
    for n, v in res["torch"][0]["params"].items():
        for r in range(2):
            got = res["dcp"][r]["params"][n]
            err = (got - v).norm() / max(v.norm().item(), 1e-12)
            assert err < 1e-4, (n, r, float(err))
        assert torch.equal(res["dcp"][0]["params"][n], res["dcp"][1]["params"][n]), n


@pytest.mark.parametrize("inject", ["syncbn", "syncbn:1"])
def test_bench_diagnostic_phase_failure_keeps_headline(inject):
    """A failure in the optional SyncBN phase -- on every rank (caught, recorded) or on rank 1 only
    (the ranks then wait in mismatched collectives until the diagnostic deadline) -- still prints
    the one JSON line with the local-BN headline."""
    env = dict(os.environ, DCP_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", DCP_BENCH_INJECT=inject,
               DCP_BENCH_EXTRA_DEADLINE="40")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "8", "--image-size", "64"]
    out = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["syncbn_value"] is None
    errs = rec["diagnostic_errors"]
    assert ("syncbn" in errs) if inject == "syncbn" else ("deadline" in errs or "syncbn" in errs), errs


def _peer_worker(rank, world, port, out_dir):
    """PeerExchange between processes sharing the GPU: gathers and rank-ordered sums of
    integer-valued floats (exact) against gloo's collectives, sizes from 1 float to a full slot,
    many back-to-back exchanges (the epoch-parity mailboxes), and a HIP graph of exchanges
    replayed (the device-side epoch advances per replay)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    from ddp_classification_pytorch_amd.parallel import peer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ex = peer.enable(dist.group.WORLD, dev)
    assert ex is not None and ex.world == world and ex.rank == rank
    errs = []
    g = torch.Generator().manual_seed(100 + rank)
    for it, n in enumerate([1, 7, 192, 6144, peer.MAX_FLOATS] * 4):
        x = torch.randint(-50, 50, (n,), generator=g).float()
        ref_g = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(ref_g, x)
        ref_r = x.clone()
        dist.all_reduce(ref_r)
        out = torch.empty(world * n, device=dev)
        ex.all_gather_into_tensor(out, x.to(dev))
        red = x.to(dev)
        ex.all_reduce(red)
        if not torch.equal(out.cpu(), torch.cat(ref_g)):
            errs.append(("gather", it, n))
        if not torch.equal(red.cpu(), ref_r):
            errs.append(("reduce", it, n))
    # captured exchanges: 3 per replay, 5 replays; the inputs change between replays
    src = torch.zeros(64, device=dev)
    outs = [torch.empty(world * 64, device=dev) for _ in range(3)]
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        for o in outs:
            ex.all_gather_into_tensor(o, src)
            src.add_(1.0)
    for rep in range(5):
        src.fill_(1000.0 * rank + 10.0 * rep)
        graph.replay()
        torch.cuda.synchronize()
        for j, o in enumerate(outs):
            want = torch.cat([torch.full((64,), 1000.0 * r + 10.0 * rep + j) for r in range(world)])
            if not torch.equal(o.cpu(), want):
                errs.append(("graph", rep, j))
    ex.check()
    torch.save({"errs": errs, "epoch": int(ex.epoch.item())}, os.path.join(out_dir, f"peer{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_peer_exchange_matches_gloo():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_peer_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = [torch.load(os.path.join(d, f"peer{r}.pt"), weights_only=True) for r in range(2)]
    for r in res:
        assert r["errs"] == [], r["errs"]
        assert r["epoch"] == 2 * 20 + 3 * 5  # every exchange (eager and replayed) advanced the epoch


def test_syncbn_peer_timeout_fails_loudly(tmp_path):
    """a rank late past the peer exchange's deadline must end the run with a
    message, never continue on a stale mailbox slot.  Two main.py ranks (gloo, one GPU) train with
    SyncBN over the peer transport; rank 1's host sleeps 6 s before its 40th exchange while the
    deadline is 1 s: rank 0's exchange kernel times out (err set, NaN written), the training loop's
    check raises, and the job exits non-zero naming the peer exchange."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", DCP_PEER_TIMEOUT_S="1", DCP_PEER_DELAY="1:6:40")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "main.py"),
           "--workload", "baseline", "--model", "resnet18", "--data", "synthetic", "--dataset", "CIFAR10",
           "--batchsize", "8", "--synthetic-train-size", "96", "--synthetic-val-size", "16", "--epochs", "1",
           "--workers", "0", "--log-interval", "2", "--num-classes", "10", "--optimizer", "SGD", "--lr", "0.05",
           "--syncbn", "--syncbn-transport", "peer", "--dist-backend", "gloo", "--no-graph", "--no-autotune",
           "--out-dir", str(tmp_path / "out")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "SyncBN peer exchange" in r.stderr and "did not publish" in r.stderr, r.stderr[-3000:]
