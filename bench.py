#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 224px DDP training throughput (images/sec, whole job).

BASELINE.json metric: "images/sec (whole node), ResNet-50 224px DDP at 1/2/4/8 MI355X".
Synthetic ImageNet-1k-shaped data (uint8 images generated on device, random
labels), random-init ResNet-50, bf16 activations / fp32 master weights, full
training step in the timed region: input normalisation (u8 NCHW -> bf16 NHWC
kernel), forward, softmax-CE, backward (DDP bucketed all-reduce over RCCL when
N > 1), fused SGD-momentum step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

``--gpus N`` without a torchrun environment launches the N ranks itself (a
``torch.distributed.run`` child process, started before anything touches the GPU);
under torchrun ``--gpus`` must equal WORLD_SIZE.

Rank 0 prints ONE JSON line; `value` = total images/s over all ranks, timed
as the MAX over ranks of K steps bracketed by barrier + device sync.  With N > 1 a
second timed phase of the same K steps runs the reference's cross-replica BN
(SyncBN on its own RCCL communicator) and reports it as ``syncbn_value``; the
headline ``value`` is local BN (per-GPU batch 4096: 156 GB of the 288 GB HBM).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import threading
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from ddp_classification_pytorch_amd import _ext, tuning  # noqa: E402
from ddp_classification_pytorch_amd.models import build_model, input_layout  # noqa: E402
from ddp_classification_pytorch_amd.ops import functional as Fn  # noqa: E402
from ddp_classification_pytorch_amd.optim import FusedSGD  # noqa: E402
from ddp_classification_pytorch_amd.parallel import ddp as pddp  # noqa: E402

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); launched here when no torchrun environment is set")
    ap.add_argument("--config", default="r50", choices=["r50", "arcface", "resnext", "r101", "tresnet"],
                    help="BASELINE.json config: r50 (headline), arcface (R50+ArcFace 10k cls @112), "
                         "resnext (ResNeXt-50 32x4d), r101 (ResNet-101 large batch), tresnet (BASELINE default)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch")
    ap.add_argument("--model", default=None)
    ap.add_argument("--image-size", type=int, default=None)
    ap.add_argument("--num-classes", type=int, default=None)
    ap.add_argument("--syncbn", action="store_true",
                    help="headline phase with cross-replica BN (reference default); off = local BN")
    ap.add_argument("--no-syncbn-phase", dest="syncbn_phase", action="store_false",
                    help="N > 1: skip the second, SyncBN-timed phase")
    ap.add_argument("--no-syncbn-peer", dest="syncbn_peer", action="store_false",
                    help="N > 1: skip the third phase, SyncBN over the peer-memory mailboxes (parallel/peer.py)")
    ap.add_argument("--syncbn-shared-group", action="store_true",
                    help="SyncBN collectives on the gradient communicator instead of their own "
                         "(DCP_SYNCBN_SHARED_GROUP=1; parallel/ddp.py bn_process_group)")
    ap.add_argument("--bucket-cap-mb", type=float, default=25.0)
    ap.add_argument("--grad-comm", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce precision (bf16: half the xGMI bytes; bucket engine: bf16 buckets, "
                         "torch engine: bf16_compress_hook)")
    ap.add_argument("--ddp-engine", default="dcp", choices=["dcp", "torch"],
                    help="dcp: this framework's bucket engine (optimizer fused per bucket, HIP-graph capturable); "
                         "torch: DistributedDataParallel's C++ Reducer")
    ap.add_argument("--force-ddp", action="store_true",
                    help="1 GPU: still run the data-parallel path -- a world-size-1 RCCL process group, the DDP "
                         "engine, the SyncBN phase and telemetry (measures the engine's own cost and its HIP-graph "
                         "capture on one box)")
    ap.add_argument("--telemetry-steps", type=int, default=5,
                    help="N > 1, dcp engine: untimed steps after the timed phase that record per-bucket HIP events "
                         "(exposed communication per rank)")
    ap.add_argument("--no-comm-probe", dest="comm_probe", action="store_false",
                    help="distributed runs: skip the untimed collective probe after the timed phases (RCCL "
                         "all-reduce bus bandwidth per bucket size; SyncBN-sized all-gather / all-reduce latency)")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--profile-dir", default=None, help="write a torch.profiler trace here")
    ap.add_argument("--graph", dest="graph", action="store_true", default=None,
                    help="capture the whole step in a HIP graph and replay it (default on one GPU: +0.5 %% at the "
                         "headline batch, profiles/r4/graph1024_ab.txt; more at small batches)")
    ap.add_argument("--eager", dest="graph", action="store_false",
                    help="launch the step eagerly (the default with several ranks: a captured side-stream bucket "
                         "fork / join costs more than replay saves at batch 1024)")
    ap.add_argument("--no-autotune", dest="autotune", action="store_false",
                    help="fixed heuristic conv configurations instead of the per-shape timing on the warm-up "
                         "steps (the reference's cudnn.benchmark=True, BASELINE/main.py:40)")
    return ap.parse_args(argv)


CONFIGS = {
    # per-GPU batches sized for 288 GB of HBM (the larger grids amortise per-kernel latency and
    # the per-step optimizer / weight refresh).  r50 (the headline), round 6, same box
    # (profiles/r6/batch_sweep_s51_s52.txt): 1024 / 1536 / 2048 / 3072 / 4096: 14.63k / 14.91k /
    # 15.05k / 15.34k / 15.41k img/s (39 / 59 / 78 / 117 / 156 GB); r101 (BASELINE config 5, "large
    # per-GPU batch") 1024 / 3072: 9.05k / 9.66k (59 / 177 GB); arcface 1024 / 2048 / 4096: 47.7k /
    # 53.2k / 56.8k (10 / 20 / 40 GB), 8192 / 16384: 58.8k / 59.6k (80 / 159 GB, s61); resnext 1024 / 2048 / 3072: 11.48k / 11.81k / 11.81k (53 / 106 /
    # 158 GB); tresnet 1024 / 2048 / 4096: 13.59k / 14.17k / 14.49k (26 / 51 / 101 GB), 8192: +0.8 %
    # (profiles/r6/config_batch_sweep_s57.txt).  Round 2
    # (profiles/meas_r2/batch_sweep.txt):
    # r50 512 / 1024 / 2048: 11.9k / 12.7k / 13.0k img/s (43 GB at 1024); arcface 256 / 512 / 1024:
    # 26.6k / 36.6k / 43.9k (11 GB); resnext 128 / 256 / 512 / 1024: 7.5k / 8.7k / 9.5k / 9.9k (56 GB);
    # r101 512 / 1024 / 1536: 7.7k / 8.4k / 8.6k (64 GB); tresnet 256 / 512 / 1024: 9.4k / 10.9k / 11.7k
    "r50": dict(model="resnet50", batch=4096, image_size=224, num_classes=1000),
    "arcface": dict(model="resnet50", batch=8192, image_size=112, num_classes=10000),
    "resnext": dict(model="resnext50_32x4d", batch=2048, image_size=224, num_classes=1000),
    "r101": dict(model="resnet101", batch=3072, image_size=224, num_classes=1000),
    "tresnet": dict(model="tresnet_m", batch=4096, image_size=224, num_classes=1000),
}
METRICS = {
    "r50": "images/sec (whole node), ResNet-50 224px DDP at 1/2/4/8 MI355X",
    "arcface": "images/sec (whole node), ResNet-50 + ArcFace head, 10k-class 112px, DDP",
    "resnext": "images/sec (whole node), ResNeXt-50 32x4d 224px, DDP",
    "r101": "images/sec (whole node), ResNet-101 224px large per-GPU batch, DDP",
    "tresnet": "images/sec (whole node), TResNet-M 224px, DDP",
}


def build_bench_model(a):
    if a.config == "arcface":
        from ddp_classification_pytorch_amd.algos.arcface import ArcFaceModel
        from ddp_classification_pytorch_amd.models.heads import ArcMarginProduct, MLPHead

        bb = build_model(a.model, num_classes=0)
        return ArcFaceModel(bb, MLPHead(bb.feat_dim, 512, 256, log_softmax=True),
                            ArcMarginProduct(256, a.num_classes, s=30.0, m=0.5, easy_margin=True))
    return build_model(a.model, num_classes=a.num_classes)


def rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n, argv):
    """Run this script as N torchrun ranks in a child process and return its exit code.  Called
    before any GPU work in this process (the parent never initialises HIP, and never execs)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def comm_probe(dev, world, bn_group, reps=5):
    """Untimed microbenchmark of the collectives this step issues, on the job's own communicators
    (SURVEY.md §5.8 items 1, 4, 6): all-reduce bus bandwidth at gradient-bucket sizes (ring
    convention 2 (n-1)/n x bytes / time) and the latency of SyncBN-sized all-gathers (forward
    statistics, 3 x 2048 floats per rank) and all-reduces (backward sums, 2 x 2048 floats) on the
    dedicated BN communicator.  The per-bucket numbers say where bucket size stops paying on xGMI."""
    out = {"allreduce_busbw_gbs": {}, "allreduce_ms": {}, "world": world}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, n):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        ev0.record()
        for _ in range(n):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / n * 1e-3  # s per call

    for mb in (4, 25, 100):
        t = torch.empty(mb * 2**20 // 4, dtype=torch.float32, device=dev)
        sec = timed(lambda: dist.all_reduce(t), reps)
        out["allreduce_ms"][f"{mb}MB"] = round(sec * 1e3, 4)
        out["allreduce_busbw_gbs"][f"{mb}MB"] = round(2.0 * (world - 1) / max(world, 1) * t.numel() * 4 / sec / 1e9, 1)
        del t
    st = torch.empty(3 * 2048, dtype=torch.float32, device=dev)
    gathered = torch.empty(world * st.numel(), dtype=torch.float32, device=dev)
    out["syncbn_allgather_us"] = round(timed(lambda: dist.all_gather_into_tensor(gathered, st, group=bn_group), 20) * 1e6, 1)
    sums = torch.empty(2 * 2048, dtype=torch.float32, device=dev)
    out["syncbn_allreduce_us"] = round(timed(lambda: dist.all_reduce(sums, group=bn_group), 20) * 1e6, 1)
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(self_launch(a.gpus, argv))
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus is not None and a.gpus != world:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks")
    # one rank per GPU over RCCL ("nccl" on ROCm).  DCP_DIST_BACKEND=gloo lets tests run
    # several ranks on one GPU (RCCL refuses duplicate devices).
    backend = os.environ.get("DCP_DIST_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    dist_on = world > 1 or a.force_ddp
    if a.syncbn_shared_group:
        os.environ["DCP_SYNCBN_SHARED_GROUP"] = "1"
    if a.graph is None:  # default: HIP-graph replay on one GPU without a process group, eager otherwise
        a.graph = not dist_on
    if dist_on:
        if a.graph:
            pddp.graph_safe_nccl_env()
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        # an explicit timeout: a rank that never arrives fails the job with a message in minutes
        # instead of running into the driver's limit (DCP_PG_TIMEOUT seconds, default 300)
        pg_timeout = datetime.timedelta(seconds=float(os.environ.get("DCP_PG_TIMEOUT", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)
        else:
            dist.init_process_group(backend, timeout=pg_timeout)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    kops = _ext.hip_ops()  # fail loudly if the gfx950 library is missing
    # per-shape conv configuration autotuning on the (untimed) warm-up steps, as the reference's
    # torch.backends.cudnn.benchmark = True (BASELINE/main.py:40); DCP_AUTOTUNE=0 / --no-autotune off
    autotune = a.autotune and os.environ.get("DCP_AUTOTUNE", "1") != "0"
    kops.set_tuning(tuning.slot("autotune"), 1 if autotune else 0)
    # A/B experiments only: DCP_TUNE="name=value,..." sets kernel-config overrides (csrc/tune.h)
    tuning.apply(kops, os.environ.get("DCP_TUNE", ""))

    torch.manual_seed(1234 + rank)
    model = build_bench_model(a).to(dev)
    if dist_on:
        model = pddp.wrap_ddp(model, local, syncbn=a.syncbn, bucket_cap_mb=a.bucket_cap_mb, engine=a.ddp_engine,
                              force=a.force_ddp,
                              comm_dtype=torch.bfloat16 if a.grad_comm == "bf16" else torch.float32)
        # created collectively now (every rank, same order) so the SyncBN phase can switch to it
        bn_group = pddp.bn_process_group()
        if a.grad_comm == "bf16" and a.ddp_engine == "torch":
            from torch.distributed.algorithms.ddp_comm_hooks import default_hooks

            model.register_comm_hook(None, default_hooks.bf16_compress_hook)
    opt = FusedSGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)
    # bucket engine: the SGD kernel runs per gradient bucket right behind its all-reduce (its
    # step() after backward is then a no-op); torch DDP / one GPU: one launch after backward
    pddp.attach_optimizer(model, opt)

    B, S = a.batch, a.image_size
    g = torch.Generator(device=dev)
    g.manual_seed(rank)
    images = torch.randint(0, 256, (B, 3, S, S), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, a.num_classes, (B,), device=dev, generator=g)
    mean = torch.tensor(IMAGENET_MEAN, device=dev)
    std = torch.tensor(IMAGENET_STD, device=dev)

    layout = input_layout(model)  # e.g. ResNets: 2x2 space-to-depth input of the s2d stem

    def step():
        x = Fn.to_device_nhwc(images, mean, std, nchw=True, in_scale=1.0 / 255.0, **layout)
        if a.config == "arcface":
            loss, _ = model(x, labels)
        else:
            loss = Fn.cross_entropy(model(x), labels)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    run = step
    graphed = None
    if a.graph:
        if dist_on and a.ddp_engine != "dcp":
            raise SystemExit("--graph with N > 1 needs the bucket engine (torch DDP's reducer is not capturable)")
        from ddp_classification_pytorch_amd.engine.graph import GraphedStep

        graphed = GraphedStep(step, warmup=max(1, a.warmup), distributed=dist_on)  # warm-up steps run inside
        run = graphed
    else:
        for _ in range(a.warmup):
            loss = step()

    def timed(n_steps):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_steps):
            out = run()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, out

    def gather_max(dt):
        """(max over ranks, every rank's seconds)"""
        if world == 1:
            return dt, [dt]
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        per = [float(v.item()) for v in allt]
        return max(per), per

    prof = None
    if a.profile_dir and rank == 0:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    dt, loss = timed(a.steps)
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(a.profile_dir, exist_ok=True)
        with open(os.path.join(a.profile_dir, "bench_profile.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    dt, per_rank = gather_max(dt)
    loss_v = float(loss.item())
    ms = dt / a.steps * 1000.0
    ips = B * world * a.steps / dt
    out = {
        "metric": METRICS[a.config],
        "value": round(ips, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,  # the reference publishes no throughput
        "dtype": "bf16",
        "data": "synthetic (uint8 ImageNet-shaped images generated on device, random labels; random-init weights)",
        "dist_backend": (dist.get_backend() if dist_on else None),
        "world_size": (dist.get_world_size() if dist_on else 1),
        "rccl_version": rccl_version(),
        "per_rank_ms": [round(v / a.steps * 1000.0, 3) for v in per_rank],
        "syncbn_value": None,
        "syncbn_ms_per_step": None,
        "syncbn_peer_value": None,
        "syncbn_peer_ms_per_step": None,
        "comm": None,
        "comm_probe": None,
        "config": {
            "model": a.model,
            "global_batch": B * world,
            "per_gpu_batch": B,
            "seq_len": None,
            "image_size": S,
            "num_classes": a.num_classes,
            "parallelism": f"dp{world}",
            "hip_graph": bool(a.graph),
            "autotune": bool(autotune),
            "syncbn": bool(a.syncbn),
            "grad_comm": a.grad_comm,
            "ddp_engine": a.ddp_engine if dist_on else None,
            "force_ddp": bool(a.force_ddp),
            "bucket_cap_mb": a.bucket_cap_mb,
            "optimizer": "fused SGD momentum 0.9 wd 1e-4",
            "final_loss": round(loss_v, 4),
            "max_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1),
        },
    }
    # The headline is measured.  What follows (bucket telemetry, the SyncBN phase, the collective
    # probe) is diagnostic and must never cost the line: each phase is guarded, and a deadline
    # watchdog prints the line and ends the rank if a phase hangs (e.g. one rank failed inside a
    # collective sequence the others are still in).
    emitted = threading.Event()

    def emit():
        if rank == 0 and not emitted.is_set():
            emitted.set()
            print(json.dumps(out), flush=True)

    errors = {}

    def watchdog():
        errors["deadline"] = f"diagnostic phases exceeded {extra_deadline:.0f} s; headline kept"
        out["diagnostic_errors"] = dict(errors)
        emit()
        sys.stdout.flush()
        sys.stderr.write(f"bench.py rank {rank}: {errors['deadline']}\n")
        sys.stderr.flush()
        os._exit(0)

    extra_deadline = float(os.environ.get("DCP_BENCH_EXTRA_DEADLINE", "240"))
    timer = threading.Timer(extra_deadline, watchdog) if dist_on else None
    if timer is not None:
        timer.daemon = True
        timer.start()
    inject = os.environ.get("DCP_BENCH_INJECT", "")  # tests: "phase" or "phase:rank" raises in that phase
    inject_rank = int(inject.split(":")[1]) if ":" in inject else None

    def guarded(name, fn):
        """Run one diagnostic phase; an exception is recorded in the line instead of ending the run.
        Afterwards the ranks agree (one all-reduce) whether any of them failed, so they all skip the
        remaining phases together instead of entering mismatched collectives."""
        ok = 1.0
        try:
            if inject.split(":")[0] == name and inject_rank in (None, rank):
                raise RuntimeError(f"injected failure in the {name} phase (DCP_BENCH_INJECT)")
            fn()
        except Exception as e:  # noqa: BLE001
            errors[name] = f"{type(e).__name__}: {e}"[:300]
            ok = 0.0
        if world > 1:
            flag = torch.tensor([ok], device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = float(flag.item())
        return ok > 0

    def telemetry_phase():
        # untimed: per-step HIP events around the bucket engine (backward end on the compute stream,
        # first bucket start / last bucket done on the communication stream), eager steps
        red = model.reducer
        red.telemetry = True
        for _ in range(a.telemetry_steps):
            step()
        red.telemetry = False
        summ = red.telemetry_summary() or {}
        t = torch.tensor([summ.get("exposed_comm_ms", 0.0), summ.get("comm_span_ms", 0.0)], device=dev,
                         dtype=torch.float64)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        out["comm"] = {"engine": "dcp", "buckets": summ.get("buckets"), "bucket_mb": summ.get("bucket_mb"),
                       "optimizer_per_bucket": True, "telemetry_steps": summ.get("steps"),
                       "exposed_comm_ms_per_rank": [round(float(v[0]), 4) for v in allt],
                       "comm_span_ms_per_rank": [round(float(v[1]), 4) for v in allt],
                       "grad_comm": a.grad_comm}

    def syncbn_phase():
        nonlocal run, graphed
        # second phase: the reference's SyncBN (BASELINE/main.py:148) on the dedicated BN communicator
        pddp.convert_sync_batchnorm(pddp.unwrap(model), bn_group)
        if a.graph:  # recapture: the BN collectives (on the BN communicator) go into the new graph
            from ddp_classification_pytorch_amd.engine.graph import GraphedStep

            run = graphed = None
            torch.cuda.empty_cache()
            run = GraphedStep(step, warmup=2, distributed=True)
        for _ in range(2):
            run()
        sdt, _ = timed(a.steps)
        sdt, sper = gather_max(sdt)
        out["syncbn_value"] = round(B * world * a.steps / sdt, 2)
        out["syncbn_ms_per_step"] = round(sdt / a.steps * 1000.0, 3)
        out["syncbn_per_rank_ms"] = [round(v / a.steps * 1000.0, 3) for v in sper]

    def bn_stats_forward(transport):
        """One no-grad training-mode forward with the SyncBN statistics exchanged over ``transport``:
        the statistics every BN layer merged (its running-stat update), BN state restored after."""
        from ddp_classification_pytorch_amd.models.layers import BatchNorm2d

        net = pddp.unwrap(model)
        pddp.convert_sync_batchnorm(net, bn_group, transport=transport)
        bns = [m for m in net.modules() if isinstance(m, BatchNorm2d)]
        saved = [(m.running_mean.clone(), m.running_var.clone(), m._nbt_pending) for m in bns]
        x = Fn.to_device_nhwc(images, mean, std, nchw=True, in_scale=1.0 / 255.0, **layout)
        with torch.no_grad():
            net(x, labels) if a.config == "arcface" else net(x)
        got = [(m.running_mean.clone(), m.running_var.clone()) for m in bns]
        for m, (rm, rv, nbt) in zip(bns, saved):
            m.running_mean.copy_(rm)
            m.running_var.copy_(rv)
            m._nbt_pending = nbt
        return got

    def peer_crosscheck(ex):
        """The peer transport against RCCL on the same inputs: the collectives themselves
        (a SyncBN-sized gather must be bitwise equal; the sums agree to fp32 summation order) and the
        BN statistics of one forward of the model.  Worst relative difference over all of them."""
        gen = torch.Generator(device=dev)
        gen.manual_seed(77 + rank)
        st = torch.randn(3 * 2048, device=dev, generator=gen)
        ref = torch.empty(world * st.numel(), device=dev)
        dist.all_gather_into_tensor(ref, st, group=bn_group)
        got = torch.empty_like(ref)
        ex.all_gather_into_tensor(got, st)
        red_ref = st.clone()
        dist.all_reduce(red_ref, group=bn_group)
        red_got = st.clone()
        ex.all_reduce(red_got)
        ex.check()

        def rel(u, v):
            return float(((u - v).abs().max() / v.abs().max().clamp_min(1e-30)).item())

        diffs = {"gather": rel(got, ref), "reduce": rel(red_got, red_ref)}
        a_st, b_st = bn_stats_forward("rccl"), bn_stats_forward("peer")
        ex.check()
        diffs["bn_stats"] = max(max(rel(p[0], q[0]), rel(p[1], q[1])) for p, q in zip(b_st, a_st))
        t = torch.tensor([max(diffs.values())], device=dev, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out["syncbn_peer_max_rel_diff"] = float(t.item())
        out["syncbn_peer_rel_diff_parts"] = {k: float(v) for k, v in diffs.items()}

    def syncbn_peer_phase():
        nonlocal run, graphed
        # third phase: the same SyncBN with its statistics exchanged through the IPC-mapped peer
        # mailboxes (parallel/peer.py: one kernel per exchange instead of an RCCL collective)
        from ddp_classification_pytorch_amd.parallel import peer

        pddp.convert_sync_batchnorm(pddp.unwrap(model), bn_group, transport="peer")
        ex = peer.exchange_for(bn_group)
        if ex is None:
            raise RuntimeError("peer mailboxes unavailable (no peer access): stayed on RCCL")
        peer_crosscheck(ex)  # leaves the peer transport on
        if a.graph:
            from ddp_classification_pytorch_amd.engine.graph import GraphedStep

            run = graphed = None
            torch.cuda.empty_cache()
            run = GraphedStep(step, warmup=2, distributed=True)
        for _ in range(2):
            run()
        sdt, _ = timed(a.steps)
        sdt, sper = gather_max(sdt)
        ex.check()
        out["syncbn_peer_value"] = round(B * world * a.steps / sdt, 2)
        out["syncbn_peer_ms_per_step"] = round(sdt / a.steps * 1000.0, 3)
        pddp.convert_sync_batchnorm(pddp.unwrap(model), bn_group, transport="rccl")

    def probe_phase():
        out["comm_probe"] = comm_probe(dev, world, bn_group)

    go = True
    if dist_on and a.ddp_engine == "dcp" and a.telemetry_steps > 0:
        go = guarded("telemetry", telemetry_phase)
    elif dist_on:
        out["comm"] = {"engine": a.ddp_engine, "bucket_mb": [round(v, 2) for v in pddp.bucket_layout_mb(model)]}
    if go and dist_on and not a.syncbn and a.syncbn_phase:
        go = guarded("syncbn", syncbn_phase)
        if go and a.syncbn_peer:
            go = guarded("syncbn_peer", syncbn_peer_phase)
    if go and dist_on and a.comm_probe and dist.get_backend() == "nccl":
        go = guarded("probe", probe_phase)
    if timer is not None:
        timer.cancel()
    if errors:
        out["diagnostic_errors"] = errors
    emit()
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
