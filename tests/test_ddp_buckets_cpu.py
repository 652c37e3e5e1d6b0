"""DDP gradient-bucket layout for ResNet-50 under the framework defaults.

Builds the real DistributedDataParallel module through ``wrap_ddp`` (1-rank
gloo), runs three forward/backward passes so the Reducer rebuilds its buckets
in gradient-ready order, and reads the sizes the Reducer reports.  This pins
the overlap argument in parallel/ddp.py: a small first bucket (the fc weight)
and only a small tail bucket (layer1 + stem side) left for after the stem's
weight gradient.  torch ignores the first-bucket limit when the cap is passed
explicitly; the second test shows that layout is worse.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from ddp_classification_pytorch_amd.models import build_model
from ddp_classification_pytorch_amd.parallel import ddp as pddp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def gloo1():
    if dist.is_initialized():
        yield
        return
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def _layout(ddp):
    torch.manual_seed(0)
    x = torch.randn(2, 32, 32, 8)
    for _ in range(3):  # buckets are rebuilt in grad-ready order before the 3rd forward
        ddp(x).float().sum().backward()
    data = ddp._get_ddp_logging_data()
    assert data.get("has_rebuilt_buckets") == 1
    return [int(v) / 2**20 for v in str(data["rebuilt_bucket_sizes"]).split(",")]


def test_resnet50_bucket_layout_leaves_small_tail(gloo1):
    ddp = pddp.wrap_ddp(build_model("resnet50", num_classes=1000), force=True, engine="torch")
    sizes = _layout(ddp)
    assert abs(sum(sizes) - 97.49) < 0.05
    assert len(sizes) == 5
    assert sizes[0] < 8.0          # fc weight + bias alone: the first all-reduce starts right after the head
    assert sizes[-1] < 0.1 * sum(sizes)  # the only bucket that cannot overlap backward
    assert pddp.bucket_layout_mb(ddp) == pytest.approx(sizes)


def test_explicit_cap_has_no_small_first_bucket(gloo1):
    """What the constructor does with an explicit 25 MiB cap: no first-bucket limit, larger tail."""
    m = build_model("resnet50", num_classes=1000)
    ddp = torch.nn.parallel.DistributedDataParallel(m, bucket_cap_mb=25, broadcast_buffers=False,
                                                    gradient_as_bucket_view=True)
    sizes = _layout(ddp)
    assert sizes[0] > 20.0 and sizes[-1] > 0.15 * sum(sizes)


def test_bucket_engine_layout_follows_gradient_order(gloo1):
    """The bucket engine (parallel/reducer.py) rebuilds its buckets after the first backward in
    gradient-ready order: the head's gradients form the first (small) bucket, 25 MiB buckets
    follow, and the tail that can only start after the stem's weight gradient stays small."""
    net = pddp.wrap_ddp(build_model("resnet50", num_classes=1000), force=True, engine="dcp")
    torch.manual_seed(0)
    x = torch.randn(2, 32, 32, 8)
    net(x).float().sum().backward()
    sizes = pddp.bucket_layout_mb(net)
    assert abs(sum(sizes) - 97.49) < 0.1
    assert sizes[0] < 8.5 and all(s < 32 for s in sizes)
    assert sizes[-1] < 0.15 * sum(sizes)
    first = net.reducer.buckets[0].params
    assert any(p is net.module.fc.weight for p in first)
