"""Per-step losses of the eager step vs StepGrapher over a sequence of distinct batches."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd.engine.graph import StepGrapher  # noqa: E402
from ddp_classification_pytorch_amd.models import build_model, input_layout  # noqa: E402
from ddp_classification_pytorch_amd.ops import functional as Fn  # noqa: E402
from ddp_classification_pytorch_amd.optim import FusedSGD  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
base = build_model("resnet18", num_classes=10).to(dev)
g = torch.Generator().manual_seed(1)
batches = []
for i in range(7):
    B = 16 if i < 6 else 8
    imgs = torch.randint(0, 256, (B, 3, 32, 32), dtype=torch.uint8, generator=g)
    batches.append((imgs, torch.randint(0, 10, (B,), generator=g)))


def make(model):
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9)
    lay = input_layout(model)

    def step(x, y):
        loss = Fn.cross_entropy(model(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    return step, lay


for mode in ("eager", "graph"):
    m = copy.deepcopy(base)
    step, lay = make(m)
    run = StepGrapher(step, warmup=2) if mode == "graph" else step
    out = []
    for imgs, y in batches:
        x = Fn.to_device_nhwc(imgs.to(dev), torch.tensor((0.5, 0.5, 0.5), device=dev),
                              torch.tensor((0.25, 0.25, 0.25), device=dev), nchw=True, in_scale=1 / 255.0, **lay)
        out.append(float(run(x, y.to(dev)).item()))
    print(mode, " ".join(f"{v:.5f}" for v in out), flush=True)
