"""main.py eager / eager / --graph in one process: checksum of the final weights of each run."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import main as entry  # noqa: E402

common = ["--workload", "baseline", "--model", "resnet18", "--data", "synthetic", "--dataset", "CIFAR10",
          "--batchsize", "16", "--synthetic-train-size", "120", "--synthetic-val-size", "32", "--epochs",
          sys.argv[1] if len(sys.argv) > 1 else "2", "--workers", "0", "--log-interval", "1", "--num-classes", "10",
          "--optimizer", "SGD", "--lr", "0.05"]
d = tempfile.mkdtemp()
for tag, extra in (("eager1", []), ("eager2", []), ("graph", ["--graph"])):
    torch.manual_seed(0)
    entry.main(common + ["--out-dir", os.path.join(d, tag)] + extra)
    sd = torch.load(os.path.join(d, tag, "last.pth"), weights_only=True)["models"]["model"]
    print(tag, "conv1", float(sd["backbone.conv1.weight"].double().abs().sum()), flush=True)
