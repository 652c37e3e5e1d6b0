"""Direct 64->64 3x3 kernel: the register-direct store epilogue (g_tune[30] = 0, default) against the
LDS-staged one (g_tune[30] = 2) -- differing output elements and BN-statistics difference per shape.

    python tools/conv3x3_epilogue_check.py   (on the GPU)
"""
import torch, sys, os
sys.path.insert(0, os.getcwd())
from ddp_classification_pytorch_amd import _ext
from ddp_classification_pytorch_amd.tuning import slot as tslot
K = _ext.hip_ops()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
for (N, H, W) in [(16, 16, 16), (2, 56, 56), (3, 7, 9), (64, 56, 56)]:
    x = (torch.randn(N, H, W, 64, device=dev) * 2).abs().bfloat16()
    w = (torch.randn(64, 3, 3, 64, device=dev) / 24).bfloat16()
    K.set_tuning(tslot("c3_epilogue"), 2); y0, p0 = K.conv_fwd(x, w, 1, 1, True)
    K.set_tuning(tslot("c3_epilogue"), 0); y1, p1 = K.conv_fwd(x, w, 1, 1, True)
    K.set_tuning(tslot("c3_epilogue"), 0)
    d = (y0.float() - y1.float()).abs()
    s0, s1 = K.bn_stats(y0, p0), K.bn_stats(y1, p1)
    print(N, H, W, "ndiff", int((d > 0).sum()), "of", d.numel(), "maxdiff", float(d.max()), "max|y|", float(y0.float().abs().max()),
          "stats diff", float((s0 - s1).abs().max()), flush=True)
