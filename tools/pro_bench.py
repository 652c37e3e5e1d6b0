"""BN-prologue (K5) A/B per ResNet-50 bottleneck conv3 shape: the separate BN-apply pass + the
plain 1x1 conv / weight gradient against the prologue kernels (conv_fwd_pro / conv_wgrad_pro).

    python tools/pro_bench.py --batch 1024
"""
import argparse
import math

import torch

from ddp_classification_pytorch_amd import _ext

SHAPES = [  # (H, C = width, Co = 4 * planes, blocks)
    (56, 64, 256, 3), (28, 128, 512, 4), (14, 256, 1024, 6), (7, 512, 2048, 3)]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    K = _ext.hip_ops()
    dev = torch.device("cuda")
    tot = [0.0] * 6
    print(f"{'shape':24s} {'bn_act':>8s} {'fwd':>8s} {'fwd_pro':>8s} | {'wgrad':>8s} {'wg_pro':>8s}   (us)")
    for H, C, Co, nb in SHAPES:
        N = a.batch
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(Co, 1, 1, C, device=dev) / math.sqrt(C)).bfloat16()
        dy = torch.randn(N, H, H, Co, device=dev).bfloat16()
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev) * 0.5
        act = K.bn_act(x, None, sc, sh, 1, 0.0)
        t_bn = timeit(lambda: K.bn_act(x, None, sc, sh, 1, 0.0), a.iters)
        t_f = timeit(lambda: K.conv_fwd(act, w, 1, 0, True), a.iters)
        t_fp = timeit(lambda: K.conv_fwd_pro(x, w, sc, sh, True), a.iters)
        t_w = timeit(lambda: K.conv_wgrad(dy, act, 1, 1, 1, 0), a.iters)
        t_wp = timeit(lambda: K.conv_wgrad_pro(dy, x, sc, sh), a.iters)
        print(f"{N}x{H}x{H}x{C}->{Co} x{nb}".ljust(24),
              f"{t_bn:8.1f} {t_f:8.1f} {t_fp:8.1f} | {t_w:8.1f} {t_wp:8.1f}", flush=True)
        for i, v in enumerate((t_bn, t_f, t_fp, t_w, t_wp)):
            tot[i] += v * nb
        del x, dy, act
    print(f"per-step totals (ms): separate = bn {tot[0] / 1e3:.2f} + fwd {tot[1] / 1e3:.2f} + wgrad {tot[3] / 1e3:.2f} = "
          f"{(tot[0] + tot[1] + tot[3]) / 1e3:.2f};  prologue = fwd {tot[2] / 1e3:.2f} + wgrad {tot[4] / 1e3:.2f} = "
          f"{(tot[2] + tot[4]) / 1e3:.2f}")


if __name__ == "__main__":
    main()
