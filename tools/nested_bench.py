#!/usr/bin/env python3
"""TestNested evaluation kernels (K19) on the reference's shape: val batch 128 x 2048 features x
2173 classes (NESTED/train.py:103-166): the rank-ballot fast path vs the one-workgroup-per-sample
scalar kernel, counts compared for equality.

    python tools/nested_bench.py [--batch 128] [--dim 2048] [--classes 2173]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd import _ext  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--classes", type=int, default=2173)
    a = ap.parse_args()
    K = _ext.hip_ops()
    torch.manual_seed(0)
    f = torch.relu(torch.randn(a.batch, a.dim, device="cuda"))
    W = torch.randn(a.dim, a.classes, device="cuda") * 0.05
    lab = torch.randint(0, a.classes, (a.batch,), device="cuda")
    fast = K.nested_eval(f, W, lab)
    slow = K.nested_eval_scalar(f, W, lab)
    t_fast = timeit(lambda: K.nested_eval(f, W, lab))
    t_slow = timeit(lambda: K.nested_eval_scalar(f, W, lab), 3)
    print(f"nested_eval B={a.batch} D={a.dim} C={a.classes}: fast {t_fast:.1f} us, scalar {t_slow:.1f} us "
          f"({t_slow / t_fast:.1f}x), counts identical: {bool(torch.equal(fast, slow))}")


if __name__ == "__main__":
    main()
