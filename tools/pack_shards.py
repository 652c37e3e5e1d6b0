"""Pack an image-folder tree (``<folder>/{train,test}/<class>/*.jpg``, the reference layout of
BASELINE/main.py:81-83,97-121) or a Clothing1M list dataset into the native loader's shard files
``<out>/train.dcps`` and ``<out>/test.dcps`` (decode once; see data/shards.py).

    python tools/pack_shards.py --folder /data/food --out /data/food --short-side 256 --workers 8
    python main.py --workload baseline --data shards --folder /data/food ...
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_classification_pytorch_amd.data.datasets import CappedImageFolder, ListDataset  # noqa: E402
from ddp_classification_pytorch_amd.data.shards import pack_image_folder  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--folder", required=True)
    ap.add_argument("--out", default=None, help="output directory (default: --folder)")
    ap.add_argument("--list", action="store_true", help="Clothing1M annotation-list layout (PLC/FolderDataset.py)")
    ap.add_argument("--imgs-limited", type=int, default=None, help="per-class cap (reference: 500 / 400)")
    ap.add_argument("--num-class-dirs", type=int, default=None)
    ap.add_argument("--short-side", type=int, default=256)
    ap.add_argument("--workers", type=int, default=4)
    a = ap.parse_args(argv)
    out = a.out or a.folder
    os.makedirs(out, exist_ok=True)
    for split, sub in (("train", "train"), ("test", "test" if not a.list else "val")):
        if a.list:
            ds = ListDataset(a.folder, sub, resize=0)
        else:
            ds = CappedImageFolder(os.path.join(a.folder, sub), None, a.imgs_limited, a.num_class_dirs)
        t0 = time.time()
        n = pack_image_folder(ds, os.path.join(out, f"{split}.dcps"), a.short_side, a.workers)
        print(f"{split}: {n} images -> {os.path.join(out, split + '.dcps')} in {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
