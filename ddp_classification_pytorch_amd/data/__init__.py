from .datasets import (CappedImageFolder, ImageFolder, ListDataset, SyntheticImages, make_fake_image_folder,
                       write_label_files)
from .loader import DevicePrefetcher, SyntheticLoader, build_loader, collate_uint8
from .sampler import ShardSampler
from .shards import ShardDataset, ShardLoader, aug_preset, pack_image_folder, write_shard
from .transforms import build_transform, norm_stats

__all__ = ["CappedImageFolder", "ImageFolder", "ListDataset", "SyntheticImages", "make_fake_image_folder",
           "write_label_files", "DevicePrefetcher", "SyntheticLoader", "build_loader", "collate_uint8",
           "ShardSampler", "build_transform", "norm_stats", "ShardDataset", "ShardLoader", "aug_preset",
           "pack_image_folder", "write_shard"]
