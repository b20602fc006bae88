"""Input-pipeline throughput: images/s through the reference's loader API,
get_train_loader(engine, RGBXDataset, config) (dataloader/dataloader.py:129-165), on a synthetic
NYUv2-shape PNG tree (480 x 640 RGB, one-channel depth, labels in [1, 40] with gt_transform),
with the reference's NYU TrainPre settings (scales 0.5..1.75, 480 x 640 crop) on the GPU.

Usage (GPU box): python scripts/bench_loader.py [--images 64] [--batch 2] [--workers 8] [--iters 40]
Prints one JSON line: images/s end to end (PNG decode in workers + upload + device TrainPre),
and the device-only TrainPre rate on pre-decoded samples."""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MEAN = [0.485, 0.456, 0.406]
STD = [0.229, 0.224, 0.225]
SCALES = [0.5, 0.75, 1, 1.25, 1.5, 1.75]


def make_tree(root: str, n: int, H: int, W: int) -> None:
    from PIL import Image
    rng = np.random.default_rng(0)
    for d in ("RGB", "Depth", "Label"):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    for i in range(n):
        # smooth-ish content so PNG compression resembles real photos more than white noise
        base = rng.integers(0, 256, (H // 8, W // 8, 3), dtype=np.uint8)
        rgb = np.kron(base, np.ones((8, 8, 1), dtype=np.uint8)) + rng.integers(0, 16, (H, W, 3), dtype=np.uint8)
        Image.fromarray(rgb).save(os.path.join(root, "RGB", f"{i}.png"))
        Image.fromarray(rgb[:, :, 0]).save(os.path.join(root, "Depth", f"{i}.png"))
        lab = np.kron(rng.integers(1, 41, (H // 16, W // 16), dtype=np.uint8), np.ones((16, 16), dtype=np.uint8))
        Image.fromarray(lab).save(os.path.join(root, "Label", f"{i}.png"))
    with open(os.path.join(root, "train.txt"), "w") as f:
        f.write("".join(f"{i}\n" for i in range(n)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images", type=int, default=64)
    p.add_argument("--batch", type=int, default=2)
    p.add_argument("--workers", type=int, default=8)
    p.add_argument("--iters", type=int, default=40)
    args = p.parse_args()
    from types import SimpleNamespace
    from rgbx_semantic_segmentation_amd.dataloader import RGBXDataset, get_train_loader
    H, W = 480, 640
    with tempfile.TemporaryDirectory() as root:
        make_tree(root, args.images, H, W)
        cfg = SimpleNamespace(rgb_root_folder=f"{root}/RGB", rgb_format=".png", gt_root_folder=f"{root}/Label",
                              gt_format=".png", gt_transform=True, x_root_folder=f"{root}/Depth", x_format=".png",
                              x_is_single_channel=True, train_source=f"{root}/train.txt",
                              eval_source=f"{root}/train.txt", background=255, num_classes=40, image_height=H,
                              image_width=W, norm_mean=MEAN, norm_std=STD, train_scale_array=SCALES,
                              batch_size=args.batch, niters_per_epoch=args.iters + 5, num_workers=args.workers)
        engine = SimpleNamespace(distributed=False, world_size=1)
        torch.manual_seed(0)
        loader, _ = get_train_loader(engine, RGBXDataset, cfg)
        it = iter(loader)
        for _ in range(5):                      # worker start-up, first PNG decodes
            next(it)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            mb = next(it)
        torch.cuda.synchronize()
        e2e = args.iters * args.batch / (time.perf_counter() - t0)
        # the device TrainPre alone on pre-decoded uint8 samples (pinned), same draws
        pre = loader.pre
        ds = loader.loader.dataset
        samples = []
        for i in range(args.batch):
            d = ds[i]
            samples.append(tuple(torch.from_numpy(np.ascontiguousarray(d[k])).pin_memory()
                                 for k in ("data", "label", "modal_x")))
        out = pre.batch(samples)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            pre.batch(samples, out=out)
        torch.cuda.synchronize()
        dev = args.iters * args.batch / (time.perf_counter() - t0)
    print(json.dumps({"metric": "input pipeline images/s (get_train_loader, RGBXDataset PNG tree, GPU TrainPre)",
                      "end_to_end_images_per_s": round(e2e, 1), "device_trainpre_images_per_s": round(dev, 1),
                      "batch": args.batch, "workers": args.workers, "image": [H, W],
                      "note": "one rank; the B2 step consumes 255-260 images/s per GPU"}))


if __name__ == "__main__":
    main()
