"""Synthetic RGB-X batches with the reference's input semantics.

RGB: uint8 uniform -> ``(x/255 - mean)/std`` in float64 then fp32 (utils/transforms.py:182-187);
X: ONE uint8 plane replicated to 3 channels (RGBXDataset.py:58-59), same ImageNet
normalisation (dataloader.py:105-106); labels: uniform in [0, K) with one 25x25 block of
ignore (255) per image (cutout, dataloader.py:61-83).
"""
from __future__ import annotations

import torch

MEAN = torch.tensor([0.485, 0.456, 0.406], dtype=torch.float64)
STD = torch.tensor([0.229, 0.224, 0.225], dtype=torch.float64)


def make_batch(B: int, H: int, W: int, K: int, seed: int = 12345, device="cpu", background: int = 255):
    g = torch.Generator().manual_seed(seed)
    rgb8 = torch.randint(0, 256, (B, 3, H, W), generator=g, dtype=torch.uint8)
    x8 = torch.randint(0, 256, (B, 1, H, W), generator=g, dtype=torch.uint8).expand(B, 3, H, W)

    def norm(t):
        return ((t.to(torch.float64) / 255.0 - MEAN[None, :, None, None]) / STD[None, :, None, None]).float()

    rgb, x = norm(rgb8), norm(x8)
    lab = torch.randint(0, K, (B, H, W), generator=g, dtype=torch.int64)
    for b in range(B):
        cy = int(torch.randint(12, max(13, H - 12), (1,), generator=g))
        cx = int(torch.randint(12, max(13, W - 12), (1,), generator=g))
        lab[b, max(0, cy - 12):cy + 13, max(0, cx - 12):cx + 13] = background
    return rgb.contiguous().to(device), x.contiguous().to(device), lab.to(device)
