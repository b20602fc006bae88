"""TrainPre on the GPU (dataloader/dataloader.py:85-112) over the HIP kernels of csrc/augment.hip.

Same interface as the reference's ``TrainPre(norm_mean, norm_std)`` plus the config values the
reference reads from its global ``config`` (num_classes, train_scale_array, image_height /
image_width, background).  ``__call__(rgb, gt, modal_x)`` takes one uint8 HWC sample (rgb / x
in the BGR channel order cv2.imread gives, gt HxW) on the host or the device and returns the
device tensors the reference's Dataset yields for it: float32 CHW rgb, int64 HxW label,
float32 CHW modal_x.

The random draws happen on the host with Python's ``random`` module in the reference's order
(mirror, scale, brightness, saturation, hue, blur, cutout + its centre), so a seeded
``random`` gives the reference's parameter sequence; the pixel work is four kernels:

  resize (mirror + label clip + random_scale)  x3 (rgb, x linear; label nearest)
  colour jitter (in place)  ->  optional 5x5 blur  ->  finalize (cutout + ensure_size +
  normalize + CHW, into the batch slot)

There is no CPU fallback: the kernels raise if the library is missing (the checker,
oracle/augment_ref.py, lives with the tests)."""
from __future__ import annotations

import random

import torch

from . import _lib as L


def draw_params(h: int, w: int, scales, rng=random, mask_size: int = 25, p: float = 0.5) -> dict:
    """The draws of TrainPre.__call__ in order: random_mirror (dataloader.py:10), random_scale
    (:17-19), random_color_jitter brightness / saturation / hue (:38,42,46),
    random_gaussian_blur (:54), cutout (:62; centre :69-70 at the scaled size, box :73-76)."""
    mirror = rng.random() >= 0.5
    scale, sh, sw = 1.0, h, w
    if scales is not None:
        scale = rng.choice(scales)
        sh, sw = int(h * scale), int(w * scale)
    bf = 1.0 + rng.uniform(-0.2, 0.2)
    sf = 1.0 + rng.uniform(-0.2, 0.2)
    hf = rng.uniform(-0.1, 0.1)
    blur = rng.random() >= 0.5
    box = None
    if not rng.random() > p:
        half = mask_size // 2
        cx = rng.randint(half, sw - half)
        cy = rng.randint(half, sh - half)
        box = (max(0, cx - half), max(0, cy - half), min(sw, cx + half), min(sh, cy + half))
    return dict(mirror=mirror, scale=scale, sh=sh, sw=sw, bf=bf, sf=sf, hf=hf, blur=blur, box=box)


def _u8(t, dev):
    if not isinstance(t, torch.Tensor):
        t = torch.from_numpy(t)
    if t.dtype != torch.uint8:
        raise TypeError(f"TrainPre expects uint8 images, got {t.dtype}")
    return t.to(dev, non_blocking=True).contiguous()


class TrainPre:
    def __init__(self, norm_mean, norm_std, num_classes: int, image_height: int, image_width: int,
                 train_scale_array=None, background: int = 255, rng=None, device=None):
        self.norm_mean = [float(v) for v in norm_mean]
        self.norm_std = [float(v) for v in norm_std]
        self.num_classes = int(num_classes)
        self.H, self.W = int(image_height), int(image_width)
        self.scales = list(train_scale_array) if train_scale_array is not None else None
        self.background = int(background)
        self.rng = rng if rng is not None else random
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())

    def apply(self, rgb, gt, modal_x, prm: dict, out=None):
        """The pixel work for given draws ``prm`` (draw_params).  ``out`` = (rgb (3,H,W) f32,
        gt (H,W) i64, x (3,H,W) f32) views to write into (a batch slot), else new tensors."""
        dev = self.device
        rgb, gt, x = _u8(rgb, dev), _u8(gt, dev), _u8(modal_x, dev)
        if rgb.dim() != 3 or rgb.shape[2] != 3 or x.shape != rgb.shape or gt.shape != rgb.shape[:2]:
            raise ValueError(f"TrainPre: rgb {tuple(rgb.shape)} / x {tuple(x.shape)} must be HxWx3 and gt "
                             f"{tuple(gt.shape)} HxW of the same size")
        h, w = rgb.shape[:2]
        sh, sw = prm["sh"], prm["sw"]
        st = L.stream()
        m = int(bool(prm["mirror"]))
        rs = torch.empty(sh, sw, 3, dtype=torch.uint8, device=dev)
        xs = torch.empty_like(rs)
        gs = torch.empty(sh, sw, dtype=torch.uint8, device=dev)
        L.call("cmx_aug_resize_u8", L.ptr(rgb), h, w, 3, L.ptr(rs), sh, sw, 0, m, -1, st)
        L.call("cmx_aug_resize_u8", L.ptr(x), h, w, 3, L.ptr(xs), sh, sw, 0, m, -1, st)
        L.call("cmx_aug_resize_u8", L.ptr(gt), h, w, 1, L.ptr(gs), sh, sw, 1, m, self.num_classes - 1, st)
        L.call("cmx_aug_color_jitter_u8", L.ptr(rs), sh, sw, float(prm["bf"]), float(prm["sf"]),
               float(prm["hf"] * 180), st)
        if prm["blur"]:
            rb = torch.empty_like(rs)
            L.call("cmx_aug_blur5_u8", L.ptr(rs), L.ptr(rb), sh, sw, 3, st)
            rs = rb
        if out is None:
            out = (torch.empty(3, self.H, self.W, dtype=torch.float32, device=dev),
                   torch.empty(self.H, self.W, dtype=torch.int64, device=dev),
                   torch.empty(3, self.H, self.W, dtype=torch.float32, device=dev))
        ro, go, xo = out
        assert ro.is_contiguous() and go.is_contiguous() and xo.is_contiguous()
        bx1, by1, bx2, by2 = prm["box"] if prm["box"] is not None else (0, 0, 0, 0)
        mn, sd = self.norm_mean, self.norm_std
        L.call("cmx_aug_finalize", L.ptr(rs), L.ptr(xs), L.ptr(gs), sh, sw, self.H, self.W, bx1, by1, bx2, by2,
               self.background, mn[0], mn[1], mn[2], sd[0], sd[1], sd[2], L.ptr(ro), L.ptr(xo), L.ptr(go), st)
        return out

    def __call__(self, rgb, gt, modal_x, out=None):
        h, w = rgb.shape[:2]
        prm = draw_params(h, w, self.scales, self.rng)
        return self.apply(rgb, gt, modal_x, prm, out)

    def batch(self, samples, out=None):
        """Augment a list of (rgb, gt, modal_x) uint8 samples into batch tensors (B,3,H,W) f32,
        (B,H,W) i64, (B,3,H,W) f32 -- the default collate of the reference's DataLoader."""
        B = len(samples)
        dev = self.device
        if out is None:
            out = (torch.empty(B, 3, self.H, self.W, dtype=torch.float32, device=dev),
                   torch.empty(B, self.H, self.W, dtype=torch.int64, device=dev),
                   torch.empty(B, 3, self.H, self.W, dtype=torch.float32, device=dev))
        for b, (rgb, gt, x) in enumerate(samples):
            self(rgb, gt, x, out=(out[0][b], out[1][b], out[2][b]))
        return out
