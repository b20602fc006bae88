"""CPU restatement of the reference's training augmentation (TrainPre) -- TEST INFRASTRUCTURE.

Nothing in the product imports this file; tests/ use it as the checker of the HIP kernels in
csrc/augment.hip (rgbx_semantic_segmentation_amd/augment.py).

Reference: dataloader/dataloader.py:9-112 (random_mirror, random_scale, ensure_size,
random_color_jitter, random_gaussian_blur, cutout, TrainPre.__call__), utils/transforms.py:
182-187 (normalize), dataloader/RGBXDataset.py:37-73 (__getitem__).

The reference's pixel work is OpenCV (cv2 4.x, an unpinned pip dependency of the reference;
cv2 is NOT installed in this image and the reference holds no fixtures of these ops).  The
algorithms below restate OpenCV's published 8-bit implementations:

  * cv2.flip(img, 1): x -> W-1-x.
  * cv2.resize INTER_NEAREST (resizeNN): src = min(floor(d * (1/(dsize/ssize))), ssize-1).
  * cv2.resize INTER_LINEAR, 8U (resizeGeneric_ / HResizeLinear / VResizeLinear): the
    source coordinate f = (d + 0.5) * scale - 0.5 in float, s = floor(f), clamped to the
    edge with weight 0; weights round((1-f)*2048), round(f*2048) (11-bit, cvRound = half to
    even); horizontal pass D = S0*a0 + S1*a1 in int32; vertical pass as the x86 SIMD kernel
    (VResizeLinearVec_32s8u): ((((D0>>4)*b0)>>16) + (((D1>>4)*b1)>>16) + 2) >> 2, saturated,
    applied to EVERY byte of a row.  cv2 rounds the bytes its vector loop leaves over at the
    end of a row with the scalar FixedPtCast ((D0*b0 + D1*b1 + (1 << 21)) >> 22) instead, which
    can differ by 1 LSB: that scalar tail is NOT modelled, so the GPU kernels are bit-exact
    against this restatement, and within 1 LSB (not bit-exact) of cv2 itself (unpinned: cv2
    is not installed).
    Same-size resize is a copy (cv2.resize returns src.copyTo for dsize == ssize).
  * cv2.cvtColor BGR2HSV, 8U (RGB2HSV_b): integer V, S = round(diff*255/V) and H via the
    12-bit sdiv/hdiv tables, H in [0, 180).
  * cv2.cvtColor HSV2BGR, 8U (HSV2RGB_b): to float (S, V / 255), sector formula with
    hscale = 6/180, fp32 without fused multiply-adds, saturate_cast<uchar>(x * 255).
  * cv2.GaussianBlur(5x5, sigma 1), 8U: the bit-exact fixed-point path (ufixedpoint16
    kernel from the error-diffused rounding of the normalised Gaussian = [14, 62, 104, 62,
    14] / 256, separable sums exact in integers, (v + 2^15) >> 16), BORDER_REFLECT_101.

Parity with cv2 itself is therefore UNPINNED (no cv2, no fixtures); the integer / label
work (clip, mirror, nearest resize, cutout box, background fill) has no rounding choices
and follows the reference's Python line by line.
"""
from __future__ import annotations

import random

import numpy as np

COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS
BLUR5 = np.array([14, 62, 104, 62, 14], dtype=np.int64)       # sigma 1, /256


# ---------------------------------------------------------------------------- resize
def _linear_tab(ssize: int, dsize: int):
    """Source index pairs and 11-bit weights of cv2's INTER_LINEAR along one axis."""
    scale = 1.0 / (dsize / ssize)
    s0 = np.empty(dsize, np.int64)
    s1 = np.empty(dsize, np.int64)
    w0 = np.empty(dsize, np.int64)
    w1 = np.empty(dsize, np.int64)
    for d in range(dsize):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0.0), 0
        if s >= ssize - 1:
            f, s = np.float32(0.0), ssize - 1
        s0[d] = s
        s1[d] = min(s + 1, ssize - 1)
        w0[d] = int(np.rint(np.float32(np.float32(1.0) - f) * np.float32(COEF_SCALE)))
        w1[d] = int(np.rint(f * np.float32(COEF_SCALE)))
    return s0, s1, w0, w1


def resize_linear_u8(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """cv2.resize(img, (ow, oh), interpolation=cv2.INTER_LINEAR) for uint8 HxW[xC]."""
    h, w = img.shape[:2]
    if (h, w) == (oh, ow):
        return img.copy()
    x0, x1, a0, a1 = _linear_tab(w, ow)
    y0, y1, b0, b1 = _linear_tab(h, oh)
    src = img.astype(np.int64)
    if src.ndim == 2:
        src = src[:, :, None]
    D = src[:, x0, :] * a0[None, :, None] + src[:, x1, :] * a1[None, :, None]      # (h, ow, C)
    v = (((D[y0] >> 4) * b0[:, None, None]) >> 16) + (((D[y1] >> 4) * b1[:, None, None]) >> 16)
    out = np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)
    return out[:, :, 0] if img.ndim == 2 else out


def resize_nearest_u8(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """cv2.resize(img, (ow, oh), interpolation=cv2.INTER_NEAREST)."""
    h, w = img.shape[:2]
    if (h, w) == (oh, ow):
        return img.copy()
    ifx, ify = 1.0 / (ow / w), 1.0 / (oh / h)
    xs = np.minimum(np.floor(np.arange(ow) * ifx).astype(np.int64), w - 1)
    ys = np.minimum(np.floor(np.arange(oh) * ify).astype(np.int64), h - 1)
    return img[ys][:, xs].copy()


# ---------------------------------------------------------------------------- colour
def _tables():
    sdiv = np.zeros(256, np.int64)
    hdiv = np.zeros(256, np.int64)
    for i in range(1, 256):
        sdiv[i] = int(np.rint((255 << 12) / float(i)))
        hdiv[i] = int(np.rint((180 << 12) / (6.0 * i)))
    return sdiv, hdiv


_SDIV, _HDIV = _tables()


def bgr2hsv_u8(img: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(img, cv2.COLOR_BGR2HSV) for uint8 (H in [0, 180))."""
    b, g, r = (img[..., i].astype(np.int64) for i in range(3))
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    vr = v == r
    vg = v == g
    s = (diff * _SDIV[v] + (1 << 11)) >> 12
    h = np.where(vr, g - b, np.where(vg, b - r + 2 * diff, r - g + 4 * diff))
    h = (h * _HDIV[diff] + (1 << 11)) >> 12
    h = np.where(h < 0, h + 180, h)
    return np.stack([h, s, v], -1).astype(np.uint8)


def hsv2bgr_u8(hsv: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(hsv, cv2.COLOR_HSV2BGR) for uint8, fp32 arithmetic as HSV2RGB_b."""
    f32 = np.float32
    h = hsv[..., 0].astype(f32)
    s = hsv[..., 1].astype(f32) * f32(1.0 / 255.0)
    v = hsv[..., 2].astype(f32) * f32(1.0 / 255.0)
    h = h * f32(6.0 / 180.0)
    h = np.fmod(h, f32(6.0))
    h = np.where(h < 0, h + f32(6.0), h).astype(f32)
    sector = np.floor(h).astype(np.int64)
    h = (h - sector.astype(f32)).astype(f32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    h = np.where(bad, f32(0.0), h).astype(f32)
    one = f32(1.0)
    tab = np.stack([v, v * (one - s), v * (one - s * h), v * (one - s * (one - h))], -1).astype(f32)
    sec = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    idx = sec[sector]                                            # (..., 3) -> b, g, r
    bgr = np.take_along_axis(tab, idx, -1)
    bgr = np.where((hsv[..., 1] == 0)[..., None], v[..., None], bgr).astype(f32)
    return np.clip(np.rint(bgr * f32(255.0)), 0, 255).astype(np.uint8)


def color_jitter_u8(img: np.ndarray, bf: float, sf: float, hf: float) -> np.ndarray:
    """random_color_jitter (dataloader.py:32-54) with its three draws given:
    bf = 1 + U(-0.2, 0.2) (brightness, V), sf = 1 + U(-0.2, 0.2) (saturation, S),
    hf = U(-0.1, 0.1) (hue shift * 180).  numpy float32 arithmetic on the HSV image."""
    hsv = bgr2hsv_u8(img).astype(np.float32)
    hsv[:, :, 2] *= np.float32(bf)
    hsv[:, :, 1] *= np.float32(sf)
    hsv[:, :, 0] += np.float32(hf * 180)
    hsv = np.clip(hsv, 0, 255)
    return hsv2bgr_u8(hsv.astype(np.uint8))


def gaussian_blur5_u8(img: np.ndarray) -> np.ndarray:
    """cv2.GaussianBlur(img, (5, 5), 1.0), 8U bit-exact path, BORDER_REFLECT_101."""
    h, w = img.shape[:2]

    def refl(i, n):
        i = np.abs(i)
        return np.where(i >= n, 2 * (n - 1) - i, i)

    src = img.astype(np.int64)
    xs = np.arange(w)
    ys = np.arange(h)
    hs = sum(BLUR5[k] * src[:, refl(xs + k - 2, w)] for k in range(5))
    vs = sum(BLUR5[k] * hs[refl(ys + k - 2, h)] for k in range(5))
    return np.clip((vs + (1 << 15)) >> 16, 0, 255).astype(np.uint8)


# ---------------------------------------------------------------------------- TrainPre
def draw_params(h: int, w: int, scales, rng=random, mask_size: int = 25, p: float = 0.5):
    """The random draws of TrainPre.__call__ in the reference's order (dataloader.py:
    90-100): mirror (:10), scale (:17), jitter b / s / h (:38,42,46), blur (:54), cutout
    (:62, then cx, cy :69-70 at the scaled size)."""
    mirror = rng.random() >= 0.5
    scale = 1.0
    sh, sw = h, w
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
        box = (max(0, cx - half), max(0, cy - half), min(sw, cx + half), min(sh, cy + half))   # x1 y1 x2 y2
    return dict(mirror=mirror, scale=scale, sh=sh, sw=sw, bf=bf, sf=sf, hf=hf, blur=blur, box=box)


def train_pre(rgb, gt, x, prm, num_classes, height, width, mean, std, background=255):
    """TrainPre.__call__ (dataloader.py:85-112) with the draws ``prm`` (draw_params).
    rgb / x: uint8 HxWx3 (BGR as cv2 reads them), gt uint8 HxW.  Returns float32 CHW rgb,
    int64 HxW gt, float32 CHW x (RGBXDataset.py:65-68 conversions)."""
    gt = np.clip(gt, 0, num_classes - 1)
    if prm["mirror"]:
        rgb, gt, x = rgb[:, ::-1], gt[:, ::-1], x[:, ::-1]
    sh, sw = prm["sh"], prm["sw"]
    rgb = resize_linear_u8(np.ascontiguousarray(rgb), sh, sw)
    gt = resize_nearest_u8(np.ascontiguousarray(gt), sh, sw)
    x = resize_linear_u8(np.ascontiguousarray(x), sh, sw)
    rgb = color_jitter_u8(rgb, prm["bf"], prm["sf"], prm["hf"])
    if prm["blur"]:
        rgb = gaussian_blur5_u8(rgb)
    if prm["box"] is not None:
        x1, y1, x2, y2 = prm["box"]
        rgb = rgb.copy(); gt = gt.copy(); x = x.copy()
        rgb[y1:y2, x1:x2, :] = 0
        gt[y1:y2, x1:x2] = background
        x[y1:y2, x1:x2, :] = 0
    rgb = resize_linear_u8(rgb, height, width)
    gt = resize_nearest_u8(gt, height, width)
    x = resize_linear_u8(x, height, width)

    def norm(img):
        img = img.astype(np.float64) / 255.0
        return ((img - np.asarray(mean)) / np.asarray(std)).transpose(2, 0, 1)

    return (np.ascontiguousarray(norm(rgb)).astype(np.float32), gt.astype(np.int64),
            np.ascontiguousarray(norm(x)).astype(np.float32))
