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

import numpy as np
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
        (B,H,W) i64, (B,3,H,W) f32 -- the default collate of the reference's DataLoader.

        The draws are made sample by sample in the reference's order (as B calls of __call__
        would); the pixel work is ONE launch per stage for the whole minibatch
        (``cmx_aug_batch``).  Host samples (numpy / CPU tensors) and the per-sample record table
        are packed into one pinned staging buffer (two, alternating, reused across batches) and
        moved to HBM by ONE host-to-device copy; samples already on the device are read in place."""
        B = len(samples)
        dev = self.device
        if out is None:
            out = (torch.empty(B, 3, self.H, self.W, dtype=torch.float32, device=dev),
                   torch.empty(B, self.H, self.W, dtype=torch.int64, device=dev),
                   torch.empty(B, 3, self.H, self.W, dtype=torch.float32, device=dev))
        ro, go, xo = out
        assert ro.is_contiguous() and go.is_contiguous() and xo.is_contiguous()
        assert ro.shape == (B, 3, self.H, self.W) and xo.shape == ro.shape and go.shape == (B, self.H, self.W)
        rec = np.zeros((B, _AUG_REC), dtype=np.int64)
        host = []                                    # (array, staging offset)
        src_off = 0
        scratch_off = 0
        max_sh = max_sw = 1
        for b, (rgb, gt, x) in enumerate(samples):
            h, w = int(rgb.shape[0]), int(rgb.shape[1])
            if (rgb.ndim != 3 or rgb.shape[2] != 3 or tuple(x.shape) != tuple(rgb.shape)
                    or tuple(gt.shape) != (h, w)):
                raise ValueError(f"TrainPre: rgb {tuple(rgb.shape)} / x {tuple(x.shape)} must be HxWx3 and gt "
                                 f"{tuple(gt.shape)} HxW of the same size")
            prm = draw_params(h, w, self.scales, self.rng)
            sh, sw = prm["sh"], prm["sw"]
            max_sh, max_sw = max(max_sh, sh), max(max_sw, sw)
            for k, a in enumerate((rgb, x, gt)):
                if isinstance(a, torch.Tensor) and a.is_cuda:
                    if a.dtype != torch.uint8 or not a.is_contiguous():
                        raise TypeError("TrainPre: device samples must be contiguous uint8")
                    rec[b, k] = a.data_ptr()
                else:
                    a = a.numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
                    if a.dtype != np.uint8:
                        raise TypeError(f"TrainPre expects uint8 images, got {a.dtype}")
                    host.append((b, k, a, src_off))
                    src_off += _align(a.size)
            n = sh * sw
            sizes = (3 * n, 3 * n, n, 3 * n if prm["blur"] else 0)
            for k, sz in enumerate(sizes):
                rec[b, 3 + k] = scratch_off if sz else -1
                scratch_off += _align(sz)
            bx1, by1, bx2, by2 = prm["box"] if prm["box"] is not None else (0, 0, 0, 0)
            rec[b, 10:19] = (h, w, sh, sw, int(bool(prm["mirror"])), bx1, by1, bx2, by2)
            rec[b, 19:22] = np.array([prm["bf"], prm["sf"], prm["hf"] * 180], dtype=np.float32).view(np.int32)
        table_bytes = rec.nbytes
        stage = torch.empty(src_off + table_bytes, dtype=torch.uint8, device=dev)
        scratch = torch.empty(max(scratch_off, 1), dtype=torch.uint8, device=dev)
        sbase, cbase = stage.data_ptr(), scratch.data_ptr()
        for b, k, a, off in host:
            rec[b, k] = sbase + off
        for k in range(4):
            col = rec[:, 3 + k]
            rec[:, 3 + k] = np.where(col >= 0, col + cbase, 0)
        rec[:, 7] = [ro[b].data_ptr() for b in range(B)]
        rec[:, 8] = [xo[b].data_ptr() for b in range(B)]
        rec[:, 9] = [go[b].data_ptr() for b in range(B)]
        pin = self._staging(src_off + table_bytes)
        view = pin.numpy()
        for b, k, a, off in host:
            view[off:off + a.size] = a.reshape(-1)
        view[src_off:src_off + table_bytes] = rec.reshape(-1).view(np.uint8)
        st = torch.cuda.current_stream(dev)
        stage.copy_(pin[:src_off + table_bytes], non_blocking=True)
        self._events[self._turn].record(st)
        mn, sd = self.norm_mean, self.norm_std
        L.call("cmx_aug_batch", sbase + src_off, B, max_sh, max_sw, self.H, self.W, self.num_classes - 1,
               self.background, mn[0], mn[1], mn[2], sd[0], sd[1], sd[2], st.cuda_stream)
        return out

    def _staging(self, nbytes: int) -> torch.Tensor:
        """The next of two pinned staging buffers, grown to ``nbytes``; waits until the copy that
        last read it has finished (its event), so a buffer is never overwritten in flight."""
        if not hasattr(self, "_pins"):
            self._pins = [None, None]
            self._events = [torch.cuda.Event(), torch.cuda.Event()]
            self._turn = 1
        self._turn ^= 1
        t = self._turn
        self._events[t].synchronize()
        if self._pins[t] is None or self._pins[t].numel() < nbytes:
            self._pins[t] = torch.empty(_align(int(nbytes * 1.25)), dtype=torch.uint8).pin_memory()
        return self._pins[t]


_AUG_REC = 24


def _align(n: int, a: int = 256) -> int:
    return (int(n) + a - 1) // a * a
