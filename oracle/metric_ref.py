"""CPU restatement of the reference's evaluation path (TEST ORACLE -- test infrastructure only).

Only tests/ may import this module; the product evaluator
(rgbx_semantic_segmentation_amd/engine/evaluator.py) runs on the HIP kernels of csrc/metric.hip.

Restated, line by line in behaviour:
  * hist_info / compute_score      -- utils/metric.py:8-29 (numpy, verbatim semantics)
  * pad_image_to_shape (constant)  -- utils/transforms.py:61-75 (cv2.copyMakeBorder CONSTANT 0)
  * normalize                      -- utils/transforms.py:182-187
  * Evaluator.sliding_eval_rgbX / scale_process_rgbX / val_func_process_rgbX /
    process_image_rgbX             -- engine/evaluator.py:306-431, including its quirks:
      - the window origin uses stride[0] for x and stride[1] for y, and the crop end uses
        crop_size[0] for x and crop_size[1] for y (:352-357); a negative start is a
        Python slice from the end (numpy img_pad[s_y:e_y] and torch data_scale[:, s_y:e_y]);
      - the image is normalised again inside process_image_rgbX (:408-412);
      - per-scale scores are summed in float64 on the host (:310, :322).
  * resize                         -- cv2.resize(..., INTER_LINEAR) on float images: half-pixel
    centres, src = (dst + 0.5) * in / out - 0.5, clamped at 0 and at the last row / column.
    opencv-python is not installed here (requirements.txt:4), so this restatement is "parity
    unpinned" against cv2 itself; it is exact for the scale factors whose output size is an
    exact multiple (0.75 / 1.25 of 480 x 640), where fx and in/out agree.
"""
from __future__ import annotations

import math

import numpy as np


def hist_info(n_cl, pred, gt):
    """utils/metric.py:8-15."""
    assert pred.shape == gt.shape
    k = (gt >= 0) & (gt < n_cl)
    labeled = int(np.sum(k))
    correct = int(np.sum(pred[k] == gt[k]))
    cm = np.bincount(n_cl * gt[k].astype(int) + pred[k].astype(int), minlength=n_cl ** 2).reshape(n_cl, n_cl)
    return cm, labeled, correct


def compute_score(hist, correct, labeled):
    """utils/metric.py:17-29."""
    with np.errstate(divide="ignore", invalid="ignore"):
        iou = np.diag(hist) / (hist.sum(1) + hist.sum(0) - np.diag(hist))
        mean_IoU = np.nanmean(iou)
        mean_IoU_no_back = np.nanmean(iou[1:])
        freq = hist.sum(1) / hist.sum()
        freq_IoU = (iou[freq > 0] * freq[freq > 0]).sum()
        classAcc = np.diag(hist) / hist.sum(axis=1)
        mean_pixel_acc = np.nanmean(classAcc)
        pixel_acc = correct / labeled
    return iou, mean_IoU, mean_IoU_no_back, freq_IoU, mean_pixel_acc, pixel_acc


def normalize(img, mean, std):
    """utils/transforms.py:182-187."""
    img = img.astype(np.float64) / 255.0
    return (img - mean) / std


def pad_image_to_shape(img, shape, value=0):
    """utils/transforms.py:61-75 with BORDER_CONSTANT."""
    margin = np.zeros(4, np.int64)
    ph = max(shape[0] - img.shape[0], 0)
    pw = max(shape[1] - img.shape[1], 0)
    margin[0], margin[1] = ph // 2, ph // 2 + ph % 2
    margin[2], margin[3] = pw // 2, pw // 2 + pw % 2
    pad = [(int(margin[0]), int(margin[1])), (int(margin[2]), int(margin[3]))] + [(0, 0)] * (img.ndim - 2)
    return np.pad(img, pad, mode="constant", constant_values=value), margin


def resize_linear(img, out_h, out_w):
    """cv2.resize INTER_LINEAR of an (H, W[, C]) array (align_corners=False rule).  cv2 returns
    the input's dtype: a uint8 image comes back rounded to uint8 values (cv2's own 11-bit
    fixed-point interpolation is not restated: opencv is absent, parity unpinned)."""
    H, W = img.shape[:2]

    def idx(n_out, n_in):
        s = (np.arange(n_out) + 0.5) * (n_in / n_out) - 0.5
        s = np.maximum(s, 0.0)
        i0 = np.minimum(np.floor(s).astype(np.int64), n_in - 1)
        i1 = np.minimum(i0 + 1, n_in - 1)
        l1 = s - i0
        return i0, i1, l1

    y0, y1, ly = idx(out_h, H)
    x0, x1, lx = idx(out_w, W)
    sh = (-1, 1) + (1,) * (img.ndim - 2)
    sw = (1, -1) + (1,) * (img.ndim - 2)
    ly, lx = ly.reshape(sh), lx.reshape(sw)
    top = img[y0][:, x0] * (1 - lx) + img[y0][:, x1] * lx
    bot = img[y1][:, x0] * (1 - lx) + img[y1][:, x1] * lx
    out = top * (1 - ly) + bot * ly
    if img.dtype == np.uint8:
        out = np.clip(np.rint(out), 0, 255)
    return out


class SlidingEvaluatorRef:
    """engine/evaluator.py:306-431 on the CPU.  ``val_func(rgb, x) -> logits`` takes and returns
    float arrays (1, 3, h, w) -> (1, K, h, w) (the network; tests pass the product model's
    forward or a deterministic stand-in)."""

    def __init__(self, class_num, norm_mean, norm_std, val_func, multi_scales, is_flip):
        self.class_num = class_num
        self.norm_mean, self.norm_std = norm_mean, norm_std
        self.val_func = val_func
        self.multi_scales = multi_scales
        self.is_flip = is_flip

    def sliding_eval_rgbX(self, img, modal_x, crop_size, stride_rate):
        ori_rows, ori_cols, _ = img.shape
        processed = np.zeros((ori_rows, ori_cols, self.class_num))
        for s in self.multi_scales:
            nh, nw = int(round(ori_rows * s)), int(round(ori_cols * s))
            img_s = resize_linear(img, nh, nw) if (nh, nw) != (ori_rows, ori_cols) else img
            x_s = resize_linear(modal_x, nh, nw) if (nh, nw) != (ori_rows, ori_cols) else modal_x
            processed += self.scale_process_rgbX(img_s, x_s, (ori_rows, ori_cols), crop_size, stride_rate)
        return processed.argmax(2)

    def scale_process_rgbX(self, img, modal_x, ori_shape, crop_size, stride_rate):
        new_rows, new_cols, _ = img.shape
        if new_cols <= crop_size[1] or new_rows <= crop_size[0]:
            d, x, margin = self.process_image_rgbX(img, modal_x, crop_size)
            score = self.val_func_process_rgbX(d, x)
            score = score[:, margin[0]:score.shape[1] - margin[1], margin[2]:score.shape[2] - margin[3]]
        else:
            stride = (int(math.ceil(crop_size[0] * stride_rate)), int(math.ceil(crop_size[1] * stride_rate)))
            img_pad, margin = pad_image_to_shape(img, crop_size)
            x_pad, _ = pad_image_to_shape(modal_x, crop_size)
            pr, pc = img_pad.shape[:2]
            r_grid = int(np.ceil((pr - crop_size[0]) / stride[0])) + 1
            c_grid = int(np.ceil((pc - crop_size[1]) / stride[1])) + 1
            data_scale = np.zeros((self.class_num, pr, pc), np.float32)
            for gy in range(r_grid):
                for gx in range(c_grid):
                    s_x = gx * stride[0]
                    s_y = gy * stride[1]
                    e_x = min(s_x + crop_size[0], pc)
                    e_y = min(s_y + crop_size[1], pr)
                    s_x = e_x - crop_size[0]
                    s_y = e_y - crop_size[1]
                    d, x, tm = self.process_image_rgbX(img_pad[s_y:e_y, s_x:e_x], x_pad[s_y:e_y, s_x:e_x], crop_size)
                    t = self.val_func_process_rgbX(d, x)
                    t = t[:, tm[0]:t.shape[1] - tm[1], tm[2]:t.shape[2] - tm[3]]
                    data_scale[:, s_y:e_y, s_x:e_x] += t
            score = data_scale[:, margin[0]:pr - margin[1], margin[2]:pc - margin[3]]
        score = score.transpose(1, 2, 0)
        if score.shape[:2] != tuple(ori_shape):
            score = resize_linear(score.astype(np.float32), ori_shape[0], ori_shape[1])
        return score

    def val_func_process_rgbX(self, d, x):
        d = np.ascontiguousarray(d[None], dtype=np.float32)
        x = np.ascontiguousarray(x[None], dtype=np.float32)
        score = self.val_func(d, x)[0].astype(np.float32)
        if self.is_flip:
            score = score + self.val_func(d[..., ::-1].copy(), x[..., ::-1].copy())[0].astype(np.float32)[..., ::-1]
        return np.exp(score).astype(np.float32)

    def process_image_rgbX(self, img, modal_x, crop_size):
        p_img = normalize(img, self.norm_mean, self.norm_std)
        p_x = normalize(modal_x, self.norm_mean, self.norm_std)
        p_img, margin = pad_image_to_shape(p_img, crop_size)
        p_x, _ = pad_image_to_shape(p_x, crop_size)
        return p_img.transpose(2, 0, 1), p_x.transpose(2, 0, 1), margin
