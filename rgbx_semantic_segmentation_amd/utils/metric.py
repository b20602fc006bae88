"""Drop-in mirror of the reference's ``utils/metric.py`` (utils/metric.py:8-29).

``hist_info`` runs on the device: one fused HIP kernel (csrc/metric.hip,
``cmx_seg_argmax_confusion``) bins labels x predictions into the n_cl x n_cl confusion
matrix with integer atomics (bit-exact, order independent).  It accepts numpy arrays (the
reference's types: copied to the current GPU) or CUDA tensors, and returns the reference's
``(confusionMatrix, labeled, correct)`` as (numpy int64 array, int, int).
``hist_info_from_score`` is the evaluator's fused form: argmax over a (K, H, W) score map on
the device plus the same binning, accumulating into device-resident counters, so a validation
pass copies only n_cl^2 + 2 integers to the host.
``compute_score`` is the reference's host arithmetic on the small matrix (unchanged).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _lib

np.seterr(divide="ignore", invalid="ignore")


def _label_code(t: torch.Tensor) -> int:
    if t.dtype == torch.int64:
        return 0
    if t.dtype == torch.uint8:
        return 1
    raise RuntimeError(f"hist_info: labels must be int64 or uint8, got {t.dtype}")


class ConfusionCounter:
    """Device-resident hist (n_cl x n_cl int64) + [labeled, correct], accumulated over a pass."""

    def __init__(self, n_cl: int, device=None):
        device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.n_cl = n_cl
        self.hist = torch.zeros(n_cl * n_cl, dtype=torch.int64, device=device)
        self.counts = torch.zeros(2, dtype=torch.int64, device=device)

    def add_score(self, score: torch.Tensor, gt: torch.Tensor, pred_out: torch.Tensor | None = None):
        """score (K, H, W) fp32 on the device; gt (H, W) int64 / uint8."""
        if score.dim() != 3 or score.dtype != torch.float32 or not score.is_cuda:
            raise RuntimeError("hist_info_from_score: score must be a (K, H, W) float32 CUDA tensor")
        K, H, W = score.shape
        gt = gt.to(score.device).contiguous()
        if gt.shape != (H, W):
            raise RuntimeError(f"hist_info_from_score: label shape {tuple(gt.shape)} != score {(H, W)}")
        score = score.contiguous()
        _lib.call("cmx_seg_argmax_confusion", _lib.ptr(score), K, H * W, _lib.ptr(gt), _label_code(gt), self.n_cl,
                  _lib.ptr(pred_out), _lib.ptr(self.hist), _lib.ptr(self.counts), _lib.stream())

    def add_pred(self, pred: torch.Tensor, gt: torch.Tensor):
        pred = pred.to(device=self.hist.device, dtype=torch.int32).contiguous()
        gt = gt.to(self.hist.device).contiguous()
        if pred.shape != gt.shape:
            raise AssertionError("hist_info: pred and gt shapes differ")
        _lib.call("cmx_seg_argmax_confusion", None, 0, pred.numel(), _lib.ptr(gt), _label_code(gt), self.n_cl,
                  _lib.ptr(pred), _lib.ptr(self.hist), _lib.ptr(self.counts), _lib.stream())

    def result(self):
        h = self.hist.cpu().numpy().reshape(self.n_cl, self.n_cl)
        c = self.counts.cpu().numpy()
        return h, int(c[0]), int(c[1])


def _as_tensor(a):
    if isinstance(a, torch.Tensor):
        return a
    a = np.ascontiguousarray(a)
    if a.dtype not in (np.int64, np.uint8):
        a = a.astype(np.int64)
    return torch.from_numpy(a)


def hist_info(n_cl, pred, gt):
    """utils/metric.py:8-15: (confusionMatrix, labeled, correct) of one prediction."""
    pred_t, gt_t = _as_tensor(pred), _as_tensor(gt)
    if tuple(pred_t.shape) != tuple(gt_t.shape):
        raise AssertionError("hist_info: pred and gt shapes differ")
    dev = pred_t.device if pred_t.is_cuda else (gt_t.device if gt_t.is_cuda else None)
    cc = ConfusionCounter(n_cl, dev)
    cc.add_pred(pred_t, gt_t)
    return cc.result()


def hist_info_from_score(n_cl, score, gt, counter: ConfusionCounter | None = None):
    """argmax over classes of a device score (K, H, W) fused with hist_info."""
    cc = counter or ConfusionCounter(n_cl, score.device)
    cc.add_score(score, _as_tensor(gt))
    return cc if counter is not None else cc.result()


def compute_score(hist, correct, labeled):
    """utils/metric.py:17-29 (host arithmetic on the n_cl x n_cl matrix)."""
    iou = np.diag(hist) / (hist.sum(1) + hist.sum(0) - np.diag(hist))
    mean_IoU = np.nanmean(iou)
    mean_IoU_no_back = np.nanmean(iou[1:])
    freq = hist.sum(1) / hist.sum()
    freq_IoU = (iou[freq > 0] * freq[freq > 0]).sum()
    classAcc = np.diag(hist) / hist.sum(axis=1)
    mean_pixel_acc = np.nanmean(classAcc)
    pixel_acc = correct / labeled
    return iou, mean_IoU, mean_IoU_no_back, freq_IoU, mean_pixel_acc, pixel_acc
