"""Roofline of the step's dominant kernel, measured live with HIP events on its launch stream.

The dominant single launch of the CMX-B2 step (rocprofv3 summary under profiles/) is the
grouped weight-gradient GEMM ``gemm_grouped_kernel`` (deferred.py): every Linear / 1x1 /
im2col-conv weight gradient of the backward pass in one launch.  ``measure_dominant`` runs
one eager training step, keeps the record table and operands of that launch, and re-launches
it standalone on the same stream (inputs resident in HBM), bracketed by torch.cuda.Event.

achieved = algorithmic FLOPs of one launch (SURVEY.md §8(d) counting: 2 * M * N * K per weight
gradient; the bias-gradient column is not counted) / average launch duration.  The
algorithmic bytes (each operand read once in bf16, each fp32 gradient written once) are
reported beside it, and ``traffic`` is the PMC-measured HBM bytes per launch from the
committed profile (profiles/*pmc*.json, FETCH_SIZE x 2 + WRITE_SIZE per the gfx950
correction in MI355X_MICROARCH.md), or None when no such profile is present."""
from __future__ import annotations

import glob
import json
import os

import torch

from . import deferred, _lib

PEAK_BF16_TFLOPS = 2516.6
PEAK_HBM_GBS = 8000.0
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pmc_traffic(kernel: str):
    for path in sorted(glob.glob(os.path.join(_ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel)
        if k and k.get("hbm_bytes_per_launch"):
            return k["hbm_bytes_per_launch"], os.path.relpath(path, _ROOT)
    return None, None


def measure_dominant(model, batch, iters: int = 20):
    """Time the grouped weight-gradient GEMM of one eager step of ``model`` on ``batch``."""
    rgb, x, lab = batch
    seen = []

    def obs(dev, nrec, blk, work, keep):
        seen.append((dev, nrec, blk, list(work), list(keep)))

    deferred.observer = obs
    try:
        loss = model(rgb, x, lab)
        loss.backward()
    finally:
        deferred.observer = None
    torch.cuda.synchronize()
    if not seen:
        return None
    dev, nrec, blk, work, keep = max(seen, key=lambda s: s[2])
    flops = 0.0
    nbytes = 0.0
    for (G, M, Nr, K) in work:
        flops += 2.0 * G * M * Nr * K
        nbytes += 2.0 * G * (M + Nr) * K + 4.0 * G * M * Nr
    launch = lambda: _lib.call("cmx_gemm_grouped", dev.data_ptr(), nrec, blk, _lib.stream())
    for _ in range(3):
        launch()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        launch()
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / iters * 1e-3
    traffic, src = _pmc_traffic("gemm_grouped_kernel")
    out = {"kernel": f"gemm_grouped_kernel (all {nrec} weight-gradient GEMM problems of the backward, one launch, "
                     f"{blk} workgroups)",
           "bound": "mfma", "achieved": round(flops / t / 1e12, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
           "frac": round(flops / t / 1e12 / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
           "avg_launch_us": round(t * 1e6, 2), "algorithmic_per_launch": flops,
           "algorithmic_bytes_per_launch": nbytes, "achieved_hbm_gbs": round(nbytes / t / 1e9, 1)}
    if src:
        out["traffic_source"] = src
    del seen, keep, work
    return out
