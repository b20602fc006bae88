"""Roofline of the step's dominant kernel, measured live with HIP events on its launch stream.

The dominant single launch of the CMX-B2 step (rocprofv3 summary under profiles/) is the
grouped weight-gradient GEMM ``gemm_grouped_kernel`` (deferred.py): every Linear / 1x1 /
im2col-conv weight gradient of the backward pass in one launch.  ``measure_dominant`` runs
one eager training step, keeps the record table and operands of that launch, and re-launches
it standalone on the same stream (inputs resident in HBM), bracketed by torch.cuda.Event.

Algorithmic work of one launch (SURVEY.md §8(d) counting): FLOP = sum of 2 * M * N * K per
weight gradient (the bias-gradient column is not counted); bytes = each bf16 operand read once
plus each fp32 gradient written once.  Their ratio against the bf16 ridge point (314.6 FLOP/B)
picks the roof: the grouped launch sits below it (~120 FLOP/B), so ``bound`` is "hbm" and
``achieved`` = algorithmic bytes / average launch duration in GB/s; the MFMA figure is
reported beside it.  ``traffic`` is the PMC-measured HBM bytes per launch from a committed
profile of the SAME workload and grid (profiles/*pmc*.json, FETCH_SIZE x 2 + WRITE_SIZE per
the gfx950 correction in MI355X_MICROARCH.md), or None when no such profile exists."""
from __future__ import annotations

import glob
import json
import os

import torch

from . import deferred, _lib

PEAK_BF16_TFLOPS = 2516.6
PEAK_HBM_GBS = 8000.0
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


RIDGE_FLOP_PER_BYTE = PEAK_BF16_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)      # 314.6


def _pmc_traffic(kernel: str, workload: str, blocks: int):
    """PMC HBM bytes per launch of ``kernel`` measured on THIS workload: a profile counts only
    when its ``workload`` tag and the launch's workgroup count match (a B5 line must never
    reuse B2 bytes).  Newest profile first."""
    for path in sorted(glob.glob(os.path.join(_ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload:
            continue
        k = d.get("kernels", {}).get(kernel)
        if k and k.get("hbm_bytes_per_launch") and k.get("blocks") in (None, blocks):
            return k["hbm_bytes_per_launch"], os.path.relpath(path, _ROOT)
    return None, None


def measure_dominant(model, batch, workload: str, iters: int = 20):
    """Time the grouped weight-gradient GEMM of one eager step of ``model`` on ``batch``.
    ``bound`` follows the launch's arithmetic intensity against the bf16 ridge point
    (algorithmic FLOP / algorithmic bytes vs 314.6 FLOP/B): below it the HBM roof binds and
    ``achieved`` / ``peak`` are GB/s, else TFLOP/s; both fractions are reported."""
    rgb, x, lab = batch
    seen = []

    def obs(dev, nrec, blk, work, keep, dcode=1):
        seen.append((dev, nrec, blk, list(work), list(keep), dcode))

    deferred.observer = obs
    try:
        loss = model(rgb, x, lab)
        loss.backward()
    finally:
        deferred.observer = None
    torch.cuda.synchronize()
    if not seen:
        return None
    # every grouped launch of the step (one per block boundary flush, deferred.flush_hook):
    # each re-timed standalone; the family's algorithmic work over its total time
    flops = nbytes = t = 0.0
    blk = nrec = 0
    for dev, nr, bl, work, keep, dcode in seen:
        for (G, M, Nr, K) in work:
            flops += 2.0 * G * M * Nr * K
            nbytes += 2.0 * G * (M + Nr) * K + 4.0 * G * M * Nr
        launch = lambda: _lib.call("cmx_gemm_grouped", dev.data_ptr(), nr, bl, dcode, _lib.stream())
        for _ in range(3):
            launch()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            launch()
        e.record()
        torch.cuda.synchronize()
        t += s.elapsed_time(e) / iters * 1e-3
        blk += bl
        nrec += nr
    n = len(seen)
    traffic, src = _pmc_traffic("gemm_grouped_kernel", workload, blk // n)
    tflops, gbs = flops / t / 1e12, nbytes / t / 1e9
    ai = flops / nbytes
    hbm = ai < RIDGE_FLOP_PER_BYTE
    out = {"kernel": f"gemm_grouped_kernel (all {nrec} weight-gradient GEMM problems of the backward in {n} grouped "
                     f"launches, {blk} workgroups)",
           "bound": "hbm" if hbm else "mfma",
           "achieved": round(gbs, 1) if hbm else round(tflops, 2),
           "peak": PEAK_HBM_GBS if hbm else PEAK_BF16_TFLOPS,
           "unit": "GB/s" if hbm else "TFLOP/s",
           "frac": round(gbs / PEAK_HBM_GBS if hbm else tflops / PEAK_BF16_TFLOPS, 4),
           "traffic": traffic,
           "arithmetic_intensity_flop_per_byte": round(ai, 1), "ridge_flop_per_byte": round(RIDGE_FLOP_PER_BYTE, 1),
           "achieved_tflops": round(tflops, 2), "mfma_frac": round(tflops / PEAK_BF16_TFLOPS, 4),
           "achieved_hbm_gbs": round(gbs, 1), "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
           "launches": n, "avg_launch_us": round(t / n * 1e6, 2), "total_us": round(t * 1e6, 1),
           "algorithmic_flop_per_launch": flops / n, "algorithmic_bytes_per_launch": nbytes / n, "workload": workload}
    if src:
        out["traffic_source"] = src
    del seen
    return out
