"""Roofline of the step's dominant kernels, measured live with HIP events on their launch stream.

1. ``measure_gemm_family`` -- the DOMINANT family of the CMX-B2 step by device time (the census
   of profiles/r05_*_step_census.txt: ~3.2 ms of ~7.3 ms): the MFMA tile GEMMs of the forward and
   input-gradient passes (``gemm_bf16_kernel`` / ``gemm_multi_kernel`` / split-K reduce: every
   Linear, 1x1 / implicit conv, the decoder's fuse products), ~250 launches per step.  During one
   eager training step every such launch is re-issued in place, right after the original (the
   caller still holds its buffers), 4 warm + 16 timed times between two HIP events on the launch
   stream; the family's device time per step is the sum of the per-launch averages.  Algorithmic
   work per step is floor.step_work's "gemm" family (each bf16 operand read once, each output
   written once: SURVEY.md §8(d) counting), so ``achieved`` = those bytes / that time.
2. ``measure_dominant`` -- the largest SINGLE launch, the grouped weight-gradient GEMM
   ``gemm_grouped_kernel`` (deferred.py): every Linear / 1x1 / im2col-conv weight gradient of
   the backward pass in one launch; its record table and operands are kept from the same eager
   step and it is re-launched standalone on the same stream.

Algorithmic work of the grouped launch (SURVEY.md §8(d) counting): FLOP = sum of 2 * M * N * K per
weight gradient (the bias-gradient column is not counted); bytes = each bf16 operand read once
plus each fp32 gradient written once.  Their ratio against the bf16 ridge point (314.6 FLOP/B)
picks the roof: both sit below it (~110-120 FLOP/B), so ``bound`` is "hbm" and ``achieved`` =
algorithmic bytes / average launch duration in GB/s; the MFMA figure is reported beside it.
``traffic`` is the PMC-measured HBM bytes per launch from a committed profile of the SAME
workload (profiles/*pmc*.json, FETCH_SIZE x 2 + WRITE_SIZE per the gfx950 correction in
MI355X_MICROARCH.md), or None when no such profile exists."""
from __future__ import annotations

import glob
import json
import os

import torch

from . import deferred, _lib
from .floor import step_work

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


# the C-ABI entry points whose launches make up the tile-GEMM family (the FFM per-head context
# products, cmx_gemm_h2, are floor.py's "ffm" family and stay out of both the time and the work)
GEMM_FAMILY = ("cmx_gemm", "cmx_gemm_ln", "cmx_gemm_multi", "cmx_conv_implicit_fwd", "cmx_decoder_fuse_fwd",
               "cmx_conv_patch_dgrad", "cmx_gemm_ln_bwd", "cmx_conv_patch_dgrad_ln_bwd")
# (the LayerNorm-epilogue launches -- cmx_gemm_ln and the two *_ln_bwd -- are timed whole: their time
# includes the norm's work, their algorithmic bytes only the GEMM's, so the family's fraction errs low)


def _family_traffic(kernels, workload: str):
    """PMC HBM bytes per launch averaged over the named kernels of one committed profile of THIS
    workload (launch-weighted), newest profile first; (bytes, source) or (None, None)."""
    for path in sorted(glob.glob(os.path.join(_ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload:
            continue
        ks = [d.get("kernels", {}).get(k) for k in kernels]
        ks = [k for k in ks if k and k.get("hbm_bytes_per_launch") and k.get("launches")]
        if ks:
            n = sum(k["launches"] for k in ks)
            return sum(k["hbm_bytes_per_launch"] * k["launches"] for k in ks) / n, os.path.relpath(path, _ROOT)
    return None, None


def measure_gemm_family(model, batch, workload: str, shape: dict, warm: int = 4, iters: int = 16):
    """Device time per step of the tile-GEMM family (GEMM_FAMILY launches of one eager training
    step of ``model``, each re-issued in place between HIP events) and its roofline."""
    import torch as _t
    rgb, x, lab = batch
    timings = []

    def obs(name, fn, args):
        if name not in GEMM_FAMILY:
            return
        for _ in range(warm):
            fn(*args)
        e0, e1 = _t.cuda.Event(enable_timing=True), _t.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn(*args)
        e1.record()
        timings.append((name, e0, e1))

    _lib.observer = obs
    try:
        loss = model(rgb, x, lab)
        loss.backward()
    finally:
        _lib.observer = None
    _t.cuda.synchronize()
    if not timings:
        return None
    per = [e0.elapsed_time(e1) / iters * 1e-3 for _, e0, e1 in timings]
    t = sum(per)
    flops, nbytes = step_work(**shape)["gemm"]
    n = len(per)
    traffic, src = _family_traffic(("gemm_bf16_kernel", "gemm_stream_kernel", "gemm_multi_kernel", "splitk_reduce_kernel"),
                                  workload)
    gbs, tflops = nbytes / t / 1e9, flops / t / 1e12
    hbm = flops / nbytes < RIDGE_FLOP_PER_BYTE
    out = {"kernel": f"tile-GEMM family: gemm_bf16_kernel / gemm_multi_kernel / splitk_reduce_kernel ({n} forward and "
                     f"input-gradient launches per step: every Linear, 1x1 / implicit conv, decoder fuse product)",
           "bound": "hbm" if hbm else "mfma",
           "achieved": round(gbs, 1) if hbm else round(tflops, 2),
           "peak": PEAK_HBM_GBS if hbm else PEAK_BF16_TFLOPS,
           "unit": "GB/s" if hbm else "TFLOP/s",
           "frac": round(gbs / PEAK_HBM_GBS if hbm else tflops / PEAK_BF16_TFLOPS, 4),
           "traffic": traffic,
           "arithmetic_intensity_flop_per_byte": round(flops / nbytes, 1),
           "ridge_flop_per_byte": round(RIDGE_FLOP_PER_BYTE, 1),
           "achieved_tflops": round(tflops, 2), "mfma_frac": round(tflops / PEAK_BF16_TFLOPS, 4),
           "achieved_hbm_gbs": round(gbs, 1), "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
           "launches": n, "avg_launch_us": round(t / n * 1e6, 2), "total_us": round(t * 1e6, 1),
           "by_entry_point_us": {k: round(sum(p for (nm, _, _), p in zip(timings, per) if nm == k) * 1e6, 1)
                                 for k in GEMM_FAMILY if any(nm == k for nm, _, _ in timings)},
           "algorithmic_flop_per_launch": flops / n, "algorithmic_bytes_per_launch": nbytes / n,
           "algorithmic_bytes_per_step": nbytes, "workload": workload,
           "timing": f"each launch re-issued in place {warm} + {iters} times; HIP events around the {iters}"}
    if src:
        out["traffic_source"] = src
    return out


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
