"""Roofline of the step's dominant kernels, measured live inside bench.py.

0. ``measure_in_step`` -- the bench line's ``roofline`` since round 6: a
   kernel trace (torch.profiler's roctracer activity records) of 10 replays of the captured
   step; every launch is classified into its family by kernel name (the census regexes of
   scripts/family_table.py), the family's device time per step is its summed kernel durations
   / 10, and ``achieved`` = its algorithmic work per step (floor.step_work) / that time.  This
   is the figure the committed ``profiles/*_family_table.md`` tables give for the same tree.
1. ``measure_gemm_family`` -- kept as ``roofline.reissue``: the DOMINANT family of the CMX-B2 step by device time (the census
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


# kernel-name -> family of the step census (the regexes of scripts/family_table.py; first match wins,
# so the grouped weight-gradient launch is not counted as a tile GEMM)
FAMILY_RE = (
    ("wgrad", r"gemm_grouped_kernel|reduce_grouped_kernel"),
    ("gemm", r"gemm_bf16_kernel|gemm_stream|gemm_multi|gemm_generic|splitk_reduce"),
    ("sra", r"sra_"),
    ("dwconv", r"dw2_|dw_"),
    ("layernorm", r"ln_fwd|ln_bwd|rowln"),
    ("adamw", r"adamw"),
    ("batchnorm", r"bn_"),
    ("frm", r"pool_|linear_fwd|linear_bwd|combine_|frm_|reduce_partials"),
    ("ffm", r"ffm_"),
    ("ce", r"ce_|upsample"),
    ("bilinear", r"bilinear|adj3_|up3_"),
    ("im2col", r"im2col|col2im"),
    ("pe1", r"pe1_"),
)


def family_of(kernel: str) -> str:
    import re
    for fam, rx in FAMILY_RE:
        if re.search(rx, kernel):
            return fam
    return "other"


def trace_kernels(run_step, steps: int):
    """Kernel records [(name, start_us, duration_us)] of ``steps`` calls of ``run_step`` (graph
    replays), from the in-process kineto / roctracer activity trace (the same dispatch
    timestamps a ``rocprofv3 --kernel-trace`` run reports).  [] when the tracer delivers none."""
    from torch.profiler import profile, ProfilerActivity
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(steps):
            run_step()
        torch.cuda.synchronize()
    out = []
    for e in prof.profiler.kineto_results.events():
        if e.device_type() != torch.autograd.DeviceType.CUDA:
            continue
        name = e.name()
        if "Memcpy" in name or "Memset" in name:
            continue
        out.append((name, e.start_ns() / 1e3, e.duration_ns() / 1e3))
    out.sort(key=lambda r: r[1])
    return out


# the first kernel of every training step (the DropPath / Dropout2d mask draw): step boundary
STEP_FIRST = "step_masks_kernel"


def split_steps(recs):
    """The traced kernels cut into steps at each STEP_FIRST launch; only COMPLETE steps are kept
    (the activity tracer can drop records: a step is complete when it holds the largest launch
    count seen, the count of the captured graph).  Returns a list of per-step record lists."""
    idx = [i for i, r in enumerate(recs) if STEP_FIRST in r[0]]
    if not idx:
        return []
    segs = [recs[a:b] for a, b in zip(idx, idx[1:] + [len(recs)])]
    full = max(len(sg) for sg in segs)
    return [sg for sg in segs if len(sg) == full]


def measure_in_step(run_step, workload: str, shape: dict, n_params: float, steps: int = 10,
                    step_us: float | None = None):
    """The step's kernel families from a kernel trace of ``steps`` graph replays: device time and
    launches per step of each family, against its algorithmic work (floor.step_work: FLOPs and
    bytes, each tensor read once and written once).  ``roofline`` is the dominant family by time:
    ``achieved`` = its algorithmic bytes (HBM-bound) or FLOPs per step / its in-step kernel time
    -- the time those launches take inside the replayed step, next to their neighbours, not
    re-issued in isolation.

    step_us (the untraced, timed step): each family's time is its share of the traced kernel
    time x step_us.  Under torch.profiler the summed kernel durations run ~10 % above the
    rocprofv3 kernel trace of the same tree (busy / wall 1.10 against 0.98 at round 6: the
    activity records stretch overlapping kernels), while the families' shares agree to < 1 %;
    the profiled sums are kept as ``profiled_us_per_step``."""
    recs = trace_kernels(run_step, steps)
    if not recs:
        return None, None
    segs = split_steps(recs)
    if segs:                         # complete steps only
        recs = [r for sg in segs for r in sg]
        steps = len(segs)
    work = step_work(n_params=n_params, **shape)
    fams = {}
    for name, _, us in recs:
        f = fams.setdefault(family_of(name), [0.0, 0])
        f[0] += us
        f[1] += 1
    busy = sum(v[0] for v in fams.values()) / steps
    # seconds per step of a family: its traced share of the step's kernel time x the timed step
    scale = (step_us / busy) if step_us else 1.0

    def fam_s(us_total):
        return us_total / steps * scale * 1e-6

    table = {}
    for fam, (us, n) in sorted(fams.items(), key=lambda kv: -kv[1][0]):
        t = fam_s(us)
        fl, by = work[fam] if fam in work else (0.0, 0.0)
        row = {"us_per_step": round(t * 1e6, 1), "profiled_us_per_step": round(us / steps, 1),
               "launches_per_step": round(n / steps, 1), "share_of_busy": round(us / steps / busy, 4)}
        if by:
            row.update({"alg_gb": round(by / 1e9, 4), "tbs": round(by / t / 1e12, 3),
                        "hbm_frac": round(by / t / (PEAK_HBM_GBS * 1e9), 4)})
        if fl:
            row.update({"alg_gflop": round(fl / 1e9, 2), "mfma_frac": round(fl / t / (PEAK_BF16_TFLOPS * 1e12), 4)})
        table[fam] = row
    dom = max((f for f in fams if f in work and work[f][1] > 0), key=lambda f: fams[f][0])
    us, n = fams[dom]
    t = fam_s(us)
    nl = n / steps
    flops, nbytes = work[dom]
    hbm = flops / nbytes < RIDGE_FLOP_PER_BYTE
    gbs, tflops = nbytes / t / 1e9, flops / t / 1e12
    kern = {"gemm": ("gemm_bf16_kernel", "gemm_stream_kernel", "gemm_multi_kernel", "splitk_reduce_kernel"),
            "wgrad": ("gemm_grouped_kernel",)}.get(dom, ())
    traffic, src = _family_traffic(kern, workload) if kern else (None, None)
    roof = {"kernel": f"{dom} family in the replayed step ({nl:.0f} launches per step; kernel trace of {steps} "
                      f"HIP-graph replays)",
            "family": dom, "bound": "hbm" if hbm else "mfma",
            "achieved": round(gbs, 1) if hbm else round(tflops, 2),
            "peak": PEAK_HBM_GBS if hbm else PEAK_BF16_TFLOPS,
            "unit": "GB/s" if hbm else "TFLOP/s",
            "frac": round(gbs / PEAK_HBM_GBS if hbm else tflops / PEAK_BF16_TFLOPS, 4),
            "traffic": traffic,
            "arithmetic_intensity_flop_per_byte": round(flops / nbytes, 1),
            "ridge_flop_per_byte": round(RIDGE_FLOP_PER_BYTE, 1),
            "achieved_tflops": round(tflops, 2), "mfma_frac": round(tflops / PEAK_BF16_TFLOPS, 4),
            "achieved_hbm_gbs": round(gbs, 1), "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
            "launches": round(nl, 1), "avg_launch_us": round(t / nl * 1e6, 2), "total_us": round(t * 1e6, 1),
            "algorithmic_flop_per_launch": flops / nl, "algorithmic_bytes_per_launch": nbytes / nl,
            "algorithmic_bytes_per_step": nbytes, "workload": workload,
            "timing": f"in-step: kernel durations of {steps} complete replayed steps (torch.profiler / roctracer "
                      f"activity records, steps cut at {STEP_FIRST}), summed per family and divided by {steps}"
                      + (f"; the family's share of that kernel time x the timed step ({step_us:.0f} us)"
                         if step_us else "")}
    if src:
        roof["traffic_source"] = src
        roof["traffic_over_algorithmic"] = round(traffic / (nbytes / nl), 3)
    walls = [sg[-1][1] + sg[-1][2] - sg[0][1] for sg in segs] if segs else []
    if step_us:
        roof["profiled_us"] = round(us / steps, 1)
    return roof, {"busy_us_per_step": round(busy, 1), "launches_per_step": round(len(recs) / steps, 1),
                  "complete_steps_traced": steps if segs else None,
                  "wall_us_per_step_median": round(sorted(walls)[len(walls) // 2], 1) if walls else None,
                  "families": table}


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
