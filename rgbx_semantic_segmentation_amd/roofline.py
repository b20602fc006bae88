"""Roofline of the dominant kernel, measured live with HIP events on the launch stream.

achieved = algorithmic work of ONE launch (SURVEY.md §8(d) counting) / average launch
duration; the kernel is re-launched standalone on the exact shapes it has in the step
(inputs resident in HBM), bracketed by torch.cuda.Event on torch's current stream (the
stream the C-ABI launches on)."""
from __future__ import annotations

import torch

from . import kernels as K

PEAK_BF16_TFLOPS = 2516.6
PEAK_HBM_GBS = 8000.0


def _time(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def measure_sra_fwd(Bt=4, N=19200, Nk=300, heads=1, D=64, dtype=torch.bfloat16):
    """Stage-1 SRA attention forward of CMX-B2 at 480x640, bs=2 (both streams: Bt = 2*2)."""
    C = heads * D
    q = torch.randn(Bt, N, C, device="cuda", dtype=dtype)
    kv = torch.randn(Bt, Nk, 2 * C, device="cuda", dtype=dtype)
    t = _time(lambda: K.sra_attn_fwd(q, kv, kv[..., C:], Bt, N, Nk, heads, D, D ** -0.5, C, 2 * C))
    flops = 4.0 * Bt * heads * N * Nk * D          # QK^T + PV
    return {"kernel": "sra_fwd_kernel<bf16,64> (stage-1 SRA attention fwd, Bt=4 N=19200 Nk=300 d=64)",
            "bound": "mfma", "achieved": round(flops / t / 1e12, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(flops / t / 1e12 / PEAK_BF16_TFLOPS, 4), "traffic": None,
            "avg_launch_us": round(t * 1e6, 2), "algorithmic_per_launch": flops}


def measure_dominant(args):
    return measure_sra_fwd()
