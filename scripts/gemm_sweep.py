"""Per-launch cost model of the bf16 GEMM: time one shape family while sweeping K (slope = cost
of one 64-deep k-step of the pipeline, intercept = fixed cost: dispatch, first DMA latency,
epilogue), beside an empty-kernel graph node.  Each time is one launch inside a HIP graph of
`iters` back-to-back launches.  Usage (GPU box): python scripts/gemm_sweep.py"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rgbx_semantic_segmentation_amd import kernels as K  # noqa: E402


def timeit(fn, iters=50, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def case(G, M, N, Kd, tB, **kw):
    A = torch.randn(G, M, Kd, device="cuda").to(torch.bfloat16)
    if tB:      # dgrad orientation: B(j, k) = W[k][j]
        B = torch.randn(G, Kd, N, device="cuda").to(torch.bfloat16).transpose(1, 2)
    else:
        B = torch.randn(G, N, Kd, device="cuda").to(torch.bfloat16)
    C = torch.empty(G, M, N, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(G, N, device="cuda") if kw.pop("bias", False) else None
    return timeit(lambda: K.gemm(A, B, C, bias=bias, **kw))


def main():
    z = torch.zeros(1, device="cuda")
    print(f"empty fill_ node: {timeit(lambda: z.zero_()):.2f} us")
    for (G, M, N, tB) in [(2, 600, 512, 1), (2, 600, 512, 0), (2, 2400, 320, 0), (2, 2400, 320, 1),
                          (2, 9600, 128, 0), (2, 38400, 64, 0), (2, 38400, 256, 0)]:
        row = []
        for Kd in (64, 128, 256, 512, 1024, 2048):
            row.append(f"K{Kd}:{case(G, M, N, Kd, tB):6.2f}")
        print(f"G{G} M{M:5d} N{N:4d} tB{tB}  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
