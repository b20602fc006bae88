"""Per-launch floor of dependent kernels inside a HIP graph on MI355X (what a step of ~800
small launches pays before any work): graphs of L back-to-back launches of a trivial kernel
(cmx_cast_f32_bf16) on one stream, on two independent streams, and at several grid sizes.
Usage (GPU box): python scripts/launch_floor.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rgbx_semantic_segmentation_amd import _lib  # noqa: E402


def graph_time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    L = 400
    for n in (8 * 256, 8 * 256 * 256, 8 * 256 * 2048):
        src = torch.randn(n, device=dev)
        dst = torch.empty(n, dtype=torch.bfloat16, device=dev)

        def one():
            for _ in range(L):
                _lib.call("cmx_cast_f32_bf16", src.data_ptr(), dst.data_ptr(), n, _lib.stream())
        t = graph_time(one)
        blocks = max(1, min(8192, n // 256))
        print(f"1 stream : {L} launches of {blocks:5d} blocks: {t / L:6.2f} us per launch")

        side = torch.cuda.Stream()
        src2 = torch.randn(n, device=dev)
        dst2 = torch.empty(n, dtype=torch.bfloat16, device=dev)

        def two():
            side.wait_stream(torch.cuda.current_stream())
            for _ in range(L // 2):
                _lib.call("cmx_cast_f32_bf16", src.data_ptr(), dst.data_ptr(), n, _lib.stream())
            with torch.cuda.stream(side):
                for _ in range(L // 2):
                    _lib.call("cmx_cast_f32_bf16", src2.data_ptr(), dst2.data_ptr(), n, _lib.stream())
            torch.cuda.current_stream().wait_stream(side)
        t2 = graph_time(two)
        print(f"2 streams: {L} launches of {blocks:5d} blocks: {t2 / L:6.2f} us per launch (wall / launches)")


if __name__ == "__main__":
    main()
