"""Standalone DWConv timing at the B2 480x640 bs=2 shapes (G=2 streams): fwd_save and
bwd_saved, HIP-event timed over graph-captured repeats, with algorithmic GB/s.
Usage (GPU box): python scripts/bench_dw.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rgbx_semantic_segmentation_amd import kernels as Kn  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
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


def main():
    G, B = 2, 2
    for (H, W, C) in [(120, 160, 256), (60, 80, 512), (30, 40, 1280), (15, 20, 2048)]:
        NI = G * B
        h = torch.randn(NI, H * W, C, device="cuda").bfloat16()
        w = torch.randn(G, C, 9, device="cuda") * 0.3
        b = torch.randn(G, C, device="cuda") * 0.1
        out, gp, da, dh = (torch.empty_like(h) for _ in range(4))
        da.normal_()
        ws = Kn._ws(Kn.query("cmx_dwconv3x3_bwd_workspace", NI, B, H, W, C), h.device)
        dw = torch.empty(G, C, 9, device="cuda")
        db = torch.empty(G, C, device="cuda")
        ACT = Kn.ACT["gelu"]

        def fwd():
            Kn.call("cmx_dwconv3x3_fwd_save", Kn.ptr(h), Kn.ptr(w), Kn.ptr(b), Kn.ptr(out), Kn.ptr(gp), NI, B, H, W,
                    C, ACT, 1, Kn.stream())

        def bwd():
            Kn.call("cmx_dwconv3x3_bwd_saved", Kn.ptr(da), Kn.ptr(h), Kn.ptr(gp), Kn.ptr(w), Kn.ptr(dh), Kn.ptr(dw),
                    Kn.ptr(db), Kn.ptr(ws), NI, B, H, W, C, 0, 1, Kn.stream())
        tf, tb = timeit(fwd), timeit(bwd)
        nb = h.numel() * 2
        print(f"H{H} W{W} C{C}: fwd_save {tf:7.1f} us {3 * nb / tf / 1e3:6.0f} GB/s   "
              f"bwd_saved(+reduce) {tb:7.1f} us {4 * nb / tb / 1e3:6.0f} GB/s  (tensor {nb / 1e6:.1f} MB)")


if __name__ == "__main__":
    main()
