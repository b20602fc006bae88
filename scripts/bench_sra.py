"""Time the SRA attention kernels at the CMX-B2 480x640 bs=2 stage shapes (both streams,
Bt = 4) with HIP events; prints per-stage fwd / bwd microseconds and TFLOP/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rgbx_semantic_segmentation_amd import kernels as K  # noqa: E402


def t(fn, iters=20):
    """GPU time per call: `iters` calls captured in one HIP graph (no host launch cost)."""
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
    Bt, D, Nk = 4, 64, 300
    tot_f = tot_b = 0.0
    stages = ((19200, 1, 3), (4800, 2, 4), (1200, 5, 6), (300, 8, 3))
    if len(sys.argv) > 2 and sys.argv[1] == "stage":          # one stage (for a rocprofv3 per-kernel split)
        stages = (stages[int(sys.argv[2]) - 1],)
    for N, heads, depth in stages:
        C = heads * D
        q = torch.randn(Bt, N, C, device="cuda").bfloat16()
        kv = torch.randn(Bt, Nk, 2 * C, device="cuda").bfloat16()
        do = torch.randn(Bt, N, C, device="cuda").bfloat16()
        o, lse = K.sra_attn_fwd(q, kv, kv[..., C:], Bt, N, Nk, heads, D, D ** -0.5, C, 2 * C)
        tf = t(lambda: K.sra_attn_fwd(q, kv, kv[..., C:], Bt, N, Nk, heads, D, D ** -0.5, C, 2 * C))
        tb = t(lambda: K.sra_attn_bwd(q, kv, kv[..., C:], o, do, lse, Bt, N, Nk, heads, D, D ** -0.5, C, 2 * C))
        fl = 4.0 * Bt * heads * N * Nk * D
        print(f"N={N:6d} h={heads}: fwd {tf:7.1f} us ({fl / tf / 1e6:6.1f} TF/s)  bwd {tb:7.1f} us "
              f"({2.5 * fl / tb / 1e6:6.1f} TF/s)")
        tot_f += depth * tf
        tot_b += depth * tb
    print(f"per step (x depth): fwd {tot_f:.0f} us, bwd {tot_b:.0f} us")




def sweep():
    Bt, D = 4, 64
    for N, heads in ((300, 8), (19200, 1)):
        for Nk in (32, 64, 128, 300):
            C = heads * D
            q = torch.randn(Bt, N, C, device="cuda").bfloat16()
            kv = torch.randn(Bt, Nk, 2 * C, device="cuda").bfloat16()
            tf = t(lambda: K.sra_attn_fwd(q, kv, kv[..., C:], Bt, N, Nk, heads, D, D ** -0.5, C, 2 * C))
            print(f"sweep N={N} h={heads} Nk={Nk}: fwd {tf:.1f} us")
    x = torch.empty(1, device="cuda")
    print(f"empty fill: {t(lambda: x.fill_(1.0)):.1f} us")


def nw_sweep():
    """SRA_NW / SRA_QW launch-shape A/B, interleaved in one process (cmx_tune)."""
    from rgbx_semantic_segmentation_amd import _lib
    for qw, nw in ((0, 0), (1, 8), (1, 10), (1, 4), (2, 8), (1, 2)):
        _lib.call("cmx_tune", b"SRA_QW", qw)
        _lib.call("cmx_tune", b"SRA_NW", nw)
        print(f"--- SRA_QW={qw} SRA_NW={nw}")
        main()


if len(sys.argv) > 1 and sys.argv[1] == "sweep":
    sweep()
elif len(sys.argv) > 1 and sys.argv[1] == "nw":
    nw_sweep()
elif __name__ == "__main__":     # all stages, or `stage S`
    main()
