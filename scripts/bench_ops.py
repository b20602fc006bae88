"""Standalone timings of single kernels at the CMX-B2 480x640 bs=2 shapes (HIP events over
many back-to-back launches on one stream), for iterating on one kernel without the step's
run-to-run scheduling noise.  Usage: python scripts/bench_ops.py [name ...]"""
import sys

import torch

sys.path.insert(0, ".")
from rgbx_semantic_segmentation_amd import kernels as K  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def ce():
    B, h, w, Kc = 2, 120, 160, 40
    H, W = 4 * h, 4 * w
    logits = torch.randn(B, h * w, Kc, device="cuda").to(torch.bfloat16)
    label = torch.randint(0, Kc, (B, H, W), device="cuda")
    label[:, :20, :20] = 255
    out = torch.empty(3, device="cuda")
    ws = K._ws(K.query("cmx_upsample_ce_workspace", B, H, W), "cuda")
    fwd = lambda: K.call("cmx_upsample_ce_fwd", K.ptr(logits), K.ptr(label), 0, K.ptr(out), K.ptr(ws), B, h, w, H, W,
                         Kc, 255, 1, K.stream())
    dloss = torch.ones(1, device="cuda")
    dl = torch.empty_like(logits)
    fwd()
    bwd = lambda: K.call("cmx_upsample_ce_bwd", K.ptr(logits), K.ptr(label), K.ptr(dloss), K.ptr(out), K.ptr(dl), B, h,
                         w, H, W, Kc, 255, 1, K.stream())
    adj = torch.empty(B, h * w, Kc, device="cuda")
    fwd_adj = lambda: K.call("cmx_upsample_ce_fwd_adj", K.ptr(logits), K.ptr(label), K.ptr(adj), K.ptr(out), K.ptr(ws),
                             B, h, w, H, W, Kc, 255, 1, K.stream())
    scale = lambda: K.call("cmx_upsample_ce_bwd_scale", K.ptr(adj), K.ptr(dloss), K.ptr(out), K.ptr(dl), dl.numel(), 1,
                           K.stream())
    return {"ce_fwd (loss only)": timeit(fwd), "ce_bwd (recompute)": timeit(bwd), "ce_fwd_adj (training)": timeit(fwd_adj),
            "ce_bwd_scale (training)": timeit(scale)}


def decoder():
    """The decoder fold's full-resolution passes at the B2 shapes: the upsample-sum (up3) + the c1
    residual GEMM against the c1 GEMM with the upsample in its epilogue, and the 3-grid adjoint
    against three 2-pass adjoints."""
    from rgbx_semantic_segmentation_amd import functions as F
    B, H, W, E = 2, 120, 160, 512
    grids = [(15, 20), (30, 40), (60, 80)]
    bf = torch.bfloat16
    zs = [torch.randn(1, B * h * w, E, device="cuda").to(bf) for (h, w) in grids]
    bias = torch.randn(E, device="cuda")
    x1 = torch.randn(1, B * H * W, 64, device="cuda").to(bf)
    M1 = torch.randn(1, E, 64, device="cuda").to(bf)
    U = torch.empty(1, B * H * W, E, device="cuda").to(bf)
    Z = torch.empty(1, B * H * W, E, device="cuda").to(bf)
    g = [v for hw in grids for v in hw]
    up3 = lambda: K.call("cmx_bilinear_up3_add", *[K.ptr(z) for z in zs], B, *g, K.ptr(bias), K.ptr(U), H, W, E, 1,
                         K.stream())
    res = lambda: K.gemm(x1, M1, Z, residual=U)
    epi = lambda: K.call("cmx_decoder_fuse_fwd", K.ptr(x1), K.ptr(M1), K.ptr(Z), K.ptr(bias), *[K.ptr(z) for z in zs],
                         B, H, W, *g, E, 64, 64, 64, 1, K.stream())
    dZ = torch.randn(1, B * H * W, E, device="cuda").to(bf)
    ys = [torch.empty(1, B * h * w, E, device="cuda").to(bf) for (h, w) in grids]
    ts = [torch.empty(B * H * w * E, device="cuda") for (h, w) in grids]
    adj3 = lambda: K.call("cmx_bilinear_adjoint3", K.ptr(dZ), *[K.ptr(t) for t in ts], *[K.ptr(y) for y in ys], B, H,
                          W, *g, E, 1, K.stream())
    adj1 = lambda: [F._adjoint_to(dZ, B, H, W, h, w, E) for (h, w) in grids]
    return {"up3_add": timeit(up3), "c1 residual gemm": timeit(res), "c1 gemm + upsample epilogue": timeit(epi),
            "adjoint3 (x + y)": timeit(adj3), "3 x adjoint_to (6 launches)": timeit(adj1)}


def bnsmall():
    """ChannelEmbed-sized BatchNorms (stage 3: 2400 x 320 ReLU, stage 4: 600 x 512 with residual):
    the one-launch small-map forms against stats + fold + apply / reduce + fold + apply."""
    out = {}
    for M, C, act, use_res in ((2400, 320, 2, False), (600, 512, 0, True)):
        x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        res = torch.randn(M, C, device="cuda").to(torch.bfloat16) if use_res else None
        g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        mean, invstd = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        sums = torch.empty(2, C, dtype=torch.float64, device="cuda")
        ws = torch.empty(max(1, K.query("cmx_bn_workspace", M, C) // 8), dtype=torch.float64, device="cuda")
        y, dx = torch.empty_like(x), torch.empty_like(x)
        dres = torch.empty_like(x) if use_res else None
        gg, gb = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        rps = M // 2

        def multi_f():
            K.call("cmx_bn_stats_finalize", K.ptr(x), K.ptr(sums), K.ptr(ws), M, C, 1e-5, 0.1, K.ptr(rm), K.ptr(rv),
                   K.ptr(mean), K.ptr(invstd), 1, K.stream())
            K.call("cmx_bn_apply", K.ptr(x), K.ptr(mean), K.ptr(invstd), K.ptr(g), K.ptr(b), K.ptr(res), 0, K.ptr(y),
                   M, C, rps, act, 1, K.stream())

        def multi_b():
            K.call("cmx_bn_bwd_reduce", K.ptr(dy), K.ptr(x), K.ptr(mean), K.ptr(invstd), K.ptr(g), K.ptr(b),
                   K.ptr(res), 0, K.ptr(sums), K.ptr(gg), K.ptr(gb), K.ptr(ws), M, C, rps, act, 0, 1, K.stream())
            K.call("cmx_bn_bwd_apply", K.ptr(dy), K.ptr(x), K.ptr(mean), K.ptr(invstd), K.ptr(g), K.ptr(b),
                   K.ptr(res), 0, K.ptr(sums), float(M), K.ptr(dx), K.ptr(dres), M, C, rps, act, 1, 1, K.stream())
        small_f = lambda: K.call("cmx_bn_small_fwd", K.ptr(x), K.ptr(res), K.ptr(g), K.ptr(b), 0, K.ptr(y), K.ptr(sums),
                                 K.ptr(mean), K.ptr(invstd), K.ptr(rm), K.ptr(rv), M, C, rps, act, 1e-5, 0.1, 1,
                                 K.stream())
        small_b = lambda: K.call("cmx_bn_small_bwd", K.ptr(dy), K.ptr(x), K.ptr(mean), K.ptr(invstd), K.ptr(g),
                                 K.ptr(b), K.ptr(res), 0, K.ptr(gg), K.ptr(gb), K.ptr(dx), K.ptr(dres), M, C, rps, act,
                                 0, 1, K.stream())
        for n, f in (("multi fwd", multi_f), ("small fwd", small_f), ("multi bwd", multi_b), ("small bwd", small_b)):
            out[f"bn {M}x{C} {n}"] = timeit(f)
    return out


def bn():
    res = {}
    for M, C in [(38400, 512), (2400, 320), (600, 512), (38400, 64)]:
        x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        mean = torch.zeros(C, device="cuda")
        invstd = torch.ones(C, device="cuda")
        gamma = torch.ones(C, device="cuda")
        beta = torch.zeros(C, device="cuda")
        sums = torch.empty(2, C, dtype=torch.float64, device="cuda")
        dg = torch.empty(C, device="cuda")
        db = torch.empty(C, device="cuda")
        for cap in (256, 512, 1024):
            K.tune("BN_NBLK", cap)
            ws = torch.empty(max(1, K.query("cmx_bn_workspace", M, C) // 8), dtype=torch.float64, device="cuda")
            f = lambda: K.call("cmx_bn_bwd_reduce", K.ptr(dy), K.ptr(x), K.ptr(mean), K.ptr(invstd), K.ptr(gamma),
                               K.ptr(beta), 0, 0, K.ptr(sums), K.ptr(dg), K.ptr(db), K.ptr(ws), M, C, 1, 0, 0, 1,
                               K.stream())
            fs = lambda: K.call("cmx_bn_stats", K.ptr(x), K.ptr(sums), K.ptr(ws), M, C, 1, K.stream())
            res[f"bn_bwd_reduce {M}x{C} nblk<={cap}"] = timeit(f)
            res[f"bn_stats {M}x{C} nblk<={cap}"] = timeit(fs)
        K.tune("BN_NBLK", 256)
    return res


if __name__ == "__main__":
    want = sys.argv[1:] or ["ce", "bn", "decoder"]
    for name in want:
        for k, v in globals()[name]().items():
            print(f"{k:32s} {v:8.2f} us")
