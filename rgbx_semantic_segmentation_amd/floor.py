"""Algorithmic work of the CMX training step AS EXECUTED here, per kernel family, and the
step's roofline floor.

Per family: FLOPs (2 x MAC of the products the kernels run: the decoder fuse after the exact
commute, the FFM per-head d x d contexts) and ALGORITHMIC HBM bytes (every tensor a kernel of
the family reads once plus every tensor it writes once, at its storage dtype: 16-bit
activations / GEMM weight shadows, fp32 master weights / gradients / statistics, int64
labels).  The floor is sum over families of max(flops / 2516.6 TFLOP/s, bytes / 8 TB/s)
(MI355X_MICROARCH.md dense bf16 MFMA, HBM); ``step_frac_of_floor`` in the bench line is that
floor over the measured step time.  Conventions follow the launches of functions.py (e.g.
LayerNorm backward reads dy + dy2 + x and writes dx + the DropPath-scaled tap, DWConv saves
act'(z)).  The whole-step FLOP count of the BENCH line's step_mfma_roofline stays the
reference's op-by-op count (flops.py)."""
from __future__ import annotations

import collections

from .models.encoders.dual_segformer import MIT_SPECS, NUM_HEADS, SR_RATIOS

PEAK_TFLOPS = 2516.6
PEAK_TBS = 8.0
A = 2                      # bytes per 16-bit activation / GEMM operand
F32 = 4


def _grid(H, W, k, s, p):
    return (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1


def step_work(backbone="mit_b2", H=480, W=640, B=2, K=40, E=512, n_params=None):
    """{family: [flops, bytes]} for one training step (forward + backward + AdamW) of one rank."""
    fam = collections.defaultdict(lambda: [0.0, 0.0])

    def add(f, flops=0.0, byts=0.0):
        fam[f][0] += flops
        fam[f][1] += byts

    def gemm(M, N, Kd, G=1, res=False, wgrad=True, dgrad=True, bias_grad=True):
        # forward y = x W^T (+ residual), dgrad dx = dy W, wgrad dW = dy^T x (fp32 out)
        add("gemm", 2 * G * M * N * Kd, G * A * (M * Kd + N * Kd + M * N + (M * N if res else 0)))
        if dgrad:
            add("gemm", 2 * G * M * N * Kd, G * A * (M * N + N * Kd + M * Kd))
        if wgrad:
            add("wgrad", 2 * G * M * N * Kd, G * (A * (M * N + M * Kd) + F32 * N * (Kd + (1 if bias_grad else 0))))

    def ln(rows, C, G=1, two=False, tap=False):
        add("layernorm", 0, G * A * rows * C * 2 + G * F32 * 2 * rows)                 # fwd: x -> y, mean / rstd
        add("layernorm", 0, G * A * rows * C * (3 + (1 if two else 0) + (1 if tap else 0)) + G * F32 * 2 * rows)

    def dw(M_pix, C, G=1):
        add("dwconv", 2 * 9 * G * M_pix * C * 3, G * A * M_pix * C * 3)              # fwd: h -> out, act'
        add("dwconv", 0, G * A * M_pix * C * 4)                                      # bwd: da, act', h -> dh

    def bn(M, C, res=False):
        add("batchnorm", 0, A * M * C * (1 + 2 + (1 if res else 0)))                  # stats + apply
        add("batchnorm", 0, A * M * C * (2 + 3 + (2 if res else 0) + (1 if res else 0)))   # reduce + apply

    dims, depths = MIT_SPECS[backbone]["embed_dims"], MIT_SPECS[backbone]["depths"]
    G = 2
    h, w, cin = H, W, 3
    grids = []
    for s in range(4):
        k, st = (7, 4) if s == 0 else (3, 2)
        h, w = _grid(h, w, k, st, k // 2)
        N, C = h * w, dims[s]
        M = B * N
        grids.append((h, w, C))
        # patch embed: stage 1 direct conv on the fp32 NCHW images (fwd; wgrad re-reads the
        # images and dy, one (C, Kp + 1) fp32 result); 3x3 s2 implicit conv
        if s == 0:
            Kp = (cin * k * k + 7) // 8 * 8
            img = F32 * B * cin * H * W
            add("pe1", 2 * G * M * C * cin * k * k, G * (img + A * C * Kp + A * M * C))
            add("pe1", 2 * G * M * C * cin * k * k, G * (img + A * M * C + F32 * C * (Kp + 1)))
        else:
            gemm(M, C, cin * k * k, G)
            add("im2col", 0, G * A * M * cin * k * k * 2)                             # col2im of the dgrad columns
        ln(M, C, G)
        R = SR_RATIOS[s]
        hk, wk = _grid(h, w, R, R, 0) if R > 1 else (h, w)
        Nk = hk * wk
        Mk = B * Nk
        for _ in range(depths[s]):
            ln(M, C, G, two=R > 1, tap=True)                                          # norm1 (+ residual tap)
            gemm(M, C, C, G)                                                          # q
            if R > 1:
                gemm(Mk, C, R * R * C, G)                                             # SR conv (implicit / patch dgrad)
                ln(Mk, C, G)
            gemm(Mk, 2 * C, C, G)                                                     # kv
            d = C // NUM_HEADS[s]
            fwd_f = 4 * G * B * N * Nk * C
            add("sra", fwd_f, G * A * (M * C + Mk * 2 * C + M * C) + G * F32 * B * NUM_HEADS[s] * N)
            add("sra", 2.5 * fwd_f, G * A * (3 * M * C + Mk * 2 * C + M * C + Mk * 2 * C) + G * F32 * B * NUM_HEADS[s] * N * 2)
            gemm(M, C, C, G, res=True)                                                # proj + residual
            ln(M, C, G, tap=True)                                                     # norm2
            gemm(M, 4 * C, C, G)                                                      # fc1
            dw(M, 4 * C, G)
            gemm(M, C, 4 * C, G, res=True)                                            # fc2 + residual
        ln(M, C, G, tap=True)                                                         # stage norm
        # CM-FRM: pool, channel MLP (fp32 weights), spatial 2C -> C GEMM, combine, backward
        add("frm", 0, G * A * M * C)                                                  # pool
        add("frm", 2 * 2 * B * (16 * C * C + 8 * C * C), F32 * 3 * (16 * C * C + 8 * C * C))   # MLP fwd + bwd (W, dW)
        gemm(M, C, 2 * C, 1)
        add("frm", 0, A * M * C * (G + 1 + G))                                        # combine fwd: x, h -> out
        add("frm", 0, A * M * C * (G + G + 1 + G + 1) + A * M * C * G * 2)            # combine bwd + pool bwd (RMW)
        # FFM: CrossPath (channel_proj, kv, per-head contexts, end_proj + residual) + ChannelEmbed
        d = C // NUM_HEADS[s]
        gemm(M, 2 * C, C, G)                                                          # channel_proj (ReLU)
        gemm(M, 2 * C, C, G, bias_grad=False)                                         # kv on u
        add("ffm", 2 * G * B * NUM_HEADS[s] * N * d * d * 2 * 3,
            G * A * (M * 2 * C + M * C * 2) * 3)                                      # k^T v, u ctx (+ bwd)
        gemm(M, C, 2 * C, G, res=True)                                                # end_proj + residual
        gemm(M, C, 2 * C, 1, bias_grad=False)                                         # ChannelEmbed.residual
        gemm(M, C, 2 * C, 1)                                                          # channel_embed[0]
        dw(M, C, 1)
        gemm(M, C, C, 1)                                                              # channel_embed[3]
        bn(M, C)
        bn(M, C, res=True)
        cin = C
    # decoder: linear_c1..4 at their own resolution, the fuse (c1 product + low-res products +
    # bilinear adds in the epilogue; adjoints in the backward), BN (+ReLU, Dropout2d), linear_pred
    h1, w1, _ = grids[0]
    N1 = B * h1 * w1
    for (hh, ww, C) in grids:
        gemm(B * hh * ww, E, C, 1)
    for (hh, ww, C) in grids[1:]:
        gemm(B * hh * ww, E, E, 1, bias_grad=False)
        add("bilinear", 0, A * (B * hh * ww * E + N1 * E) * 2)                       # fwd add (read) + adjoint
    gemm(N1, E, E, 1)
    bn(N1, E)
    gemm(N1, K, E, 1)
    # upsample x4 + CE (fused): low-res logits + int64 labels; backward writes the low-res gradient
    add("ce", 0, A * N1 * K * 3 + 8 * B * H * W * 2)
    if n_params:
        add("adamw", 0, n_params * 30)
    return fam


def floor_table(**kw):
    """[(family, flops, bytes, floor_us, bound)] and the total floor in us."""
    rows, tot = [], 0.0
    for f, (fl, by) in sorted(step_work(**kw).items(), key=lambda kv: -max(kv[1][0] / PEAK_TFLOPS / 1e6,
                                                                            kv[1][1] / PEAK_TBS / 1e6)):
        tf, tb = fl / (PEAK_TFLOPS * 1e6), by / (PEAK_TBS * 1e6)
        rows.append((f, fl, by, max(tf, tb), "mfma" if tf > tb else "hbm"))
        tot += max(tf, tb)
    return rows, tot


if __name__ == "__main__":
    rows, tot = floor_table(n_params=66.58e6)
    for f, fl, by, us, bd in rows:
        print(f"{f:10s} {fl / 1e9:9.1f} GFLOP {by / 1e9:8.3f} GB  floor {us:8.1f} us ({bd})")
    print(f"step floor {tot:.0f} us")
