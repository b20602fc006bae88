"""Mix-FFN band kernels (csrc/mixffn.hip) against the separate launches they replace.

Forward (cmx_mixffn_fwd): h = fc1(x) against cmx_gemm (bit for bit where the separate GEMM runs
the same one-group k-loop: grids above 512 tiles, every B2 / B4 stage-3/4 shape), and a / act'(z)
against cmx_dwconv3x3_fwd_save run on the band kernel's own h -- bit for bit (same taps, same
order, same rounding points).  Backward (cmx_mixffn_bwd): dh against fc2's dgrad (cmx_gemm) +
cmx_dwconv3x3_bwd_saved (bit for bit where the dgrad GEMM is one-group), the DW weight / bias
gradient partials summed against that kernel's (fp32, summation order differs: 1e-5).
Reference: dual_segformer.py:27-33,67-74 (Mlp: fc1 -> DWConv 3x3 -> GELU -> fc2)."""
import math

import pytest
import torch

from rgbx_semantic_segmentation_amd import kernels as K

pytestmark = pytest.mark.gpu

# (G, images per group, H, W, C, hidden): B2 / B4 480x640 stages 3 and 4, B0 stage 4, B5 1024^2
# stage 4, and a ragged band count
SHAPES = [(2, 2, 30, 40, 320, 1280), (2, 2, 15, 20, 512, 2048), (2, 4, 30, 40, 320, 1280), (2, 1, 8, 10, 256, 1024),
          (2, 1, 32, 32, 512, 2048), (1, 3, 17, 24, 128, 512),
          # 2-D tiles (cmx_mixffn_mode 2): B2 480 x 640 stages 1 / 2, B0 stage 1, a ragged wide image
          (2, 2, 120, 160, 64, 256), (2, 2, 60, 80, 128, 512), (2, 1, 60, 80, 32, 256), (1, 3, 37, 50, 64, 256)]


def _setup(G, B, H, W, C, Ch, dtype, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    M = B * H * W
    x = torch.randn(G, M, C, device="cuda", generator=g).to(dtype)
    W1 = (torch.randn(G, Ch, C, device="cuda", generator=g) / math.sqrt(C)).to(dtype)
    b1 = torch.randn(G, Ch, device="cuda", generator=g) * 0.1
    wdw = torch.randn(G, Ch, 9, device="cuda", generator=g) * 0.3
    bdw = torch.randn(G, Ch, device="cuda", generator=g) * 0.1
    W2 = (torch.randn(G, C, Ch, device="cuda", generator=g) / math.sqrt(Ch)).to(dtype)
    dz2 = torch.randn(G, M, C, device="cuda", generator=g).to(dtype)
    return x, W1, b1, wdw, bdw, W2, dz2


def _one_group_gemm(G, M, N, K_):
    """the separate cmx_gemm runs the plain one-group k-loop (no k-group split) for this shape"""
    return G * math.ceil(M / 64) * math.ceil(N / 64) > 512 or math.ceil(K_ / 64) < 4


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("G,B,H,W,C,Ch", SHAPES)
def test_mixffn_fwd(dev, G, B, H, W, C, Ch, dtype):
    x, W1, b1, wdw, bdw, _, _ = _setup(G, B, H, W, C, Ch, dtype)
    M = B * H * W
    h, gp, a = (torch.empty(G, M, Ch, device="cuda", dtype=dtype) for _ in range(3))
    K.call("cmx_mixffn_fwd", K.ptr(x), K.ptr(W1), K.ptr(b1), K.ptr(wdw), K.ptr(bdw), K.ptr(h), K.ptr(gp), K.ptr(a),
           G, B, H, W, C, Ch, W1.stride(0), b1.stride(0), wdw.stride(0), K.dtype_code(x), K.stream())
    h0 = torch.empty_like(h)
    K.gemm(x, W1, h0, bias=b1)
    a0, g0 = torch.empty_like(h), torch.empty_like(h)
    K.call("cmx_dwconv3x3_fwd_save", K.ptr(h), K.ptr(wdw), K.ptr(bdw), K.ptr(a0), K.ptr(g0), G * B, B, H, W, Ch,
           K.ACT["gelu"], K.dtype_code(h), K.stream())
    torch.cuda.synchronize()
    if _one_group_gemm(G, M, Ch, C):
        assert torch.equal(h, h0), (h.float() - h0.float()).abs().max().item()
    else:
        assert ((h.float() - h0.float()).abs().max() / h0.float().abs().max()).item() < 1e-2
    assert torch.equal(a, a0), (a.float() - a0.float()).abs().max().item()
    assert torch.equal(gp, g0), (gp.float() - g0.float()).abs().max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("G,B,H,W,C,Ch", SHAPES)
def test_mixffn_bwd(dev, G, B, H, W, C, Ch, dtype):
    x, W1, b1, wdw, bdw, W2, dz2 = _setup(G, B, H, W, C, Ch, dtype, seed=1)
    M = B * H * W
    h, gp, a = (torch.empty(G, M, Ch, device="cuda", dtype=dtype) for _ in range(3))
    K.call("cmx_mixffn_fwd", K.ptr(x), K.ptr(W1), K.ptr(b1), K.ptr(wdw), K.ptr(bdw), K.ptr(h), K.ptr(gp), K.ptr(a),
           G, B, H, W, C, Ch, W1.stride(0), b1.stride(0), wdw.stride(0), K.dtype_code(x), K.stream())
    dh = torch.empty_like(h)
    nb = K.query("cmx_mixffn_bwd_workspace", G, B, H, W, Ch)
    ws = torch.empty(nb // 4, device="cuda")
    K.call("cmx_mixffn_bwd", K.ptr(dz2), K.ptr(W2), K.ptr(wdw), K.ptr(h), K.ptr(gp), K.ptr(dh), K.ptr(ws), G, B, H, W,
           C, Ch, W2.stride(0), wdw.stride(0), K.dtype_code(h), K.stream())
    # the separate launches: da = dz2 W2 (fc2's dgrad), then the saved-act DW backward
    da = torch.empty_like(h)
    K.gemm(dz2, W2.transpose(1, 2), da)
    dh0 = torch.empty_like(h)
    nb0 = K.query("cmx_dwconv3x3_bwd_workspace", G * B, B, H, W, Ch)
    ws0 = torch.empty(nb0 // 4, device="cuda")
    K.call("cmx_dwconv3x3_bwd_saved", K.ptr(da), K.ptr(h), K.ptr(gp), K.ptr(wdw), K.ptr(dh0), 0, 0, K.ptr(ws0),
           G * B, B, H, W, Ch, 0, K.dtype_code(h), K.stream())
    torch.cuda.synchronize()
    if _one_group_gemm(G, M, Ch, C):
        assert torch.equal(dh, dh0), (dh.float() - dh0.float()).abs().max().item()
    else:
        assert ((dh.float() - dh0.float()).abs().max() / dh0.float().abs().max()).item() < 2e-2
    P = nb // (40 * G * Ch)
    P0 = K.query("cmx_dwconv3x3_bwd_saved_tiles", B, H, W)
    s = ws[:G * P * Ch * 10].view(G, P, Ch, 10).double().sum(1)
    s0 = ws0[:G * P0 * Ch * 10].view(G, P0, Ch, 10).double().sum(1)
    tol = 1e-5 if _one_group_gemm(G, M, Ch, C) else 2e-2
    assert ((s - s0).abs().max() / s0.abs().max()).item() < tol
