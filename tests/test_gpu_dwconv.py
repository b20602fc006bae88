"""cmx_dwconv3x3_fwd / _bwd (csrc/dwconv.hip) against a plain PyTorch fp32 reference of the
same op: depthwise Conv2d(C, C, 3, 1, 1, groups=C) + bias + act on NHWC tokens, per modality
group weights (dual_segformer.py:27-33 DWConv + GELU; net_utils.py:315-318 DW + ReLU).

Covers the LDS-tiled path (C % 32 == 0: 32- and 64-channel blocks, tiles ragged in H and W,
fused backward with dz kept on chip) and the strip path (C = 36), both dtypes and every
activation.  Tolerances: fp32 1e-5 relative (dW sums over up to 2x2x30x44 pixels), bf16
2e-2 relative (bf16 storage of out / dh)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30)).item()


def ref_dw(h, w, b, act, G, B, H, W):
    """h (G*B, H*W, C) -> act(dwconv(h) + b) in the same layout, fp32 autograd."""
    C = h.shape[-1]
    outs = []
    for g in range(G):
        x = h[g * B:(g + 1) * B].view(B, H, W, C).permute(0, 3, 1, 2)
        y = F.conv2d(x, w[g].view(C, 1, 3, 3), b[g], padding=1, groups=C)
        y = {"none": y, "gelu": F.gelu(y), "relu": F.relu(y)}[act]
        outs.append(y.permute(0, 2, 3, 1).reshape(B, H * W, C))
    return torch.cat(outs)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C,H,W", [(64, 30, 44), (256, 17, 16), (160, 9, 33), (320, 8, 10), (36, 12, 12)])
@pytest.mark.parametrize("act", ["gelu", "relu", "none"])
def test_dwconv_fwd_bwd(dev, dtype, C, H, W, act):
    from rgbx_semantic_segmentation_amd import kernels as Kn
    torch.manual_seed(0)
    G, B = 2, 2
    NI = G * B
    h = torch.randn(NI, H * W, C, device="cuda")
    w = torch.randn(G, C, 9, device="cuda") * 0.3
    b = torch.randn(G, C, device="cuda") * 0.1
    da = torch.randn(NI, H * W, C, device="cuda")
    hq, daq = h.to(dtype), da.to(dtype)
    hr = hq.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    out_ref = ref_dw(hr, wr, br, act, G, B, H, W)
    out_ref.backward(daq.float())
    out = torch.empty_like(hq)
    Kn.call("cmx_dwconv3x3_fwd", Kn.ptr(hq), Kn.ptr(w), Kn.ptr(b), Kn.ptr(out), NI, B, H, W, C, Kn.ACT[act],
            Kn.dtype_code(hq), Kn.stream())
    dz = torch.empty_like(hq)
    dh = torch.empty_like(hq)
    dw = torch.empty(G, C, 9, device="cuda")
    db = torch.empty(G, C, device="cuda")
    ws = Kn._ws(Kn.query("cmx_dwconv3x3_bwd_workspace", NI, B, H, W, C), h.device)
    Kn.call("cmx_dwconv3x3_bwd", Kn.ptr(daq), Kn.ptr(hq), Kn.ptr(w), Kn.ptr(b), Kn.ptr(dz), Kn.ptr(dh), Kn.ptr(dw),
            Kn.ptr(db), Kn.ptr(ws), NI, B, H, W, C, Kn.ACT[act], 0, Kn.dtype_code(hq), Kn.stream())
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel(out, out_ref) < tol
    assert rel(dh, hr.grad) < tol
    assert rel(dw, wr.grad) < (tol if dtype == torch.float32 else 1e-2)
    assert rel(db, br.grad) < (tol if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype,C,H,W", [(torch.float16, 64, 30, 44), (torch.float16, 512, 15, 20),
                                         (torch.bfloat16, 64, 30, 44), (torch.bfloat16, 256, 17, 16),
                                         (torch.bfloat16, 320, 9, 33), (torch.bfloat16, 512, 15, 20),
                                         (torch.float32, 32, 8, 10), (torch.float32, 160, 9, 33),
                                         (torch.float32, 64, 30, 44)])
@pytest.mark.parametrize("act", ["gelu", "relu"])
def test_dwconv_fwd_save_bwd_saved(dev, dtype, C, H, W, act):
    """The training path: forward saves act'(z); the backward forms dz = da * act'(z) and the
    transposed conv and dW / db from one LDS image (tiles ragged in H and W)."""
    from rgbx_semantic_segmentation_amd import kernels as Kn
    torch.manual_seed(1)
    G, B = 2, 2
    NI = G * B
    h = torch.randn(NI, H * W, C, device="cuda")
    w = torch.randn(G, C, 9, device="cuda") * 0.3
    b = torch.randn(G, C, device="cuda") * 0.1
    da = torch.randn(NI, H * W, C, device="cuda")
    hq, daq = h.to(dtype), da.to(dtype)
    hr = hq.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    out_ref = ref_dw(hr, wr, br, act, G, B, H, W)
    out_ref.backward(daq.float())
    out = torch.empty_like(hq)
    gp = torch.empty_like(hq)
    Kn.call("cmx_dwconv3x3_fwd_save", Kn.ptr(hq), Kn.ptr(w), Kn.ptr(b), Kn.ptr(out), Kn.ptr(gp), NI, B, H, W, C,
            Kn.ACT[act], Kn.dtype_code(hq), Kn.stream())
    dh = torch.empty_like(hq)
    dw = torch.empty(G, C, 9, device="cuda")
    db = torch.empty(G, C, device="cuda")
    ws = Kn._ws(Kn.query("cmx_dwconv3x3_bwd_workspace", NI, B, H, W, C), h.device)
    Kn.call("cmx_dwconv3x3_bwd_saved", Kn.ptr(daq), Kn.ptr(hq), Kn.ptr(gp), Kn.ptr(w), Kn.ptr(dh), Kn.ptr(dw),
            Kn.ptr(db), Kn.ptr(ws), NI, B, H, W, C, 0, Kn.dtype_code(hq), Kn.stream())
    torch.cuda.synchronize()
    # dz = da * act'(z) is rounded to the storage dtype once (as the reference's autograd
    # under autocast stores it): bf16 2e-2 relative, fp32 1e-5
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel(out, out_ref) < tol
    assert rel(dh, hr.grad) < tol
    assert rel(dw, wr.grad) < (tol if dtype == torch.float32 else 1e-2)
    assert rel(db, br.grad) < (tol if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("C,H,W", [(64, 30, 44), (256, 17, 16), (512, 15, 20)])
def test_dwconvf_deferred_reduce_matches_immediate(dev, C, H, W):
    """functions.DWConvF backward with the deferred grouped reduce (deferred.py, the step's
    path) against the immediate reduce, on tiles ragged in H and W: the grouped reduce reads
    P = cmx_dwconv3x3_bwd_saved_tiles partial slabs of the shared workspace."""
    from rgbx_semantic_segmentation_amd import deferred
    from rgbx_semantic_segmentation_amd import functions as Fn
    torch.manual_seed(2)
    G, B = 2, 2
    NI = G * B
    h = torch.randn(NI, H * W, C, device="cuda").to(torch.bfloat16)
    w = torch.randn(G, C, 9, device="cuda") * 0.3
    b = torch.randn(G, C, device="cuda") * 0.1
    da = torch.randn(NI, H * W, C, device="cuda").to(torch.bfloat16)
    anchor = torch.nn.Parameter(torch.zeros(1, device="cuda"))
    res = {}
    saved = deferred.ENABLED
    try:
        for mode in (False, True):
            deferred.ENABLED = mode
            wg = torch.full((G, C, 9), float("nan"), device="cuda")
            bg = torch.full((G, C), float("nan"), device="cuda")
            hx = h.clone().requires_grad_(True)
            out = Fn.DWConvF.apply(hx, w, b, wg, bg, NI, B, H, W, "gelu", anchor)
            out.backward(da)
            deferred.flush()
            torch.cuda.synchronize()
            res[mode] = (hx.grad.float(), wg.clone(), bg.clone())
    finally:
        deferred.ENABLED = saved
    for a, c in zip(res[False], res[True]):
        assert torch.isfinite(c).all()
        assert rel(c, a) < 1e-6, rel(c, a)
