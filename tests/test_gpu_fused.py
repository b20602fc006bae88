"""Fused kernels of round 2 against plain PyTorch fp32 references of the same ops.

* functions.DecoderFuseF (cmx_decoder_fuse_fwd + low-resolution branch GEMMs + bilinear
  adjoints): DecoderHead's upsample + concat + linear_fuse 1x1 conv (MLPDecoder.py:66-77) with
  the conv commuted ahead of the upsample -- forward and every input / weight / bias gradient.
* functions.DecoderFoldF (linear_c{1..4} folded into linear_fuse, decoder_fold.hip): the whole
  decode head up to the fuse conv against linear -> upsample -> concat -> conv in fp32.
* cmx_conv_patch_dgrad: dx of the SRA spatial-reduction conv (kernel = stride = R, pad 0,
  dual_segformer.py:95-96) with the col2im folded into the GEMM epilogue, incl. grids that R
  does not divide (the remainder pixels get zero gradient, as torch's conv backward gives).
Tolerances: fp32 1e-5 relative; bf16 2e-2 (bf16 storage of the low-resolution products and
of the outputs)."""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H1,W1,E", [(2, 120, 160, 64), (1, 32, 40, 128), (2, 30, 17, 32)])
def test_decoder_fuse_matches_upsample_concat_conv(dev, dtype, B, H1, W1, E):
    from rgbx_semantic_segmentation_amd import deferred
    from rgbx_semantic_segmentation_amd import functions as Fn
    torch.manual_seed(0)
    grids = [(H1, W1), ((H1 + 1) // 2, (W1 + 1) // 2), ((H1 + 3) // 4, (W1 + 3) // 4), ((H1 + 7) // 8, (W1 + 7) // 8)]
    es = [torch.randn(B, h * w, E, device=dev) for (h, w) in grids]           # e1, e2, e3, e4
    Wf = torch.randn(1, E, 4 * E, device=dev) * (4 * E) ** -0.5
    bf = torch.randn(1, E, device=dev) * 0.1
    dZ = torch.randn(B * H1 * W1, E, device=dev)
    # reference: up(e4), up(e3), up(e2), e1 concatenated -> 1x1 conv (fp32 autograd on the rounded inputs)
    er = [e.to(dtype).float().requires_grad_(True) for e in es]
    Wr = Wf.to(dtype).float().requires_grad_(True)
    br = bf.clone().requires_grad_(True)

    def nchw(e, hw):
        return e.view(B, hw[0], hw[1], E).permute(0, 3, 1, 2)
    ups = [TF.interpolate(nchw(er[i], grids[i]), size=(H1, W1), mode="bilinear", align_corners=False)
           for i in (3, 2, 1)]
    cat = torch.cat(ups + [nchw(er[0], grids[0])], 1)
    Zr = TF.conv2d(cat, Wr[0].view(E, 4 * E, 1, 1), br[0]).permute(0, 2, 3, 1).reshape(B * H1 * W1, E)
    Zr.backward(dZ.to(dtype).float())
    # product
    eq = [e.to(dtype).requires_grad_(True) for e in es]
    Wq = Wf.to(dtype)
    Wg = torch.zeros(1, E, 4 * E, device=dev)
    bg = torch.zeros(1, E, device=dev)
    anchor = torch.nn.Parameter(torch.zeros(1, device=dev))
    Z = Fn.DecoderFuseF.apply(eq[3], eq[2], eq[1], eq[0], Wq, Wg, bf, bg, grids, anchor)
    Z.backward(dZ.to(dtype))
    deferred.flush()
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel(Z, Zr) < tol, rel(Z, Zr)
    for i in range(4):
        assert rel(eq[i].grad, er[i].grad) < tol, (i, rel(eq[i].grad, er[i].grad))
    assert rel(Wg, Wr.grad) < tol, rel(Wg, Wr.grad)
    assert rel(bg, br.grad) < tol, rel(bg, br.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H1,W1,E,Cs", [(2, 120, 160, 512, (64, 128, 320, 512)), (1, 32, 40, 128, (32, 64, 160, 256)),
                                          (2, 30, 17, 64, (32, 64, 160, 256)), (2, 30, 17, 128, (32, 64, 160, 256))])
def test_decoder_fold_matches_mlp_upsample_concat_conv(dev, dtype, B, H1, W1, E, Cs):
    """functions.DecoderFoldF against the reference decode head's op sequence in fp32
    (MLPDecoder.py:60-77: linear_c{1..4} -> upsample -> concat c4, c3, c2, c1 -> 1x1 conv):
    the output, the four feature gradients and the gradients of all ten weights and biases
    (the chain-rule terms run after deferred.flush, as in the step)."""
    from rgbx_semantic_segmentation_amd import deferred
    from rgbx_semantic_segmentation_amd import functions as Fn
    torch.manual_seed(0)
    grids = [(H1, W1), ((H1 + 1) // 2, (W1 + 1) // 2), ((H1 + 3) // 4, (W1 + 3) // 4), ((H1 + 7) // 8, (W1 + 7) // 8)]
    xs = [torch.randn(B, h * w, C, device=dev) for (h, w), C in zip(grids, Cs)]      # x1..x4
    Wcs = [torch.randn(E, C, device=dev) * C ** -0.5 for C in Cs]
    bcs = [torch.randn(E, device=dev) * 0.1 for _ in Cs]
    Wf = torch.randn(E, 4 * E, device=dev) * (4 * E) ** -0.5
    bf = torch.randn(E, device=dev) * 0.1
    dZ = torch.randn(B * H1 * W1, E, device=dev)
    xr = [x.to(dtype).float().requires_grad_(True) for x in xs]
    Wcr = [w.to(dtype).float().requires_grad_(True) for w in Wcs]
    bcr = [b.clone().requires_grad_(True) for b in bcs]
    Wr = Wf.to(dtype).float().requires_grad_(True)
    br = bf.clone().requires_grad_(True)

    def nchw(e, hw):
        return e.view(B, hw[0], hw[1], E).permute(0, 3, 1, 2)
    cs = [xr[i] @ Wcr[i].t() + bcr[i] for i in range(4)]
    ups = [TF.interpolate(nchw(cs[i], grids[i]), size=(H1, W1), mode="bilinear", align_corners=False)
           for i in (3, 2, 1)]
    cat = torch.cat(ups + [nchw(cs[0], grids[0])], 1)
    Zr = TF.conv2d(cat, Wr.view(E, 4 * E, 1, 1), br).permute(0, 2, 3, 1).reshape(B * H1 * W1, E)
    Zr.backward(dZ.to(dtype).float())
    # product (slot order c4, c3, c2, c1)
    xq = [x.to(dtype).requires_grad_(True) for x in xs]
    order = (3, 2, 1, 0)
    Wq = Wf.to(dtype)
    Wcq = tuple(Wcs[i].to(dtype) for i in order)
    Wfg = torch.full((1, E, 4 * E), float("nan"), device=dev)
    bfg = torch.full((E,), float("nan"), device=dev)
    Wcg = [torch.full((1, E, C), float("nan"), device=dev) for C in Cs]
    bcg = [torch.full((E,), float("nan"), device=dev) for _ in Cs]
    grads = (Wfg, bfg, tuple(Wcg[i] for i in order), tuple(bcg[i] for i in order))
    anchor = torch.nn.Parameter(torch.zeros(1, device=dev))
    Z = Fn.DecoderFoldF.apply(xq[3], xq[2], xq[1], xq[0], Wq, Wcq, bf, tuple(bcs[i] for i in order), grads, grids,
                              anchor)
    Z.backward(dZ.to(dtype))
    deferred.flush()
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel(Z, Zr) < tol, rel(Z, Zr)
    for i in range(4):
        assert rel(xq[i].grad, xr[i].grad) < tol, (i, rel(xq[i].grad, xr[i].grad))
        assert rel(Wcg[i][0], Wcr[i].grad) < tol, (i, rel(Wcg[i][0], Wcr[i].grad))
        assert rel(bcg[i], bcr[i].grad) < tol, (i, rel(bcg[i], bcr[i].grad))
    assert rel(Wfg[0], Wr.grad) < tol, rel(Wfg[0], Wr.grad)
    assert rel(bfg, br.grad) < tol, rel(bfg, br.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,W,C", [(2, 120, 160, 512), (1, 30, 17, 128), (2, 64, 64, 256)])
def test_bilinear_up3_and_adjoint3(dev, dtype, B, H, W, C):
    """cmx_bilinear_up3_add (bias + the sum of three bilinear upsamples, MLPDecoder.py:67-73) and
    cmx_bilinear_adjoint3 (its backward to the three grids from one read of dZ) against
    F.interpolate and its autograd adjoint in fp32, incl. non-integer scale factors."""
    from rgbx_semantic_segmentation_amd import kernels as K
    torch.manual_seed(3)
    grids = [((H + 7) // 8, (W + 7) // 8), ((H + 3) // 4, (W + 3) // 4), ((H + 1) // 2, (W + 1) // 2)]
    zs = [torch.randn(B, h, w, C, device=dev).to(dtype) for (h, w) in grids]
    bias = torch.randn(C, device=dev)
    U = torch.empty(B, H, W, C, dtype=dtype, device=dev)
    K.call("cmx_bilinear_up3_add", *[K.ptr(z) for z in zs], B, *[v for g in grids for v in g], K.ptr(bias), K.ptr(U),
           H, W, C, K.dtype_code(U), K.stream())
    zr = [z.float().permute(0, 3, 1, 2).requires_grad_(True) for z in zs]
    Ur = bias.view(1, C, 1, 1) + sum(TF.interpolate(z, size=(H, W), mode="bilinear", align_corners=False) for z in zr)
    dZ = torch.randn(B, H, W, C, device=dev).to(dtype)
    Ur.backward(dZ.float().permute(0, 3, 1, 2))
    ys = [torch.empty(B, h, w, C, dtype=dtype, device=dev) for (h, w) in grids]
    ts = [torch.empty(B * H * w * C, device=dev) for (h, w) in grids]
    K.call("cmx_bilinear_adjoint3", K.ptr(dZ), *[K.ptr(t) for t in ts], *[K.ptr(y) for y in ys], B, H, W,
           *[v for g in grids for v in g], C, K.dtype_code(dZ), K.stream())
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(U, Ur.detach().permute(0, 2, 3, 1)) < tol, rel(U, Ur.detach().permute(0, 2, 3, 1))
    for y, z in zip(ys, zr):
        ref = z.grad.permute(0, 2, 3, 1)
        assert rel(y, ref) < tol, rel(y, ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("NI,G,H,W,C,R,N", [(4, 2, 120, 160, 64, 8, 64), (4, 2, 60, 80, 128, 4, 128),
                                            (2, 2, 30, 40, 320, 2, 320), (2, 1, 60, 81, 32, 8, 32),
                                            (4, 2, 13, 9, 64, 2, 64)])
def test_conv_patch_dgrad_matches_conv_backward(dev, dtype, NI, G, H, W, C, R, N):
    from rgbx_semantic_segmentation_amd import kernels as Kn
    torch.manual_seed(1)
    Ho, Wo = H // R, W // R
    NIg = NI // G
    Wt = torch.randn(G, N, R, R, C, device=dev) * (R * R * C) ** -0.5          # tap-major storage
    dy = torch.randn(G, NIg * Ho * Wo, N, device=dev)
    Wq, dyq = Wt.to(dtype), dy.to(dtype)
    ref = []
    for g in range(G):
        w = Wq[g].float().permute(0, 3, 1, 2)                                     # (N, C, R, R)
        d = dyq[g].float().view(NIg, Ho, Wo, N).permute(0, 3, 1, 2)
        ref.append(torch.nn.grad.conv2d_input((NIg, C, H, W), w, d, stride=R).permute(0, 2, 3, 1))
    ref = torch.cat(ref)
    exact = H % R == 0 and W % R == 0
    dx = (torch.empty if exact else torch.zeros)(NI, H, W, C, dtype=dtype, device=dev)
    Kn.call("cmx_conv_patch_dgrad", Kn.ptr(dyq), Kn.ptr(Wq), Kn.ptr(dx), G, NIg, H, W, C, R, Ho, Wo, N,
            dyq.stride(0), Wq.stride(0), NIg * H * W * C, Kn.dtype_code(dyq), Kn.stream())
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(dx, ref) < tol, rel(dx, ref)
