"""Op-level parity of the HIP kernels against fp64 PyTorch CPU restatements of the
reference ops (each test cites the reference op it checks).  Tolerances: fp32 mode
1e-4 relative to max |ref|; bf16 mode 3e-2 (bf16 storage, fp32 accumulate)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 1e-4, torch.bfloat16: 3e-2}
DTYPES = [torch.float32, torch.bfloat16]


def relerr(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("C,eps", [(32, 1e-6), (64, 1e-6), (160, 1e-5), (320, 1e-6), (512, 1e-5)])
def test_layernorm(dev, dtype, C, eps):
    from rgbx_semantic_segmentation_amd import kernels as K
    torch.manual_seed(0)
    G, R = 2, 777
    x = (torch.randn(G, R, C, dtype=torch.float64) * 2 + 0.5)
    g = torch.randn(G, C, dtype=torch.float64)
    b = torch.randn(G, C, dtype=torch.float64)
    dy = torch.randn(G, R, C, dtype=torch.float64)
    xr = x.clone().requires_grad_(True); gr = g.clone().requires_grad_(True); br = b.clone().requires_grad_(True)
    yr = torch.stack([torch.nn.functional.layer_norm(xr[i], (C,), gr[i], br[i], eps) for i in range(G)])
    yr.backward(dy)
    xd = x.to(dev, dtype)
    y, mu, rs = K.layernorm_fwd(xd, g.float().to(dev), b.float().to(dev), eps, G=G)
    assert relerr(y, yr) < TOL[dtype]
    dg = torch.empty(G, C, device=dev); db = torch.empty(G, C, device=dev)
    dx = K.layernorm_bwd(dy.to(dev, dtype), xd, g.float().to(dev), mu, rs, G, dg, db)
    assert relerr(dx, xr.grad) < TOL[dtype] * 3
    assert relerr(dg, gr.grad) < TOL[dtype] * 3
    assert relerr(db, br.grad) < TOL[dtype] * 3


def sra_ref(q, kv, heads, D):
    """Attention core of dual_segformer.py:125-134 on token-major tensors (fp64)."""
    Bt, N, C = q.shape
    Nk = kv.shape[1]
    qh = q.view(Bt, N, heads, D).transpose(1, 2)
    kvh = kv.view(Bt, Nk, 2, heads, D).permute(2, 0, 3, 1, 4)
    a = ((qh @ kvh[0].transpose(-2, -1)) * D ** -0.5).softmax(-1)
    return (a @ kvh[1]).transpose(1, 2).reshape(Bt, N, C)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("Bt,N,Nk,heads,D", [(4, 19200 // 16, 300, 1, 64), (2, 333, 70, 2, 32),
                                              (4, 300, 300, 8, 64), (2, 1200, 300, 5, 64),
                                              (1, 65, 80, 8, 32)])
def test_sra_attention(dev, dtype, Bt, N, Nk, heads, D):
    from rgbx_semantic_segmentation_amd import kernels as K
    torch.manual_seed(1)
    C = heads * D
    q = torch.randn(Bt, N, C, dtype=torch.float64)
    kv = torch.randn(Bt, Nk, 2 * C, dtype=torch.float64)
    do = torch.randn(Bt, N, C, dtype=torch.float64)
    qr = q.clone().requires_grad_(True); kvr = kv.clone().requires_grad_(True)
    o_ref = sra_ref(qr, kvr, heads, D)
    o_ref.backward(do)
    qd = q.to(dev, dtype); kvd = kv.to(dev, dtype).contiguous()
    o, lse = K.sra_attn_fwd(qd, kvd, kvd[..., C:], Bt, N, Nk, heads, D, D ** -0.5, C, 2 * C)
    torch.cuda.synchronize()
    assert relerr(o, o_ref) < TOL[dtype], relerr(o, o_ref)
    dq, dkv = K.sra_attn_bwd(qd, kvd, kvd[..., C:], o, do.to(dev, dtype), lse, Bt, N, Nk, heads, D,
                             D ** -0.5, C, 2 * C)
    torch.cuda.synchronize()
    assert relerr(dq, qr.grad) < TOL[dtype] * 2, relerr(dq, qr.grad)
    assert relerr(dkv[..., :C], kvr.grad[..., :C]) < TOL[dtype] * 2, relerr(dkv[..., :C], kvr.grad[..., :C])
    assert relerr(dkv[..., C:], kvr.grad[..., C:]) < TOL[dtype] * 2, relerr(dkv[..., C:], kvr.grad[..., C:])


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("B,h,w,K", [(2, 120, 160, 40), (1, 15, 20, 9), (2, 16, 24, 19)])
@pytest.mark.parametrize("fused", [True, False])
def test_upsample_ce(dev, dtype, B, h, w, K, fused):
    """Final x4 bilinear upsample + CrossEntropyLoss(mean, ignore_index=255) (builder.py:233,249;
    train.py:72-73): loss and d logits against torch fp64 autograd.  fused=True: loss-only
    forward + tile-recomputing backward (ce_fused.hip); False: the materialised-gradient path
    (forced by a non-x4 output size)."""
    import torch.nn.functional as Fn
    from rgbx_semantic_segmentation_amd.functions import UpsampleCEF
    torch.manual_seed(7)
    H, W = (4 * h, 4 * w) if fused else (4 * h - 2, 4 * w + 3)
    lg = torch.randn(B, h, w, K, dtype=torch.float64) * 3
    lab = torch.randint(0, K, (B, H, W))
    lab[:, 5:30, 7:40] = 255
    ref = lg.clone().requires_grad_(True)
    up = Fn.interpolate(ref.permute(0, 3, 1, 2), size=(H, W), mode="bilinear", align_corners=False)
    loss_ref = Fn.cross_entropy(up, lab, reduction="mean", ignore_index=255)
    (loss_ref * 0.7).backward()
    x = lg.to(dev, dtype).requires_grad_(True)
    loss = UpsampleCEF.apply(x, lab.to(dev), (B, h, w, H, W, K), 255)
    (loss * 0.7).backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref.item()) / loss_ref.item() < (1e-5 if dtype == torch.float32 else 1e-2)
    assert relerr(x.grad, ref.grad) < TOL[dtype] * 2, relerr(x.grad, ref.grad)
