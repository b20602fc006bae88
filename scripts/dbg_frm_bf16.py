"""Step through FRMF.backward in both dtypes on identical inputs / weights and compare every intermediate."""
import torch, sys
sys.path.insert(0, ".")
from oracle import cmx_ref as R
from rgbx_semantic_segmentation_amd.models.net_utils import FeatureRectifyModule
from rgbx_semantic_segmentation_amd.params import ParamStore
from rgbx_semantic_segmentation_amd import functions as F, deferred
from rgbx_semantic_segmentation_amd import kernels as K
C, B, H, W = 32, 2, 32, 40
N = H * W
torch.manual_seed(0)
ref = R.FeatureRectifyModule(C); ref.apply(R.segformer_init)
g0 = torch.Generator().manual_seed(1)
x = torch.randn(2, B, N, C, generator=g0).to(torch.bfloat16)
dout_all = torch.randn(2, B, N, C, generator=g0).to(torch.bfloat16)
res = {}
for cdt in (torch.float32, torch.bfloat16):
    prod = FeatureRectifyModule(C); prod.load_state_dict(ref.state_dict())
    store = ParamStore(prod, "cuda", cdt)
    r = x.to(cdt).cuda()
    cwm, swm = prod.channel_weights.mlp, prod.spatial_weights.mlp
    f32 = lambda p: store.w(p, stacked=False, compute=False)
    cmp = lambda p: store.w(p, stacked=False)
    W1, b1, W2, b2, W0, b0, w2s, b2s = (f32(cwm[0].weight), f32(cwm[0].bias), f32(cwm[2].weight), f32(cwm[2].bias),
                                        cmp(swm[0].weight).view(C, 2 * C), f32(swm[0].bias), f32(swm[2].weight).view(2, C), f32(swm[2].bias))
    dt = K.dtype_code(r)
    st = {}
    pooled = torch.empty(B, 4 * C, device="cuda"); argmax = torch.empty(B, 2 * C, dtype=torch.int32, device="cuda")
    ws = K._ws(K.query("cmx_frm_pool_workspace", B, N, C), "cuda")
    K.call("cmx_frm_pool_fwd", K.ptr(r), K.ptr(pooled), K.ptr(argmax), K.ptr(ws), 0, B, N, C, dt, K.stream())
    y1 = torch.empty(B, 4 * C, device="cuda")
    K.call("cmx_small_linear_fwd", K.ptr(pooled), K.ptr(W1), K.ptr(b1), K.ptr(y1), B, 4 * C, 4 * C, 2, K.stream())
    cw = torch.empty(B, 2 * C, device="cuda")
    K.call("cmx_small_linear_fwd", K.ptr(y1), K.ptr(W2), K.ptr(b2), K.ptr(cw), B, 4 * C, 2 * C, 3, K.stream())
    h = torch.empty(1, B * N, C, dtype=r.dtype, device="cuda")
    K.gemm(r[0].view(1, B * N, C), W0[None], h, bias=b0[None], A2=r[1].view(1, B * N, C))
    h = h[0]
    sw = torch.empty(B * N, 2, device="cuda"); out = torch.empty_like(r)
    K.call("cmx_frm_combine_fwd", K.ptr(r), K.ptr(cw), K.ptr(h), K.ptr(w2s), K.ptr(b2s), K.ptr(sw), K.ptr(out), B, N, C, dt, K.stream())
    st.update(pooled=pooled.clone(), y1=y1.clone(), cw=cw.clone(), h=h.clone(), sw=sw.clone(), out=out.clone())
    dout = dout_all.to(cdt).cuda()
    dx = torch.empty_like(r); dh = torch.empty_like(h)
    nb = K.query("cmx_frm_combine_bwd_nblk", N, C, dt)
    ws = K._ws(K.query("cmx_frm_combine_bwd_workspace", B, N, C, dt), "cuda")
    K.call("cmx_frm_combine_bwd", K.ptr(dout), 0, K.ptr(r), K.ptr(cw), K.ptr(sw), K.ptr(h), K.ptr(w2s), K.ptr(dx), K.ptr(dh), K.ptr(ws), B, N, C, dt, K.stream())
    torch.cuda.synchronize(); st.update(dx_direct=dx.clone(), dh=dh.clone(), pcw=ws[:B * nb * 2 * C].clone())
    Wd = W0.view(C, 2, C).permute(1, 0, 2); dx2 = dx.view(2, B * N, C)
    K.gemm(dh[None].expand(2, B * N, C), Wd.transpose(1, 2), dx2, residual=dx2)
    torch.cuda.synchronize(); st.update(dx_gemm=dx.clone())
    ns = K.query("cmx_small_linear_nslice")
    gW1 = torch.empty_like(W1); gb1 = torch.empty_like(b1); gW2 = torch.empty_like(W2); gb2 = torch.empty_like(b2)
    dy1p = torch.empty(ns, B, 4 * C, device="cuda")
    K.call("cmx_small_linear_bwd", K.ptr(ws), nb, 2 * C, nb * 2 * C, K.ptr(cw), K.ptr(y1), K.ptr(W2), K.ptr(dy1p), K.ptr(gW2), K.ptr(gb2), B, 4 * C, 2 * C, 3, 0, K.stream())
    dpp = torch.empty(ns, B, 4 * C, device="cuda")
    K.call("cmx_small_linear_bwd", K.ptr(dy1p), ns, B * 4 * C, 4 * C, K.ptr(y1), K.ptr(pooled), K.ptr(W1), K.ptr(dpp), K.ptr(gW1), K.ptr(gb1), B, 4 * C, 4 * C, 2, 0, K.stream())
    torch.cuda.synchronize(); st.update(dy1=dy1p.sum(0), dp=dpp.sum(0), gW2=gW2.clone(), gW1=gW1.clone())
    K.call("cmx_frm_pool_bwd", K.ptr(dpp), ns, B * 4 * C, K.ptr(argmax), K.ptr(dx), B, N, C, dt, K.stream())
    torch.cuda.synchronize(); st.update(dx_final=dx.clone(), argmax=argmax.clone())
    res[cdt] = st
a, b = res[torch.bfloat16], res[torch.float32]
for k in a:
    u, v = a[k].double(), b[k].double()
    e = ((u - v).abs().max() / v.abs().max().clamp_min(1e-30)).item()
    extra = ""
    if k == "argmax":
        extra = f" mismatches {int((a[k] != b[k]).sum())}"
    print(f"{k:10s} {e:.3e}{extra}")
