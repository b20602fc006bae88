"""CrossAttentionF (MFMA GEMM cross attention) against an fp64 torch restatement of
CrossAttention.forward (net_utils.py:199-214), forward and backward, per shape."""
import sys
import torch
sys.path.insert(0, ".")
from rgbx_semantic_segmentation_amd.functions import CrossAttentionF


def ref(u, kv, B, N, heads, D):
    G, M, C = u.shape
    s = D ** -0.5
    k, v = kv[..., :C], kv[..., C:]
    sh = lambda t: t.reshape(G, B, N, heads, D).permute(0, 1, 3, 2, 4)      # G B h N D
    q, k, v = sh(u), sh(k), sh(v)
    ctx = (k.transpose(-1, -2) @ v * s).softmax(dim=-2)                       # G B h D D
    out = q @ ctx.flip(0)
    return out.permute(0, 1, 3, 2, 4).reshape(G, M, C)


for C, heads, B, H, W in [(32, 1, 2, 32, 40), (160, 5, 2, 8, 10), (320, 5, 2, 30, 40), (512, 8, 2, 15, 20),
                          (320, 5, 2, 8, 10), (320, 5, 1, 30, 40), (128, 2, 2, 30, 40)]:
    for dt in (torch.float32, torch.bfloat16):
        torch.manual_seed(0)
        N = H * W
        D = C // heads
        u = torch.randn(2, B * N, C).to(dt).double().requires_grad_(True)
        kv = torch.randn(2, B * N, 2 * C).to(dt).double().requires_grad_(True)
        w = torch.randn(2, B * N, C).to(dt).double()
        o = ref(u, kv, B, N, heads, D)
        (o * w).sum().backward()
        ug = u.detach().to(dt).cuda().requires_grad_(True)
        kg = kv.detach().to(dt).cuda().requires_grad_(True)
        og = CrossAttentionF.apply(ug, kg, B, N, heads, D)
        (og * w.to(dt).cuda()).sum().backward()
        torch.cuda.synchronize()
        e = lambda a, b: ((a.double().cpu() - b).abs().max() / b.abs().max()).item()
        print(f"C={C} h={heads} B={B} N={N} {str(dt)[6:]}: out {e(og, o):.2e} du {e(ug.grad, u.grad):.2e} "
              f"dk {e(kg.grad[..., :C], kv.grad[..., :C]):.2e} dv {e(kg.grad[..., C:], kv.grad[..., C:]):.2e}")
