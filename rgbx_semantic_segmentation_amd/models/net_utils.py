"""CM-FRM and FFM parameter containers + FFM execution (reference: models/net_utils.py).

Containers reproduce the reference module names (``channel_weights.mlp.0``,
``cross.cross_attn.kv1``, ``channel_emb.channel_embed.4`` ...).  ``FeatureFusionModule.run``
executes CrossPath + ChannelEmbed for the modality pair in grouped launches and returns
the fused map as (B*N, C) tokens (the reference returns NCHW; the decoder consumes
tokens directly, MLPDecoder.py:17-18 flattens it anyway).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import functions as F


def trunc_normal_(t, std=0.02):
    with torch.no_grad():
        return nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2.0, b=2.0)


def init_segformer(m):
    """MiT/FFM ``_init_weights`` (dual_segformer.py:52-65, net_utils.py:360-373)."""
    if isinstance(m, nn.Linear):
        trunc_normal_(m.weight, std=0.02)
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)
    elif isinstance(m, nn.LayerNorm):
        nn.init.constant_(m.bias, 0)
        nn.init.constant_(m.weight, 1.0)
    elif isinstance(m, nn.Conv2d):
        fan_out = m.kernel_size[0] * m.kernel_size[1] * m.out_channels // m.groups
        with torch.no_grad():
            m.weight.normal_(0, math.sqrt(2.0 / fan_out))
            if m.bias is not None:
                m.bias.zero_()


class ChannelWeights(nn.Module):                  # net_utils.py:10-30
    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.mlp = nn.Sequential(nn.Linear(4 * dim, 4 * dim), nn.ReLU(inplace=True),
                                 nn.Linear(4 * dim, 2 * dim), nn.Sigmoid())


class SpatialWeights(nn.Module):                  # net_utils.py:69-83
    def __init__(self, dim):
        super().__init__()
        self.mlp = nn.Sequential(nn.Conv2d(2 * dim, dim, 1), nn.ReLU(inplace=True),
                                 nn.Conv2d(dim, 2, 1), nn.Sigmoid())


class FeatureRectifyModule(nn.Module):            # net_utils.py:124-152
    def __init__(self, dim, reduction=1, lambda_c=0.5, lambda_s=0.5):
        super().__init__()
        self.lambda_c, self.lambda_s = lambda_c, lambda_s
        self.channel_weights = ChannelWeights(dim)
        self.spatial_weights = SpatialWeights(dim)


class CrossAttention(nn.Module):                  # net_utils.py:187-214
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.kv1 = nn.Linear(dim, 2 * dim, bias=False)
        self.kv2 = nn.Linear(dim, 2 * dim, bias=False)


class CrossPath(nn.Module):                       # net_utils.py:260-281
    def __init__(self, dim, num_heads):
        super().__init__()
        self.channel_proj1 = nn.Linear(dim, 2 * dim)
        self.channel_proj2 = nn.Linear(dim, 2 * dim)
        self.act1 = nn.ReLU(inplace=True)
        self.act2 = nn.ReLU(inplace=True)
        self.cross_attn = CrossAttention(dim, num_heads)
        self.end_proj1 = nn.Linear(2 * dim, dim)
        self.end_proj2 = nn.Linear(2 * dim, dim)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)


class ChannelEmbed(nn.Module):                    # net_utils.py:309-329
    def __init__(self, cin, cout):
        super().__init__()
        self.residual = nn.Conv2d(cin, cout, 1, bias=False)
        self.channel_embed = nn.Sequential(
            nn.Conv2d(cin, cout, 1, bias=True),
            nn.Conv2d(cout, cout, 3, 1, 1, bias=True, groups=cout),
            nn.ReLU(inplace=True),
            nn.Conv2d(cout, cout, 1, bias=True),
            nn.BatchNorm2d(cout))                 # plain BN, eps 1e-5 (norm_fuse not forwarded)
        self.norm = nn.BatchNorm2d(cout)


class FeatureFusionModule(nn.Module):             # net_utils.py:354-384
    def __init__(self, dim, num_heads, reduction=1, norm_layer=None):
        super().__init__()
        self.dim, self.num_heads = dim, num_heads
        self.cross = CrossPath(dim, num_heads)
        self.channel_emb = ChannelEmbed(2 * dim, dim)
        self.apply(init_segformer)

    def run(self, store, r, B, H, W, training):
        """r: (2, B, N, C) rectified pair -> fused (B*N, C) tokens."""
        G, _, N, C = r.shape
        M = B * N
        cp, ce = self.cross, self.channel_emb
        heads = self.num_heads
        x = r.view(G, M, C)
        # relu(channel_proj) -> chunk -> kv + cross attention -> x + end_proj(cat(y, v)): one node
        e = F.cross_path(store, cp, x, B, N, heads)
        o = F.layernorm(store, cp.norm1, e, G)
        res, t = F.pair_embed(store, ce, o)             # residual / channel_embed[0] on cat(o[0], o[1])
        t = F.dwconv(store, ce.channel_embed[1], t, B, B, H, W, "relu")
        t = F.glinear(store, ce.channel_embed[3].weight, ce.channel_embed[3].bias, t)
        s = F.batchnorm(store, ce.channel_embed[4], t.view(M, C), training, res=res.view(M, C))
        return F.batchnorm(store, ce.norm, s, training)


# ---- improved variants: config.feature_rectify_module = 'IFRM' / feature_fusion_module = 'IFFM'
#      (config.py:57-58, selected in dual_segformer.py:316-329)
class ImprovedChannelWeights(nn.Module):          # net_utils.py:33-66
    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.mlp = nn.Sequential(nn.Linear(4 * dim, 4 * dim), nn.LayerNorm(4 * dim), nn.GELU(),
                                 nn.Linear(4 * dim, 2 * dim), nn.LayerNorm(2 * dim))
        self.gate = nn.Sequential(nn.Linear(2 * dim, 2 * dim), nn.Sigmoid())


class ImprovedSpatialWeights(nn.Module):          # net_utils.py:86-121
    def __init__(self, dim):
        super().__init__()
        self.conv1 = nn.Conv2d(2 * dim, dim, 1)
        self.norm1 = nn.BatchNorm2d(dim)
        self.conv2 = nn.Conv2d(dim, dim, 1)
        self.norm2 = nn.BatchNorm2d(dim)
        self.conv3 = nn.Conv2d(dim, 2, 1)


class ImprovedFeatureRectifyModule(nn.Module):    # net_utils.py:155-180
    def __init__(self, dim, reduction=1):
        super().__init__()
        self.channel_weights = ImprovedChannelWeights(dim)
        self.spatial_weights = ImprovedSpatialWeights(dim)
        self.lambda_channel = nn.Parameter(torch.tensor(0.5))
        self.lambda_spatial = nn.Parameter(torch.tensor(0.5))
        self.norm = nn.LayerNorm(dim)

    def rectify(self, store, x, training):
        """x (2, B, N, C) -> rectified pair (2, B, N, C).  ImprovedSpatialWeights runs as
        cat-free GEMM -> BN + GELU (fused apply) -> GEMM -> BN + GELU -> residual add -> C -> 2
        GEMM; the channel MLP + rectification as IFRMF; the shared LayerNorm over both
        modalities' rows at once (one gamma / beta: G = 1)."""
        G, B, N, C = x.shape
        sp = self.spatial_weights
        x1, x2 = F.split(x.view(G, 1, B * N, C), 1, 0)
        h = F.glinear(store, sp.conv1.weight, sp.conv1.bias, x1[0], x2[0])[0]          # (B*N, C)
        a1 = F.batchnorm(store, sp.norm1, h, training, act="gelu")
        h = F.glinear(store, sp.conv2.weight, sp.conv2.bias, a1[None])[0]
        a2 = F.batchnorm(store, sp.norm2, h, training, act="gelu")
        y = F.ResidualF.apply(a2, a1, None, a2.numel())
        sw = F.glinear(store, sp.conv3.weight, sp.conv3.bias, y[None])[0]              # (B*N, 2)
        cwm, gate = self.channel_weights.mlp, self.channel_weights.gate
        f32 = lambda p: store.w(p, stacked=False, compute=False)
        g = lambda p: store.g(p, stacked=False)
        prm = {
            "w": (f32(cwm[0].weight), f32(cwm[0].bias), f32(cwm[1].weight), f32(cwm[1].bias),
                  f32(cwm[3].weight), f32(cwm[3].bias), f32(cwm[4].weight), f32(cwm[4].bias),
                  f32(gate[0].weight), f32(gate[0].bias), f32(self.lambda_channel).view(1),
                  f32(self.lambda_spatial).view(1), cwm[1].eps, cwm[4].eps),
            "g": (g(cwm[0].weight), g(cwm[0].bias), g(cwm[1].weight), g(cwm[1].bias),
                  g(cwm[3].weight), g(cwm[3].bias), g(cwm[4].weight), g(cwm[4].bias),
                  g(gate[0].weight), g(gate[0].bias), g(self.lambda_channel).view(1),
                  g(self.lambda_spatial).view(1)),
        }
        o = F.IFRMF.apply(x, sw, prm, cwm[0].weight)
        return F.layernorm(store, self.norm, o.view(1, G * B * N, C), 1).view(G, B, N, C)


class ImprovedCrossAttention(nn.Module):          # net_utils.py:216-257
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.q1 = nn.Linear(dim, dim, bias=False)
        self.kv1 = nn.Linear(dim, 2 * dim, bias=False)
        self.q2 = nn.Linear(dim, dim, bias=False)
        self.kv2 = nn.Linear(dim, 2 * dim, bias=False)
        self.attn_drop = nn.Dropout(0.0)
        self.proj1 = nn.Linear(dim, dim)
        self.proj2 = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(0.0)


class ImprovedCrossPath(nn.Module):               # net_utils.py:283-306
    def __init__(self, dim, num_heads):
        super().__init__()
        self.channel_proj1 = nn.Linear(dim, 2 * dim)
        self.channel_proj2 = nn.Linear(dim, 2 * dim)
        self.act1 = nn.GELU()
        self.act2 = nn.GELU()
        self.cross_attn = ImprovedCrossAttention(dim, num_heads)
        self.end_proj1 = nn.Linear(2 * dim, dim)
        self.end_proj2 = nn.Linear(2 * dim, dim)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)


class ImprovedChannelEmbed(nn.Module):            # net_utils.py:331-351
    def __init__(self, cin, cout):
        super().__init__()
        self.residual = nn.Conv2d(cin, cout, 1, bias=False)
        self.channel_embed = nn.Sequential(
            nn.Conv2d(cin, cout, 1, bias=True),
            nn.Conv2d(cout, cout, 3, 1, 1, bias=True, groups=cout),
            nn.GELU(),
            nn.Conv2d(cout, cout, 1, bias=True),
            nn.BatchNorm2d(cout))
        self.norm = nn.BatchNorm2d(cout)


class ImprovedFeatureFusionModule(nn.Module):     # net_utils.py:387-417
    def __init__(self, dim, num_heads, reduction=1, norm_layer=None):
        super().__init__()
        self.dim, self.num_heads = dim, num_heads
        self.cross = ImprovedCrossPath(dim, num_heads)
        self.channel_emb = ImprovedChannelEmbed(2 * dim, dim)
        self.apply(init_segformer)

    def run(self, store, r, B, H, W, training):
        """r: (2, B, N, C) rectified pair -> fused (B*N, C) tokens.  As FeatureFusionModule.run
        with GELU for ReLU and the full cross attention (q / kv projections, softmax over the
        other modality's tokens, output projection) in place of the context attention."""
        G, _, N, C = r.shape
        M = B * N
        cp, ce = self.cross, self.channel_emb
        ca = cp.cross_attn
        heads = self.num_heads
        x = r.view(G, M, C)
        a = F.ActF.apply(F.glinear(store, cp.channel_proj1.weight, cp.channel_proj1.bias, x), "gelu")
        y, u = F.split(a, C, -1)
        q = F.glinear(store, ca.q1.weight, None, u)
        kv = F.glinear(store, ca.kv1.weight, None, u)
        o = F.CrossFlashAttnF.apply(q, kv, B, N, heads, C // heads)
        v = F.glinear(store, ca.proj1.weight, ca.proj1.bias, o)
        e = F.glinear(store, cp.end_proj1.weight, cp.end_proj1.bias, y, v, res=x)     # x + end_proj(cat(y, v))
        o = F.layernorm(store, cp.norm1, e, G)
        o1, o2 = F.split(o, 1, 0)
        res = F.glinear(store, ce.residual.weight, None, o1, o2)
        t = F.glinear(store, ce.channel_embed[0].weight, ce.channel_embed[0].bias, o1, o2)
        t = F.dwconv(store, ce.channel_embed[1], t, B, B, H, W, "gelu")
        t = F.glinear(store, ce.channel_embed[3].weight, ce.channel_embed[3].bias, t)
        s = F.batchnorm(store, ce.channel_embed[4], t.view(M, C), training, res=res.view(M, C))
        return F.batchnorm(store, ce.norm, s, training)
