"""Module-form CPU restatement of the CMX RGB-X segmentation model (TEST ORACLE).

Test infrastructure only (see ``oracle/__init__.py``).  Every class restates one
reference component; the attribute names reproduce the reference ``state_dict`` keys
exactly (e.g. ``backbone.block1.0.attn.kv.weight``,
``backbone.FFMs.2.cross.cross_attn.kv1.weight``,
``decode_head.linear_fuse.1.running_var``) so checkpoints interoperate.

Numerics follow the reference op order in fp32 (or fp64 via ``.double()``):
  * Block / stage LayerNorms eps 1e-6 (``dual_segformer.py:503`` partial(LayerNorm, 1e-6)),
    OverlapPatchEmbed / SRA ``sr`` / CrossPath LayerNorms eps 1e-5 (defaults,
    ``dual_segformer.py:97,198``; ``net_utils.py:270-271``).
  * FFM BatchNorms are plain ``nn.BatchNorm2d`` eps 1e-5 (``mit_b*`` drops ``norm_fuse``,
    ``dual_segformer.py:499-504``); the decoder BN gets eps 1e-3 / momentum 0.1 from
    ``init_weight`` (``builder.py:204-206``, ``init_func.py:10-19``).
  * FFM cross attention normalises over dim -2 (``net_utils.py:207,209``) and crosses
    the contexts (``:211-212``).

Stochastic layers take injectable masks so train-mode parity can be checked:
``DropPath.masks`` (list of per-sample keep flags (B,), one per call) and ``Dropout2d.mask``
(per-(B,C) keep flags).  With ``mask is None`` they draw from torch's RNG.

Deviation (documented in DESIGN.md): decoder input channels come from the encoder's
``embed_dims``; the reference hard-codes [96,192,384,768] for mit_b4/b5
(``builder.py:66-75``), which cannot run, and aliases mit_b1 to mit_b0
(``builder.py:84-87``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

# --------------------------------------------------------------------------------------
# Backbone hyper-parameters: dual_segformer.py:483-528
# --------------------------------------------------------------------------------------
MIT_SPECS = {
    "mit_b0": dict(embed_dims=[32, 64, 160, 256], depths=[2, 2, 2, 2]),
    "mit_b1": dict(embed_dims=[64, 128, 320, 512], depths=[2, 2, 2, 2]),
    "mit_b2": dict(embed_dims=[64, 128, 320, 512], depths=[3, 4, 6, 3]),
    "mit_b3": dict(embed_dims=[64, 128, 320, 512], depths=[3, 4, 18, 3]),
    "mit_b4": dict(embed_dims=[64, 128, 320, 512], depths=[3, 8, 27, 3]),
    "mit_b5": dict(embed_dims=[64, 128, 320, 512], depths=[3, 6, 40, 3]),
}
NUM_HEADS = [1, 2, 5, 8]
SR_RATIOS = [8, 4, 2, 1]
MLP_RATIO = 4
DROP_PATH_RATE = 0.1


@dataclass
class CMXConfig:
    """Subset of ``config.py`` fields consumed on the hot path."""
    backbone: str = "mit_b2"
    num_classes: int = 40
    decoder_embed_dim: int = 512
    bn_eps: float = 1e-3          # config.py:80
    bn_momentum: float = 0.1      # config.py:81
    background: int = 255         # config.py:42
    lr: float = 6e-5              # config.py:68
    lr_power: float = 0.9
    weight_decay: float = 0.01
    drop_path_rate: float = DROP_PATH_RATE
    decoder_dropout: float = 0.1  # MLPDecoder.py:26
    feature_rectify_module: str = "FRM"   # config.py:57 (FRM | IFRM)
    feature_fusion_module: str = "FFM"    # config.py:58 (FFM | IFFM)


def drop_path_table(depths: List[int], rate: float = DROP_PATH_RATE):
    """Per-stage, per-stream drop-path probabilities, reproducing the reference
    indexing including the stage-2 quirk (``dual_segformer.py:249-311``): every
    ``block2[i]`` uses ``dpr[cur]`` and every ``extra_block2[i]`` uses ``dpr[cur+1]``.
    Returns ``[(rgb_probs, x_probs)]`` per stage."""
    dpr = [x.item() for x in torch.linspace(0, rate, sum(depths))]
    out, cur = [], 0
    for s, d in enumerate(depths):
        if s == 1:
            rgb = [dpr[cur]] * d
            ext = [dpr[cur + 1]] * d
        else:
            rgb = [dpr[cur + i] for i in range(d)]
            ext = list(rgb)
        out.append((rgb, ext))
        cur += d
    return out


def trunc_normal_(t: torch.Tensor, std: float = 0.02):
    # timm trunc_normal_(std=.02, a=-2, b=2): truncation at +-2 absolute (i.e. +-100 std)
    with torch.no_grad():
        return nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2.0, b=2.0)


def segformer_init(m: nn.Module):
    """``_init_weights`` of the MiT modules (``dual_segformer.py:52-65``)."""
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
            with torch.no_grad():
                m.bias.zero_()


class DropPath(nn.Module):
    """timm DropPath restated: x / keep * floor(keep + U) per sample.  One module serves
    both residual branches of a Block (two independent draws per forward,
    dual_segformer.py:177-178), so injected masks are a list consumed in call order."""

    def __init__(self, p: float):
        super().__init__()
        self.p = p
        self.masks: List[torch.Tensor] = []        # [(B,) keep flags in {0,1}] per call

    def forward(self, x):
        if self.p == 0.0 or not self.training:
            return x
        keep = 1.0 - self.p
        if self.masks:
            m = self.masks.pop(0).to(x.dtype)
        else:
            m = torch.floor(keep + torch.rand(x.shape[0], dtype=x.dtype))
        return x.div(keep) * m.view(-1, *([1] * (x.dim() - 1)))


class Dropout2d(nn.Module):
    """nn.Dropout2d restated with an injectable (B, C) keep mask."""

    def __init__(self, p: float):
        super().__init__()
        self.p = p
        self.mask: Optional[torch.Tensor] = None

    def forward(self, x):
        if not self.training or self.p == 0.0:
            return x
        if self.mask is not None:
            m = self.mask.to(x.dtype)
        else:
            m = torch.bernoulli(torch.full(x.shape[:2], 1 - self.p, dtype=x.dtype))
        return x * m[:, :, None, None] / (1 - self.p)


# --------------------------------------------------------------------------------------
# Encoder pieces: dual_segformer.py:19-225
# --------------------------------------------------------------------------------------
class DWConv(nn.Module):                                   # dual_segformer.py:19-33
    def __init__(self, dim):
        super().__init__()
        self.dwconv = nn.Conv2d(dim, dim, 3, 1, 1, bias=True, groups=dim)

    def forward(self, x, H, W):
        B, N, C = x.shape
        y = self.dwconv(x.transpose(1, 2).reshape(B, C, H, W))
        return y.flatten(2).transpose(1, 2)


class Mlp(nn.Module):                                      # dual_segformer.py:36-74
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.dwconv = DWConv(hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x, H, W):
        return self.fc2(F.gelu(self.dwconv(self.fc1(x), H, W)))


class Attention(nn.Module):                                # dual_segformer.py:77-138
    def __init__(self, dim, num_heads, sr_ratio):
        super().__init__()
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.q = nn.Linear(dim, dim, bias=True)
        self.kv = nn.Linear(dim, 2 * dim, bias=True)
        self.proj = nn.Linear(dim, dim)
        self.sr_ratio = sr_ratio
        if sr_ratio > 1:
            self.sr = nn.Conv2d(dim, dim, sr_ratio, sr_ratio)
            self.norm = nn.LayerNorm(dim)          # eps 1e-5

    def forward(self, x, H, W):
        B, N, C = x.shape
        h = self.num_heads
        q = self.q(x).view(B, N, h, C // h).transpose(1, 2)
        if self.sr_ratio > 1:
            xs = self.sr(x.transpose(1, 2).reshape(B, C, H, W)).flatten(2).transpose(1, 2)
            xs = self.norm(xs)
        else:
            xs = x
        kv = self.kv(xs).view(B, -1, 2, h, C // h).permute(2, 0, 3, 1, 4)
        k, v = kv[0], kv[1]
        a = ((q @ k.transpose(-2, -1)) * self.scale).softmax(dim=-1)
        return self.proj((a @ v).transpose(1, 2).reshape(B, N, C))


class Block(nn.Module):                                    # dual_segformer.py:141-180
    def __init__(self, dim, num_heads, sr_ratio, drop_path):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads, sr_ratio)
        self.drop_path = DropPath(drop_path) if drop_path > 0 else nn.Identity()
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, dim * MLP_RATIO)

    def forward(self, x, H, W):
        x = x + self.drop_path(self.attn(self.norm1(x), H, W))
        x = x + self.drop_path(self.mlp(self.norm2(x), H, W))
        return x


class OverlapPatchEmbed(nn.Module):                        # dual_segformer.py:183-225
    def __init__(self, patch_size, stride, in_chans, embed_dim):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, embed_dim, patch_size, stride, patch_size // 2)
        self.norm = nn.LayerNorm(embed_dim)        # eps 1e-5

    def forward(self, x):
        x = self.proj(x)
        _, _, H, W = x.shape
        return self.norm(x.flatten(2).transpose(1, 2)), H, W


# --------------------------------------------------------------------------------------
# Fusion modules: net_utils.py
# --------------------------------------------------------------------------------------
class ChannelWeights(nn.Module):                           # net_utils.py:10-30
    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.mlp = nn.Sequential(nn.Linear(4 * dim, 4 * dim), nn.ReLU(),
                                 nn.Linear(4 * dim, 2 * dim), nn.Sigmoid())

    def forward(self, x1, x2):
        B = x1.shape[0]
        x = torch.cat((x1, x2), 1)
        # AdaptiveAvgPool2d(1) / AdaptiveMaxPool2d(1) (net_utils.py:14-15,25-26): the max pool
        # routes its gradient to ONE index (the first maximum in scan order), unlike amax
        # which splits it over ties
        avg = F.adaptive_avg_pool2d(x, 1).view(B, 2 * self.dim)
        mx = F.adaptive_max_pool2d(x, 1).view(B, 2 * self.dim)
        y = torch.cat((avg, mx), 1)
        return self.mlp(y).view(B, 2, self.dim, 1, 1).permute(1, 0, 2, 3, 4)


class SpatialWeights(nn.Module):                           # net_utils.py:69-83
    def __init__(self, dim):
        super().__init__()
        self.mlp = nn.Sequential(nn.Conv2d(2 * dim, dim, 1), nn.ReLU(),
                                 nn.Conv2d(dim, 2, 1), nn.Sigmoid())

    def forward(self, x1, x2):
        B, _, H, W = x1.shape
        return self.mlp(torch.cat((x1, x2), 1)).view(B, 2, 1, H, W).permute(1, 0, 2, 3, 4)


class FeatureRectifyModule(nn.Module):                     # net_utils.py:124-152
    def __init__(self, dim, lambda_c=0.5, lambda_s=0.5):
        super().__init__()
        self.lambda_c, self.lambda_s = lambda_c, lambda_s
        self.channel_weights = ChannelWeights(dim)
        self.spatial_weights = SpatialWeights(dim)

    def forward(self, x1, x2):
        cw = self.channel_weights(x1, x2)
        sw = self.spatial_weights(x1, x2)
        o1 = x1 + self.lambda_c * cw[1] * x2 + self.lambda_s * sw[1] * x2
        o2 = x2 + self.lambda_c * cw[0] * x1 + self.lambda_s * sw[0] * x1
        return o1, o2


class CrossAttention(nn.Module):                           # net_utils.py:187-214
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.kv1 = nn.Linear(dim, 2 * dim, bias=False)
        self.kv2 = nn.Linear(dim, 2 * dim, bias=False)

    def forward(self, x1, x2):
        B, N, C = x1.shape
        h, d = self.num_heads, C // self.num_heads
        q1 = x1.view(B, N, h, d).transpose(1, 2)
        q2 = x2.view(B, N, h, d).transpose(1, 2)
        k1, v1 = self.kv1(x1).view(B, N, 2, h, d).permute(2, 0, 3, 1, 4)
        k2, v2 = self.kv2(x2).view(B, N, 2, h, d).permute(2, 0, 3, 1, 4)
        ctx1 = ((k1.transpose(-2, -1) @ v1) * self.scale).softmax(dim=-2)
        ctx2 = ((k2.transpose(-2, -1) @ v2) * self.scale).softmax(dim=-2)
        o1 = (q1 @ ctx2).transpose(1, 2).reshape(B, N, C)
        o2 = (q2 @ ctx1).transpose(1, 2).reshape(B, N, C)
        return o1, o2


class CrossPath(nn.Module):                                # net_utils.py:260-281
    def __init__(self, dim, num_heads):
        super().__init__()
        self.channel_proj1 = nn.Linear(dim, 2 * dim)
        self.channel_proj2 = nn.Linear(dim, 2 * dim)
        self.cross_attn = CrossAttention(dim, num_heads)
        self.end_proj1 = nn.Linear(2 * dim, dim)
        self.end_proj2 = nn.Linear(2 * dim, dim)
        self.norm1 = nn.LayerNorm(dim)             # eps 1e-5
        self.norm2 = nn.LayerNorm(dim)

    def forward(self, x1, x2):
        y1, u1 = F.relu(self.channel_proj1(x1)).chunk(2, dim=-1)
        y2, u2 = F.relu(self.channel_proj2(x2)).chunk(2, dim=-1)
        v1, v2 = self.cross_attn(u1, u2)
        o1 = self.norm1(x1 + self.end_proj1(torch.cat((y1, v1), -1)))
        o2 = self.norm2(x2 + self.end_proj2(torch.cat((y2, v2), -1)))
        return o1, o2


class ChannelEmbed(nn.Module):                             # net_utils.py:309-329
    def __init__(self, cin, cout):
        super().__init__()
        self.residual = nn.Conv2d(cin, cout, 1, bias=False)
        self.channel_embed = nn.Sequential(
            nn.Conv2d(cin, cout, 1, bias=True),
            nn.Conv2d(cout, cout, 3, 1, 1, bias=True, groups=cout),
            nn.ReLU(),
            nn.Conv2d(cout, cout, 1, bias=True),
            nn.BatchNorm2d(cout))                  # eps 1e-5 (norm_fuse not forwarded)
        self.norm = nn.BatchNorm2d(cout)

    def forward(self, x, H, W):
        B, N, C = x.shape
        x = x.transpose(1, 2).reshape(B, C, H, W)
        return self.norm(self.residual(x) + self.channel_embed(x))


class FeatureFusionModule(nn.Module):                      # net_utils.py:354-384
    def __init__(self, dim, num_heads):
        super().__init__()
        self.cross = CrossPath(dim, num_heads)
        self.channel_emb = ChannelEmbed(2 * dim, dim)
        self.apply(segformer_init)

    def forward(self, x1, x2):
        B, C, H, W = x1.shape
        a, b = self.cross(x1.flatten(2).transpose(1, 2), x2.flatten(2).transpose(1, 2))
        return self.channel_emb(torch.cat((a, b), -1), H, W)


# ---- improved variants (config.py:57-58, dual_segformer.py:316-329) ----------------------
class ImprovedChannelWeights(nn.Module):                   # net_utils.py:33-66
    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.mlp = nn.Sequential(nn.Linear(4 * dim, 4 * dim), nn.LayerNorm(4 * dim), nn.GELU(),
                                 nn.Linear(4 * dim, 2 * dim), nn.LayerNorm(2 * dim))
        self.gate = nn.Sequential(nn.Linear(2 * dim, 2 * dim), nn.Sigmoid())

    def forward(self, x1, x2):
        B = x1.shape[0]
        x = torch.cat((x1, x2), 1)
        avg = F.adaptive_avg_pool2d(x, 1).view(B, 2 * self.dim)
        mx = F.adaptive_max_pool2d(x, 1).view(B, 2 * self.dim)
        y = self.mlp(torch.cat((avg, mx), 1))
        y = y * self.gate(y)                                # gating (:61-63)
        return y.view(B, 2, self.dim, 1, 1).permute(1, 0, 2, 3, 4)


class ImprovedSpatialWeights(nn.Module):                   # net_utils.py:86-121
    def __init__(self, dim):
        super().__init__()
        self.conv1 = nn.Conv2d(2 * dim, dim, 1)
        self.norm1 = nn.BatchNorm2d(dim)
        self.conv2 = nn.Conv2d(dim, dim, 1)
        self.norm2 = nn.BatchNorm2d(dim)
        self.conv3 = nn.Conv2d(dim, 2, 1)

    def forward(self, x1, x2):
        B, _, H, W = x1.shape
        y = F.gelu(self.norm1(self.conv1(torch.cat((x1, x2), 1))))
        y = F.gelu(self.norm2(self.conv2(y))) + y           # residual (:107-115)
        return self.conv3(y).view(B, 2, 1, H, W).permute(1, 0, 2, 3, 4)     # no sigmoid (:118)


class ImprovedFeatureRectifyModule(nn.Module):             # net_utils.py:155-180
    def __init__(self, dim):
        super().__init__()
        self.channel_weights = ImprovedChannelWeights(dim)
        self.spatial_weights = ImprovedSpatialWeights(dim)
        self.lambda_channel = nn.Parameter(torch.tensor(0.5))
        self.lambda_spatial = nn.Parameter(torch.tensor(0.5))
        self.norm = nn.LayerNorm(dim)                       # eps 1e-5, shared by both outputs

    def forward(self, x1, x2):
        cw = self.channel_weights(x1, x2)
        sw = self.spatial_weights(x1, x2)
        o1 = x1 + self.lambda_channel * cw[1] * x2 + self.lambda_spatial * sw[1] * x2
        o2 = x2 + self.lambda_channel * cw[0] * x1 + self.lambda_spatial * sw[0] * x1
        o1 = self.norm(o1.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        o2 = self.norm(o2.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        return o1, o2


class ImprovedCrossAttention(nn.Module):                   # net_utils.py:216-257
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.q1 = nn.Linear(dim, dim, bias=False)
        self.kv1 = nn.Linear(dim, 2 * dim, bias=False)
        self.q2 = nn.Linear(dim, dim, bias=False)
        self.kv2 = nn.Linear(dim, 2 * dim, bias=False)
        self.proj1 = nn.Linear(dim, dim)
        self.proj2 = nn.Linear(dim, dim)                    # attn_drop / proj_drop: p = 0

    def forward(self, x1, x2):
        B, N, C = x1.shape
        h, d = self.num_heads, C // self.num_heads
        q1 = self.q1(x1).view(B, N, h, d).transpose(1, 2)
        k1, v1 = self.kv1(x1).view(B, N, 2, h, d).permute(2, 0, 3, 1, 4)
        q2 = self.q2(x2).view(B, N, h, d).transpose(1, 2)
        k2, v2 = self.kv2(x2).view(B, N, 2, h, d).permute(2, 0, 3, 1, 4)
        a1 = ((q1 @ k2.transpose(-2, -1)) * self.scale).softmax(dim=-1)
        a2 = ((q2 @ k1.transpose(-2, -1)) * self.scale).softmax(dim=-1)
        o1 = self.proj1((a1 @ v2).transpose(1, 2).reshape(B, N, C))
        o2 = self.proj2((a2 @ v1).transpose(1, 2).reshape(B, N, C))
        return o1, o2


class ImprovedCrossPath(nn.Module):                        # net_utils.py:283-306
    def __init__(self, dim, num_heads):
        super().__init__()
        self.channel_proj1 = nn.Linear(dim, 2 * dim)
        self.channel_proj2 = nn.Linear(dim, 2 * dim)
        self.cross_attn = ImprovedCrossAttention(dim, num_heads)
        self.end_proj1 = nn.Linear(2 * dim, dim)
        self.end_proj2 = nn.Linear(2 * dim, dim)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)

    def forward(self, x1, x2):
        y1, u1 = F.gelu(self.channel_proj1(x1)).chunk(2, dim=-1)
        y2, u2 = F.gelu(self.channel_proj2(x2)).chunk(2, dim=-1)
        v1, v2 = self.cross_attn(u1, u2)
        o1 = self.norm1(x1 + self.end_proj1(torch.cat((y1, v1), -1)))
        o2 = self.norm2(x2 + self.end_proj2(torch.cat((y2, v2), -1)))
        return o1, o2


class ImprovedChannelEmbed(ChannelEmbed):                  # net_utils.py:331-351: GELU for ReLU
    def __init__(self, cin, cout):
        super().__init__(cin, cout)
        self.channel_embed[2] = nn.GELU()


class ImprovedFeatureFusionModule(nn.Module):              # net_utils.py:387-417
    def __init__(self, dim, num_heads):
        super().__init__()
        self.cross = ImprovedCrossPath(dim, num_heads)
        self.channel_emb = ImprovedChannelEmbed(2 * dim, dim)
        self.apply(segformer_init)

    def forward(self, x1, x2):
        B, C, H, W = x1.shape
        a, b = self.cross(x1.flatten(2).transpose(1, 2), x2.flatten(2).transpose(1, 2))
        return self.channel_emb(torch.cat((a, b), -1), H, W)


class RGBXTransformer(nn.Module):                          # dual_segformer.py:228-446
    def __init__(self, embed_dims, depths, drop_path_rate=DROP_PATH_RATE, frm="FRM", ffm="FFM"):
        super().__init__()
        self.depths = depths
        dp = drop_path_table(depths, drop_path_rate)
        cins = [3] + embed_dims[:3]
        for pre in ("", "extra_"):                    # registration order of :238-246
            for s in range(4):
                k, st = (7, 4) if s == 0 else (3, 2)
                setattr(self, f"{pre}patch_embed{s + 1}",
                        OverlapPatchEmbed(k, st, cins[s], embed_dims[s]))
        for s in range(4):
            for pre, probs in (("", dp[s][0]), ("extra_", dp[s][1])):
                setattr(self, f"{pre}block{s + 1}", nn.ModuleList(
                    [Block(embed_dims[s], NUM_HEADS[s], SR_RATIOS[s], probs[i])
                     for i in range(depths[s])]))
                setattr(self, f"{pre}norm{s + 1}", nn.LayerNorm(embed_dims[s], eps=1e-6))
        # dual_segformer.py:316-340: anything but 'FRM' / 'FFM' selects the improved variant
        rect = FeatureRectifyModule if frm == "FRM" else ImprovedFeatureRectifyModule
        fuse = FeatureFusionModule if ffm == "FFM" else ImprovedFeatureFusionModule
        self.FRMs = nn.ModuleList([rect(d) for d in embed_dims])
        self.FFMs = nn.ModuleList([fuse(d, NUM_HEADS[s]) for s, d in enumerate(embed_dims)])
        self.apply(segformer_init)

    def forward(self, x_rgb, x_e, return_stages=False):
        B = x_rgb.shape[0]
        outs, stages = [], []
        for s in range(4):
            x_rgb, H, W = getattr(self, f"patch_embed{s + 1}")(x_rgb)
            x_e, _, _ = getattr(self, f"extra_patch_embed{s + 1}")(x_e)
            for blk in getattr(self, f"block{s + 1}"):
                x_rgb = blk(x_rgb, H, W)
            for blk in getattr(self, f"extra_block{s + 1}"):
                x_e = blk(x_e, H, W)
            x_rgb = getattr(self, f"norm{s + 1}")(x_rgb)
            x_e = getattr(self, f"extra_norm{s + 1}")(x_e)
            x_rgb = x_rgb.reshape(B, H, W, -1).permute(0, 3, 1, 2)
            x_e = x_e.reshape(B, H, W, -1).permute(0, 3, 1, 2)
            stages.append((x_rgb, x_e))
            x_rgb, x_e = self.FRMs[s](x_rgb, x_e)
            outs.append(self.FFMs[s](x_rgb, x_e))
        return (outs, stages) if return_stages else outs


# --------------------------------------------------------------------------------------
# Decoder: MLPDecoder.py:8-81
# --------------------------------------------------------------------------------------
class MLP(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.proj = nn.Linear(cin, cout)

    def forward(self, x):
        return self.proj(x.flatten(2).transpose(1, 2))


class DecoderHead(nn.Module):
    def __init__(self, in_channels, num_classes, embed_dim, dropout_ratio=0.1, bn_eps=1e-3,
                 bn_momentum=0.1):
        super().__init__()
        c1, c2, c3, c4 = in_channels
        self.dropout = Dropout2d(dropout_ratio)
        self.linear_c4 = MLP(c4, embed_dim)
        self.linear_c3 = MLP(c3, embed_dim)
        self.linear_c2 = MLP(c2, embed_dim)
        self.linear_c1 = MLP(c1, embed_dim)
        self.linear_fuse = nn.Sequential(nn.Conv2d(4 * embed_dim, embed_dim, 1),
                                         nn.BatchNorm2d(embed_dim, eps=bn_eps,
                                                        momentum=bn_momentum),
                                         nn.ReLU())
        self.linear_pred = nn.Conv2d(embed_dim, num_classes, 1)

    def forward(self, inputs):
        c1, c2, c3, c4 = inputs
        n = c4.shape[0]
        size = c1.shape[2:]

        def lin(m, c, up):
            t = m(c).transpose(1, 2).reshape(n, -1, c.shape[2], c.shape[3])
            return F.interpolate(t, size=size, mode="bilinear", align_corners=False) if up else t

        cat = torch.cat([lin(self.linear_c4, c4, True), lin(self.linear_c3, c3, True),
                         lin(self.linear_c2, c2, True), lin(self.linear_c1, c1, False)], 1)
        return self.linear_pred(self.dropout(self.linear_fuse(cat)))


def decoder_init(head: nn.Module, bn_eps, bn_momentum):
    """``init_weight(decode_head, kaiming_normal_, BN, eps, momentum, fan_in, relu)``
    (``builder.py:204-206`` / ``init_func.py:10-19``)."""
    for m in head.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm2d):
            m.eps, m.momentum = bn_eps, bn_momentum
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)


class EncoderDecoder(nn.Module):                           # builder.py:14-253
    def __init__(self, cfg: CMXConfig = None, criterion=None):
        super().__init__()
        cfg = cfg or CMXConfig()
        spec = MIT_SPECS[cfg.backbone]
        self.cfg = cfg
        self.channels = list(spec["embed_dims"])
        self.backbone = RGBXTransformer(spec["embed_dims"], spec["depths"], cfg.drop_path_rate,
                                        cfg.feature_rectify_module, cfg.feature_fusion_module)
        self.aux_head = None
        self.decode_head = DecoderHead(self.channels, cfg.num_classes, cfg.decoder_embed_dim,
                                       cfg.decoder_dropout, cfg.bn_eps, cfg.bn_momentum)
        self.criterion = criterion if criterion is not None else nn.CrossEntropyLoss(
            reduction="mean", ignore_index=cfg.background)
        decoder_init(self.decode_head, cfg.bn_eps, cfg.bn_momentum)

    def encode_decode(self, rgb, modal_x):
        out = self.decode_head(self.backbone(rgb, modal_x))
        return F.interpolate(out, size=rgb.shape[2:], mode="bilinear", align_corners=False)

    def forward(self, rgb, modal_x, label=None):
        out = self.encode_decode(rgb, modal_x)
        if label is not None:
            return self.criterion(out, label.long())
        return out

    # ---- helpers for injecting stochastic masks --------------------------------------
    def stochastic_modules(self):
        """Ordered list of (name, module) for DropPath/Dropout2d with p > 0."""
        return [(n, m) for n, m in self.named_modules()
                if isinstance(m, (DropPath, Dropout2d)) and m.p > 0]


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
