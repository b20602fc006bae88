"""Dual-stream MiT encoder (mit_b0..b5) of CMX, executed with both modality streams in
every kernel launch.

Parameter containers keep the reference module tree (``dual_segformer.py:19-528``), so
``state_dict`` keys match (``backbone.block2.3.attn.sr.weight``,
``backbone.extra_patch_embed1.proj.weight``, ...).  The containers hold parameters only;
``RGBXTransformer.run`` executes a stage for BOTH streams at once: the RGB module's
parameters are addressed through the ParamStore as (2, ...) stacked views that include
the ``extra_*`` twin, activations are (2, B*N, C) token-major tensors.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn as nn

from ... import functions as F
from ... import streams
from ..net_utils import (FeatureRectifyModule, FeatureFusionModule, ImprovedFeatureRectifyModule,
                         ImprovedFeatureFusionModule, init_segformer)

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


def drop_path_probs(depths: List[int], rate: float):
    """Per stage: (rgb_probs, x_probs) per block.  Reproduces dual_segformer.py:249-311,
    including the stage-2 indexing (block2[i] -> dpr[cur], extra_block2[i] -> dpr[cur+1])."""
    dpr = [x.item() for x in torch.linspace(0, rate, sum(depths))]
    out, cur = [], 0
    for s, d in enumerate(depths):
        if s == 1:
            out.append(([dpr[cur]] * d, [dpr[cur + 1]] * d))
        else:
            p = [dpr[cur + i] for i in range(d)]
            out.append((p, list(p)))
        cur += d
    return out


class DWConv(nn.Module):                          # dual_segformer.py:19-33
    def __init__(self, dim):
        super().__init__()
        self.dwconv = nn.Conv2d(dim, dim, 3, 1, 1, bias=True, groups=dim)


class Mlp(nn.Module):                             # dual_segformer.py:36-74
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.dwconv = DWConv(hidden)
        self.fc2 = nn.Linear(hidden, dim)


class Attention(nn.Module):                       # dual_segformer.py:77-138
    def __init__(self, dim, num_heads, sr_ratio):
        super().__init__()
        self.num_heads = num_heads
        self.q = nn.Linear(dim, dim, bias=True)
        self.kv = nn.Linear(dim, 2 * dim, bias=True)
        self.proj = nn.Linear(dim, dim)
        self.sr_ratio = sr_ratio
        if sr_ratio > 1:
            self.sr = nn.Conv2d(dim, dim, sr_ratio, sr_ratio)
            self.norm = nn.LayerNorm(dim)


class Block(nn.Module):                           # dual_segformer.py:141-180
    def __init__(self, dim, num_heads, sr_ratio, drop_path):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads, sr_ratio)
        self.drop_path_prob = drop_path
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, dim * MLP_RATIO)


class OverlapPatchEmbed(nn.Module):               # dual_segformer.py:183-225
    def __init__(self, patch_size, stride, in_chans, embed_dim):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, embed_dim, patch_size, stride, patch_size // 2)
        self.norm = nn.LayerNorm(embed_dim)
        self.stride = stride
        self.pad = patch_size // 2


class RGBXTransformer(nn.Module):                 # dual_segformer.py:228-446
    def __init__(self, embed_dims, depths, drop_path_rate=0.1, frm="FRM", ffm="FFM"):
        super().__init__()
        self.embed_dims, self.depths = list(embed_dims), list(depths)
        self.dp = drop_path_probs(depths, drop_path_rate)
        cins = [3] + list(embed_dims[:3])
        for pre in ("", "extra_"):
            for s in range(4):
                k, st = (7, 4) if s == 0 else (3, 2)
                setattr(self, f"{pre}patch_embed{s + 1}", OverlapPatchEmbed(k, st, cins[s], embed_dims[s]))
        for s in range(4):
            for pre, probs in (("", self.dp[s][0]), ("extra_", self.dp[s][1])):
                setattr(self, f"{pre}block{s + 1}", nn.ModuleList(
                    [Block(embed_dims[s], NUM_HEADS[s], SR_RATIOS[s], probs[i]) for i in range(depths[s])]))
                setattr(self, f"{pre}norm{s + 1}", nn.LayerNorm(embed_dims[s], eps=1e-6))
        # config.feature_rectify_module / feature_fusion_module (dual_segformer.py:316-340):
        # anything but 'FRM' / 'FFM' selects the improved variant, as in the reference
        rect = FeatureRectifyModule if frm == "FRM" else ImprovedFeatureRectifyModule
        fuse = FeatureFusionModule if ffm == "FFM" else ImprovedFeatureFusionModule
        self.FRMs = nn.ModuleList([rect(d) for d in embed_dims])
        self.FFMs = nn.ModuleList([fuse(d, NUM_HEADS[s]) for s, d in enumerate(embed_dims)])
        self.apply(init_segformer)

    # ------------------------------------------------------------------------ execution
    def drop_path_keep_probs(self):
        """(n_blocks_total, 2) keep probabilities in execution order (stage, block)."""
        rows = []
        for s in range(4):
            for i in range(self.depths[s]):
                rows.append((1.0 - self.dp[s][0][i], 1.0 - self.dp[s][1][i]))
        return rows

    def run_block(self, store, blk: Block, x, B, H, W, s_attn, s_mlp, prev=(None, None), tail=None,
                  next_norm=None):
        """One Block (dual_segformer.py:166-180) for both streams.  ``prev`` = (DropPath scale,
        GradTap) of the residual branch that produced ``x`` (the previous block's fc2): norm1's
        backward writes that branch's scaled gradient.  ``tail``: the LNTail of norm1 when the
        producer of x normalised it in its launch; ``next_norm``: the norm that consumes this
        block's output (the next block's norm1 or the stage norm), computed in fc2's launch.
        Returns (x_out, (s_mlp, tap), LNTail of next_norm or None) for the next consumer of x_out."""
        G, M, C = x.shape
        N = H * W
        a = blk.attn
        # norm1 also passes x through for the attention residual: its backward sums both gradients
        # (q and the SR path read norm1's output through separate handles: the norm's backward
        # sums their gradients on load)
        # norm1's backward rides on the SR conv's input-gradient launch (C 64 / 128, exact patches)
        stap = F.DgradTap() if (a.sr_ratio > 1 and F.ln_bwd_fusable(x, (H, W, a.sr_ratio))) else None
        h, h2, xr = F.layernorm_res(store, blk.norm1, x, G, scale=prev[0], rps=N, tap=prev[1], tail=tail, dtap=stap)

        if a.sr_ratio > 1:
            xs, Hk, Wk = F.conv(store, a.sr, h2, G, G * B, H, W, C, a.sr_ratio, 0, dtap=stap)
            xs, Nk = F.layernorm(store, a.norm, xs, G), Hk * Wk
        else:
            xs, Nk = h2, N
        # q and kv as ONE GEMM launch (and their input gradients as another)
        q, kv = F.glinear_multi(store, [(a.q.weight, a.q.bias, h), (a.kv.weight, a.kv.bias, xs)])
        o = F.SRAttentionF.apply(q, kv, G * B, N, Nk, a.num_heads, C // a.num_heads)
        # x + drop_path(proj(o)): residual and DropPath scale fused into the proj GEMM epilogue
        tap_a = F.GradTap() if s_attn is not None else None
        t2 = F.LNTail(blk.norm2)
        x = F.glinear(store, a.proj.weight, a.proj.bias, o, res=xr, rscale=s_attn, rps=N, tap=tap_a, ln_tail=t2)
        # norm2's backward rides on fc1's dgrad launch (C <= 128): fc1 hands (dz, W1) over
        ltap = F.DgradTap() if F.ln_bwd_fusable(x) else None
        h, _, xr = F.layernorm_res(store, blk.norm2, x, G, scale=s_attn, rps=N, tap=tap_a, tail=t2, dtap=ltap)
        f = F.glinear(store, blk.mlp.fc1.weight, blk.mlp.fc1.bias, h, dgrad_tap=ltap)
        f = F.dwconv(store, blk.mlp.dwconv.dwconv, f, G * B, B, H, W, "gelu")
        tap_m = F.GradTap() if s_mlp is not None else None
        tn = F.LNTail(next_norm) if next_norm is not None else None
        x = F.glinear(store, blk.mlp.fc2.weight, blk.mlp.fc2.bias, f, res=xr, rscale=s_mlp, rps=N, tap=tap_m,
                      ln_tail=tn)
        return x, (s_mlp, tap_m), tn

    def run(self, store, images, B, H, W, training, dp_scales: Optional[torch.Tensor], bn_group=None):
        """images: (2*B, 3, H, W) fp32 NCHW (RGB batch then X batch), or the pair of (B, 3, H, W)
        batches (rgb, modal_x) read by the stage-1 im2col in place.
        dp_scales: (n_blocks_total, 2, 2*? ) per-block (attn, mlp) per-sample scales or None.
        Returns the 4 fused maps [(B*N_s, C_s) tokens] and their grids."""
        G = 2
        x2 = None
        if isinstance(images, (tuple, list)):
            x, x2 = images
        else:
            x = images
        outs, grids = [], []
        bi = 0
        Hc, Wc, Cin = H, W, 3
        sync = getattr(self, "grad_sync", None)     # dist.BucketedGradSync (data parallel) or None
        main = torch.cuda.current_stream() if x.is_cuda else None
        side = streams.ffm_stream(main.device) if (main is not None and streams.FFM_SIDE) else None
        for s in range(4):
            pe = getattr(self, f"patch_embed{s + 1}")
            if sync is not None and s > 0 and x.requires_grad:
                # the gradient of this stage's input exists once the backward has passed the
                # stage (segment 3 - s): its gradients can be all-reduced while stages < s run
                x.register_hook(sync.segment_hook(3 - s))
            if s == 0:      # conv on the NCHW images + LayerNorm in one launch where eligible
                x, Ho, Wo = F.patch_embed1(store, pe, x, G, G * B, Hc, Wc, x2=x2)
            else:
                x, Ho, Wo = F.conv(store, pe.proj, x, G, G * B, Hc, Wc, Cin, pe.stride, pe.pad)
                x = F.layernorm(store, pe.norm, x, G)
            Hc, Wc, Cin = Ho, Wo, self.embed_dims[s]
            prev = (None, None)
            blocks = getattr(self, f"block{s + 1}")
            snorm = getattr(self, f"norm{s + 1}")
            tail = None
            for i, blk in enumerate(blocks):
                sa = sm = None
                if dp_scales is not None:
                    sa, sm = dp_scales[bi, 0], dp_scales[bi, 1]
                nxt = blocks[i + 1].norm1 if i + 1 < len(blocks) else snorm
                x, prev, tail = self.run_block(store, blk, x, B, Hc, Wc, sa, sm, prev, tail=tail, next_norm=nxt)
                bi += 1
            # stage norm: its backward also writes the last block's DropPath-scaled gradient
            x, _, _ = F.layernorm_res(store, snorm, x, G, scale=prev[0], rps=Hc * Wc, tap=prev[1], tail=tail)
            C = self.embed_dims[s]
            fr = self.FRMs[s]
            if isinstance(fr, ImprovedFeatureRectifyModule):
                r = rn = fr.rectify(store, x.view(G, B, Hc * Wc, C), training)
            else:
                r, rn = F.frm(store, fr, x.view(G, B, Hc * Wc, C))     # rn: the next stage's handle
            if side is not None:
                # FFM_s only feeds the decoder: run it beside stage s + 1 on the side stream
                # (its backward then runs there too, beside the encoder's backward)
                side.wait_stream(main)
                r.record_stream(side)
                with torch.cuda.stream(side):
                    outs.append(self.FFMs[s].run(store, r, B, Hc, Wc, training))
            else:
                outs.append(self.FFMs[s].run(store, r, B, Hc, Wc, training))
            grids.append((Hc, Wc))
            x = rn.view(G, B * Hc * Wc, C)
        if side is not None:
            main.wait_stream(side)
            for o in outs:
                o.record_stream(main)
        return outs, grids


class mit_b0(RGBXTransformer):
    def __init__(self, fuse_cfg=None, frm="FRM", ffm="FFM", **kwargs):
        super().__init__(**MIT_SPECS["mit_b0"], drop_path_rate=0.1, frm=frm, ffm=ffm)


class mit_b1(RGBXTransformer):
    def __init__(self, fuse_cfg=None, frm="FRM", ffm="FFM", **kwargs):
        super().__init__(**MIT_SPECS["mit_b1"], drop_path_rate=0.1, frm=frm, ffm=ffm)


class mit_b2(RGBXTransformer):
    def __init__(self, fuse_cfg=None, frm="FRM", ffm="FFM", **kwargs):
        super().__init__(**MIT_SPECS["mit_b2"], drop_path_rate=0.1, frm=frm, ffm=ffm)


class mit_b3(RGBXTransformer):
    def __init__(self, fuse_cfg=None, frm="FRM", ffm="FFM", **kwargs):
        super().__init__(**MIT_SPECS["mit_b3"], drop_path_rate=0.1, frm=frm, ffm=ffm)


class mit_b4(RGBXTransformer):
    def __init__(self, fuse_cfg=None, frm="FRM", ffm="FFM", **kwargs):
        super().__init__(**MIT_SPECS["mit_b4"], drop_path_rate=0.1, frm=frm, ffm=ffm)


class mit_b5(RGBXTransformer):
    def __init__(self, fuse_cfg=None, frm="FRM", ffm="FFM", **kwargs):
        super().__init__(**MIT_SPECS["mit_b5"], drop_path_rate=0.1, frm=frm, ffm=ffm)


BACKBONES = {"mit_b0": mit_b0, "mit_b1": mit_b1, "mit_b2": mit_b2, "mit_b3": mit_b3, "mit_b4": mit_b4,
             "mit_b5": mit_b5}


def load_dualpath_model(model: nn.Module, model_file):
    """Pretrained MiT weights duplicated into both streams (dual_segformer.py:449-480).
    ``model_file`` is a path (loaded with weights_only=True) or a state dict."""
    raw = torch.load(model_file, map_location="cpu", weights_only=True) if isinstance(model_file, str) \
        else model_file
    if "model" in raw:
        raw = raw["model"]
    sd = {}
    for k, v in raw.items():
        if "patch_embed" in k:
            sd[k] = v
            sd[k.replace("patch_embed", "extra_patch_embed")] = v
        elif "block" in k:
            sd[k] = v
            sd[k.replace("block", "extra_block")] = v
        elif "norm" in k:
            sd[k] = v
            sd[k.replace("norm", "extra_norm")] = v
    return model.load_state_dict(sd, strict=False)
