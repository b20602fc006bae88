"""Functional/einsum restatement of the CMX forward (TEST ORACLE, independent form).

Test infrastructure only.  Driven by a reference-format ``state_dict`` and written
without ``nn.Module``s, token-major (B, N, C) throughout and with explicit einsums,
so that it shares no code path with ``oracle/cmx_ref.py``.  The two must agree to
~1e-6 (fp64) — tests/test_oracle_selfcheck.py.

``bn_mode``: "eval" uses running statistics, "batch" uses biased batch statistics
(train-mode forward without dropout / drop-path).
Reference lines restated are cited per function.
"""
from __future__ import annotations

import math
import torch

from .cmx_ref import MIT_SPECS, NUM_HEADS, SR_RATIOS


def _ln(x, w, b, eps):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def _lin(x, sd, p, bias=True):
    y = torch.einsum("...k,nk->...n", x, sd[p + ".weight"])
    return y + sd[p + ".bias"] if bias else y


def _conv_tok(x, B, H, W, w, b, stride, pad):
    """Dense conv on token-major input via explicit im2col (unfold) + einsum."""
    C = x.shape[-1]
    img = x.reshape(B, H, W, C).permute(0, 3, 1, 2)
    kh, kw = w.shape[2], w.shape[3]
    cols = torch.nn.functional.unfold(img, (kh, kw), padding=pad, stride=stride)  # B, C*kh*kw, L
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    y = torch.einsum("bkl,ok->blo", cols, w.reshape(w.shape[0], -1))
    if b is not None:
        y = y + b
    return y, Ho, Wo


def _dw3(x, B, H, W, w, b):
    """Depthwise 3x3 pad 1 on tokens (dual_segformer.py:27-33, net_utils.py:317)."""
    C = x.shape[-1]
    img = x.reshape(B, H, W, C)
    pad = torch.nn.functional.pad(img, (0, 0, 1, 1, 1, 1))
    out = torch.zeros_like(img)
    for i in range(3):
        for j in range(3):
            out = out + pad[:, i:i + H, j:j + W, :] * w[:, 0, i, j]
    return (out + b).reshape(B, H * W, C)


def _bn(x, sd, p, eps, mode):
    """BatchNorm over token-major (B, N, C)."""
    if mode == "eval":
        mu, var = sd[p + ".running_mean"], sd[p + ".running_var"]
    else:
        mu = x.mean(dim=(0, 1))
        var = ((x - mu) ** 2).mean(dim=(0, 1))
    return (x - mu) / torch.sqrt(var + eps) * sd[p + ".weight"] + sd[p + ".bias"]


def _gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def _bilinear_tok(x, B, H, W, Ho, Wo):
    """Bilinear, align_corners=False, PyTorch source-index rule, on tokens."""
    def axis(n_in, n_out):
        s = n_in / n_out
        src = (torch.arange(n_out, dtype=torch.float64) + 0.5) * s - 0.5
        src = src.clamp(min=0)
        i0 = src.floor().long().clamp(max=n_in - 1)
        i1 = torch.where(i0 < n_in - 1, i0 + 1, i0)
        l1 = src - i0
        return i0, i1, 1 - l1, l1
    C = x.shape[-1]
    img = x.reshape(B, H, W, C)
    y0, y1, wy0, wy1 = axis(H, Ho)
    x0, x1, wx0, wx1 = axis(W, Wo)
    wx0 = wx0.to(x.dtype)[None, None, :, None]
    wx1 = wx1.to(x.dtype)[None, None, :, None]
    rows = img[:, y0] * wy0.to(x.dtype)[None, :, None, None] + img[:, y1] * wy1.to(x.dtype)[None, :, None, None]
    out = rows[:, :, x0] * wx0 + rows[:, :, x1] * wx1
    return out.reshape(B, Ho * Wo, C)


def _block(x, sd, p, B, H, W, heads, R):
    """Block (dual_segformer.py:176-180) with SRA (:116-138) and Mix-FFN (:67-74)."""
    N, C = x.shape[1], x.shape[2]
    d = C // heads
    h = _ln(x, sd[p + ".norm1.weight"], sd[p + ".norm1.bias"], 1e-6)
    q = _lin(h, sd, p + ".attn.q").reshape(B, N, heads, d)
    if R > 1:
        xs, _, _ = _conv_tok(h, B, H, W, sd[p + ".attn.sr.weight"], sd[p + ".attn.sr.bias"], R, 0)
        xs = _ln(xs, sd[p + ".attn.norm.weight"], sd[p + ".attn.norm.bias"], 1e-5)
    else:
        xs = h
    kv = _lin(xs, sd, p + ".attn.kv").reshape(B, -1, 2, heads, d)
    k, v = kv[:, :, 0], kv[:, :, 1]
    s = torch.einsum("bnhd,bmhd->bhnm", q, k) * d ** -0.5
    a = torch.softmax(s, -1)
    o = torch.einsum("bhnm,bmhd->bnhd", a, v).reshape(B, N, C)
    x = x + _lin(o, sd, p + ".attn.proj")
    h = _ln(x, sd[p + ".norm2.weight"], sd[p + ".norm2.bias"], 1e-6)
    h = _lin(h, sd, p + ".mlp.fc1")
    h = _gelu(_dw3(h, B, H, W, sd[p + ".mlp.dwconv.dwconv.weight"], sd[p + ".mlp.dwconv.dwconv.bias"]))
    return x + _lin(h, sd, p + ".mlp.fc2")


def _frm(x1, x2, sd, p):
    """FeatureRectifyModule (net_utils.py:124-152) on tokens (B, N, C)."""
    B, N, C = x1.shape
    cat = torch.cat([x1, x2], -1)
    pooled = torch.cat([cat.mean(1), cat.amax(1)], -1)
    y = torch.relu(_lin(pooled, sd, p + ".channel_weights.mlp.0"))
    cw = torch.sigmoid(_lin(y, sd, p + ".channel_weights.mlp.2"))       # (B, 2C)
    cw0, cw1 = cw[:, None, :C], cw[:, None, C:]
    w0 = sd[p + ".spatial_weights.mlp.0.weight"][:, :, 0, 0]
    hsp = torch.relu(torch.einsum("bnk,ok->bno", cat, w0) + sd[p + ".spatial_weights.mlp.0.bias"])
    w2 = sd[p + ".spatial_weights.mlp.2.weight"][:, :, 0, 0]
    sw = torch.sigmoid(torch.einsum("bnk,ok->bno", hsp, w2) + sd[p + ".spatial_weights.mlp.2.bias"])
    sw0, sw1 = sw[..., 0:1], sw[..., 1:2]
    o1 = x1 + 0.5 * cw1 * x2 + 0.5 * sw1 * x2
    o2 = x2 + 0.5 * cw0 * x1 + 0.5 * sw0 * x1
    return o1, o2


def _ffm(x1, x2, sd, p, B, H, W, heads, bn_mode):
    """FeatureFusionModule (net_utils.py:354-384) = CrossPath + ChannelEmbed."""
    N, C = x1.shape[1], x1.shape[2]
    d = C // heads
    c = p + ".cross"
    a1 = torch.relu(_lin(x1, sd, c + ".channel_proj1"))
    a2 = torch.relu(_lin(x2, sd, c + ".channel_proj2"))
    y1, u1 = a1[..., :C], a1[..., C:]
    y2, u2 = a2[..., :C], a2[..., C:]
    kv1 = _lin(u1, sd, c + ".cross_attn.kv1", bias=False).reshape(B, N, 2, heads, d)
    kv2 = _lin(u2, sd, c + ".cross_attn.kv2", bias=False).reshape(B, N, 2, heads, d)
    ctx1 = torch.softmax(torch.einsum("bnhi,bnhj->bhij", kv1[:, :, 0], kv1[:, :, 1]) * d ** -0.5, 2)
    ctx2 = torch.softmax(torch.einsum("bnhi,bnhj->bhij", kv2[:, :, 0], kv2[:, :, 1]) * d ** -0.5, 2)
    v1 = torch.einsum("bnhi,bhij->bnhj", u1.reshape(B, N, heads, d), ctx2).reshape(B, N, C)
    v2 = torch.einsum("bnhi,bhij->bnhj", u2.reshape(B, N, heads, d), ctx1).reshape(B, N, C)
    o1 = _ln(x1 + _lin(torch.cat([y1, v1], -1), sd, c + ".end_proj1"),
             sd[c + ".norm1.weight"], sd[c + ".norm1.bias"], 1e-5)
    o2 = _ln(x2 + _lin(torch.cat([y2, v2], -1), sd, c + ".end_proj2"),
             sd[c + ".norm2.weight"], sd[c + ".norm2.bias"], 1e-5)
    m = torch.cat([o1, o2], -1)
    e = p + ".channel_emb"
    res = torch.einsum("bnk,ok->bno", m, sd[e + ".residual.weight"][:, :, 0, 0])
    t = torch.einsum("bnk,ok->bno", m, sd[e + ".channel_embed.0.weight"][:, :, 0, 0]) + sd[e + ".channel_embed.0.bias"]
    t = torch.relu(_dw3(t, B, H, W, sd[e + ".channel_embed.1.weight"], sd[e + ".channel_embed.1.bias"]))
    t = torch.einsum("bnk,ok->bno", t, sd[e + ".channel_embed.3.weight"][:, :, 0, 0]) + sd[e + ".channel_embed.3.bias"]
    t = _bn(t, sd, e + ".channel_embed.4", 1e-5, bn_mode)
    return _bn(res + t, sd, e + ".norm", 1e-5, bn_mode)


def forward(sd, rgb, modal_x, backbone="mit_b2", bn_mode="eval", dec_bn_eps=1e-3,
            return_features=False):
    """Logits (B, K, H, W) of EncoderDecoder.encode_decode (builder.py:212-238)."""
    spec = MIT_SPECS[backbone]
    dims, depths = spec["embed_dims"], spec["depths"]
    B, _, Hi, Wi = rgb.shape
    xs = [rgb.permute(0, 2, 3, 1).reshape(B, Hi * Wi, 3), modal_x.permute(0, 2, 3, 1).reshape(B, Hi * Wi, 3)]
    H, W = Hi, Wi
    feats = []
    for s in range(4):
        k, st = (7, 4) if s == 0 else (3, 2)
        nxt = []
        for g, pre in enumerate(("", "extra_")):
            pe = f"backbone.{pre}patch_embed{s + 1}"
            t, Ho, Wo = _conv_tok(xs[g], B, H, W, sd[pe + ".proj.weight"], sd[pe + ".proj.bias"], st, k // 2)
            t = _ln(t, sd[pe + ".norm.weight"], sd[pe + ".norm.bias"], 1e-5)
            for i in range(depths[s]):
                t = _block(t, sd, f"backbone.{pre}block{s + 1}.{i}", B, Ho, Wo, NUM_HEADS[s], SR_RATIOS[s])
            t = _ln(t, sd[f"backbone.{pre}norm{s + 1}.weight"], sd[f"backbone.{pre}norm{s + 1}.bias"], 1e-6)
            nxt.append(t)
        H, W = Ho, Wo
        x1, x2 = _frm(nxt[0], nxt[1], sd, f"backbone.FRMs.{s}")
        xs = [x1, x2]
        feats.append((_ffm(x1, x2, sd, f"backbone.FFMs.{s}", B, H, W, NUM_HEADS[s], bn_mode), H, W))
    # MLPDecoder.py:59-81 on tokens
    H1, W1 = feats[0][1], feats[0][2]
    parts = []
    for idx in (3, 2, 1, 0):
        f, h, w = feats[idx]
        t = _lin(f, sd, f"decode_head.linear_c{idx + 1}.proj")
        parts.append(_bilinear_tok(t, B, h, w, H1, W1) if idx > 0 else t)
    cat = torch.cat(parts, -1)
    t = torch.einsum("bnk,ok->bno", cat, sd["decode_head.linear_fuse.0.weight"][:, :, 0, 0]) + sd["decode_head.linear_fuse.0.bias"]
    t = torch.relu(_bn(t, sd, "decode_head.linear_fuse.1", dec_bn_eps, bn_mode))
    t = torch.einsum("bnk,ok->bno", t, sd["decode_head.linear_pred.weight"][:, :, 0, 0]) + sd["decode_head.linear_pred.bias"]
    out = _bilinear_tok(t, B, H1, W1, Hi, Wi)
    logits = out.reshape(B, Hi, Wi, -1).permute(0, 3, 1, 2)
    return (logits, feats) if return_features else logits


def cross_entropy(logits, label, ignore=255):
    """nn.CrossEntropyLoss(mean, ignore_index=255): mean over non-ignored pixels."""
    lp = torch.log_softmax(logits, 1)
    valid = label != ignore
    tgt = torch.where(valid, label, torch.zeros_like(label))
    nll = -lp.gather(1, tgt[:, None]).squeeze(1)
    return (nll * valid).sum() / valid.sum()
