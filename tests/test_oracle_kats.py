"""Hand-derived known-answer tests pinning the CPU oracle (oracle/cmx_ref.py) to behaviours
read from the reference source.  The reference publishes no fixtures
and could not be imported (denied), so these KATs plus the two-restatement
cross-check (test_oracle_selfcheck.py) are what pins the oracle."""
import math

import pytest
import torch
import torch.nn as nn

from oracle import cmx_ref as R
from oracle import cmx_functional as FN
from oracle.train_ref import WarmUpPolyLR, group_weight


def test_ffm_softmax_axis_and_crossing():
    """net_utils.py:206-212: ctx = softmax over dim -2 (the key-feature row), out1 = q1 @ ctx2."""
    torch.manual_seed(0)
    ca = R.CrossAttention(4, 1).double()
    x1 = torch.randn(1, 5, 4, dtype=torch.float64)
    x2 = torch.randn(1, 5, 4, dtype=torch.float64)
    o1, o2 = ca(x1, x2)
    kv2 = ca.kv2(x2)
    k2, v2 = kv2[..., :4], kv2[..., 4:]
    A = (k2[0].t() @ v2[0]) * 4 ** -0.5
    ctx2 = torch.exp(A) / torch.exp(A).sum(0, keepdim=True)       # columns sum to 1
    assert torch.allclose(ctx2.sum(0), torch.ones(4, dtype=torch.float64))
    assert torch.allclose(o1[0], x1[0] @ ctx2, atol=1e-12)        # q1 with the OTHER context
    kv1 = ca.kv1(x1)
    A1 = (kv1[0, :, :4].t() @ kv1[0, :, 4:]) * 0.5
    ctx1 = torch.softmax(A1, 0)
    assert torch.allclose(o2[0], x2[0] @ ctx1, atol=1e-12)
    assert ca.kv1.bias is None and ca.kv2.bias is None            # qkv_bias=False


def test_sra_kv_split_and_heads():
    """dual_segformer.py:125-128: kv output channels are [K(h0..hH) | V(h0..hH)]."""
    torch.manual_seed(0)
    att = R.Attention(8, 2, 1).double()
    with torch.no_grad():
        att.q.weight.copy_(torch.eye(8)); att.q.bias.zero_()
        att.kv.weight.zero_(); att.kv.bias.zero_()
        att.kv.weight[:8] = torch.eye(8) * 0.0                     # K = 0 -> uniform attention
        att.kv.weight[8:] = torch.eye(8)                           # V = x
        att.proj.weight.copy_(torch.eye(8)); att.proj.bias.zero_()
    x = torch.randn(1, 6, 8, dtype=torch.float64)
    out = att(x, 2, 3)
    assert torch.allclose(out, x.mean(1, keepdim=True).expand_as(x), atol=1e-12)


def test_stage_grids_floor_semantics_b0_240x320():
    """OverlapPatchEmbed / SR conv floor sizes at 240x320: 60x80, 30x40, 15x20, 8x10, Nk=70."""
    from rgbx_semantic_segmentation_amd.flops import _grid
    h, w = 240, 320
    grids = []
    for s in range(4):
        k, st = (7, 4) if s == 0 else (3, 2)
        h, w = _grid(h, w, k, st, k // 2)
        grids.append((h, w))
    assert grids == [(60, 80), (30, 40), (15, 20), (8, 10)]
    hk, wk = _grid(60, 80, 8, 8, 0)
    assert hk * wk == 70
    conv = nn.Conv2d(1, 1, 8, 8)
    assert conv(torch.zeros(1, 1, 60, 80)).shape[-2:] == (7, 10)


def test_norm_eps_values():
    m = R.EncoderDecoder(R.CMXConfig(backbone="mit_b0", num_classes=3))
    bb = m.backbone
    assert bb.block1[0].norm1.eps == 1e-6 and bb.norm1.eps == 1e-6 and bb.extra_norm4.eps == 1e-6
    assert bb.patch_embed1.norm.eps == 1e-5 and bb.block1[0].attn.norm.eps == 1e-5
    assert bb.FFMs[0].cross.norm1.eps == 1e-5
    assert bb.FFMs[0].channel_emb.norm.eps == 1e-5 and bb.FFMs[0].channel_emb.channel_embed[4].eps == 1e-5
    assert m.decode_head.linear_fuse[1].eps == 1e-3 and m.decode_head.linear_fuse[1].momentum == 0.1


def test_bilinear_align_corners_false_hand_values():
    """src = max(0, (dst+0.5)*in/out - 0.5): upsampling [0, 10] (1x2) to width 4."""
    x = torch.tensor([[[[0.0, 10.0]]]], dtype=torch.float64)
    y = torch.nn.functional.interpolate(x, size=(1, 4), mode="bilinear", align_corners=False)
    # dst 0: src -0.25 -> 0 -> 0 ; dst 1: 0.25 -> 2.5 ; dst 2: 0.75 -> 7.5 ; dst 3: 1.25 -> clamp 10
    assert torch.allclose(y.flatten(), torch.tensor([0.0, 2.5, 7.5, 10.0], dtype=torch.float64))
    t = x.permute(0, 2, 3, 1).reshape(1, 2, 1)
    z = FN._bilinear_tok(t, 1, 1, 2, 1, 4)
    assert torch.allclose(z.flatten(), y.flatten())


def test_ce_mean_over_valid_pixels_with_ignore():
    logits = torch.zeros(1, 2, 1, 3, dtype=torch.float64)
    logits[0, 0, 0, 0] = math.log(3.0)                        # p(class0) = 3/4 at pixel 0
    lab = torch.tensor([[[0, 1, 255]]])
    ce = nn.CrossEntropyLoss(reduction="mean", ignore_index=255)(logits, lab)
    expect = (-math.log(0.75) - math.log(0.5)) / 2            # ignored pixel excluded from the mean
    assert abs(ce.item() - expect) < 1e-12
    assert abs(FN.cross_entropy(logits, lab).item() - expect) < 1e-12


def test_frm_index_pairing():
    """net_utils.py:150-151: out1 = x1 + .5*cw[1]*x2 + .5*sw[1]*x2 (cw/sw index 1 -> applied to x2)."""
    torch.manual_seed(0)
    frm = R.FeatureRectifyModule(2).double()
    x1 = torch.randn(1, 2, 2, 2, dtype=torch.float64)
    x2 = torch.randn(1, 2, 2, 2, dtype=torch.float64)
    cw = frm.channel_weights(x1, x2)
    sw = frm.spatial_weights(x1, x2)
    o1, o2 = frm(x1, x2)
    assert torch.allclose(o1, x1 + 0.5 * cw[1] * x2 + 0.5 * sw[1] * x2)
    assert torch.allclose(o2, x2 + 0.5 * cw[0] * x1 + 0.5 * sw[0] * x1)
    # channel weights come from [avg(cat) | max(cat)] -> mlp -> (B, 2C) split as [cw0 | cw1]
    cat = torch.cat([x1, x2], 1)
    y = frm.channel_weights.mlp(torch.cat([cat.mean((2, 3)), cat.amax((2, 3))], 1))
    assert torch.allclose(cw[0].flatten(), y[0, :2]) and torch.allclose(cw[1].flatten(), y[0, 2:])


def test_drop_path_table_stage2_quirk():
    """dual_segformer.py:249-311: block2[i] -> dpr[cur], extra_block2[i] -> dpr[cur+1]."""
    dpr = [x.item() for x in torch.linspace(0, 0.1, 16)]
    t = R.drop_path_table([3, 4, 6, 3], 0.1)
    assert t[0][0] == dpr[0:3] and t[0][1] == dpr[0:3]
    assert t[1][0] == [dpr[3]] * 4 and t[1][1] == [dpr[4]] * 4
    assert t[2][0] == dpr[7:13] and t[3][0] == dpr[13:16]
    from rgbx_semantic_segmentation_amd.models.encoders.dual_segformer import drop_path_probs
    assert drop_path_probs([3, 4, 6, 3], 0.1) == t


def test_lr_applied_one_step_late():
    """train.py:201-207: step 0 uses the constructor LR, step 1 uses get_lr(0) = 0."""
    p = nn.Parameter(torch.ones(1))
    opt = torch.optim.AdamW([p], lr=6e-5, weight_decay=0.0)
    pol = WarmUpPolyLR(6e-5, 0.9, 1000, 10)
    used = []
    for idx in range(3):
        used.append(opt.param_groups[0]["lr"])
        p.grad = torch.ones(1)
        opt.step()
        for g in opt.param_groups:
            g["lr"] = pol.get_lr(idx)
    assert used == [6e-5, 0.0, 6e-6]


def test_group_weight_partition():
    m = R.EncoderDecoder(R.CMXConfig(backbone="mit_b0", num_classes=3))
    groups = group_weight(m, 6e-5)
    n_decay, n_no = len(groups[0]["params"]), len(groups[1]["params"])
    assert n_decay + n_no == len(list(m.parameters()))
    assert groups[1]["weight_decay"] == 0.0
    decay_ids = {id(p) for p in groups[0]["params"]}
    for mod in m.modules():
        if isinstance(mod, (nn.Linear, nn.Conv2d)):
            assert id(mod.weight) in decay_ids
            if mod.bias is not None:
                assert id(mod.bias) not in decay_ids


def test_param_count_b2():
    assert R.count_params(R.EncoderDecoder(R.CMXConfig(backbone="mit_b2", num_classes=40))) == 66581424


def test_fast_erf_table():
    """cmx_erf (csrc/cmx_common.h) evaluated in float32 with the coefficients parsed from
    the header: max |erf error| <= 5e-7 on [-6, 6] (the GELU kernels' accuracy budget)."""
    import math
    import os
    import re
    import numpy as np
    src = open(os.path.join(os.path.dirname(__file__), "..", "rgbx_semantic_segmentation_amd", "csrc",
                            "cmx_common.h")).read()
    body = src[src.index("float cmx_erf(float x)"):]
    body = body[:body.index("return x * p")]
    lits = [np.float32(v) for v in re.findall(r"(-?\d\.\d+e-\d+)f", body)]
    assert len(lits) == 12
    f = np.float32
    x = np.linspace(-6, 6, 40001).astype(f)
    xc = np.clip(x, f(-4), f(4))
    x2 = xc * xc
    p = np.full_like(x2, lits[0])
    for a in lits[1:7]:
        p = p * x2 + a
    q = np.full_like(x2, lits[7])
    for b in lits[8:]:
        q = q * x2 + b
    r = xc * p * (f(1) / q)
    ref = np.array([math.erf(float(v)) for v in x])
    assert np.abs(r.astype(np.float64) - ref).max() < 5e-7
