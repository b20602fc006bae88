"""SegFormer all-MLP decode head (reference: models/decoders/MLPDecoder.py:8-81).

Execution on tokens: linear_c{1..4}, the upsample, the concat and the linear_fuse 1x1 conv as
functions.DecoderFoldF (each projection folded into its slot of the conv: M_i = Wf_i Wc_i, the
composed products at each branch's own resolution, the bilinear upsample added in the c1 GEMM's
epilogue; neither the projections nor the (B, N1, 4E) concat are formed).  CMX_DECODER_FOLD=0:
linear_c{1..4} as one multi GEMM launch (functions.GLinearMulti) ahead of functions.DecoderFuseF;
BatchNorm (SyncBN across ranks when a process group is given) + ReLU + Dropout2d fused into
one apply kernel; linear_pred GEMM.  Returns low-resolution logits (B*N1, K).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import functions as F


class MLP(nn.Module):
    def __init__(self, input_dim=2048, embed_dim=768):
        super().__init__()
        self.proj = nn.Linear(input_dim, embed_dim)


class DecoderHead(nn.Module):
    def __init__(self, in_channels=(64, 128, 320, 512), num_classes=40, dropout_ratio=0.1,
                 norm_layer=nn.BatchNorm2d, embed_dim=768, align_corners=False):
        super().__init__()
        self.num_classes = num_classes
        self.dropout_ratio = dropout_ratio
        self.in_channels = list(in_channels)
        self.embed_dim = embed_dim
        c1, c2, c3, c4 = in_channels
        self.linear_c4 = MLP(c4, embed_dim)
        self.linear_c3 = MLP(c3, embed_dim)
        self.linear_c2 = MLP(c2, embed_dim)
        self.linear_c1 = MLP(c1, embed_dim)
        self.linear_fuse = nn.Sequential(nn.Conv2d(4 * embed_dim, embed_dim, 1), nn.BatchNorm2d(embed_dim),
                                         nn.ReLU(inplace=True))
        self.linear_pred = nn.Conv2d(embed_dim, num_classes, 1)

    def run(self, store, feats, grids, B, training, dscale=None, group=None):
        E = self.embed_dim
        lin = (self.linear_c1, self.linear_c2, self.linear_c3, self.linear_c4)
        H1, W1 = grids[0]
        M = B * H1 * W1
        conv = self.linear_fuse[0]
        G = 1
        Wf = store.w(conv.weight).view(G, E, 4 * E)
        Wfg = store.g(conv.weight).view(G, E, 4 * E)
        bf = store.w(conv.bias, compute=False).view(G, E)
        bfg = store.g(conv.bias).view(G, E)
        sizes = [grids[0]] + list(grids[1:])
        if F.DECODER_FOLD:
            # linear_c{1..4} folded into linear_fuse: M_i = Wf_i Wc_i formed per step (DecoderFoldF)
            order = (3, 2, 1, 0)                  # Wf's column slots: c4, c3, c2, c1
            Wc = tuple(store.w(lin[i].proj.weight, stacked=False) for i in order)
            bc = tuple(store.w(lin[i].proj.bias, stacked=False, compute=False) for i in order)
            grads = (Wfg, bfg.view(E), tuple(store.g(lin[i].proj.weight) for i in order),
                     tuple(store.g(lin[i].proj.bias, stacked=False) for i in order))
            x = [t.view(B, -1, t.shape[-1]) for t in feats]
            f = F.DecoderFoldF.apply(x[3], x[2], x[1], x[0], Wf[0], Wc, bf.view(E), bc, grads, sizes, conv.weight)
        else:
            # the four projections as ONE GEMM launch (and their input gradients as another)
            outs = F.glinear_multi(store, [(lin[i].proj.weight, lin[i].proj.bias,
                                            feats[i].view(1, -1, feats[i].shape[-1])) for i in range(4)])
            proj = [t.view(B, -1, E) for t in outs]
            f = F.DecoderFuseF.apply(proj[3], proj[2], proj[1], proj[0], Wf, Wfg, bf, bfg, sizes, conv.weight)
        f = F.batchnorm(store, self.linear_fuse[1], f.view(M, E), training, act="relu", dscale=dscale,
                        rps=H1 * W1, group=group)
        return F.glinear(store, self.linear_pred.weight, self.linear_pred.bias, f.view(1, M, E)).view(M, -1)
