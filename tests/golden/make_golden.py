"""Generate tests/golden/cmx_b0_64x96.npz from the CPU oracle.

The reference ships no golden vectors and may not be imported here, so
these fixtures are produced by the build's own restatement (oracle/cmx_ref.py, fp64) and
pin it across environments; the GPU tests then check the HIP path against the same
vectors.  Weights are regenerated from the seed (segformer_init / decoder_init under
torch.manual_seed(0)); `sd_sha256` pins that regeneration bit-for-bit.

Contents (CMX-B0, K=9, bs=2, 64x96, eval mode = BN running statistics, no DropPath):
  rgb, x (2,3,64,96) f32 | label (2,64,96) i64 with a 255 block | sd_sha256
  stage{1..4}: fused encoder outputs (FFM) f64 | logits (2,9,64,96) f64 | loss f64
  grad/<name>: fp32 gradients of the eval-mode loss (first 32 output rows, flattened per row)
               for a few parameters spread over the path

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle.cmx_ref import CMXConfig, EncoderDecoder  # noqa: E402

OUT = os.path.join(HERE, "cmx_b0_64x96.npz")
K, B, H, W = 9, 2, 64, 96
GRAD_PARAMS = [
    "backbone.patch_embed1.proj.weight",
    "backbone.block1.0.attn.q.weight",
    "backbone.extra_block2.1.mlp.dwconv.dwconv.weight",
    "backbone.FRMs.2.channel_weights.mlp.0.weight",
    "backbone.FFMs.3.channel_emb.channel_embed.0.weight",
    "decode_head.linear_fuse.0.weight",
    "decode_head.linear_pred.weight",
]


GRAD_ROWS = 32


def state_dict_sha256(sd) -> str:
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(v.detach().to(torch.float64 if v.is_floating_point() else torch.int64).contiguous().numpy().tobytes())
    return h.hexdigest()


def build_model():
    torch.manual_seed(0)
    return EncoderDecoder(CMXConfig(backbone="mit_b0", num_classes=K))


def make_inputs():
    g = torch.Generator().manual_seed(1)
    rgb = torch.randn(B, 3, H, W, generator=g)
    x = torch.randn(B, 1, H, W, generator=g).expand(B, 3, H, W).contiguous()
    lab = torch.randint(0, K, (B, H, W), generator=g)
    lab[:, 3:9, 5:17] = 255
    return rgb, x, lab


def compute():
    model = build_model()
    sha = state_dict_sha256(model.state_dict())
    model = model.double().eval()
    rgb, x, lab = make_inputs()
    out = {"rgb": rgb.numpy(), "x": x.numpy(), "label": lab.numpy(), "sd_sha256": np.array(sha)}
    with torch.no_grad():
        stages = model.backbone(rgb.double(), x.double())
        for i, s in enumerate(stages):
            out[f"stage{i + 1}"] = s.numpy()
        out["logits"] = model(rgb.double(), x.double()).numpy()
    loss = model(rgb.double(), x.double(), lab)
    loss.backward()
    out["loss"] = np.array(loss.item())
    params = dict(model.named_parameters())
    for n in GRAD_PARAMS:
        g = params[n].grad.view(params[n].shape[0], -1)[:GRAD_ROWS]
        out[f"grad/{n}"] = g.float().numpy()          # fp32, first GRAD_ROWS output rows
    return out


if __name__ == "__main__":
    data = compute()
    np.savez_compressed(OUT, **data)
    print(f"wrote {OUT} ({os.path.getsize(OUT) / 1e6:.2f} MB), sha {data['sd_sha256']}, loss {float(data['loss']):.8f}")
