"""cmx_step_masks: the per-step DropPath / Dropout2d masks and the BatchNorm batch counter in
one launch (replaces torch.rand draws inside the captured step).  Checked: values are exactly
{0, 1/keep} and {0, 1/(1-p)}, the keep fractions follow the probabilities (binomial bounds),
successive steps draw different masks (the step counter lives on the device, so this holds
across HIP-graph replays), and every BatchNorm's num_batches_tracked advances by one per
training forward.  Reference: timm DropPath (dual_segformer.py:141-180), Dropout2d
(MLPDecoder.py:63), BatchNorm2d.forward."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_step_masks(dev):
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    torch.manual_seed(0)
    m = EncoderDecoder(dict(backbone="mit_b2", num_classes=9, compute_dtype="bfloat16",
                            decoder_embed_dim=512)).to(dev)
    m.train()
    B = 64                                          # many samples: tight binomial bounds
    keep = torch.tensor(m.backbone.drop_path_keep_probs(), dtype=torch.float32)      # (nb, 2)
    p = m.decode_head.dropout_ratio
    draws = []
    for _ in range(3):
        m._nbt_bumped = False
        dp, d2 = m._stochastic(B, dev)
        torch.cuda.synchronize()
        draws.append((dp.cpu(), d2.cpu()))
    dp, d2 = draws[0]
    kp = keep[:, None, :, None].expand(-1, 2, -1, B).reshape(dp.shape)
    assert torch.all((dp == 0) | torch.isclose(dp, 1 / kp)), "DropPath scales must be 0 or 1/keep"
    assert torch.all((d2 == 0) | torch.isclose(d2, torch.tensor(1 / (1 - p)))), "Dropout2d values"
    for (a, b), (c, d) in zip(draws, draws[1:]):
        assert not torch.equal(a, c) and not torch.equal(b, d), "masks must change from step to step"
    # keep fractions: mean over samples of (scale > 0) vs keep, 6-sigma binomial bound
    kept = torch.stack([(x[0] > 0).float() for x in draws]).mean(0)
    n = 3
    dev_ok = (kept - kp).abs() <= 6 * torch.sqrt(kp * (1 - kp) / n) + 1e-6
    frac = (torch.stack([(x[0] > 0).float() for x in draws]).mean() - kp.mean()).abs()
    assert frac < 0.02 and dev_ok.float().mean() > 0.99, (frac, dev_ok.float().mean())
    d2k = torch.stack([(x[1] > 0).float() for x in draws]).mean()
    assert abs(d2k - (1 - p)) < 0.01, d2k
    # the BN batch counter: one increment per training forward, every BatchNorm
    before = [b.num_batches_tracked.item() for b in m.modules() if isinstance(b, torch.nn.modules.batchnorm._BatchNorm)]
    m._nbt_bumped = False
    m._stochastic(2, dev)
    after = [b.num_batches_tracked.item() for b in m.modules() if isinstance(b, torch.nn.modules.batchnorm._BatchNorm)]
    assert len(before) > 0 and all(a == b + 1 for a, b in zip(after, before)), (before[:4], after[:4])
