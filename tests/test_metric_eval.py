"""Evaluation path: mIoU confusion matrix and the sliding-window evaluator.

CPU: the oracle (oracle/metric_ref.py) against hand-computed known answers of
utils/metric.py:8-29 and the window geometry of engine/evaluator.py:326-372.
GPU: the HIP kernels (csrc/metric.hip) through the C-ABI -- confusion matrix bit-exact
against the oracle; the device evaluator against the oracle evaluator on the same
(deterministic, per-pixel linear) network: fp32 tolerance 1e-5 relative on the summed
probabilities, identical class maps where the oracle's top-2 margin exceeds 1e-4.
cv2 itself is not installed (requirements.txt:4): resizes are pinned to the half-pixel rule,
"parity unpinned" against cv2 proper (see the oracle's header).
"""
import numpy as np
import pytest
import torch

from oracle import metric_ref as R


# ---------------------------------------------------------------------------- CPU
def test_hist_info_kat():
    gt = np.array([[0, 1, 2], [2, 255, 1]])
    pred = np.array([[0, 2, 2], [1, 0, 1]])
    cm, labeled, correct = R.hist_info(3, pred, gt)
    assert labeled == 5 and correct == 3
    assert cm.tolist() == [[1, 0, 0], [0, 1, 1], [0, 1, 1]]
    iou, miou, _, fiou, macc, pacc = R.compute_score(cm.astype(np.float64), correct, labeled)
    np.testing.assert_allclose(iou, [1.0, 1 / 3, 1 / 3])
    assert abs(miou - 5 / 9) < 1e-12 and abs(pacc - 0.6) < 1e-12
    np.testing.assert_allclose(macc, np.mean([1.0, 0.5, 0.5]))
    np.testing.assert_allclose(fiou, 0.2 * 1.0 + 0.4 / 3 + 0.4 / 3)


def test_pad_margins_and_resize_identity():
    a = np.arange(12, dtype=np.float64).reshape(3, 4)
    p, m = R.pad_image_to_shape(a, (6, 5))
    assert m.tolist() == [1, 2, 0, 1] and p.shape == (6, 5) and p[1:4, 0:4].tolist() == a.tolist()
    np.testing.assert_array_equal(R.resize_linear(a, 3, 4), a)
    # 2x upscale of a ramp: half-pixel centres, edges clamped
    r = R.resize_linear(np.array([[0.0, 4.0]]), 1, 4)
    np.testing.assert_allclose(r, [[0.0, 1.0, 3.0, 4.0]])


class LinearNet:
    """Deterministic stand-in network: per-pixel linear logits of rgb and x (K x 3 each)."""

    def __init__(self, K, seed=0):
        g = np.random.default_rng(seed)
        self.Wr = g.standard_normal((K, 3)).astype(np.float32) * 0.5
        self.Wx = g.standard_normal((K, 3)).astype(np.float32) * 0.5
        self.b = g.standard_normal(K).astype(np.float32) * 0.1

    def np_forward(self, d, x):
        return (np.einsum("kc,bchw->bkhw", self.Wr, d) + np.einsum("kc,bchw->bkhw", self.Wx, x)
                + self.b[None, :, None, None])


def test_oracle_window_quirk_covers_bottom_band_only():
    """The reference's swapped-index window loop (evaluator.py:352-357) on a 600 x 800 image with a
    480 x 640 crop covers only the bottom 40 rows; the oracle reproduces that."""
    K = 3
    net = LinearNet(K)
    ev = R.SlidingEvaluatorRef(K, np.zeros(3), np.ones(3) / 255.0, net.np_forward, [1.0], False)
    img = np.ones((600, 800, 3))
    s = ev.scale_process_rgbX(img, img, (600, 800), (480, 640), 2 / 3)
    assert np.all(s[:560] == 0) and np.all(s[560:] > 0)


# ---------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("K,H,W,ldt", [(40, 61, 83, torch.int64), (9, 480, 640, torch.uint8), (3, 7, 5, torch.int64)])
def test_argmax_confusion_bit_exact(dev, K, H, W, ldt):
    from rgbx_semantic_segmentation_amd.utils.metric import ConfusionCounter, hist_info
    g = torch.Generator().manual_seed(K)
    score = torch.rand(K, H, W, generator=g)
    score[:, :2, :3] = 0.5                                   # ties: first maximum wins
    score[1, 0, 0] = float("nan")                            # NaN wins, as numpy argmax
    gt = torch.randint(0, K, (H, W), generator=g)
    gt[torch.rand(H, W, generator=g) < 0.1] = 255
    gt = gt.to(ldt)
    cc = ConfusionCounter(K, dev)
    pred = torch.empty(H, W, dtype=torch.int32, device=dev)
    cc.add_score(score.to(dev), gt.to(dev), pred_out=pred)
    cc.add_score(score.to(dev), gt.to(dev))                  # counts accumulate
    h, lab, cor = cc.result()
    pred_ref = score.numpy().argmax(0)
    np.testing.assert_array_equal(pred.cpu().numpy(), pred_ref)
    cm, l_ref, c_ref = R.hist_info(K, pred_ref, gt.numpy().astype(np.int64))
    np.testing.assert_array_equal(h, 2 * cm)
    assert (lab, cor) == (2 * l_ref, 2 * c_ref)
    # hist_info on a given class map (numpy in, numpy out), as utils/metric.py
    cm2, l2, c2 = hist_info(K, pred_ref, gt.numpy())
    np.testing.assert_array_equal(cm2, cm)
    assert (l2, c2) == (l_ref, c_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("flip", [False, True])
def test_window_accumulate(dev, flip):
    from rgbx_semantic_segmentation_amd import _lib
    K, ch, cw, PH, PW = 5, 20, 24, 40, 50
    m = (3, 2, 4, 1)
    s1 = torch.randn(K, ch, cw, device=dev)
    s2 = torch.randn(K, ch, cw, device=dev) if flip else None
    acc = torch.rand(K, PH, PW, device=dev)
    ref = acc.clone()
    sc = s1 + s2.flip(-1) if flip else s1
    h, w = ch - m[0] - m[1], cw - m[2] - m[3]
    ref[:, 7:7 + h, 11:11 + w] += torch.exp(sc)[:, m[0]:ch - m[1], m[2]:cw - m[3]]
    _lib.call("cmx_seg_window_accumulate", _lib.ptr(s1), _lib.ptr(s2), _lib.ptr(acc), K, ch, cw, *m, PH, PW, 7, 11,
              _lib.stream())
    torch.cuda.synchronize()
    torch.testing.assert_close(acc, ref, rtol=1e-6, atol=0)
    with pytest.raises(RuntimeError):
        _lib.call("cmx_seg_window_accumulate", _lib.ptr(s1), None, _lib.ptr(acc), K, ch, cw, *m, PH, PW, 30, 40,
                  _lib.stream())


class TorchLinearNet(torch.nn.Module):
    def __init__(self, ref: LinearNet, dev):
        super().__init__()
        self.Wr = torch.tensor(ref.Wr, device=dev)
        self.Wx = torch.tensor(ref.Wx, device=dev)
        self.b = torch.tensor(ref.b, device=dev)

    def forward(self, d, x):
        return (torch.einsum("kc,bchw->bkhw", self.Wr, d) + torch.einsum("kc,bchw->bkhw", self.Wx, x)
                + self.b[None, :, None, None])


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,crop,scales,flip", [
    (48, 64, (48, 64), [0.75, 1, 1.25], False),              # NYU geometry scaled by 1/10 (quirky sliding at 1.25)
    (50, 70, (32, 32), [1.0], True),                         # square crop: regular sliding windows, flip
    (30, 20, (32, 32), [1.0, 1.5], False),                   # image smaller than the crop: padded
])
def test_evaluator_matches_oracle(dev, H, W, crop, scales, flip):
    from rgbx_semantic_segmentation_amd.engine.evaluator import Evaluator
    K = 6
    net = LinearNet(K, seed=H)
    rng = np.random.default_rng(W)
    img = rng.uniform(0, 255, (H, W, 3))
    x = rng.uniform(0, 255, (H, W, 3))
    gt = rng.integers(0, K, (H, W))
    mean, std = np.array([0.485, 0.456, 0.406]), np.array([0.229, 0.224, 0.225])
    ref = R.SlidingEvaluatorRef(K, mean, std, net.np_forward, scales, flip)
    pred_ref = ref.sliding_eval_rgbX(img, x, crop, 2 / 3)
    # summed probabilities of the oracle, to find near-ties
    tot = sum(ref.scale_process_rgbX(R.resize_linear(img, int(round(H * s)), int(round(W * s))) if s != 1 else img,
                                     R.resize_linear(x, int(round(H * s)), int(round(W * s))) if s != 1 else x,
                                     (H, W), crop, 2 / 3) for s in scales)
    ev = Evaluator(None, K, mean, std, TorchLinearNet(net, dev), scales, flip, [0])
    score = ev.sliding_scores_rgbX(img, x, crop, 2 / 3, dev).cpu().numpy().transpose(1, 2, 0)
    np.testing.assert_allclose(score, tot, rtol=1e-5, atol=1e-6 * np.abs(tot).max())
    pred = ev.sliding_eval_rgbX(img, x, crop, 2 / 3, dev)
    srt = np.sort(tot, axis=2)
    clear = (srt[..., -1] - srt[..., -2]) > 1e-4 * srt[..., -1]
    np.testing.assert_array_equal(pred[clear], pred_ref[clear])
    # and the dataset pass: confusion matrix of the device argmax
    from rgbx_semantic_segmentation_amd.utils.metric import compute_score

    class DS:
        def get_length(self):
            return 1

        def __getitem__(self, i):
            return {"data": img, "modal_x": x, "label": gt}
    res = ev.run(DS(), crop, 2 / 3, dev)
    cm, lab, cor = R.hist_info(K, pred, gt)
    exp = compute_score(cm.astype(np.float64), cor, lab)
    np.testing.assert_allclose(res[1], exp[1])


@pytest.mark.gpu
def test_evaluator_runs_hip_model(dev):
    """The evaluator drives the HIP EncoderDecoder forward (eval mode) end to end."""
    from rgbx_semantic_segmentation_amd.engine.evaluator import Evaluator
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    torch.manual_seed(0)
    K = 9
    model = EncoderDecoder(dict(backbone="mit_b0", num_classes=K, compute_dtype="bfloat16",
                                decoder_embed_dim=256)).to(dev)
    rng = np.random.default_rng(0)
    img = rng.uniform(0, 255, (64, 96, 3))
    ev = Evaluator(None, K, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225], model, [1.0, 0.5], True, [0])
    pred = ev.sliding_eval_rgbX(img, img, (64, 64), 2 / 3, dev)
    assert pred.shape == (64, 96) and pred.min() >= 0 and pred.max() < K
    # batched crops (one forward over every crop and mirror) against one bs=1 forward per crop:
    # the same scores up to the bf16 network's batch-shape-dependent GEMM splits
    sb = ev.sliding_scores_rgbX(img, img, (64, 64), 2 / 3, dev)
    assert len(ev._graphs) > 0                       # the crop batches replayed HIP graphs
    sb2 = ev.sliding_scores_rgbX(img, img, (64, 64), 2 / 3, dev)
    assert torch.equal(sb, sb2)                      # replays of the cached graphs: identical
    ev.eval_graph = False
    se = ev.sliding_scores_rgbX(img, img, (64, 64), 2 / 3, dev)
    assert torch.equal(sb, se)                       # graph replay = the eager launches
    ev.eval_batch = 1
    s1 = ev.sliding_scores_rgbX(img, img, (64, 64), 2 / 3, dev)
    torch.testing.assert_close(sb, s1, rtol=2e-2, atol=2e-2 * float(s1.abs().max()))


@pytest.mark.gpu
def test_evaluator_graph_cache_of_one(dev):
    """CMX_EVAL_GRAPHS=1: with a one-graph cache, a second crop shape must capture
    while the first shape's graph -- the shared pool's only user -- is still alive, and then
    evict it; both shapes replay the eager result."""
    from rgbx_semantic_segmentation_amd.engine.evaluator import Evaluator
    from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder
    torch.manual_seed(0)
    K = 9
    model = EncoderDecoder(dict(backbone="mit_b0", num_classes=K, compute_dtype="bfloat16",
                                decoder_embed_dim=256)).to(dev)
    rng = np.random.default_rng(2)
    img = rng.uniform(0, 255, (64, 96, 3))
    ev = Evaluator(None, K, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225], model, [1.0], False, [0])
    ev.eval_graph_cap = 1
    got = [ev.sliding_scores_rgbX(img, img, c, 2 / 3, dev).clone() for c in ((64, 64), (64, 96), (64, 64))]
    assert len(ev._graphs) == 1
    ev.eval_graph = False
    exp = [ev.sliding_scores_rgbX(img, img, c, 2 / 3, dev) for c in ((64, 64), (64, 96), (64, 64))]
    for a, b in zip(got, exp):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("flip", [False, True])
def test_evaluator_batched_windows_match_single(dev, flip):
    """Crops of every scale batched into shared forwards give the per-crop result (a network
    whose per-image output does not depend on the batch: exact up to fp32 einsum order)."""
    from rgbx_semantic_segmentation_amd.engine.evaluator import Evaluator
    K, H, W = 5, 50, 70
    net = TorchLinearNet(LinearNet(K, seed=3), dev)
    rng = np.random.default_rng(1)
    img = rng.uniform(0, 255, (H, W, 3))
    x = rng.uniform(0, 255, (H, W, 3))
    ev = Evaluator(None, K, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225], net, [0.75, 1.0, 1.5], flip, [0])
    outs = []
    for nb in (1, 3, 64):
        ev.eval_batch = nb
        outs.append(ev.sliding_scores_rgbX(img, x, (32, 32), 2 / 3, dev))
    for o in outs[1:]:
        torch.testing.assert_close(o, outs[0], rtol=1e-6, atol=1e-6 * float(outs[0].abs().max()))
