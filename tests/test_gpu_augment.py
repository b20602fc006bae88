"""GPU TrainPre (csrc/augment.hip via augment.TrainPre) against the CPU restatement
(oracle/augment_ref.py), bit-exact: uint8 outputs of every kernel, the int64 labels and the
float32 normalised images of the whole pipeline (the fp64 normalisation rounds once to fp32
on both sides).  Reference: dataloader/dataloader.py:9-112, utils/transforms.py:182-187.
Sizes: the configs' 480 x 640 under every train_scale_array factor, and ragged 37 x 53 / 57 x 75."""
import random

import numpy as np
import pytest
import gc
import torch

from oracle import augment_ref as A

pytestmark = pytest.mark.gpu

MEAN = [0.485, 0.456, 0.406]
STD = [0.229, 0.224, 0.225]
SCALES = [0.5, 0.75, 1, 1.25, 1.5, 1.75]


def _img(rng, h, w, c=3, hi=256):
    shape = (h, w, c) if c else (h, w)
    return rng.integers(0, hi, shape, dtype=np.uint8)


def _call(name, *args):
    from rgbx_semantic_segmentation_amd import _lib as L
    L.call(name, *args, L.stream())


@pytest.mark.parametrize("h,w,oh,ow", [(480, 640, 240, 320), (480, 640, 840, 1120), (480, 640, 600, 800),
                                       (37, 53, 18, 26), (37, 53, 64, 92), (37, 53, 37, 53), (300, 400, 480, 640)])
@pytest.mark.parametrize("mirror", [0, 1])
def test_resize(dev, h, w, oh, ow, mirror):
    from rgbx_semantic_segmentation_amd import _lib as L
    rng = np.random.default_rng(h * w + oh + mirror)
    img = _img(rng, h, w)
    lab = _img(rng, h, w, 0)
    src = img[:, ::-1] if mirror else img
    lsrc = lab[:, ::-1] if mirror else lab
    g_img, g_lab = torch.from_numpy(img).cuda(), torch.from_numpy(lab).cuda()
    out = torch.empty(oh, ow, 3, dtype=torch.uint8, device="cuda")
    _call("cmx_aug_resize_u8", L.ptr(g_img), h, w, 3, L.ptr(out), oh, ow, 0, mirror, -1)
    assert np.array_equal(out.cpu().numpy(), A.resize_linear_u8(np.ascontiguousarray(src), oh, ow))
    lo = torch.empty(oh, ow, dtype=torch.uint8, device="cuda")
    _call("cmx_aug_resize_u8", L.ptr(g_lab), h, w, 1, L.ptr(lo), oh, ow, 1, mirror, 39)
    assert np.array_equal(lo.cpu().numpy(), A.resize_nearest_u8(np.clip(np.ascontiguousarray(lsrc), 0, 39), oh, ow))


@pytest.mark.parametrize("bf,sf,hf", [(1.0, 1.0, 0.0), (1.2, 0.8, 0.1), (0.8, 1.2, -0.1), (1.137, 0.93, 0.0371),
                                      (0.9, 1.05, -0.0625)])
def test_color_jitter(dev, bf, sf, hf):
    from rgbx_semantic_segmentation_amd import _lib as L
    rng = np.random.default_rng(7)
    img = _img(rng, 61, 83)
    img[0, :27] = [[b, g, r] for b in (0, 128, 255) for g in (0, 128, 255) for r in (0, 128, 255)]   # greys, primaries
    t = torch.from_numpy(img).cuda()
    _call("cmx_aug_color_jitter_u8", L.ptr(t), 61, 83, float(bf), float(sf), float(hf * 180))
    assert np.array_equal(t.cpu().numpy(), A.color_jitter_u8(img, bf, sf, hf))


@pytest.mark.parametrize("h,w", [(480, 640), (37, 53), (5, 5), (3, 7)])
def test_blur(dev, h, w):
    from rgbx_semantic_segmentation_amd import _lib as L
    img = _img(np.random.default_rng(h), h, w)
    t = torch.from_numpy(img).cuda()
    o = torch.empty_like(t)
    _call("cmx_aug_blur5_u8", L.ptr(t), L.ptr(o), h, w, 3)
    assert np.array_equal(o.cpu().numpy(), A.gaussian_blur5_u8(img))


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("h,w,H,W", [(480, 640, 480, 640), (57, 75, 48, 64)])
def test_train_pre_pipeline(dev, seed, h, w, H, W):
    """The whole TrainPre for seeded draws (every scale factor shows up across the seeds):
    GPU TrainPre.apply vs oracle.train_pre with the same parameters, bit-exact."""
    from rgbx_semantic_segmentation_amd.augment import TrainPre, draw_params
    rng = np.random.default_rng(100 + seed)
    rgb, x = _img(rng, h, w), _img(rng, h, w)
    gt = _img(rng, h, w, 0)
    gt[:5, :5] = 255                                     # ignore pixels: clipped to K-1 first (dataloader.py:88)
    pre = TrainPre(MEAN, STD, 40, H, W, SCALES, 255)
    prm = draw_params(h, w, SCALES, random.Random(seed))
    r_g, g_g, x_g = pre.apply(rgb, gt, x, prm)
    r_o, g_o, x_o = A.train_pre(rgb, gt, x, prm, 40, H, W, MEAN, STD)
    assert np.array_equal(g_g.cpu().numpy(), g_o)
    assert np.array_equal(r_g.cpu().numpy(), r_o)
    assert np.array_equal(x_g.cpu().numpy(), x_o)


@pytest.mark.parametrize("seed", range(3))
def test_train_pre_batch_bit_exact(dev, seed):
    """TrainPre.batch (one cmx_aug_batch launch per stage for the whole minibatch, pinned
    staging) vs oracle.train_pre sample by sample with the same draws: bit-exact.  Mixed source
    sizes, host numpy and device samples in one batch, and three batches in a row so both
    staging buffers are reused."""
    from rgbx_semantic_segmentation_amd.augment import TrainPre, draw_params
    H, W = 48, 64
    pre = TrainPre(MEAN, STD, 40, H, W, SCALES, 255, rng=random.Random(seed))
    shadow = random.Random(seed)                       # replays the batch's draws in order
    rng = np.random.default_rng(200 + seed)
    for it in range(3):
        shapes = [(57, 75), (48, 64), (40, 90), (61, 61)][: 2 + it]
        samples, host = [], []
        for j, (h, w) in enumerate(shapes):
            rgb, x = _img(rng, h, w), _img(rng, h, w)
            gt = _img(rng, h, w, 0)
            gt[:3, :4] = 255
            host.append((rgb, gt, x))
            if j % 2:
                samples.append(tuple(torch.from_numpy(a).cuda() for a in (rgb, gt, x)))
            else:
                samples.append((rgb, gt, x[:, :, ::-1].copy()[:, :, ::-1]))   # non-contiguous-safe copy path
        r_g, g_g, x_g = pre.batch(samples)
        for b, (rgb, gt, x) in enumerate(host):
            prm = draw_params(rgb.shape[0], rgb.shape[1], SCALES, shadow)
            r_o, g_o, x_o = A.train_pre(rgb, gt, x, prm, 40, H, W, MEAN, STD)
            assert np.array_equal(g_g[b].cpu().numpy(), g_o), (it, b)
            assert np.array_equal(r_g[b].cpu().numpy(), r_o), (it, b)
            assert np.array_equal(x_g[b].cpu().numpy(), x_o), (it, b)


def test_train_pre_batch_and_loader(dev, tmp_path):
    """get_train_loader(engine, RGBXDataset, config) on PNG files: device batches of the
    reference's dict shape, label values in [0, K-1] or the cutout background."""
    from types import SimpleNamespace
    from PIL import Image
    from rgbx_semantic_segmentation_amd.dataloader import RGBXDataset, get_train_loader
    for d in ("RGB", "Label", "Depth"):
        (tmp_path / d).mkdir()
    rng = np.random.default_rng(9)
    for n in range(3):
        Image.fromarray(_img(rng, 60, 80)).save(tmp_path / "RGB" / f"{n}.png")
        Image.fromarray(_img(rng, 60, 80, 0)).save(tmp_path / "Depth" / f"{n}.png")
        Image.fromarray(_img(rng, 60, 80, 0, 12)).save(tmp_path / "Label" / f"{n}.png")
    (tmp_path / "train.txt").write_text("0\n1\n2\n")
    cfg = SimpleNamespace(rgb_root_folder=str(tmp_path / "RGB"), rgb_format=".png",
                          gt_root_folder=str(tmp_path / "Label"), gt_format=".png", gt_transform=False,
                          x_root_folder=str(tmp_path / "Depth"), x_format=".png", x_is_single_channel=True,
                          train_source=str(tmp_path / "train.txt"), eval_source=str(tmp_path / "train.txt"),
                          background=255, num_classes=9, image_height=48, image_width=64, norm_mean=MEAN,
                          norm_std=STD, train_scale_array=SCALES, batch_size=2, niters_per_epoch=2, num_workers=0)
    engine = SimpleNamespace(distributed=False, world_size=1)
    loader, sampler = get_train_loader(engine, RGBXDataset, cfg)
    assert sampler is None and len(loader) == 2
    n = 0
    for mb in loader:
        assert mb["data"].shape == (2, 3, 48, 64) and mb["modal_x"].shape == (2, 3, 48, 64)
        assert mb["data"].is_cuda and mb["data"].dtype == torch.float32 and mb["label"].dtype == torch.int64
        lab = mb["label"]
        assert bool(((lab >= 0) & (lab <= 8) | (lab == 255)).all())
        assert torch.isfinite(mb["data"]).all() and len(mb["fn"]) == 2
        n += 1
    assert n == 2
    # release the loader's pinned host buffers now, not at a later test's garbage collection
    del loader, mb
    gc.collect()
    torch.cuda.synchronize()
