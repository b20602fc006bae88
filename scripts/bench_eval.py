"""Evaluator throughput: CMX-B2 480x640, the reference's NYU eval settings (config.py:84-88:
scales [0.75, 1, 1.25], crop 480 x 640, stride 2/3, no flip), random-init weights, synthetic
images; images/s of sliding_scores + argmax/confusion, and the two metric kernels timed alone.
Usage (GPU box): python scripts/bench_eval.py [--images 8] [--flip]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rgbx_semantic_segmentation_amd import _lib  # noqa: E402
from rgbx_semantic_segmentation_amd.engine.evaluator import Evaluator  # noqa: E402
from rgbx_semantic_segmentation_amd.models.builder import EncoderDecoder  # noqa: E402
from rgbx_semantic_segmentation_amd.utils.metric import ConfusionCounter  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=8)
    ap.add_argument("--flip", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    K = 40
    torch.manual_seed(0)
    model = EncoderDecoder(dict(backbone="mit_b2", num_classes=K, compute_dtype="bfloat16",
                                decoder_embed_dim=512)).to(dev)
    ev = Evaluator(None, K, [0.485, 0.456, 0.406], [0.229, 0.224, 0.225], model, [0.75, 1, 1.25], a.flip, [0])
    rng = np.random.default_rng(0)
    imgs = [rng.uniform(0, 255, (480, 640, 3)).astype(np.float32) for _ in range(2)]
    gt = torch.randint(0, K, (480, 640), device=dev)
    cc = ConfusionCounter(K, dev)
    for i in range(2):                                   # warm-up
        cc.add_score(ev.sliding_scores_rgbX(imgs[i % 2], imgs[i % 2], (480, 640), 2 / 3, dev), gt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.images):
        cc.add_score(ev.sliding_scores_rgbX(imgs[i % 2], imgs[i % 2], (480, 640), 2 / 3, dev), gt)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # kernels alone
    score = torch.rand(K, 480, 640, device=dev)
    s1 = torch.randn(K, 480, 640, device=dev)
    acc = torch.zeros(K, 480, 640, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    e0.record()
    for _ in range(n):
        cc.add_score(score, gt)
    e1.record()
    torch.cuda.synchronize()
    t_conf = e0.elapsed_time(e1) / n * 1e3
    e0.record()
    for _ in range(n):
        _lib.call("cmx_seg_window_accumulate", _lib.ptr(s1), None, _lib.ptr(acc), K, 480, 640, 0, 0, 0, 0, 480, 640,
                  0, 0, _lib.stream())
    e1.record()
    torch.cuda.synchronize()
    t_win = e0.elapsed_time(e1) / n * 1e3
    nb_conf = K * 480 * 640 * 4 + 480 * 640 * 8
    nb_win = K * 480 * 640 * 4 * 3
    print(f"eval CMX-B2 480x640 scales [0.75,1,1.25] flip={a.flip}: {a.images / dt:.2f} images/s "
          f"({dt / a.images * 1e3:.1f} ms/image, {a.images} images)")
    print(f"argmax+confusion (K=40, 480x640, int64 labels): {t_conf:.1f} us, {nb_conf / t_conf / 1e3:.0f} GB/s")
    print(f"window accumulate (K=40, 480x640 crop, no flip): {t_win:.1f} us, {nb_win / t_win / 1e3:.0f} GB/s")


if __name__ == "__main__":
    main()
