"""Drop-in mirror of the reference's sliding-window evaluator (engine/evaluator.py:18-431) on
the device.

Same class, constructor and method names as the reference; the network runs through the HIP
forward (``EncoderDecoder.forward(rgb, x)`` in eval mode), and the two per-pixel passes the
reference runs on the host or as eager torch ops are HIP kernels (csrc/metric.hip):
  * ``cmx_seg_window_accumulate`` -- exp(score (+ mirrored flip score)) of one crop, minus its
    padding margin, added into the scale accumulator (evaluator.py:345-368, 374-396);
  * ``cmx_seg_argmax_confusion``  -- argmax over classes + hist_info (evaluator.py:322,
    eval.py:35, utils/metric.py:8-15), accumulating on the device.
Resizes (cv2.resize INTER_LINEAR, evaluator.py:311-316, 371) use the bilinear kernel of the
decoder (csrc/bilinear.hip, the same half-pixel rule); padding and the per-channel normalise
are torch elementwise plumbing.

Kept from the reference, deliberately: the window origin / end index quirk (stride[0] and
crop_size[0] on x, evaluator.py:352-357; negative starts are Python slices from the end), the
second normalisation inside ``process_image_rgbX`` (:408-412).  Differences: scores of the
scales are summed in fp32 on the device (the reference sums float64 on the host), and a
scale's image size is round(s * size) with the in/out resize rule (cv2 uses 1/fx; identical
when s * size is an integer, as for 0.75 / 1.25 of 480 x 640).  One process per GPU (the
reference's spawn pool of per-device workers is replaced by the Engine's one-process-per-GPU
launch); ``run`` evaluates a dataset and returns the metric line.
"""
from __future__ import annotations

import math
import collections
import os

import numpy as np
import torch
import torch.nn.functional as TF

from .. import _lib
from ..utils.metric import ConfusionCounter, compute_score


def _pad_margin(h, w, crop):
    """utils/transforms.py:61-70 margins (top, bottom, left, right) padding (h, w) up to crop."""
    ph, pw = max(crop[0] - h, 0), max(crop[1] - w, 0)
    return ph // 2, ph // 2 + ph % 2, pw // 2, pw // 2 + pw % 2


def _resize_chw(x: torch.Tensor, oh: int, ow: int, as_uint8: bool = False) -> torch.Tensor:
    """(C, H, W) fp32 -> (C, oh, ow) fp32, bilinear align_corners=False (cv2 INTER_LINEAR).
    ``as_uint8``: the source image was uint8, and cv2.resize returns the input's dtype, so
    the result is rounded and clamped to uint8 values.  cv2 interpolates uint8 images in
    11-bit fixed point; this kernel interpolates in fp32, so a value on a .5 rounding boundary
    can land one level apart (no cv2 here to pin it: parity unpinned)."""
    C, H, W = x.shape
    if (H, W) == (oh, ow):
        return x
    src = x.permute(1, 2, 0).contiguous()                    # NHWC input of the kernel
    out = torch.empty(C, oh, ow, device=x.device, dtype=torch.float32)
    _lib.call("cmx_bilinear_fwd_nchw_f32", _lib.ptr(src), _lib.ptr(out), 1, H, W, oh, ow, C, 0, _lib.stream())
    if as_uint8:
        out = out.round_().clamp_(0, 255)
    return out


def _is_uint8(a) -> bool:
    return (a.dtype == torch.uint8) if isinstance(a, torch.Tensor) else (np.asarray(a).dtype == np.uint8)


class Evaluator(object):
    def __init__(self, dataset, class_num, norm_mean, norm_std, network, multi_scales, is_flip, devices,
                 verbose=False, save_path=None, show_image=False):
        self.eval_time = 0
        self.dataset = dataset
        self.ndata = dataset.get_length() if dataset is not None and hasattr(dataset, "get_length") else 0
        self.class_num = class_num
        self.norm_mean = np.asarray(norm_mean, dtype=np.float64)
        self.norm_std = np.asarray(norm_std, dtype=np.float64)
        self.multi_scales = multi_scales
        self.is_flip = is_flip
        self.network = network
        self.devices = devices
        self.val_func = network
        self.verbose = verbose
        self.save_path = save_path
        self.show_image = show_image
        # crops per network forward (both mirrors of a crop count as two): batched sliding windows
        self.eval_batch = int(os.environ.get("CMX_EVAL_BATCH", "8"))
        # one HIP graph per crop-batch shape for capturable networks (CMX_EVAL_GRAPH=0: eager)
        self.eval_graph = os.environ.get("CMX_EVAL_GRAPH", "1") != "0"
        # at most CMX_EVAL_GRAPHS cached shapes (least recently used evicted); every graph after
        # the first allocates from the first one's private memory pool
        self.eval_graph_cap = max(1, int(os.environ.get("CMX_EVAL_GRAPHS", "4")))
        self._graphs = collections.OrderedDict()
        self._graph_pool = None

    # ------------------------------------------------------------------ per-sample API
    def func_per_iteration(self, data, device):
        raise NotImplementedError           # subclass (eval.py:22-66)

    def compute_metric(self, results):
        raise NotImplementedError           # subclass (eval.py:69-83)

    def _device(self, device):
        if device is None:
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cuda", device) if isinstance(device, int) else torch.device(device)

    def _chw(self, a, dev):
        """HWC (numpy or tensor, any numeric dtype) -> (C, H, W) float32 on the device."""
        t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
        t = t.to(device=dev, dtype=torch.float32)
        if t.dim() == 2:
            t = t[..., None]
        return t.permute(2, 0, 1).contiguous()

    def sliding_scores_rgbX(self, img, modal_x, crop_size, stride_rate, device=None) -> torch.Tensor:
        """Sum over scales of the per-scale score maps, (K, H, W) fp32 on the device.  The crops
        of every scale (all of one shape, crop_size) run through the network in batches of
        ``eval_batch`` (one forward per batch instead of one bs=1 forward per crop); each crop's
        scores are then added into its scale's accumulator in the reference's window order."""
        dev = self._device(device)
        crop = (int(crop_size[0]), int(crop_size[1])) if not isinstance(crop_size, int) else (crop_size, crop_size)
        img_c, x_c = self._chw(img, dev), self._chw(modal_x, dev)
        u8_img, u8_x = _is_uint8(img), _is_uint8(modal_x)
        _, ori_rows, ori_cols = img_c.shape
        plans = []
        for s in self.multi_scales:
            nh, nw = int(round(ori_rows * s)), int(round(ori_cols * s))
            plans.append(self._scale_plan(_resize_chw(img_c, nh, nw, u8_img), _resize_chw(x_c, nh, nw, u8_x), crop,
                                            stride_rate))
        self._run_windows([w for pl in plans for w in pl["windows"]], crop)
        processed = torch.zeros(self.class_num, ori_rows, ori_cols, device=dev, dtype=torch.float32)
        for pl in plans:
            processed += self._scale_result(pl, (ori_rows, ori_cols))
        return processed

    def sliding_eval_rgbX(self, img, modal_x, crop_size, stride_rate, device=None):
        """evaluator.py:306-324: the (H, W) class map (numpy int64, as the reference returns)."""
        score = self.sliding_scores_rgbX(img, modal_x, crop_size, stride_rate, device)
        pred = torch.empty(score.shape[1:], dtype=torch.int32, device=score.device)
        cc = ConfusionCounter(self.class_num, score.device)
        dummy = torch.full(score.shape[1:], 255, dtype=torch.uint8, device=score.device)
        cc.add_score(score, dummy, pred_out=pred)            # argmax only (every label ignored)
        return pred.cpu().numpy().astype(np.int64)

    def scale_process_rgbX(self, img, modal_x, ori_shape, crop_size, stride_rate, device=None):
        """evaluator.py:326-372 on (C, h, w) device images; returns (K, H, W) at ori_shape."""
        crop = (int(crop_size[0]), int(crop_size[1])) if not isinstance(crop_size, int) else (crop_size, crop_size)
        pl = self._scale_plan(img, modal_x, crop, stride_rate)
        self._run_windows(pl["windows"], crop)
        return self._scale_result(pl, ori_shape)

    def _scale_plan(self, img, modal_x, crop_size, stride_rate):
        """The windows of one scale (evaluator.py:326-368): each one's normalised, padded crop
        pair and where its scores land in the scale's accumulator."""
        dev = img.device
        _, new_rows, new_cols = img.shape
        K = self.class_num
        wins = []
        if new_cols <= crop_size[1] or new_rows <= crop_size[0]:
            m = _pad_margin(new_rows, new_cols, crop_size)
            acc = torch.zeros(K, new_rows, new_cols, device=dev, dtype=torch.float32)
            wins.append((img, modal_x, acc, 0, 0, m))
            view = None
        else:
            stride = (int(math.ceil(crop_size[0] * stride_rate)), int(math.ceil(crop_size[1] * stride_rate)))
            m = _pad_margin(new_rows, new_cols, crop_size)
            img_pad = TF.pad(img, (m[2], m[3], m[0], m[1]))
            x_pad = TF.pad(modal_x, (m[2], m[3], m[0], m[1]))
            pad_rows, pad_cols = img_pad.shape[1], img_pad.shape[2]
            r_grid = int(np.ceil((pad_rows - crop_size[0]) / stride[0])) + 1
            c_grid = int(np.ceil((pad_cols - crop_size[1]) / stride[1])) + 1
            acc = torch.zeros(K, pad_rows, pad_cols, device=dev, dtype=torch.float32)
            for gy in range(r_grid):
                for gx in range(c_grid):
                    s_x = gx * stride[0]                      # (sic) evaluator.py:352-357
                    s_y = gy * stride[1]
                    e_x = min(s_x + crop_size[0], pad_cols)
                    e_y = min(s_y + crop_size[1], pad_rows)
                    s_x = e_x - crop_size[0]
                    s_y = e_y - crop_size[1]
                    # Python slice semantics of a negative start (numpy / torch in the reference)
                    sy0 = s_y if s_y >= 0 else max(pad_rows + s_y, 0)
                    sx0 = s_x if s_x >= 0 else max(pad_cols + s_x, 0)
                    if e_y <= sy0 or e_x <= sx0:
                        continue
                    wins.append((img_pad[:, sy0:e_y, sx0:e_x], x_pad[:, sy0:e_y, sx0:e_x], acc, sy0, sx0,
                                 _pad_margin(e_y - sy0, e_x - sx0, crop_size)))
            view = (m[0], pad_rows - m[1], m[2], pad_cols - m[3])
        return {"windows": wins, "acc": acc, "view": view}

    def _scale_result(self, plan, ori_shape):
        acc, v = plan["acc"], plan["view"]
        score = acc if v is None else acc[:, v[0]:v[1], v[2]:v[3]]
        return _resize_chw(score.contiguous(), ori_shape[0], ori_shape[1])

    def _run_windows(self, wins, crop_size):
        """process_image_rgbX + a batched val_func_process_rgbX + margin crop + window add (one
        kernel per window, in list order)."""
        nb = max(1, int(self.eval_batch) // (2 if self.is_flip else 1))
        pairs = [self.process_image_rgbX(w[0], w[1], crop_size) for w in wins]
        c0 = 0
        while c0 < len(wins):
            # runs of consecutive crops of one shape (a scale smaller than the crop on one side
            # only keeps its other side: that whole-image crop is not crop-sized)
            c1 = c0 + 1
            while c1 < len(wins) and c1 - c0 < nb and pairs[c1][0].shape == pairs[c0][0].shape \
                    and pairs[c1][1].shape == pairs[c0][1].shape:
                c1 += 1
            chunk = wins[c0:c1]
            d = torch.stack([p[0] for p in pairs[c0:c1]])
            x = torch.stack([p[1] for p in pairs[c0:c1]])
            c0 = c1
            s1, s2 = self._val_batch(d, x)
            for i, (_, _, acc, sy, sx, tm) in enumerate(chunk):
                a, b = s1[i], (s2[i] if s2 is not None else None)
                K, ch, cw = a.shape
                _lib.call("cmx_seg_window_accumulate", _lib.ptr(a), _lib.ptr(b), _lib.ptr(acc), K, ch, cw,
                          tm[0], tm[1], tm[2], tm[3], acc.shape[1], acc.shape[2], sy, sx, _lib.stream())

    def _val_batch(self, d, x):
        """(n, 3, h, w) crops -> their logits (n, K, h, w) fp32 and (is_flip) those of the mirrored
        crops, from one forward over the n (or 2n) images."""
        net = self.val_func
        was_training = net.training
        net.eval()
        n = d.shape[0]
        with torch.no_grad():
            if self.is_flip:
                out = self._forward(net, torch.cat([d, d.flip(-1)]), torch.cat([x, x.flip(-1)])).float()
                s1, s2 = out[:n].contiguous(), out[n:].contiguous()
            else:
                s1, s2 = self._forward(net, d, x).float().contiguous(), None
        if was_training:
            net.train()
        return s1, s2

    def _forward(self, net, d, x):
        """net(d, x); for a network that declares itself graph-capturable (EncoderDecoder), one
        HIP graph per input shape, replayed from static input buffers (the eager forward of a
        crop batch is bound by the host's ~600 launches).  The returned logits live in the
        graph's output buffer: the caller consumes them on this stream before the next replay."""
        if not (self.eval_graph and getattr(net, "cmx_capturable", False)):
            return net(d.contiguous(), x.contiguous())
        key = (tuple(d.shape), tuple(x.shape), str(d.device), id(net))
        g = self._graphs.get(key)
        if g is None:
            # Bounded cache: images of many sizes give many whole-image crop shapes,
            # and each graph would otherwise keep its own pool holding a full set of forward
            # activations.  Sharing one pool is safe: replays run in order on this stream and
            # each output is consumed (window-accumulated) before the next replay.  The new graph
            # is captured BEFORE the oldest are evicted: a graph sharing the pool must
            # stay alive across the capture, or at cap 1 the pool's last user goes and the capture
            # would draw on a released pool handle.
            sd, sx = d.contiguous().clone(), x.contiguous().clone()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                net(sd, sx)                          # warm-up: workspaces and allocator pools
            torch.cuda.current_stream().wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, pool=self._graph_pool, capture_error_mode="thread_local"):
                out = net(sd, sx)
            if self._graph_pool is None:
                self._graph_pool = graph.pool()
            g = self._graphs[key] = (graph, sd, sx, out)
            while len(self._graphs) > self.eval_graph_cap:
                self._graphs.popitem(last=False)
        self._graphs.move_to_end(key)
        graph, sd, sx, out = g
        sd.copy_(d)
        sx.copy_(x)
        graph.replay()
        return out

    def val_func_process_rgbX(self, input_data, input_modal_x, device=None):
        """evaluator.py:374-396 up to the exp: the logits of the crop and (is_flip) of its mirror,
        (K, h, w) fp32 each; the sum, mirror and exp are fused into cmx_seg_window_accumulate."""
        net = self.val_func
        was_training = net.training
        net.eval()
        with torch.no_grad():
            score = net(input_data[None].contiguous(), input_modal_x[None].contiguous())[0].float().contiguous()
            flip = None
            if self.is_flip:
                flip = net(input_data.flip(-1)[None].contiguous(),
                           input_modal_x.flip(-1)[None].contiguous())[0].float().contiguous()
        if was_training:
            net.train()
        return score, flip

    def process_image_rgbX(self, img, modal_x, crop_size=None):
        """evaluator.py:398-431 on (3, h, w) device images: normalise (utils/transforms.py:182-187,
        applied to whatever the dataset produced, as the reference does) and pad to crop_size."""
        mean = torch.as_tensor(self.norm_mean, dtype=torch.float32, device=img.device).view(-1, 1, 1)
        std = torch.as_tensor(self.norm_std, dtype=torch.float32, device=img.device).view(-1, 1, 1)
        p_img = (img / 255.0 - mean) / std
        if modal_x.shape[0] == 1:                   # a 2-D modal map: normalize(x, 0, 1) (:404-406)
            p_x = modal_x / 255.0
        else:
            p_x = (modal_x / 255.0 - mean) / std
        if crop_size is not None:
            m = _pad_margin(p_img.shape[1], p_img.shape[2], crop_size)
            p_img = TF.pad(p_img, (m[2], m[3], m[0], m[1]))
            p_x = TF.pad(p_x, (m[2], m[3], m[0], m[1]))
        return p_img.contiguous(), p_x.contiguous()

    # ------------------------------------------------------------------ dataset pass
    def run(self, dataset=None, crop_size=None, stride_rate=2 / 3, device=None):
        """Evaluate every sample (dict with data / modal_x / label, HWC / HW) and return
        (iou, mean_IoU, mean_IoU_no_back, freq_IoU, mean_pixel_acc, pixel_acc)."""
        dataset = dataset if dataset is not None else self.dataset
        dev = self._device(device)
        cc = ConfusionCounter(self.class_num, dev)
        n = dataset.get_length() if hasattr(dataset, "get_length") else len(dataset)
        for i in range(n):
            d = dataset[i]
            img = d["data"].transpose(1, 2, 0) if d["data"].ndim == 3 and d["data"].shape[0] == 3 else d["data"]
            score = self.sliding_scores_rgbX(img, d["modal_x"], crop_size, stride_rate, dev)
            cc.add_score(score, torch.as_tensor(np.ascontiguousarray(d["label"])))
        hist, labeled, correct = cc.result()
        return compute_score(hist, correct, labeled)
