"""Side HIP stream of the FFM branch.

FFM_s (net_utils.py:354-384) only feeds the decoder, so ``RGBXTransformer.run`` runs it on
its own stream beside stage s + 1 of the encoder (its backward then runs there too, beside
the encoder's backward); inside the step's HIP graph the fork / join are graph edges.
``CMX_FFM_STREAM=0`` keeps everything on the current stream (A/B switch for measurements).

(A second side stream for the weight-gradient GEMMs was measured and removed: the ~230
fork / join edges per step cost more than the overlap won, and the weight gradients now
run as one deferred grouped launch per segment, deferred.py.)
"""
from __future__ import annotations

import os

import torch

FFM_SIDE = os.environ.get("CMX_FFM_STREAM", "1") == "1"
# CMX_SR_STREAM=1: each Attention's key/value path (SR conv -> norm -> kv Linear,
# dual_segformer.py:114-124) on a second side stream beside the q Linear (:111), forward and
# (autograd follows the forward's streams) backward
SR_SIDE = os.environ.get("CMX_SR_STREAM", "0") == "1"
_ffm: dict = {}
_sr: dict = {}


def sr_stream(device) -> torch.cuda.Stream:
    idx = torch.device(device).index
    if idx not in _sr:
        _sr[idx] = torch.cuda.Stream(device=device)
    return _sr[idx]


def ffm_stream(device) -> torch.cuda.Stream:
    idx = torch.device(device).index
    if idx not in _ffm:
        _ffm[idx] = torch.cuda.Stream(device=device)
    return _ffm[idx]
