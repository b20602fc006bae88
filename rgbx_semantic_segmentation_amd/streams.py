"""Side HIP stream of the FFM branch.

FFM_s (net_utils.py:354-384) only feeds the decoder, so ``RGBXTransformer.run`` runs it on
its own stream beside stage s + 1 of the encoder (its backward then runs there too, beside
the encoder's backward); inside the step's HIP graph the fork / join are graph edges.
``CMX_FFM_STREAM=0`` keeps everything on the current stream (A/B switch for measurements).

(Measured and removed: a side stream for the weight-gradient GEMMs -- the fork / join edges
cost more than the overlap won, and the weight gradients run as one deferred grouped launch,
deferred.py -- and one for each Attention's key/value path beside the q Linear, -5 % per
step in round 3.)
"""
from __future__ import annotations

import os

import torch

FFM_SIDE = os.environ.get("CMX_FFM_STREAM", "1") == "1"
_ffm: dict = {}


def ffm_stream(device) -> torch.cuda.Stream:
    idx = torch.device(device).index
    if idx not in _ffm:
        _ffm[idx] = torch.cuda.Stream(device=device)
    return _ffm[idx]
