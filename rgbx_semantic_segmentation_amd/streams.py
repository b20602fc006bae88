"""Side HIP stream for the backward pass's off-critical-path work.

Weight gradients (the wgrad GEMMs of every Linear / conv) are not consumed by the rest of the
backward pass, only by the optimizer step.  They are launched on a second stream that first
waits for everything already queued on the current stream (so dz and x are ready), and the
current stream waits for the side stream once, at the end of the backward pass (an autograd
engine callback).  The small-output, long-K wgrads then overlap the dgrad / elementwise
chain instead of serialising with it; inside a HIP graph capture the fork / join become
graph edges.  Off by default (CMX_SIDE_STREAM=1 enables it): measured on MI355X inside the
step's HIP graph it LOST 11 % (139 -> 124 img/s, B2 480x640 bs=2) -- the ~230 fork / join
edges cost more than the overlap wins while the wgrads hold whole CUs (128 KB LDS rings).

This is the single-GPU analogue of the reference's DDP reducer overlap (train.py:145-146):
the gradient all-reduce of a multi-GPU step is issued after the join (dist.GradAllReduce).
"""
from __future__ import annotations

import os

import torch

ENABLED = os.environ.get("CMX_SIDE_STREAM", "0") == "1"
# FFM (the fusion branch feeding only the decoder) on its own stream beside the encoder
FFM_SIDE = os.environ.get("CMX_FFM_STREAM", "1") == "1"
_ffm: dict = {}


def ffm_stream(device) -> torch.cuda.Stream:
    idx = torch.device(device).index
    if idx not in _ffm:
        _ffm[idx] = torch.cuda.Stream(device=device)
    return _ffm[idx]
_side: dict = {}
_pending: set = set()


def side_stream(device) -> torch.cuda.Stream:
    idx = torch.device(device).index
    if idx not in _side:
        _side[idx] = torch.cuda.Stream(device=device)
    return _side[idx]


def _join(main: torch.cuda.Stream, side: torch.cuda.Stream, key) -> None:
    main.wait_stream(side)
    _pending.discard(key)


def run_side(fn, *keep) -> None:
    """Run ``fn()`` (kernel launches only, no host sync) on the side stream, ordered after the
    work already queued on the current stream.  ``keep``: tensors ``fn`` reads that the caller
    may free afterwards (marked as in use by the side stream for the caching allocator).
    Must be called from inside a backward pass: the join is queued as an engine callback."""
    if not ENABLED:
        fn()
        return
    main = torch.cuda.current_stream()
    side = side_stream(main.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        fn()
    for t in keep:
        if t is not None:
            t.record_stream(side)
    key = (main.cuda_stream, side.cuda_stream)
    if key not in _pending:
        _pending.add(key)
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _join(main, side, key))
