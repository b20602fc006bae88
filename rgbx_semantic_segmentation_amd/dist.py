"""Data parallelism over RCCL (torch.distributed "nccl" backend = RCCL on ROCm).

Replaces DistributedDataParallel (train.py:141-149) for this model: parameters live in
one flat buffer, so the gradient exchange is a SUM all-reduce of the flat fp32 gradient
buffer (one large collective per step instead of ~11 DDP buckets) followed by a 1/P scale
folded into the fused AdamW kernel.  SyncBatchNorm of the decoder's linear_fuse BN is in
functions.BatchNormF (all-reduce of the fp64 channel sums, forward and backward).
The FFM BatchNorms stay local, like the reference (mit_b* drops norm_fuse).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradAllReduce:
    """Callable used by FusedAdamW.step(): all-reduce(SUM) the flat gradient buffer and
    return the scale (1/world) the optimizer applies."""

    def __init__(self, store, group=None):
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group)

    def __call__(self, flat_grad: torch.Tensor) -> float:
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=self.group)
        return 1.0 / self.world


@torch.no_grad()
def broadcast_parameters(model, group=None, src: int = 0):
    """DDP's construction-time broadcast of parameters and buffers from rank 0."""
    dist.broadcast(model.store.flat, src=src, group=group)
    for b in model.buffers():
        dist.broadcast(b, src=src, group=group)
    model.store.refresh_shadow()


def all_reduce_tensor(tensor, op=dist.ReduceOp.SUM, world_size=1):
    """utils/pyt_utils.py:119-124: mean of a (loss) tensor over ranks."""
    t = tensor.clone()
    dist.all_reduce(t, op)
    t.div_(world_size)
    return t
