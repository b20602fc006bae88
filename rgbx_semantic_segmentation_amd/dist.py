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


class BucketedGradSync:
    """Gradient all-reduce overlapped with the backward pass (the DDP reducer's bucketed
    overlap, train.py:145-146, restated for the flat ParamStore).

    The store lays parameters out by backward-completion segment (models.builder.
    backward_segment): decode head + stage 4, stage 3, stage 2, stage 1.  When the backward
    has passed a stage's patch embed (a tensor hook on that stage's input), the segment's
    queued weight gradients are flushed (deferred.flush) and its contiguous gradient range
    is all-reduced on a side stream (RCCL) while the backward of the earlier stages
    continues.  The last segment goes at the end of the backward.  ``__call__`` (from
    FusedAdamW.step) joins the side stream into the current one and returns the 1/P scale
    the AdamW kernel applies."""

    def __init__(self, store, group=None, overlap=None, payload=None, chunk_mb=None, groups=None):
        import os
        self.store = store
        self.group = group
        self.world = self._world()
        # CMX_DP_OVERLAP=0: one blocking all-reduce per segment at optimizer time (no overlap)
        self.overlap = (os.environ.get("CMX_DP_OVERLAP", "1") == "1") if overlap is None else overlap
        # gradient payload on the wire: "fp32" (SUM all-reduce of the fp32 gradients, DDP's
        # semantics) or "bf16" (fp32 reduce-scatter + bf16 all-gather: 6 instead of 8 bytes per
        # element over xGMI; one rounding of the fp32 sum to bf16)
        self.payload = (payload or os.environ.get("CMX_DP_PAYLOAD", "fp32")).lower()
        if self.payload not in ("fp32", "bf16"):
            raise ValueError(f"gradient payload {self.payload!r}: fp32 or bf16")
        # collectives of at most ~chunk_mb of payload each (DDP's 25 MB bucket cap): a long
        # segment is exchanged as a sequence of bounded messages
        mb = float(chunk_mb if chunk_mb is not None else os.environ.get("CMX_DP_CHUNK_MB", "25"))
        # a multiple of 64 elements, so every chunk of the flat buffer stays 16-byte aligned for
        # the vectorized cast / shard-sum kernels (a fractional MB would otherwise misalign)
        self.chunk = max(1024, (int(mb * 2 ** 20) // (2 if self.payload == "bf16" else 4)) // 64 * 64)
        self.ranges = {sid: (a, b) for sid, a, b in store.segments}
        # CMX_DP_GROUPS (default 2): the backward-completion segments are exchanged in this many
        # groups of consecutive segments -- each group's queued weight gradients flushed as ONE
        # grouped launch and all-reduced together once the backward has passed the group's last
        # stage.  4 = one exchange per segment (round 5: the per-segment flushes cut the grouped
        # weight-gradient launch in four and the side-stream joins left the CUs idle, 6 % off the
        # step at world size 1); 2 = decode head + stage 4 + stage 3 mid-backward, stages 2 + 1 at
        # the end of the backward
        ng = int(os.environ.get("CMX_DP_GROUPS", "2")) if groups is None else int(groups)
        sids = sorted(self.ranges)
        ng = max(1, min(ng, len(sids)))
        per = -(-len(sids) // ng)
        self.group_of = {sid: i // per for i, sid in enumerate(sids)}
        self.group_last = {}
        for sid in sids:
            self.group_last[self.group_of[sid]] = sid
        self.works = []
        self.launched = set()
        self._armed = False
        self.side = None

    def _launch(self, sid):
        """Flush the queued gradient work, then all-reduce the group of segments ending at
        ``sid`` on the side stream: the side stream waits for the backward so far, the blocking
        all-reduce blocks only the side stream, and the main stream runs on.  (A plain stream
        fork/join, so it is also captured into the step's HIP graph; async_op works are not
        capture-safe here.)"""
        from . import deferred
        if sid in self.launched or sid not in self.ranges:
            return
        g = self.group_of[sid]
        members = [s for s in sorted(self.ranges) if self.group_of[s] == g and s not in self.launched]
        deferred.flush()
        # the group's segments are consecutive in the flat buffer: one range
        a = min(self.ranges[s][0] for s in members)
        b = max(self.ranges[s][1] for s in members)
        main = torch.cuda.current_stream() if self.store.grad.is_cuda else None
        if main is None:                         # CPU tensors (gloo tests): blocking, in order
            self._reduce(self.store.grad[a:b])
        else:
            if self.side is None:
                self.side = torch.cuda.Stream(device=main.device)
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                self._reduce(self.store.grad[a:b])
            self.works.append(self.side)
        self.launched.update(members)

    def _world(self) -> int:
        return dist.get_world_size(self.group)

    def _reduce(self, seg: torch.Tensor) -> None:
        for a in range(0, seg.numel(), self.chunk):
            part = seg[a:a + self.chunk]
            # the bf16 protocol runs at every world size (at P = 1 the all-to-all and the
            # all-gather are copies), so a one-GPU run exercises its kernels and collectives
            if self.payload == "fp32":
                dist.all_reduce(part, op=dist.ReduceOp.SUM, group=self.group)
            else:
                self._reduce_bf16(part)

    def _reduce_bf16(self, t: torch.Tensor) -> None:
        """SUM over ranks of fp32 ``t`` in place with a bf16 return leg: a reduce-scatter of the
        fp32 gradients (each rank ends with the fp32 sum of its shard, accumulated in fp32 along
        the ring), one rounding of that sum to bf16, and an all-gather of the bf16 shards (4 + 2
        bytes per element on the wire vs 4 + 4 for an fp32 ring all-reduce; every rank, the
        shard's owner too, takes the gathered bf16 value, so the ranks stay bit-identical).
        Both collectives are safe inside a HIP-graph capture; an all-to-all was not (RCCL
        all_to_all_single inside a capture crashed at capture end or hung at exit even at world
        size 1: scripts/rccl_capture_probe.py).  On the GPU the casts are HIP
        kernels (cmx_cast_f32_bf16 / cmx_cast_bf16_f32); the CPU branch is the gloo rehearsal."""
        P = self.world
        n = t.numel()
        shard = -(-n // (8 * P)) * 8                 # per-rank shard, a multiple of 8 elements
        if n == P * shard:
            send = t
        else:
            send = torch.zeros(P * shard, dtype=torch.float32, device=t.device)
            send[:n].copy_(t)
        mine = torch.empty(shard, dtype=torch.float32, device=t.device)
        dist.reduce_scatter_tensor(mine, send, op=dist.ReduceOp.SUM, group=self.group)
        mine16 = torch.empty(shard, dtype=torch.bfloat16, device=t.device)
        out = torch.empty(P * shard, dtype=torch.bfloat16, device=t.device)
        if t.is_cuda:
            from . import _lib
            _lib.call("cmx_cast_f32_bf16", _lib.ptr(mine), _lib.ptr(mine16), shard, _lib.stream())
        else:
            mine16.copy_(mine)
        dist.all_gather_into_tensor(out, mine16, group=self.group)
        if t.is_cuda and n % 8 == 0:
            _lib.call("cmx_cast_bf16_f32", _lib.ptr(out), _lib.ptr(t), n, _lib.stream())
        else:
            t.copy_(out[:n])

    def _finish_backward(self):
        self._armed = False
        for sid in sorted(self.ranges):
            self._launch(sid)

    def segment_hook(self, sid):
        """Tensor hook: the backward is past segment ``sid`` (and every earlier segment)."""
        def hook(grad):
            if not self.overlap:
                return None
            if not self._armed:
                self._armed = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finish_backward)
            # every group whose last segment the backward has passed
            for s in sorted(self.ranges):
                if s <= sid and self.group_last[self.group_of[s]] <= sid:
                    self._launch(s)
            return None
        return hook

    def __call__(self, flat_grad: torch.Tensor) -> float:
        for sid in sorted(self.ranges):       # whatever the backward's hooks / callback did not launch
            self._launch(sid)
        if self.works:
            torch.cuda.current_stream().wait_stream(self.side)
        self.works, self.launched = [], set()
        return 1.0 / self.world


def flatten_bn_buffers(model, device=None):
    """Every BatchNorm's running_mean / running_var as views of ONE contiguous fp32 tensor
    (returned; None without BatchNorms), so DDP's per-forward buffer broadcast is one
    collective.  state_dict keys and shapes are unchanged; in-place updates of the running
    statistics (the BN kernels, load_state_dict) land in the flat tensor."""
    bns = [m for m in model.modules() if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)
           and m.running_mean is not None]
    if not bns:
        return None
    parts = []
    for m in bns:
        parts += [m.running_mean, m.running_var]
    dev = torch.device(device) if device is not None else parts[0].device
    flat = torch.cat([p.detach().to(device=dev, dtype=torch.float32).reshape(-1) for p in parts])
    off = 0
    for m in bns:
        for k in ("running_mean", "running_var"):
            n = m._buffers[k].numel()
            m._buffers[k] = flat[off:off + n].view(m._buffers[k].shape)
            off += n
    return flat


@torch.no_grad()
def broadcast_buffers(flat, group=None, src: int = 0):
    """DDP's per-forward buffer sync (DistributedDataParallel(broadcast_buffers=True), the
    default the reference uses, train.py:145-146): every rank's BatchNorm running statistics
    are replaced by rank ``src``'s at the start of each training forward -- one broadcast of the
    flat buffer (flatten_bn_buffers).  num_batches_tracked is not sent: every rank increments
    it in lockstep, so it is equal already."""
    if flat is not None:
        dist.broadcast(flat, src=group_src_rank(group, src), group=group)


def group_src_rank(group, src: int = 0) -> int:
    """Global rank of group rank ``src`` (torch.distributed.broadcast takes a GLOBAL src even with
    a subgroup; DDP broadcasts from the group's first member, which need not be global rank 0)."""
    if group is None or group is dist.group.WORLD:
        return src
    return dist.get_global_rank(group, src)


@torch.no_grad()
def broadcast_parameters(model, group=None, src: int = 0):
    """DDP's construction-time broadcast of parameters and buffers from rank 0."""
    gsrc = group_src_rank(group, src)
    dist.broadcast(model.store.flat, src=gsrc, group=group)
    for b in model.buffers():
        dist.broadcast(b, src=gsrc, group=group)
    model.store.refresh_shadow()


def all_reduce_tensor(tensor, op=dist.ReduceOp.SUM, world_size=1):
    """utils/pyt_utils.py:119-124: mean of a (loss) tensor over ranks."""
    t = tensor.clone()
    dist.all_reduce(t, op)
    t.div_(world_size)
    return t
