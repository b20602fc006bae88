"""Flat parameter store: one fp32 master buffer, one fp32 gradient buffer, one bf16 / fp16 shadow.

MI355X-first layout decisions (the reference keeps 66.6 M parameters as ~600 separate
tensors, ``train.py:104-149``):
  * every parameter is a view into a single contiguous fp32 buffer (64-element aligned
    segments), so AdamW is ONE fused kernel and the DDP gradient all-reduce is a handful
    of large contiguous RCCL buckets;
  * the RGB-stream and X-stream copies of each encoder weight (``block1.0.attn.q`` /
    ``extra_block1.0.attn.q``, ``cross.channel_proj1`` / ``channel_proj2``, ...) sit next to
    each other with equal strides, so a (2, N, K) stacked view feeds one grouped GEMM /
    one kernel launch for both modalities;
  * conv weights are stored tap-major ``(Cout, kh, kw, Cin)`` (the im2col order of NHWC
    activations); the ``nn.Parameter`` the module exposes is a permuted view with the
    reference shape ``(Cout, Cin, kh, kw)``, so ``state_dict`` keys, shapes and values are
    those of the reference and checkpoints interoperate;
  * gradients are written by the kernels straight into ``param.grad`` (a view of the flat
    gradient buffer): no zero-fill and no accumulate pass per step.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

ALIGN = 64


def _pad(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def partner_name(name: str) -> Optional[str]:
    """Name of the other-modality twin of an RGB-stream parameter, or None."""
    m = re.match(r"backbone\.(patch_embed\d|block\d|norm\d)(\..*)$", name)
    if m:
        return f"backbone.extra_{m.group(1)}{m.group(2)}"
    for a, b in (("channel_proj1", "channel_proj2"), ("end_proj1", "end_proj2"),
                 ("cross_attn.kv1", "cross_attn.kv2"), ("cross.norm1", "cross.norm2"),
                 ("cross_attn.q1", "cross_attn.q2"), ("cross_attn.proj1", "cross_attn.proj2")):      # IFFM
        if a in name:
            return name.replace(a, b)
    return None


@dataclass
class Slot:
    name: str
    offset: int           # element offset of the first member in the flat buffer
    stride: int           # element stride between stacked members (== padded size)
    count: int            # 1 or 2 stacked members
    index: int            # this parameter's member index
    storage_shape: Tuple[int, ...]
    kind: str             # "plain", "conv_taps", "conv_pad"
    decay: bool
    frozen: bool = False  # in neither group_weight group: the optimizer never updates it


class ParamStore:
    def __init__(self, model: nn.Module, device, compute_dtype=torch.float32,
                 conv_pad: Dict[str, int] | None = None, segment_of=None):
        """segment_of(name) -> int: optional backward-completion segment of each parameter.
        The flat buffers are laid out segment by segment (0 first), so each segment's
        gradients form ONE contiguous range (``self.segments``) that the data-parallel
        gradient exchange can all-reduce as soon as that part of the backward is done."""
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        conv_pad = conv_pad or {}
        named = list(model.named_parameters())
        self._ref_shape = {n: tuple(p.shape) for n, p in named}
        by_name = dict(named)
        owner = {}
        for mname, mod in model.named_modules():
            for pname, _ in mod.named_parameters(recurse=False):
                owner[f"{mname}.{pname}" if mname else pname] = (mod, pname)
        # utils/init_func.py:33-57 group_weight: Linear / Conv weights decay; their biases and
        # norm affine parameters do not; any other parameter (IFRM's lambdas) is in NEITHER
        # group, so the reference's optimizer never steps it: a frozen slot here
        decay_ids, grouped = set(), set()
        for mod in model.modules():
            if isinstance(mod, (nn.Linear, nn.Conv2d)):
                decay_ids.add(id(mod.weight))
                grouped.update(id(p) for p in mod.parameters(recurse=False))
            elif isinstance(mod, (nn.BatchNorm2d, nn.LayerNorm, nn.GroupNorm, nn.SyncBatchNorm)):
                grouped.update(id(p) for p in mod.parameters(recurse=False))

        self.slots: Dict[str, Slot] = {}
        placed = set()
        off = 0
        order: List[Tuple[str, int]] = []
        seg_of = segment_of or (lambda n: 0)
        placement = sorted(named, key=lambda kv: seg_of(kv[0]))      # stable: module order within a segment
        seg_bounds: Dict[int, List[int]] = {}
        for name, p in placement:
            if name in placed:
                continue
            sid = seg_of(name)
            seg_bounds.setdefault(sid, [off, off])
            pn = partner_name(name)
            group = [name] + ([pn] if pn and pn in by_name and pn not in placed else [])
            kind, sshape = self._storage(name, p, conv_pad)
            numel = 1
            for d in sshape:
                numel *= d
            # a modality pair is packed back to back (member stride = numel, a multiple of 8
            # elements for every CMX parameter, so both members stay 16-byte aligned) and the
            # pair is padded to 64 elements; (G, ...) views of it are then plain views.
            assert numel % 8 == 0 or len(group) == 1, (name, numel)
            stride = numel if len(group) == 2 else _pad(numel)
            for i, n in enumerate(group):
                assert by_name[n].shape == p.shape, (name, n)
                self.slots[n] = Slot(n, off, stride, len(group), i, sshape, kind, id(by_name[n]) in decay_ids,
                                     id(by_name[n]) not in grouped)
                placed.add(n)
            off += _pad(stride * len(group))
            seg_bounds[sid][1] = off
        self.numel = off
        # [(segment id, start, end)] in element offsets, in layout order
        self.segments = [(sid, b[0], b[1]) for sid, b in sorted(seg_bounds.items())]
        self.flat = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=self.device)
        # the GEMM-operand copy of the weights in a 16-bit compute dtype (bf16, or fp16 for the
        # reference's AMP configuration), refreshed by every optimizer step
        self.shadow = (torch.zeros(off, dtype=compute_dtype, device=self.device)
                       if compute_dtype in (torch.bfloat16, torch.float16) else None)
        self.shadow_code = {torch.bfloat16: 1, torch.float16: 2}.get(compute_dtype, 0)
        self.decay64 = torch.zeros(off // ALIGN, dtype=torch.uint8)
        # copy values, rebind parameters as views
        self.params: Dict[str, nn.Parameter] = {}
        for name, p in named:
            s = self.slots[name]
            if s.decay or s.frozen:         # 1: decay, 2: frozen (the AdamW kernel skips it)
                self.decay64[s.offset // ALIGN:(s.offset + _pad(s.stride * s.count)) // ALIGN] = 2 if s.frozen else 1
            with torch.no_grad():
                self._param_view(self.flat, s).copy_(p.detach().to(self.device))
            newp = nn.Parameter(self._param_view(self.flat, s))
            newp.grad = self._param_view(self.grad, s)
            mod, pname = owner[name]
            mod._parameters[pname] = newp
            self.params[name] = newp
        self.decay64 = self.decay64.to(self.device)
        self.by_id = {id(p): n for n, p in self.params.items()}
        self.refresh_shadow()

    # ------------------------------------------------------------------ layouts
    @staticmethod
    def _storage(name, p, conv_pad):
        if p.dim() == 4 and (p.shape[2] > 1 or p.shape[3] > 1) and p.shape[1] > 1:
            co, ci, kh, kw = p.shape
            if name in conv_pad:                   # NCHW-image conv: (c, kh, kw) order, padded K
                return "conv_pad", (co, conv_pad[name])
            return "conv_taps", (co, kh, kw, ci)
        if p.dim() == 4:                           # 1x1 conv / depthwise: same memory order
            return "plain", (p.shape[0], p.shape[1] * p.shape[2] * p.shape[3])
        return "plain", tuple(p.shape) or (1,)          # 0-dim (IFRM's lambdas): one element

    def _storage_view(self, buf, s: Slot, stacked: bool):
        n = 1
        for d in s.storage_shape:
            n *= d
        if stacked:
            return buf.narrow(0, s.offset, n * s.count).view(s.count, *s.storage_shape)
        base = s.offset + s.index * s.stride
        return buf.narrow(0, base, n).view(*s.storage_shape)

    def _param_view(self, buf, s: Slot):
        st = self._storage_view(buf, s, stacked=False)
        if s.kind == "conv_taps":
            return st.permute(0, 3, 1, 2)
        if s.kind == "conv_pad":
            co, kp = s.storage_shape
            ref = self._ref_shape[s.name]
            k = ref[1] * ref[2] * ref[3]
            return st[:, :k].as_strided(ref, (kp, ref[2] * ref[3], ref[3], 1))
        return st.view(torch.Size(self._ref_shape[s.name]))

    # ------------------------------------------------------------------ accessors
    def slot(self, p: nn.Parameter) -> Slot:
        return self.slots[self.by_id[id(p)]]

    def w(self, p: nn.Parameter, stacked: bool = True, compute: bool = True):
        """Storage-layout view in the compute dtype (bf16 shadow or fp32 master).  With
        ``stacked`` the result always has a leading group dim G (2 for a modality pair)."""
        s = self.slot(p)
        buf = self.shadow if (compute and self.shadow is not None) else self.flat
        if stacked and s.count == 2:
            return self._storage_view(buf, s, True)
        v = self._storage_view(buf, s, False)
        return v[None] if stacked else v

    def g(self, p: nn.Parameter, stacked: bool = True):
        s = self.slot(p)
        if stacked and s.count == 2:
            return self._storage_view(self.grad, s, True)
        v = self._storage_view(self.grad, s, False)
        return v[None] if stacked else v

    def ensure_grads(self):
        """Re-attach ``param.grad`` to the flat gradient buffer if a caller detached it
        (e.g. ``torch.optim.Optimizer.zero_grad(set_to_none=True)``)."""
        for n, p in self.params.items():
            if p.grad is None:
                p.grad = self._param_view(self.grad, self.slots[n])

    def refresh_shadow(self):
        if self.shadow is not None:
            from . import kernels as K
            K.cast_f32_h16(self.flat, self.shadow)
