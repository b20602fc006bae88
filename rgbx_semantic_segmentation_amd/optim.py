"""Fused AdamW over the ParamStore's flat buffers (reference: train.py:107-139).

``FusedAdamW(model, lr, betas, weight_decay)`` reproduces the two parameter groups of
``utils/init_func.py:group_weight`` (decay: Linear/Conv weights; no decay: biases and
norm affine params) and ``torch.optim.AdamW``'s single-tensor update, in ONE kernel launch
over all parameters (csrc/adamw.hip), which also refreshes the bf16 weight shadow.

Host-visible state the reference loop touches is kept compatible:
  * ``param_groups[i]['lr'] = lr`` (train.py:206-207) updates a device scalar, so a HIP
    graph that replays the step picks up the new LR (the step reads it from memory);
  * ``zero_grad()`` is a no-op: the backward kernels OVERWRITE the flat gradient buffer;
  * ``state_dict()`` / ``load_state_dict()`` use torch.optim.AdamW's format (per-parameter
    ``step``/``exp_avg``/``exp_avg_sq``) so checkpoints written by either side load.
With a process group of world size > 1, ``step()`` first averages gradients (RCCL
all-reduce of the flat buffer, see dist.py) unless the caller already did.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import _lib
from ._lib import call, ptr, query, stream

# set by GradScaler.scale() while a loss-scaled backward is pending: its updates must wait for
# the whole-gradient inf / nan check, so the per-segment overlap stands aside
_scaled_backward = [False]


class SegmentUpdate:
    """AdamW per backward-completion segment, overlapped with the rest of the backward.

    The ParamStore lays parameters out by segment (models.builder.backward_segment: decode head
    + stage 4, stage 3, stage 2, stage 1).  Once the backward has passed a stage (a tensor hook
    on the stage's input, installed by the encoder), nothing later in the step reads that
    segment's weights or gradients: its queued weight-gradient GEMMs (deferred.flush) and its
    AdamW update are issued on a side stream, beside the latency-bound backward of the earlier
    stages, each launch capped to a share of the chip (CMX_SIDE_WGRAD_BLOCKS,
    CMX_SIDE_ADAMW_BLOCKS workgroups; 0 = uncapped) so the critical path keeps the rest.  The
    last segment (stage 1) goes at optimizer.step() and stores the step count.  Per element the
    update is torch.optim.AdamW's, exactly as the one-launch form (csrc/adamw.hip): results are
    bit-identical.  Armed by optimizer.zero_grad() (train.py:188's order: the step follows the
    backward), so a bare backward never moves the weights."""

    def __init__(self, opt):
        self.opt = opt
        self.ranges = {sid: (a, b) for sid, a, b in opt.store.segments}
        self.last_sid = max(self.ranges)
        self.side = None
        self.armed = False
        self.done = []
        self.wgrad_blocks = int(os.environ.get("CMX_SIDE_WGRAD_BLOCKS", "0"))
        self.adamw_blocks = int(os.environ.get("CMX_SIDE_ADAMW_BLOCKS", "0"))
        # CMX_SIDE_WGRAD=0: a segment's weight-gradient launches stay on the main stream (in
        # backward order, at the segment boundary); only its AdamW update goes to the side stream
        self.wgrad_side = os.environ.get("CMX_SIDE_WGRAD", "1") == "1"

    def arm(self):
        self.armed, self.done = True, []

    def disarm(self):
        self.armed = False

    def segment_hook(self, sid):
        """Tensor hook: the backward is past segment ``sid`` (and every earlier segment)."""
        def hook(grad):
            if self.armed and not _scaled_backward[0]:
                for s in sorted(self.ranges):
                    if s <= sid and s != self.last_sid and s not in self.done:
                        self._launch(s, last=False, gscale=1.0)
            return None
        return hook

    def _launch(self, sid, last, gscale):
        from . import deferred
        main = torch.cuda.current_stream()
        if self.side is None:
            self.side = torch.cuda.Stream(device=main.device)
        if not self.wgrad_side:
            deferred.flush()
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            deferred.flush(max_blocks=0 if last else self.wgrad_blocks)
            a, b = self.ranges[sid]
            self.opt._adamw_range(a, b, gscale, store_step=last, max_blocks=0 if last else self.adamw_blocks)
        self.done.append(sid)

    def finish(self, gscale=1.0):
        """optimizer.step(): the segments the hooks did not issue (the last one stores the step
        count), then the main stream joins the side stream."""
        rest = [s for s in sorted(self.ranges) if s not in self.done]
        for i, s in enumerate(rest):
            self._launch(s, last=i == len(rest) - 1, gscale=gscale)
        torch.cuda.current_stream().wait_stream(self.side)
        self.armed = False


class _Group(dict):
    """param_group dict whose 'lr' writes through to the device scalar."""

    def __init__(self, owner, *a, **k):
        super().__init__(*a, **k)
        self._owner = owner

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        if key == "lr" and getattr(self, "_owner", None) is not None:
            self._owner._set_lr(float(value))


class FusedAdamW:
    def __init__(self, model, lr=6e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, params=None,
                 grad_sync=None, overlap=None):
        store = model.store
        if store is None:
            raise RuntimeError("model.cuda() must be called before building the optimizer")
        self.store = store
        self.betas, self.eps, self.weight_decay = tuple(betas), float(eps), float(weight_decay)
        dev = store.device
        self.exp_avg = torch.zeros_like(store.flat)
        self.exp_avg_sq = torch.zeros_like(store.flat)
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        # this optimizer's own step-count arrival counters (zero; every launch leaves them zero)
        self.tickets = torch.zeros(query("cmx_adamw_tickets"), dtype=torch.int32, device=dev)
        self.grad_sync = grad_sync          # callable(flat_grad) -> grad scale, or None
        names = list(store.params.keys())
        decay = [store.params[n] for n in names if store.slots[n].decay]
        no_decay = [store.params[n] for n in names if not store.slots[n].decay and not store.slots[n].frozen]
        self._order = decay + no_decay      # index order used by state_dict (group_weight order)
        self.param_groups = [
            _Group(self, params=decay, lr=float(lr), betas=self.betas, eps=self.eps, weight_decay=self.weight_decay,
                   amsgrad=False, maximize=False, foreach=None, capturable=False, differentiable=False, fused=None),
            _Group(self, params=no_decay, lr=float(lr), betas=self.betas, eps=self.eps, weight_decay=0.0,
                   amsgrad=False, maximize=False, foreach=None, capturable=False, differentiable=False, fused=None),
        ]
        self.defaults = dict(lr=float(lr), betas=self.betas, eps=self.eps, weight_decay=self.weight_decay)
        # per-segment updates overlapped with the backward (SegmentUpdate; CMX_OPT_OVERLAP=1 or
        # overlap=True).  Off by default: on the B2 step the side stream's grouped weight-gradient
        # and AdamW launches slowed the latency-bound backward kernels they shared the CUs with by
        # more than they hid (-9 %).  Single-process path: with a gradient
        # all-reduce (grad_sync) the update waits for the whole exchange, as DDP's step does.
        ov = overlap if overlap is not None else os.environ.get("CMX_OPT_OVERLAP", "0") == "1"
        self._seg = None
        backbone = getattr(model, "backbone", None)
        if ov and grad_sync is None and store.flat.is_cuda and len(store.segments) > 1 and backbone is not None:
            self._seg = SegmentUpdate(self)
            backbone.seg_update = self._seg

    # ------------------------------------------------------------------ lr
    def _set_lr(self, lr: float):
        self.lr_t.fill_(lr)          # eager write, outside any captured graph
        for g in self.param_groups:
            dict.__setitem__(g, "lr", lr)

    # ------------------------------------------------------------------ step
    def zero_grad(self, set_to_none: bool = False):
        """Gradients are overwritten by every backward (see module docstring), so nothing is
        cleared; it arms the per-segment update of the coming backward (SegmentUpdate)."""
        if self._seg is not None:
            self._seg.arm()

    def _adamw_range(self, a: int, b: int, gscale: float, store_step: bool, max_blocks: int = 0):
        """cmx_adamw_step_segment over elements [a, b) of the flat buffers (64-aligned)."""
        s = self.store
        f4 = s.flat.element_size()
        sh = ptr(s.shadow) + a * s.shadow.element_size() if s.shadow is not None else 0
        call("cmx_adamw_step_segment", ptr(s.flat) + f4 * a, ptr(s.grad) + f4 * a, ptr(self.exp_avg) + f4 * a,
             ptr(self.exp_avg_sq) + f4 * a, sh, s.shadow_code, ptr(s.decay64) + a // 64, b - a, ptr(self.lr_t),
             ptr(self.step_t), self.betas[0], self.betas[1], self.eps, self.weight_decay, float(gscale),
             int(store_step), int(max_blocks), ptr(self.tickets), stream())

    @torch.no_grad()
    def step(self, closure=None, scaler: "GradScaler | None" = None):
        s = self.store
        gscale = 1.0
        if self.grad_sync is not None:
            gscale = float(self.grad_sync(s.grad))
        seg = self._seg
        if seg is not None and seg.armed and not (scaler is not None and scaler.enabled):
            seg.finish(gscale)
            return None
        if seg is not None:
            seg.disarm()
        if scaler is not None and scaler.enabled:
            # GradScaler.step: skip the update if any (scaled) gradient is inf / nan, else unscale
            # the frozen slots (IFRM lambdas, in no param group) are not checked, as
            # GradScaler.unscale_ only checks the optimizer's parameters
            call("cmx_grad_nonfinite", ptr(s.grad), s.numel, ptr(s.decay64), ptr(scaler.found_inf), stream())
            call("cmx_adamw_step_scaled", ptr(s.flat), ptr(s.grad), ptr(self.exp_avg), ptr(self.exp_avg_sq),
                 ptr(s.shadow), s.shadow_code, ptr(s.decay64), s.numel, ptr(self.lr_t), ptr(self.step_t), self.betas[0],
                 self.betas[1], self.eps, self.weight_decay, gscale, ptr(scaler.scale_t), ptr(scaler.found_inf),
                 ptr(self.tickets), stream())
            return None
        call("cmx_adamw_step", ptr(s.flat), ptr(s.grad), ptr(self.exp_avg), ptr(self.exp_avg_sq), ptr(s.shadow),
             s.shadow_code, ptr(s.decay64), s.numel, ptr(self.lr_t), ptr(self.step_t), self.betas[0], self.betas[1], self.eps,
             self.weight_decay, gscale, ptr(self.tickets), stream())
        return None

    # ------------------------------------------------------------------ checkpoint format
    def state_dict(self):
        s = self.store
        state = {}
        step = self.step_t.detach().cpu().reshape(())
        for i, p in enumerate(self._order):
            sl = s.slot(p)
            state[i] = {"step": step.clone(),
                        "exp_avg": s._param_view(self.exp_avg, sl).detach().clone(),
                        "exp_avg_sq": s._param_view(self.exp_avg_sq, sl).detach().clone()}
        groups, idx = [], 0
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(idx, idx + len(g["params"])))
            idx += len(g["params"])
            groups.append(d)
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, sd):
        s = self.store
        for i, p in enumerate(self._order):
            st = sd["state"].get(i, sd["state"].get(str(i)))
            if st is None:
                continue
            sl = s.slot(p)
            s._param_view(self.exp_avg, sl).copy_(st["exp_avg"])
            s._param_view(self.exp_avg_sq, sl).copy_(st["exp_avg_sq"])
            self.step_t.fill_(float(st["step"]))
        for g, gs in zip(self.param_groups, sd["param_groups"]):
            g["lr"] = gs["lr"]


class GradScaler:
    """Dynamic loss scaling with the API of ``torch.cuda.amp.GradScaler`` as the reference's
    AMP path uses it (train.py:13,56,185-198: ``scaler.scale(loss).backward();
    scaler.step(optimizer); scaler.update()``), defaults init_scale 2**16, growth x2 every
    2000 clean steps, backoff x0.5 on inf / nan.

    The scale, growth tracker and found-inf flag are device tensors updated by kernels
    (csrc/adamw.hip), so a scaled training step never syncs the host and can be replayed
    from a HIP graph.  ``scale(loss)`` multiplies the loss by the device scale (its backward
    carries the scale into every gradient); ``step`` checks the gradients for inf / nan and
    runs the fused AdamW unscaled by 1 / scale, skipping the update on overflow; ``update``
    applies backoff / growth.  The compute dtype stays the model's (bf16 here; fp16 storage
    is not built)."""

    def __init__(self, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True, device="cuda"):
        self.enabled = bool(enabled)
        self.growth_factor, self.backoff_factor = float(growth_factor), float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self.scale_t = torch.full((1,), float(init_scale), dtype=torch.float32, device=device)
        self.tracker = torch.zeros(1, dtype=torch.int32, device=device)
        self.found_inf = torch.zeros(1, dtype=torch.float32, device=device)

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        if self.enabled:
            _scaled_backward[0] = True          # the per-segment update overlap stands aside
        return loss * self.scale_t[0] if self.enabled else loss

    def step(self, optimizer, *args, **kwargs):
        return optimizer.step(scaler=self)

    def update(self, new_scale=None):
        _scaled_backward[0] = False
        if not self.enabled:
            return
        if new_scale is not None:
            self.scale_t.fill_(float(new_scale))
            return
        call("cmx_loss_scale_update", ptr(self.scale_t), ptr(self.tracker), ptr(self.found_inf), self.growth_factor,
             self.backoff_factor, self.growth_interval, stream())

    def get_scale(self) -> float:
        return float(self.scale_t.item()) if self.enabled else 1.0

    def is_enabled(self) -> bool:
        return self.enabled

    def state_dict(self):
        return {"scale": self.get_scale(), "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": int(self.tracker.item())}

    def load_state_dict(self, sd):
        self.scale_t.fill_(float(sd["scale"]))
        self.tracker.fill_(int(sd.get("_growth_tracker", 0)))
        self.growth_factor = float(sd.get("growth_factor", self.growth_factor))
        self.backoff_factor = float(sd.get("backoff_factor", self.backoff_factor))
        self.growth_interval = int(sd.get("growth_interval", self.growth_interval))
