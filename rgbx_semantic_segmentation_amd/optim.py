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

import torch

from . import _lib
from ._lib import call, ptr, query, stream

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
                 grad_sync=None):
        store = model.store
        if store is None:
            raise RuntimeError("model.cuda() must be called before building the optimizer")
        self.store = store
        self.betas, self.eps, self.weight_decay = tuple(betas), float(eps), float(weight_decay)
        dev = store.device
        self.exp_avg = torch.zeros_like(store.flat)
        self.exp_avg_sq = torch.zeros_like(store.flat)
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        self._lr_written = float(lr)
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

    # ------------------------------------------------------------------ lr
    def _set_lr(self, lr: float):
        # eager write, outside any captured graph; the reference loop sets the same value on every
        # param group (train.py:206-207), so only a changed value launches the device write
        if lr != getattr(self, "_lr_written", None):
            self.lr_t.fill_(lr)
            self._lr_written = lr
        for g in self.param_groups:
            dict.__setitem__(g, "lr", lr)

    # ------------------------------------------------------------------ step
    def zero_grad(self, set_to_none: bool = False):
        """Gradients are overwritten by every backward (see module docstring): nothing to clear."""

    @torch.no_grad()
    def step(self, closure=None, scaler: "GradScaler | None" = None):
        s = self.store
        gscale = 1.0
        if self.grad_sync is not None:
            gscale = float(self.grad_sync(s.grad))
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
        return loss * self.scale_t[0] if self.enabled else loss

    def step(self, optimizer, *args, **kwargs):
        return optimizer.step(scaler=self)

    def update(self, new_scale=None):
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
