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

from typing import Optional

import torch

from . import _lib
from ._lib import call, ptr, stream


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
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self.grad_sync = grad_sync          # callable(flat_grad) -> grad scale, or None
        names = list(store.params.keys())
        decay = [store.params[n] for n in names if store.slots[n].decay]
        no_decay = [store.params[n] for n in names if not store.slots[n].decay]
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
        self.lr_t.fill_(lr)          # eager write, outside any captured graph
        for g in self.param_groups:
            dict.__setitem__(g, "lr", lr)

    # ------------------------------------------------------------------ step
    def zero_grad(self, set_to_none: bool = False):
        """No-op: gradients are overwritten by every backward (see module docstring)."""

    @torch.no_grad()
    def step(self, closure=None):
        s = self.store
        gscale = 1.0
        if self.grad_sync is not None:
            gscale = float(self.grad_sync(s.grad))
        call("cmx_adamw_step", ptr(s.flat), ptr(s.grad), ptr(self.exp_avg), ptr(self.exp_avg_sq), ptr(s.shadow),
             ptr(s.decay64), s.numel, ptr(self.lr_t), ptr(self.step_t), self.betas[0], self.betas[1], self.eps,
             self.weight_decay, gscale, stream())
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
