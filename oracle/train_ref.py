"""CPU restatement of the reference training step (TEST ORACLE / CPU baseline).

Test infrastructure only.  Restates ``train.py:104-223``:
  * parameter groups of ``utils/init_func.py:33-57`` (``group_weight``): Linear/Conv
    weights decay, biases and norm affine params do not;
  * ``torch.optim.AdamW(betas=(0.9, 0.999), weight_decay=0.01)`` (``train.py:128-129``);
  * ``WarmUpPolyLR`` (``utils/lr_policy.py:30-42``) with the LR written into the param
    groups AFTER ``optimizer.step()`` (``train.py:201-207``), i.e. one step late.
"""
from __future__ import annotations

import time
import torch
import torch.nn as nn

from .cmx_ref import EncoderDecoder, CMXConfig


class WarmUpPolyLR:
    def __init__(self, start_lr, lr_power, total_iters, warmup_steps):
        self.start_lr, self.lr_power = start_lr, lr_power
        self.total_iters, self.warmup_steps = float(total_iters), warmup_steps

    def get_lr(self, cur_iter):
        if cur_iter < self.warmup_steps:
            return self.start_lr * (cur_iter / self.warmup_steps)
        return self.start_lr * ((1 - float(cur_iter) / self.total_iters) ** self.lr_power)


def group_weight(model: nn.Module, lr: float):
    decay, no_decay = [], []
    for m in model.modules():
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            decay.append(m.weight)
            if m.bias is not None:
                no_decay.append(m.bias)
        elif isinstance(m, (nn.BatchNorm2d, nn.LayerNorm)):
            if m.weight is not None:
                no_decay.append(m.weight)
            if m.bias is not None:
                no_decay.append(m.bias)
    return [dict(params=decay, lr=lr), dict(params=no_decay, weight_decay=0.0, lr=lr)]


def make_optimizer(model, cfg: CMXConfig):
    return torch.optim.AdamW(group_weight(model, cfg.lr), lr=cfg.lr, betas=(0.9, 0.999),
                             weight_decay=cfg.weight_decay, foreach=False)


def train_steps(model, optimizer, lr_policy, batches, start_iter=0):
    """Run the reference loop body over ``batches`` [(rgb, x, label)]; returns losses."""
    model.train()
    losses = []
    for i, (rgb, x, gt) in enumerate(batches):
        loss = model(rgb, x, gt)
        optimizer.zero_grad()
        loss.backward()
        optimizer.step()
        lr = lr_policy.get_lr(start_iter + i)
        for g in optimizer.param_groups:
            g["lr"] = lr
        losses.append(float(loss.detach()))
    return losses


def time_cpu_steps(cfg: CMXConfig, batch, warmup=1, steps=2, threads=None, seed=0):
    """Wall-clock CPU train steps (fp32) of the restated reference loop."""
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    model = EncoderDecoder(cfg)
    opt = make_optimizer(model, cfg)
    pol = WarmUpPolyLR(cfg.lr, cfg.lr_power, 200 * 148, 148 * 10)
    train_steps(model, opt, pol, [batch] * warmup)
    t0 = time.perf_counter()
    train_steps(model, opt, pol, [batch] * steps, start_iter=warmup)
    return (time.perf_counter() - t0) / steps
