"""LR schedule used by the training loop (reference: utils/lr_policy.py:30-42)."""


class WarmUpPolyLR:
    """lr = start * it / warmup during warm-up, else start * (1 - it / total) ** power."""

    def __init__(self, start_lr, lr_power, total_iters, warmup_steps):
        self.start_lr = start_lr
        self.lr_power = lr_power
        self.total_iters = total_iters + 0.0
        self.warmup_steps = warmup_steps

    def get_lr(self, cur_iter):
        if cur_iter < self.warmup_steps:
            return self.start_lr * (cur_iter / self.warmup_steps)
        return self.start_lr * ((1 - float(cur_iter) / self.total_iters) ** self.lr_power)
