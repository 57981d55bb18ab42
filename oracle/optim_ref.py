"""Restatement of the optimizer step of the hot path (TEST INFRASTRUCTURE).

Oracle only (tests/, smoke(), bench cpu_baseline). The reference step is PyTorch-Lightning's
`gradient_clip_val: 1.0` (torch.nn.utils.clip_grad_norm_, norm type 2) followed by torch
`AdamW` (registry.optimizer["adamw"], src/utils/registry.py:3; built in
train.py:462-542 with lr 5e-4, weight_decay 1e-5, betas (0.9, 0.999), eps 1e-8 defaults) and
`LinearLRSchedulerWarmup` (src/utils/optim/schedulers.py:92-147), stepped every optimizer step.
The tests pin `clip_and_adamw` against torch.optim.AdamW + clip_grad_norm_ directly.
"""
import math

import numpy as np


def clip_coef(grads, max_norm=1.0):
    """torch.nn.utils.clip_grad_norm_: total L2 norm over all grads; coef clamped to 1."""
    total = math.sqrt(sum(float(np.sum(np.asarray(g, np.float64) ** 2)) for g in grads))
    return min(1.0, max_norm / (total + 1e-6)), total


def adamw_step(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0):
    """One torch.optim.AdamW step (decoupled weight decay, bias-corrected), in float64."""
    p = p * (1.0 - lr * weight_decay)
    m = beta1 * m + (1.0 - beta1) * g
    v = beta2 * v + (1.0 - beta2) * g * g
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    denom = np.sqrt(v) / math.sqrt(bc2) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v


def linear_warmup_lr(t, base_lr, warmup_t, t_initial, warmup_lr_init=0.0, lr_min=0.0):
    """LinearLRSchedulerWarmup._get_lr (schedulers.py:113-132) with cycle_decay = 1 and no
    cycle limit -- the values the reference would compute had `self.cycle_limit` /
    `self.cycle_decay` been set (they are not: the reference raises AttributeError once
    t >= warmup_t)."""
    if t < warmup_t:
        return warmup_lr_init + t * (base_lr - warmup_lr_init) / warmup_t
    cycle = math.floor(1 + (t - warmup_t) / t_initial)
    t_curr = t - warmup_t - (cycle - 1) * t_initial
    return lr_min + (base_lr - lr_min) * (1 - t_curr / t_initial)
