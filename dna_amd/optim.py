"""Fused optimizer step and LR schedule of the DNABERT-2 pretraining path.

FusedAdamW = Lightning `gradient_clip_val: 1.0` (torch.nn.utils.clip_grad_norm_) + torch AdamW
(reference: train.py:462-542, registry.optimizer["adamw"], configs/optimizer/adamw.yaml,
experiment overrides lr 5e-4 / weight_decay 1e-5) over the flat buffers of dna_amd.flat: one
sum-of-squares launch and one AdamW launch per step, clip coefficient read on the device.

LinearLRSchedulerWarmup restates src/utils/optim/schedulers.py:92-147 (timm Scheduler subclass,
stepped per optimizer step with t_in_epochs False). The reference leaves `cycle_limit` and
`cycle_decay` unset and raises AttributeError once t >= warmup_t; here they default to
no limit / decay 1, the values the formula needs.
"""
import math

import torch

from . import _native as N


class FusedAdamW:
    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 max_grad_norm=1.0):
        self.flat = flat
        dev = flat.flat.device
        self.exp_avg = torch.zeros_like(flat.flat)
        self.exp_avg_sq = torch.zeros_like(flat.flat)
        self.param_groups = [dict(lr=float(lr), betas=tuple(betas), eps=float(eps),
                                  weight_decay=float(weight_decay), initial_lr=float(lr))]
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        nws = N.lib().dna_sumsq_workspace(flat.numel)
        self._ws = torch.empty(nws // 4 + 4, dtype=torch.float32, device=dev)
        self._nws = nws

    def grad_norm_sq(self):
        """Launch the global sum of squares of the gradient (device scalar, no sync)."""
        N.call("dna_sumsq", self.flat.grad.data_ptr(), self.flat.numel, self._sumsq.data_ptr(),
               self._ws.data_ptr(), self._nws, N.stream_ptr())
        return self._sumsq

    def step(self, grad_scale: float = 1.0):
        g = self.param_groups[0]
        self.step_count += 1
        clip = self.max_grad_norm is not None and self.max_grad_norm > 0
        if clip:
            self.grad_norm_sq()
        shadow = self.flat.shadow
        N.call("dna_adamw_step", self.flat.flat.data_ptr(), self.flat.grad.data_ptr(),
               self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
               None if shadow is None else shadow.data_ptr(), self.flat.numel, g["lr"],
               g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"], self.step_count,
               self._sumsq.data_ptr() if clip else None,
               float(self.max_grad_norm or 0.0), float(grad_scale), N.stream_ptr())

    def zero_grad(self, set_to_none=False):
        self.flat.zero_grad()

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "param_groups": [dict(g) for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.param_groups = [dict(g) for g in sd["param_groups"]]


class LinearLRSchedulerWarmup:
    """Linear warmup from warmup_lr_init to the base lr over warmup_t steps, then linear decay to
    lr_min over t_initial steps (schedulers.py:113-132), applied to optimizer.param_groups."""

    def __init__(self, optimizer, t_initial, warmup_t=0, warmup_lr_init=0.0, lr_min=0.0,
                 t_in_epochs=False, cycle_limit=None, cycle_decay=1.0, **unused):
        self.optimizer = optimizer
        self.t_initial = t_initial
        self.warmup_t = warmup_t
        self.warmup_lr_init = warmup_lr_init
        self.lr_min = lr_min
        self.t_in_epochs = t_in_epochs
        self.cycle_limit = cycle_limit
        self.cycle_decay = cycle_decay
        self.base_values = [g.get("initial_lr", g["lr"]) for g in optimizer.param_groups]
        self._last_epoch = 0
        self.step(epoch=0)

    def _get_lr(self, t):
        if t < self.warmup_t:
            return [self.warmup_lr_init + t * (lr - self.warmup_lr_init) / self.warmup_t
                    for lr in self.base_values]
        if self.cycle_limit is not None and t >= self.cycle_limit * self.t_initial:
            return [self.lr_min for _ in self.base_values]
        cycle = math.floor(1 + (t - self.warmup_t) / self.t_initial)
        t_curr = t - self.warmup_t - (cycle - 1) * self.t_initial
        gamma = self.cycle_decay ** cycle
        return [self.lr_min + (lr * gamma - self.lr_min) * (1 - t_curr / self.t_initial)
                for lr in self.base_values]

    def step(self, epoch=None):
        self._last_epoch = self._last_epoch + 1 if epoch is None else epoch
        for g, lr in zip(self.optimizer.param_groups, self._get_lr(self._last_epoch)):
            g["lr"] = lr

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        return {"last_epoch": self._last_epoch}

    def load_state_dict(self, sd):
        self.step(epoch=sd["last_epoch"])
