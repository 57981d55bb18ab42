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
        self.flat.refresh_transposed()

    def zero_grad(self, set_to_none=False):
        self.flat.zero_grad()

    def _ordered_params(self):
        """Parameters in module registration order = torch's optimizer param indices for the
        reference's single AdamW group (train.py:462-473: list(self.parameters()))."""
        return self.flat.params[::-1]

    def state_dict(self, torch_layout=True):
        """torch.optim.AdamW layout ({"state": {i: {step, exp_avg, exp_avg_sq}}, "param_groups"}),
        which Lightning's checkpoint loader and torch AdamW.load_state_dict accept; per-parameter
        moments are copied out of the flat buffers. torch_layout=False: the flat form."""
        g = dict(self.param_groups[0])
        if not torch_layout:
            return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                    "param_groups": [g]}
        params = self._ordered_params()
        state = {}
        if self.step_count > 0:
            for i, p in enumerate(params):
                o, n, shape = self.flat.slice_of(p)
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": self.exp_avg[o:o + n].view(shape).detach().cpu().clone(),
                            "exp_avg_sq": self.exp_avg_sq[o:o + n].view(shape).detach().cpu().clone()}
        g.setdefault("amsgrad", False)
        g.setdefault("maximize", False)
        g.setdefault("foreach", None)
        g.setdefault("capturable", False)
        g.setdefault("differentiable", False)
        g.setdefault("fused", None)
        g["params"] = list(range(len(params)))
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, sd):
        """Accepts the flat form and torch's AdamW layout (a Lightning checkpoint of the
        reference: one param group, indices in registration order)."""
        if "state" in sd:
            params = self._ordered_params()
            groups = sd["param_groups"]
            n_idx = sum(len(g["params"]) for g in groups)
            if n_idx != len(params):
                raise ValueError(f"optimizer state holds {n_idx} parameters, model has {len(params)}")
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            step = 0
            for i, p in enumerate(params):
                st = sd["state"].get(i, sd["state"].get(str(i)))
                if not st:
                    continue
                o, n, shape = self.flat.slice_of(p)
                if tuple(st["exp_avg"].shape) != tuple(shape):
                    raise ValueError(f"optimizer state {i}: shape {tuple(st['exp_avg'].shape)} "
                                     f"!= parameter shape {tuple(shape)}")
                self.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                step = max(step, int(float(st["step"])))
            self.step_count = step
            g0 = groups[0]
            self.param_groups = [dict(lr=float(g0["lr"]), betas=tuple(g0["betas"]),
                                      eps=float(g0["eps"]), weight_decay=float(g0["weight_decay"]),
                                      initial_lr=float(g0.get("initial_lr", g0["lr"])))]
            return
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.param_groups = [{k: v for k, v in g.items() if k != "params"} for g in sd["param_groups"]]


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
        """timm Scheduler.state_dict keys (the instance __dict__ minus the optimizer)."""
        return {"_last_epoch": self._last_epoch, "t_initial": self.t_initial,
                "warmup_t": self.warmup_t, "warmup_lr_init": self.warmup_lr_init,
                "lr_min": self.lr_min, "t_in_epochs": self.t_in_epochs,
                "cycle_limit": self.cycle_limit, "cycle_decay": self.cycle_decay,
                "base_values": list(self.base_values)}

    def load_state_dict(self, sd):
        """Resumes the step counter; accepts the reference's timm layout (`_last_epoch`) and the
        round-1 form of this file (`last_epoch`)."""
        t = sd["_last_epoch"] if "_last_epoch" in sd else sd["last_epoch"]
        self.step(epoch=int(t))
