"""Training step engine for DNABERT-2 MLM pretraining (replaces the Lightning fit loop's
per-batch work: SequenceLightningModule._shared_step/training_step, train.py:339-440, plus
Lightning's backward, DDP gradient all-reduce, clip_grad_norm_ and AdamW/scheduler steps).

One step = embedding/encoder/head forward on HIP kernels -> fused masked-CE loss -> backward
(gradient buckets all-reduced over RCCL as they complete) -> global-norm clip + AdamW on the
flat buffers -> LR schedule. No host synchronisation inside a step: the batch's row indices
(MLMIndex) are computed on the host while it is collated.
"""
import math
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .bert_layers import BertForMaskedLM, MLMIndex
from .ddp import GradBucketReducer, broadcast_
from .flat import FlatParams
from .optim import FusedAdamW, LinearLRSchedulerWarmup


@dataclass
class DeviceBatch:
    masked_ids: torch.Tensor  # [b, S] int64 on device
    mask: torch.Tensor        # [b, S] bool
    labels: torch.Tensor      # [b, S] int64
    target: torch.Tensor      # [b, S] int64 (original ids)
    index: MLMIndex           # on device
    n_mask: int
    n_unk_masked: int

    @staticmethod
    def from_host(masked_ids, mask, labels, target, device, pad_token_id=3):
        """Collated CPU tensors -> device batch; row bookkeeping done on the host (no GPU sync)."""
        idx = MLMIndex.build(masked_ids, labels, pad_token_id)
        n_mask = int(mask.sum())
        n_unk = n_mask - int(idx.target.numel())
        pin = lambda t: t.pin_memory() if torch.cuda.is_available() else t
        dev = lambda t: pin(t).to(device, non_blocking=True)
        return DeviceBatch(dev(masked_ids), dev(mask), dev(labels), dev(target),
                           MLMIndex(*(dev(t) for t in (idx.subset_idx, idx.head_idx, idx.target,
                                                       idx.flat_masked))), n_mask, n_unk)


def _sync_shadow(flat, versions):
    """Re-derive the bf16 parameter copy when a parameter was changed in place outside the fused
    AdamW step (load_state_dict, a manual edit): torch bumps the tensor's version counter then, the
    AdamW kernel (raw pointers) does not. Returns the versions to compare against next step."""
    if flat.shadow is None:
        return None
    v = [p._version for p in flat.params]
    if v != versions:
        flat.refresh_shadow()
    return v


class ModuleTrainer:
    """The same data-parallel step for any model (BASELINE configs D / E: HyenaDNA, Caduceus):
    parameters and gradients in one flat buffer (FlatParams), gradient buckets all-reduced over
    RCCL as they complete in the backward (GradBucketReducer, fp32 or bf16 wire), global-norm clip
    + AdamW in one fused launch (FusedAdamW), the 1/world average folded into it. `loss_fn(model,
    batch)` returns the scalar loss; with `autocast` set it runs under torch.autocast (the configs'
    bf16 mixed precision: fp32 master weights, bf16 compute)."""

    def __init__(self, model, device, loss_fn, lr=1e-3, weight_decay=0.0, betas=(0.9, 0.999),
                 eps=1e-8, max_grad_norm=1.0, bucket_mb=25.0, wire_dtype="fp32",
                 autocast=torch.bfloat16):
        self.model = model.to(device).train()
        self.device = torch.device(device)
        self.loss_fn = loss_fn
        self.autocast = autocast
        # bf16 autocast: a persistent bf16 copy of every parameter, rewritten by the fused AdamW
        # step, stands in for autocast's per-forward weight casts where the kernels read it
        # (mamba._lowp: `_dna_lp` on the parameter)
        lowp = autocast == torch.bfloat16 and torch.device(device).type == "cuda"
        self.flat = FlatParams(self.model, device, shadow_dtype=torch.bfloat16 if lowp else None)
        if lowp:
            for p in self.flat.params:
                p._dna_lp = self.flat.lp(p)
        # weight gradients the hand-written kernels can write into the flat buffer go there
        # directly (no returned dW, no AccumulateGrad add); others return theirs as before
        self.flat.enable_direct_grad(True)
        self.opt = FusedAdamW(self.flat, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                              max_grad_norm=max_grad_norm)
        self.reducer = GradBucketReducer(self.flat, bucket_mb=bucket_mb, wire_dtype=wire_dtype)
        self.world = self.reducer.world
        if self.reducer.enabled:  # DDP construction broadcast
            broadcast_(self.flat.flat, src=0)
        self._versions = _sync_shadow(self.flat, None)  # bf16 copy of the (broadcast) weights
        self.global_step = 0

    def step(self, batch) -> torch.Tensor:
        self._versions = _sync_shadow(self.flat, self._versions)
        self.opt.zero_grad()
        self.reducer.prepare(sync=True)
        if self.autocast is not None:
            with torch.autocast(self.device.type, dtype=self.autocast):
                loss = self.loss_fn(self.model, batch)
        else:
            loss = self.loss_fn(self.model, batch)
        loss.backward()
        self.reducer.finish()
        self.opt.step(grad_scale=self.reducer.grad_scale)
        self.global_step += 1
        return loss.detach()


class MLMTrainer:
    def __init__(self, model: BertForMaskedLM, device, lr=5e-4, weight_decay=1e-5,
                 betas=(0.9, 0.999), eps=1e-8, max_grad_norm=1.0, scheduler=None,
                 bucket_mb=25.0, seed=None, wire_dtype="fp32"):
        self.model = model.to(device).train()
        self.device = device
        self.flat = FlatParams(self.model, device)
        self.flat.enable_direct_grad(True)
        self.opt = FusedAdamW(self.flat, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                              max_grad_norm=max_grad_norm)
        self.sched = None
        if scheduler is not None:
            self.sched = LinearLRSchedulerWarmup(self.opt, **scheduler)
        self.reducer = GradBucketReducer(self.flat, bucket_mb=bucket_mb, wire_dtype=wire_dtype)
        self.world = self.reducer.world
        if self.reducer.enabled:  # DDP construction broadcast (C2 in SURVEY §2.2)
            broadcast_(self.flat.flat, src=0)
        # dropout stream: derived from train.seed when given, and distinct per rank
        rank = dist.get_rank() if dist.is_initialized() else 0
        base = self.model.dropout_rng.seed if seed is None else int(seed) + 0x5EED
        self.model.dropout_rng.seed = (base * 1000003 + rank) & (2 ** 63 - 1)
        self.global_step = 0
        self._versions = _sync_shadow(self.flat, None)
        self.micro_losses = []  # undivided loss of each micro-batch of the last step (metrics)

    def rng_state(self):
        """Dropout stream position, saved in checkpoints so a resume does not replay masks."""
        r = self.model.dropout_rng
        return {"seed": int(r.seed), "offset": int(r.offset)}

    def load_rng_state(self, st):
        self.model.dropout_rng.seed = int(st["seed"])
        self.model.dropout_rng.offset = int(st["offset"])

    def step(self, batch, accum=None) -> torch.Tensor:
        """One optimizer step over one micro-batch or a list of them (accumulate_grad_batches:
        each micro-batch loss is divided by `accum` -- default their number -- like Lightning,
        which divides by accumulate_grad_batches even in an epoch's short last window;
        gradients are all-reduced only during the last micro-batch's backward, like DDP
        no_sync)."""
        micro = batch if isinstance(batch, (list, tuple)) else [batch]
        div = len(micro) if accum is None else int(accum)
        self._versions = _sync_shadow(self.flat, self._versions)
        self.opt.zero_grad()
        total = None
        self.micro_losses = []
        for i, mb in enumerate(micro):
            last = i == len(micro) - 1
            self.reducer.prepare(sync=last)
            loss, _ = self.model.mlm_loss(mb.masked_ids, mb.mask, mb.index, mb.n_mask,
                                          mb.n_unk_masked)
            self.micro_losses.append(loss.detach())
            if div > 1:
                loss = loss / div
            loss.backward()
            total = loss.detach() if total is None else total + loss.detach()
        self.reducer.finish()
        self.opt.step(grad_scale=self.reducer.grad_scale)
        if self.sched is not None:
            self.sched.step()
        self.global_step += 1
        return total
