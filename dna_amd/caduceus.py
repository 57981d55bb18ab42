"""Caduceus masked-LM around the HIP BiMamba mixer (BASELINE config E).

Mirrors the reference's `CaduceusForMaskedLM` (src/models/caduceus/modeling_caduceus.py:373-470)
for rcps=False: token embeddings (:124-144), `n_layer` mamba_ssm pre-norm Blocks
[add -> norm -> BiMambaWrapper] (create_block :25-65; the fused_add_norm Triton path computes the
same add + norm), the final add + norm_f (:214-216), an LM head tied to the embeddings (HF
tie_weights) and cross entropy ignoring pad_token_id (:257-262). Parameter names follow the
reference (`caduceus.backbone.layers.{i}.mixer.mamba_fwd.*`, `...norm.weight`, `lm_head.weight`).
mamba_ssm (Mamba, Block, RMSNorm) is not vendored: their forward is restated, parity unpinned.
The RC-equivariant variant (rcps=True: RCPSEmbedding / RCPSMambaBlock / RCPSLMHead) is not built.
"""
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as DF
from .hyena_lm import _LN_COLS, LayerNorm
from .mamba import BiMambaWrapper

_TORCH_NORM = os.environ.get("DNA_CADUCEUS_TORCH_NORM", "0") == "1"  # A/B switch: torch norms


class RMSNorm(nn.Module):
    """mamba_ssm RMSNorm: x * rsqrt(mean(x^2) + eps) * weight."""

    def __init__(self, hidden_size, eps=1e-5, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden_size, device=device, dtype=dtype))
        self.register_parameter("bias", None)

    def forward(self, x):
        d = x.shape[-1]
        if (_TORCH_NORM or d not in _LN_COLS or self.weight.dtype != torch.float32
                or x.dtype not in (torch.float32, torch.bfloat16)):
            xf = x.float()
            return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps) * self.weight).to(x.dtype)
        # HIP kernel (dna_rms_fwd/bwd). Out of autocast: x.dtype as above. Under CUDA bf16
        # autocast the next op is the mixer's in_proj Linear, which casts this output to bf16:
        # the kernel writes that rounding directly (x is the fp32 residual in every Block).
        bf16_out = (torch.is_autocast_enabled("cuda")
                    and torch.get_autocast_dtype("cuda") == torch.bfloat16)
        y32, yb = DF.RMSNormFn.apply(x.reshape(-1, d), self.weight, self.eps,
                                     not bf16_out, bf16_out)
        y = yb if bf16_out else y32.to(x.dtype)
        return y.view(*x.shape[:-1], d)


class MambaBlock(nn.Module):
    """mamba_ssm.modules.mamba_simple.Block: (hidden, residual) -> (mixer(norm(add)), add)."""

    def __init__(self, dim, mixer, norm, residual_in_fp32=True):
        super().__init__()
        self.mixer = mixer
        self.norm = norm
        self.residual_in_fp32 = residual_in_fp32

    def forward(self, hidden_states, residual=None):
        residual = hidden_states + residual if residual is not None else hidden_states
        hidden_states = self.norm(residual.to(dtype=self.norm.weight.dtype))
        if self.residual_in_fp32:
            residual = residual.to(torch.float32)
        return self.mixer(hidden_states), residual


class CaduceusEmbeddings(nn.Module):
    def __init__(self, vocab_size, d_model):
        super().__init__()
        self.word_embeddings = nn.Embedding(vocab_size, d_model)

    def forward(self, input_ids):
        return self.word_embeddings(input_ids)


class CaduceusMixerModel(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.residual_in_fp32 = cfg["residual_in_fp32"]
        self.embeddings = CaduceusEmbeddings(cfg["vocab_size"], cfg["d_model"])
        norm_cls = RMSNorm if cfg["rms_norm"] else LayerNorm
        ssm = dict(cfg.get("ssm_cfg") or {})
        self.layers = nn.ModuleList([
            MambaBlock(cfg["d_model"],
                       BiMambaWrapper(cfg["d_model"], bidirectional=cfg["bidirectional"],
                                      bidirectional_strategy=cfg["bidirectional_strategy"],
                                      bidirectional_weight_tie=cfg["bidirectional_weight_tie"],
                                      layer_idx=i, **ssm),
                       norm_cls(cfg["d_model"], eps=cfg["norm_epsilon"]),
                       residual_in_fp32=cfg["residual_in_fp32"])
            for i in range(cfg["n_layer"])])
        self.norm_f = norm_cls(cfg["d_model"], eps=cfg["norm_epsilon"])

    def forward(self, input_ids):
        hidden_states = self.embeddings(input_ids)
        residual = None
        for layer in self.layers:
            hidden_states, residual = layer(hidden_states, residual)
        residual = hidden_states + residual if residual is not None else hidden_states
        return self.norm_f(residual.to(dtype=self.norm_f.weight.dtype))


class Caduceus(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.backbone = CaduceusMixerModel(cfg)

    def forward(self, input_ids):
        return self.backbone(input_ids)


DEFAULTS = dict(d_model=2560, n_layer=64, vocab_size=50277, ssm_cfg=None, rms_norm=True,
                residual_in_fp32=True, fused_add_norm=True, pad_vocab_size_multiple=8,
                norm_epsilon=1e-5, initializer_cfg=None, bidirectional=True,
                bidirectional_strategy="add", bidirectional_weight_tie=True, rcps=False,
                complement_map=None, pad_token_id=-100, tie_word_embeddings=True)


def _init_weights(module, n_layer, initializer_range=0.02, rescale_prenorm_residual=True,
                  n_residuals_per_layer=1):
    """CaduceusPreTrainedModel._init_weights (modeling_caduceus.py:283-322)."""
    if isinstance(module, nn.Linear):
        if module.bias is not None and not getattr(module.bias, "_no_reinit", False):
            nn.init.zeros_(module.bias)
    elif isinstance(module, nn.Embedding):
        nn.init.normal_(module.weight, std=initializer_range)
    if rescale_prenorm_residual:
        for name, p in module.named_parameters():
            if name in ["out_proj.weight", "fc2.weight"]:
                nn.init.kaiming_uniform_(p, a=math.sqrt(5))
                with torch.no_grad():
                    p /= math.sqrt(n_residuals_per_layer * n_layer)


class CaduceusForMaskedLM(nn.Module):
    """CaduceusForMaskedLM (rcps=False). forward(input_ids, labels=None) -> (loss, logits)."""

    def __init__(self, **config):
        super().__init__()
        cfg = dict(DEFAULTS)
        unknown = set(config) - set(DEFAULTS)
        if unknown:
            raise TypeError(f"CaduceusForMaskedLM: unknown config keys {sorted(unknown)}")
        cfg.update(config)
        if cfg["rcps"]:
            raise NotImplementedError("Caduceus rcps=True (RC-equivariant RCPS layers) is not built")
        if cfg["vocab_size"] % cfg["pad_vocab_size_multiple"]:
            cfg["vocab_size"] += cfg["pad_vocab_size_multiple"] - cfg["vocab_size"] % cfg["pad_vocab_size_multiple"]
        self.config = cfg
        self.caduceus = Caduceus(cfg)
        self.lm_head = nn.Linear(cfg["d_model"], cfg["vocab_size"], bias=False)
        ic = cfg["initializer_cfg"] or {}
        self.apply(lambda m: _init_weights(m, cfg["n_layer"], **ic))
        if cfg["tie_word_embeddings"]:
            self.lm_head.weight = self.caduceus.backbone.embeddings.word_embeddings.weight

    def forward(self, input_ids, labels=None):
        logits = self.lm_head(self.caduceus(input_ids)).float()
        loss = None
        if labels is not None:
            loss = F.cross_entropy(logits.view(-1, logits.shape[-1]), labels.view(-1),
                                   ignore_index=self.config["pad_token_id"])
        return loss, logits
