"""Caduceus masked-LM around the HIP BiMamba mixer (BASELINE config E).

Mirrors the reference's `CaduceusForMaskedLM` (src/models/caduceus/modeling_caduceus.py:373-470)
for rcps=False: token embeddings (:124-144), `n_layer` mamba_ssm pre-norm Blocks
[add -> norm -> BiMambaWrapper] (create_block :25-65; the fused_add_norm Triton path computes the
same add + norm), the final add + norm_f (:214-216), an LM head tied to the embeddings (HF
tie_weights) and cross entropy ignoring pad_token_id (:260-264), optionally weighted per token
(weighted_cross_entropy :267-275). Parameter names follow the reference
(`caduceus.backbone.layers.{i}.mixer.mamba_fwd.*`, `...norm.weight`, `lm_head.weight`).
mamba_ssm (Mamba, Block, RMSNorm) is not vendored: their forward is restated, parity unpinned.

rcps=True builds the reverse-complement parameter-sharing variant (modeling_rcps.py): the hidden
state carries 2*d_model channels, [forward strand | reverse complement flipped over length AND
channels]; every sub-layer runs once per half with shared weights. Its fused_add_norm block
(RCPSMambaBlock.forward, modeling_rcps.py:157-197) feeds the SECOND half to the forward-strand
norm and the flipped first half to the RC norm, so the two halves trade places at every fused
block; the non-fused RCPSAddNormWrapper (:99-127) keeps them in place. Both are mirrored as
written -- each preserves RC equivariance (tests/test_gpu_caduceus.py checks it exactly).
"""
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as DF
from .hyena_lm import _LN_COLS, LayerNorm
from .hyena import HipLinear, hip_linear
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

    def add_ok(self, x, residual):
        """add_norm applies: kernel widths / dtypes and an fp32 residual stream (torch's
        x + residual is then fp32 too)."""
        return (not _TORCH_NORM and x.is_cuda and residual is not None
                and residual.dtype == torch.float32 and x.dtype in (torch.float32, torch.bfloat16)
                and x.shape[-1] in _LN_COLS and self.weight.dtype == torch.float32
                and residual.shape == x.shape)

    def add_norm(self, x, residual):
        """(x + residual, self(x + residual)) in one kernel (functional.AddLayerNorm, RMS mode)."""
        d = x.shape[-1]
        bf16_out = (torch.is_autocast_enabled("cuda")
                    and torch.get_autocast_dtype("cuda") == torch.bfloat16)
        s, y = DF.AddLayerNorm.apply(x.reshape(-1, d), residual.reshape(-1, d), self.weight, None,
                                     self.eps, bf16_out)
        return s.view(*x.shape), y.view(*x.shape)


class MambaBlock(nn.Module):
    """mamba_ssm.modules.mamba_simple.Block: (hidden, residual) -> (mixer(norm(add)), add)."""

    def __init__(self, dim, mixer, norm, residual_in_fp32=True):
        super().__init__()
        self.mixer = mixer
        self.norm = norm
        self.residual_in_fp32 = residual_in_fp32

    def forward(self, hidden_states, residual=None):
        if hasattr(self.norm, "add_ok") and self.norm.add_ok(hidden_states, residual):
            # add + norm in one kernel (fp32 residual stream: the same sum and norm)
            residual, hidden_states = self.norm.add_norm(hidden_states, residual)
            return self.mixer(hidden_states), residual
        residual = hidden_states + residual if residual is not None else hidden_states
        hidden_states = self.norm(residual.to(dtype=self.norm.weight.dtype))
        if self.residual_in_fp32:
            residual = residual.to(torch.float32)
        return self.mixer(hidden_states), residual


def _rc(x):
    """RCPSWrapper.rc (modeling_rcps.py:77-80): flip length (dim -2) and channels (dim -1)."""
    return torch.flip(x, dims=[-2, -1])


def _complement_tensor(complement_map):
    """torch.tensor(list(OrderedDict(complement_map).values())) as modeling_rcps.py:27-30 builds
    it; a list/tuple is taken as already ordered by token id."""
    vals = list(complement_map.values()) if isinstance(complement_map, dict) else list(complement_map)
    return torch.tensor(vals, dtype=torch.long)


class RCPSEmbedding(nn.Module):
    """modeling_rcps.py:18-64: [emb(ids) | flip_{L,C}(emb(rc(ids)))], 2*d_model channels."""

    def __init__(self, vocab_size, d_model, complement_map):
        super().__init__()
        cm = _complement_tensor(complement_map)
        if cm.numel() != vocab_size:
            raise ValueError(f"complement_map has {cm.numel()} entries for a vocabulary of {vocab_size}")
        self.register_buffer("complement_map", cm)
        self.embedding = DF.HipEmbedding(vocab_size, d_model)

    @property
    def weight(self):
        return self.embedding.weight

    def set_weight(self, value):
        self.embedding.weight = value

    def rc(self, x):
        """Flip along length and complement every id (modeling_rcps.py:43-49)."""
        return self.complement_map[torch.flip(x, dims=[-1])]

    def forward(self, input_ids):
        return torch.cat([self.embedding(input_ids), _rc(self.embedding(self.rc(input_ids)))], dim=-1)


class RCPSWrapper(nn.Module):
    """modeling_rcps.py:67-96: submodule on the first half and on rc(second half); the RC output
    is flipped back. Shared weights, 2x the channels out."""

    def __init__(self, submodule):
        super().__init__()
        self.submodule = submodule

    def forward(self, x, **kwargs):
        c = x.shape[-1] // 2
        fwd = self.submodule(x[..., :c], **kwargs)
        rc = self.submodule(_rc(x[..., c:]), **kwargs)
        return torch.cat([fwd, _rc(rc)], dim=-1)


def _add_norm(norm, x, residual, residual_in_fp32):
    """mamba_ssm's fused add + norm (prenorm=True): (norm(x + residual), x + residual), the
    residual kept in fp32 when residual_in_fp32 -- the same arithmetic MambaBlock.forward uses."""
    if hasattr(norm, "add_ok") and norm.add_ok(x, residual):
        residual, y = norm.add_norm(x, residual)  # one kernel, fp32 residual stream
        return y, residual
    residual = x if residual is None else x + residual
    y = norm(residual.to(dtype=norm.weight.dtype))
    return y, (residual.to(torch.float32) if residual_in_fp32 else residual)


class RCPSAddNormWrapper(RCPSWrapper):
    """modeling_rcps.py:99-127: add + norm per half, halves kept in place."""

    def forward(self, x, residual=None, prenorm=False):
        c = x.shape[-1] // 2
        norm = self.submodule
        if residual is None:
            residual = x
            y = torch.cat([norm(x[..., :c].to(dtype=norm.weight.dtype)),
                           _rc(norm(_rc(x[..., c:]).to(dtype=norm.weight.dtype)))], dim=-1)
        else:
            r_fwd = x[..., :c] + residual[..., :c]
            r_rc = _rc(x[..., c:]) + _rc(residual[..., c:])
            y = torch.cat([norm(r_fwd.to(dtype=norm.weight.dtype)),
                           _rc(norm(r_rc.to(dtype=norm.weight.dtype)))], dim=-1)
            residual = torch.cat([r_fwd, _rc(r_rc)], dim=-1)
        return (y, residual) if prenorm else y


class RCPSMambaBlock(nn.Module):
    """modeling_rcps.py:130-203 (the RCPS mamba_ssm Block)."""

    def __init__(self, dim, mixer, norm, fused_add_norm=True, residual_in_fp32=True):
        super().__init__()
        self.residual_in_fp32 = residual_in_fp32
        self.fused_add_norm = fused_add_norm
        self.mixer = RCPSWrapper(mixer)
        self.norm = norm if fused_add_norm else RCPSAddNormWrapper(norm)

    def forward(self, hidden_states, residual=None):
        if not self.fused_add_norm:
            hidden_states, residual = self.norm(hidden_states, residual=residual, prenorm=True)
            if self.residual_in_fp32:
                residual = residual.to(torch.float32)
        else:
            c = hidden_states.shape[-1] // 2
            h_fwd, r_fwd = _add_norm(self.norm, hidden_states[..., c:],
                                     None if residual is None else residual[..., c:],
                                     self.residual_in_fp32)
            h_rc, r_rc = _add_norm(self.norm, _rc(hidden_states[..., :c]),
                                   None if residual is None else _rc(residual[..., :c]),
                                   self.residual_in_fp32)
            hidden_states = torch.cat([h_fwd, _rc(h_rc)], dim=-1)
            residual = torch.cat([r_fwd, _rc(r_rc)], dim=-1)
        return self.mixer(hidden_states), residual


class RCPSLMHead(nn.Module):
    """modeling_rcps.py:206-243: W x_fwd + W[complement_map] flip_C(x_rc)."""

    def __init__(self, true_dim, vocab_size, complement_map):
        super().__init__()
        self.register_buffer("complement_map", _complement_tensor(complement_map))
        self.true_dim = true_dim
        self.lm_head = HipLinear(true_dim, vocab_size, bias=False)

    @property
    def weight(self):
        return self.lm_head.weight

    def set_weight(self, value):
        self.lm_head.weight = value

    def forward(self, x):
        c = x.shape[-1]
        if c != 2 * self.true_dim:
            raise ValueError(f"RCPSLMHead: input has {c} channels, expected 2 * {self.true_dim}")
        fwd = hip_linear(x[..., :c // 2], self.weight, self.lm_head.bias)
        rc = hip_linear(torch.flip(x[..., c // 2:], dims=[-1]), self.weight[self.complement_map, :],
                        self.lm_head.bias)
        return fwd + rc


class CaduceusEmbeddings(nn.Module):
    def __init__(self, vocab_size, d_model, rcps=False, complement_map=None):
        super().__init__()
        self.word_embeddings = (RCPSEmbedding(vocab_size, d_model, complement_map) if rcps
                                else DF.HipEmbedding(vocab_size, d_model))

    def forward(self, input_ids):
        return self.word_embeddings(input_ids)


class CaduceusMixerModel(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.residual_in_fp32 = cfg["residual_in_fp32"]
        self.fused_add_norm = cfg["fused_add_norm"]
        self.rcps = cfg["rcps"]
        self.embeddings = CaduceusEmbeddings(cfg["vocab_size"], cfg["d_model"], cfg["rcps"],
                                             cfg["complement_map"])
        norm_cls = RMSNorm if cfg["rms_norm"] else LayerNorm
        ssm = dict(cfg.get("ssm_cfg") or {})
        layers = []
        for i in range(cfg["n_layer"]):
            mixer = BiMambaWrapper(cfg["d_model"], bidirectional=cfg["bidirectional"],
                                   bidirectional_strategy=cfg["bidirectional_strategy"],
                                   bidirectional_weight_tie=cfg["bidirectional_weight_tie"],
                                   layer_idx=i, **ssm)
            norm = norm_cls(cfg["d_model"], eps=cfg["norm_epsilon"])
            if self.rcps:   # create_block :56 picks RCPSMambaBlock
                layers.append(RCPSMambaBlock(cfg["d_model"], mixer, norm, cfg["fused_add_norm"],
                                             cfg["residual_in_fp32"]))
            else:
                layers.append(MambaBlock(cfg["d_model"], mixer, norm, cfg["residual_in_fp32"]))
        self.layers = nn.ModuleList(layers)
        norm_f = norm_cls(cfg["d_model"], eps=cfg["norm_epsilon"])
        # modeling_caduceus.py:195
        self.norm_f = norm_f if (self.fused_add_norm or not self.rcps) else RCPSAddNormWrapper(norm_f)

    def forward(self, input_ids):
        hidden_states = self.embeddings(input_ids)
        residual = None
        for layer in self.layers:
            hidden_states, residual = layer(hidden_states, residual)
        if self.rcps:
            # :214-243 -- fused or not, the final norm keeps the halves in place
            norm = self.norm_f if self.fused_add_norm else self.norm_f.submodule
            c = hidden_states.shape[-1] // 2
            fwd, _ = _add_norm(norm, hidden_states[..., :c],
                               None if residual is None else residual[..., :c], self.residual_in_fp32)
            rc, _ = _add_norm(norm, _rc(hidden_states[..., c:]),
                              None if residual is None else _rc(residual[..., c:]),
                              self.residual_in_fp32)
            return torch.cat([fwd, _rc(rc)], dim=-1)
        if hasattr(self.norm_f, "add_ok") and self.norm_f.add_ok(hidden_states, residual):
            return self.norm_f.add_norm(hidden_states, residual)[1]
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


def weighted_cross_entropy(logits, y, loss_weights, ignore_index=-100):
    """modeling_caduceus.py:267-275: per-token CE scaled by loss_weights normalised over the
    non-ignored tokens (the reference zeroes the ignored weights in place; this does not mutate
    the caller's tensor)."""
    logits = logits.view(-1, logits.shape[-1])
    y = y.view(-1)
    ce = F.cross_entropy(logits, y, ignore_index=ignore_index, reduction="none")
    w = loss_weights.reshape(-1).masked_fill(y == ignore_index, 0.0)
    return (ce * (w / w.sum())).sum()


class CaduceusForMaskedLM(nn.Module):
    """CaduceusForMaskedLM. forward(input_ids, labels=None, loss_weights=None) -> (loss, logits)."""

    def __init__(self, **config):
        super().__init__()
        cfg = dict(DEFAULTS)
        unknown = set(config) - set(DEFAULTS)
        if unknown:
            raise TypeError(f"CaduceusForMaskedLM: unknown config keys {sorted(unknown)}")
        cfg.update(config)
        if cfg["rcps"] and cfg["complement_map"] is None:
            raise ValueError("Complement map must be provided for RCPS.")   # :331
        if cfg["vocab_size"] % cfg["pad_vocab_size_multiple"]:
            cfg["vocab_size"] += cfg["pad_vocab_size_multiple"] - cfg["vocab_size"] % cfg["pad_vocab_size_multiple"]
        if cfg["complement_map"] is not None:   # :336-338 -- padded ids complement to themselves
            cm = cfg["complement_map"]
            cm = dict(cm) if isinstance(cm, dict) else dict(enumerate(cm))
            for i in range(len(cm), cfg["vocab_size"]):
                cm[i] = i
            cfg["complement_map"] = cm
        self.config = cfg
        self.caduceus = Caduceus(cfg)
        if cfg["rcps"]:
            self.lm_head = RCPSLMHead(cfg["d_model"], cfg["vocab_size"], cfg["complement_map"])
        else:
            self.lm_head = HipLinear(cfg["d_model"], cfg["vocab_size"], bias=False)
        ic = cfg["initializer_cfg"] or {}
        self.apply(lambda m: _init_weights(m, cfg["n_layer"], **ic))
        emb = self.caduceus.backbone.embeddings.word_embeddings
        if cfg["rcps"]:   # tie_weights :415-420 -- always tied for RCPS
            self.lm_head.set_weight(emb.weight)
        elif cfg["tie_word_embeddings"]:
            self.lm_head.weight = emb.weight

    def forward(self, input_ids, labels=None, loss_weights=None):
        logits = self.lm_head(self.caduceus(input_ids)).float()
        loss = None
        if labels is not None:
            if loss_weights is not None:
                loss = weighted_cross_entropy(logits, labels, loss_weights,
                                              ignore_index=self.config["pad_token_id"])
            elif os.environ.get("DNA_CE_SUM_COUNT", "1") == "0":  # torch's fused mean (A/B)
                loss = F.cross_entropy(logits.view(-1, logits.shape[-1]), labels.view(-1),
                                       ignore_index=self.config["pad_token_id"])
            else:
                # F.cross_entropy(..., ignore_index) with its mean over the non-ignored tokens,
                # spelled as per-token losses summed and divided by their count: torch's fused
                # mean reduction runs as one workgroup (121 + 57 us per step at L = 131,072)
                y = labels.view(-1)
                ig = self.config["pad_token_id"]
                ce = F.cross_entropy(logits.view(-1, logits.shape[-1]), y, ignore_index=ig,
                                     reduction="none")
                loss = ce.sum() / (y != ig).sum()
        return loss, logits
