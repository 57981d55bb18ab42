"""HyenaDNA language model around the HIP Hyena operator (BASELINE config D).

Mirrors the reference's `LMBackbone` / `BertLMHeadModel` (registry model "blm",
src/models/sequence/long_conv_lm.py:320-682) as configs/experiment/hyena-dna/*.yaml build it:
token embeddings (GPT2Embeddings, no positions), `n_layer` pre-norm blocks of
[dropout -> add -> LayerNorm -> HyenaOperator] and [dropout -> add -> LayerNorm -> Mlp(fc1, GELU
tanh, fc2)], a final dropout -> add -> LayerNorm, and an LM head tied to the embedding table.
The Block / Mlp / GPT2Embeddings modules come from flash_attn in the reference (not installed
here), so their forward is restated from flash_attn's published code (prenorm Block with
residual_in_fp32) with the same parameter names -- parity of the backbone is unpinned; the
Hyena operator inside is pinned (oracle/hyena_operator_ref.py). The long convolution and the
operator's data movement and the LayerNorms run on HIP kernels; embeddings, MLP and head are
torch ops.
"""
import os
from collections import namedtuple
from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as DF
from .functional import HipEmbedding
from .hyena import HipLinear, HyenaOperator, hip_linear


CausalLMOutput = namedtuple("CausalLMOutput", ["logits"])


class GPT2Embeddings(nn.Module):
    """flash_attn.modules.embedding.GPT2Embeddings: word (+ optional learned position)."""

    def __init__(self, embed_dim, vocab_size, max_position_embeddings, padding_idx=None,
                 device=None, dtype=None):
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.word_embeddings = HipEmbedding(vocab_size, embed_dim, padding_idx=padding_idx, **fk)
        self.max_position_embeddings = max_position_embeddings
        if max_position_embeddings > 0:
            self.position_embeddings = nn.Embedding(max_position_embeddings, embed_dim, **fk)

    def forward(self, input_ids, position_ids=None):
        h = self.word_embeddings(input_ids)
        if self.max_position_embeddings > 0:
            if position_ids is None:
                position_ids = torch.arange(input_ids.shape[1], device=input_ids.device)
            h = h + self.position_embeddings(position_ids)
        return h


_LN_COLS = {64, 128, 192, 256, 512, 768, 1024}  # widths dna_ln_fwd/bwd are instantiated for
_TORCH_LN = os.environ.get("DNA_HYENA_TORCH_LN", "0") == "1"  # A/B switch: torch's LayerNorm
# A/B switch: the Mlp's act + fc2 as separate torch GELU + HipLinear nodes
_TORCH_LINEAR_MLP = (os.environ.get("DNA_HYENA_TORCH_LINEAR", "0") == "1"
                     or os.environ.get("DNA_GELU_BWD_FUSED", "1") == "0")


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (the Block's norm1 / norm2 and LMBackbone.ln_f; same parameters and
    state_dict) on the HIP kernels `dna_ln_fwd` / `dna_ln_bwd` (fp32 statistics, no bias /
    dropout / residual terms). Under CUDA bf16 autocast the reference's layer_norm runs in fp32
    and the next op (a Linear: in_proj, fc1, lm_head) casts its output to bf16; the kernel writes
    that bf16 rounding directly, so one cast pass and the fp32 activation disappear. Widths the
    kernels are not built for stay on torch's GPU LayerNorm; CPU tensors raise (no CPU path)."""

    def forward(self, x):
        d = x.shape[-1]
        if _TORCH_LN or not (self.elementwise_affine and self.bias is not None and d in _LN_COLS
                and x.dtype in (torch.float32, torch.bfloat16)
                and self.weight.dtype == torch.float32):
            return super().forward(x)
        from . import functional as DF
        bf16_out = (torch.is_autocast_enabled("cuda")
                    and torch.get_autocast_dtype("cuda") == torch.bfloat16)
        y32, yb = DF.FusedLayerNorm.apply(x.reshape(-1, d), None, None, self.weight, self.bias,
                                          self.eps, 0, 0.0, 0, 0, not bf16_out, bf16_out)
        y = yb if bf16_out else y32
        return y.view(*x.shape[:-1], d)

    def add_ok(self, x, residual):
        """Whether add_norm(x, residual) applies: the fused kernel's widths and dtypes, an fp32
        residual stream (then `x + residual` is fp32 in torch too)."""
        return (not _TORCH_LN and x.is_cuda and residual is not None
                and residual.dtype == torch.float32 and x.dtype in (torch.float32, torch.bfloat16)
                and self.elementwise_affine and self.bias is not None
                and x.shape[-1] in _LN_COLS and self.weight.dtype == torch.float32
                and residual.shape == x.shape)

    def add_norm(self, x, residual):
        """(residual + x, self(residual + x)) in one pass (functional.AddLayerNorm): the fp32 sum
        is the new residual stream, the LN output is bf16 under bf16 autocast (as forward)."""
        from . import functional as DF
        d = x.shape[-1]
        bf16_out = (torch.is_autocast_enabled("cuda")
                    and torch.get_autocast_dtype("cuda") == torch.bfloat16)
        s, y = DF.AddLayerNorm.apply(x.reshape(-1, d), residual.reshape(-1, d), self.weight,
                                     self.bias, self.eps, bf16_out)
        return s.view(*x.shape), y.view(*x.shape)


class Mlp(nn.Module):
    """flash_attn.modules.mlp.Mlp: fc2(act(fc1(x)))."""

    def __init__(self, in_features, hidden_features=None, out_features=None,
                 activation=partial(F.gelu, approximate="tanh"), device=None, dtype=None):
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        hidden_features = hidden_features or in_features * 4
        self.fc1 = HipLinear(in_features, hidden_features, **fk)
        self.activation = activation
        self.fc2 = HipLinear(hidden_features, out_features or in_features, **fk)

    def forward(self, x):
        if self._tanh_gelu_bf16() and isinstance(self.fc1, HipLinear):
            # fc1's GEMM also writes gelu(h) (dna_linear_gelu_fwd): no separate GELU pass
            h = hip_linear(x, self.fc1.weight, self.fc1.bias, gelu=True)
        else:
            h = self.fc1(x)
        if self._tanh_gelu_bf16() and DF.gelu_linear_ok(h, self.fc2.weight):
            # act + fc2 as one node: fc2's data gradient carries the GELU backward (GeluLinear)
            return DF.gelu_linear(h, self.fc2.weight, self.fc2.bias, getattr(h, "_dna_gelu", None))
        return self.fc2(self.activation(h))

    def _tanh_gelu_bf16(self):
        act = self.activation
        return (isinstance(act, partial) and act.func is F.gelu and not act.args
                and act.keywords == {"approximate": "tanh"} and isinstance(self.fc2, HipLinear)
                and not _TORCH_LINEAR_MLP and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16)


class Block(nn.Module):
    """flash_attn.modules.block.Block with prenorm=True (the reference's create_block,
    long_conv_lm.py:205-267): returns (hidden_states, residual)."""

    def __init__(self, dim, mixer, mlp, norm_eps=1e-5, resid_dropout1=0.0, resid_dropout2=0.0,
                 residual_in_fp32=False):
        super().__init__()
        self.mixer = mixer
        self.dropout1 = nn.Dropout(resid_dropout1)
        self.norm1 = LayerNorm(dim, eps=norm_eps)
        self.mlp = mlp
        self.dropout2 = nn.Dropout(resid_dropout2)
        self.norm2 = LayerNorm(dim, eps=norm_eps)
        self.residual_in_fp32 = residual_in_fp32

    def forward(self, hidden_states, residual=None):
        # add + norm in one kernel when the residual stream is fp32 and the dropout is a no-op
        # (norm1 / norm2 .add_norm: the same fp32 sum and LN, functional.AddLayerNorm)
        if _no_drop(self.dropout1) and self.norm1.add_ok(hidden_states, residual):
            residual, hidden_states = self.norm1.add_norm(hidden_states, residual)
        else:
            dropped = self.dropout1(hidden_states)
            residual = dropped + residual if residual is not None else dropped
            hidden_states = self.norm1(residual.to(dtype=self.norm1.weight.dtype))
            if self.residual_in_fp32:
                residual = residual.to(torch.float32)
        hidden_states = self.mixer(hidden_states)
        if _no_drop(self.dropout2) and self.norm2.add_ok(hidden_states, residual):
            residual, hidden_states = self.norm2.add_norm(hidden_states, residual)
        else:
            dropped = self.dropout2(hidden_states)
            residual = dropped + residual
            hidden_states = self.norm2(residual.to(dtype=self.norm2.weight.dtype))
            if self.residual_in_fp32:
                residual = residual.to(torch.float32)
        return self.mlp(hidden_states), residual


def _no_drop(m):
    return m.p == 0.0 or not m.training


def _init_weights(module, n_layer, initializer_range=0.02, rescale_prenorm_residual=True):
    """long_conv_lm.py:270-318 (reseeds with 2222 per module, as the reference does)."""
    torch.manual_seed(2222)
    if isinstance(module, nn.Linear):
        nn.init.normal_(module.weight, std=initializer_range)
        if module.bias is not None:
            nn.init.zeros_(module.bias)
    elif isinstance(module, nn.Embedding):
        nn.init.normal_(module.weight, std=initializer_range)
    if rescale_prenorm_residual:
        for name, p in module.named_parameters():
            if name in ["out_proj.weight", "fc2.weight"]:
                nn.init.kaiming_normal_(p)


class LMBackbone(nn.Module):
    """long_conv_lm.py:320-576 (layer = a Hyena operator config; no attention layers)."""

    def __init__(self, d_model, n_layer, d_inner, vocab_size, layer=None, attn_layer_idx=None,
                 attn_cfg=None, max_position_embeddings=0, resid_dropout=0.0, embed_dropout=0.1,
                 layer_norm_epsilon=1e-5, initializer_cfg=None, fused_mlp=False,
                 fused_dropout_add_ln=False, residual_in_fp32=False, checkpoint_mlp=False,
                 checkpoint_mixer=False, device=None, dtype=None, **kwargs):
        super().__init__()
        if attn_layer_idx:
            raise NotImplementedError("LMBackbone: attention layers (flash_attn MHA) are out of scope")
        if fused_mlp or fused_dropout_add_ln:
            raise NotImplementedError("fused_mlp / fused_dropout_add_ln (flash_attn CUDA extensions)")
        layer = dict(layer or {})
        name = layer.pop("_name_", "hyena")
        if name != "hyena":
            raise NotImplementedError(f"LMBackbone layer {name!r} (hyena only)")
        self.residual_in_fp32 = residual_in_fp32
        self.embeddings = GPT2Embeddings(d_model, vocab_size, max_position_embeddings)
        self.layers = nn.ModuleList([
            Block(d_model, HyenaOperator(d_model, layer_idx=i, **layer),
                  Mlp(d_model, hidden_features=d_inner), norm_eps=layer_norm_epsilon,
                  resid_dropout1=embed_dropout if i == 0 else resid_dropout,
                  resid_dropout2=resid_dropout, residual_in_fp32=residual_in_fp32)
            for i in range(n_layer)])
        self.drop_f = nn.Dropout(resid_dropout)
        self.ln_f = LayerNorm(d_model, eps=layer_norm_epsilon)
        self.apply(partial(_init_weights, n_layer=n_layer, **(initializer_cfg or {})))

    def forward(self, input_ids, position_ids=None):
        hidden_states = self.embeddings(input_ids, position_ids=position_ids)
        residual = None
        for layer in self.layers:
            hidden_states, residual = layer(hidden_states, residual)
        if _no_drop(self.drop_f) and self.ln_f.add_ok(hidden_states, residual):
            return self.ln_f.add_norm(hidden_states, residual)[1]
        dropped = self.drop_f(hidden_states)
        residual = dropped + residual if residual is not None else dropped
        return self.ln_f(residual.to(dtype=self.ln_f.weight.dtype))


class BertLMHeadModel(nn.Module):
    """Registry model "blm" (long_conv_lm.py:578-682): backbone + LM head tied to the
    embeddings; forward((input_ids, mask)) -> (CausalLMOutput(logits=(logits, mask)), None)."""

    def __init__(self, d_model, n_layer, d_inner, vocab_size, pad_vocab_size_multiple=1, **kwargs):
        super().__init__()
        if vocab_size % pad_vocab_size_multiple:
            vocab_size += pad_vocab_size_multiple - vocab_size % pad_vocab_size_multiple
        self.backbone = LMBackbone(d_model, n_layer, d_inner, vocab_size, **kwargs)
        self.lm_head = HipLinear(d_model, vocab_size, bias=False)
        self.apply(partial(_init_weights, n_layer=n_layer,
                           **(kwargs.get("initializer_cfg") or {})))
        self.lm_head.weight = self.backbone.embeddings.word_embeddings.weight

    def forward(self, input_ids, position_ids=None, inference_params=None, state=None):
        mask = input_ids[1]
        ids = input_ids[0]
        logits = self.lm_head(self.backbone(ids, position_ids=position_ids))
        return CausalLMOutput(logits=(logits, mask)), None
