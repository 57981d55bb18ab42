"""DNABERT-2 (MosaicBERT) masked-LM model on dna_amd HIP kernels.

Drop-in for the reference's registry.model["dnabert2"] =
src.models.DNABERT2.bert_layers.BertForMaskedLM (src/utils/registry.py:39):
  * same constructor (`cls(config=<dict-like model.config>)`, bert_layers.py:693-716),
  * same module tree and state_dict keys (tied decoder weight),
  * same forward protocol (`forward(batch, state=None)` with batch = (masked_ids, mask, labels)
    -> (MaskedLMOutput(loss, logits=(scores [b,S,V] zero at labels<=0 rows, mask)), None),
    bert_layers.py:756-843), including the last-layer subset computation (:469-488), the
    zero logit rows for masked [UNK] tokens, and the -10000 key-pad bias.
Differences by design (documented in DESIGN.md): the pad mask comes from `ids != pad_token`
without reloading the tokenizer each forward (reference :786-787); the batch stays in padded
layout (no unpad/pad round trips) because pad keys are excluded inside the attention kernel.

Compute precision: "bf16" (default; MFMA bf16 kernels, fp32 master weights / LayerNorm /
residual stream, like PL `precision: bf16` autocast) or "fp32" (exact-fp32 kernels; the 1e-3
logit-parity mode).
"""
import math
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn

from . import functional as DF
from .config import BertConfig, alibi_slopes

try:  # the reference returns transformers' MaskedLMOutput (bert_layers.py:838-843)
    from transformers.modeling_outputs import MaskedLMOutput
except Exception:  # pragma: no cover - transformers is part of the image; keep a twin anyway
    @dataclass
    class MaskedLMOutput:
        loss: Optional[torch.Tensor] = None
        logits: Optional[object] = None
        hidden_states: Optional[object] = None
        attentions: Optional[object] = None

        def __getitem__(self, i):
            return (self.loss, self.logits)[i]

PAD_TOKEN_ID = 3  # DNABERT-2 tokenizer [PAD] (tokenizer.json added_tokens)


class BertEmbeddings(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.word_embeddings = nn.Embedding(config.vocab_size, config.hidden_size,
                                            padding_idx=config.pad_token_id)
        self.token_type_embeddings = nn.Embedding(config.type_vocab_size, config.hidden_size)
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)


class BertUnpadSelfAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        if config.hidden_size % config.num_attention_heads != 0:
            raise ValueError(f"The hidden size ({config.hidden_size}) is not a multiple of the "
                             f"number of attention heads ({config.num_attention_heads})")
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = config.hidden_size // config.num_attention_heads
        self.p_dropout = config.attention_probs_dropout_prob
        self.Wqkv = nn.Linear(config.hidden_size, 3 * config.hidden_size)


class BertSelfOutput(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)


class BertUnpadAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.self = BertUnpadSelfAttention(config)
        self.output = BertSelfOutput(config)


class BertGatedLinearUnitMLP(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.gated_layers = nn.Linear(config.hidden_size, config.intermediate_size * 2, bias=False)
        self.wo = nn.Linear(config.intermediate_size, config.hidden_size)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.layernorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)


class BertLayer(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.attention = BertUnpadAttention(config)
        self.mlp = BertGatedLinearUnitMLP(config)


class BertEncoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.layer = nn.ModuleList([BertLayer(config) for _ in range(config.num_hidden_layers)])
        self.num_attention_heads = config.num_attention_heads
        # ALiBi slopes (bert_layers.py:378-396); the [H,S,S] bias itself is never materialised
        self.register_buffer("alibi_slopes",
                             torch.tensor(alibi_slopes(config.num_attention_heads),
                                          dtype=torch.float32), persistent=False)


class BertModel(nn.Module):
    def __init__(self, config, add_pooling_layer=False):
        super().__init__()
        if add_pooling_layer:
            raise NotImplementedError("pooler is outside the MLM hot path")
        self.config = config
        self.embeddings = BertEmbeddings(config)
        self.encoder = BertEncoder(config)


class BertPredictionHeadTransform(nn.Module):
    def __init__(self, config):
        super().__init__()
        if config.hidden_act not in ("gelu", "gelu_python"):
            raise NotImplementedError(f"head activation {config.hidden_act!r} (gelu only)")
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)
        self.LayerNorm = nn.LayerNorm(config.hidden_size, eps=1e-12)


class BertLMPredictionHead(nn.Module):
    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.transform = BertPredictionHeadTransform(config)
        self.decoder = nn.Linear(bert_model_embedding_weights.size(1),
                                 bert_model_embedding_weights.size(0))
        self.decoder.weight = bert_model_embedding_weights


class BertOnlyMLMHead(nn.Module):
    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.predictions = BertLMPredictionHead(config, bert_model_embedding_weights)


@dataclass
class MLMIndex:
    """Row bookkeeping of one batch, computable on the host before the batch reaches the GPU.

    subset_idx   rows (flattened b*S) entering the last layer's output/MLP: (masked | col 0) & valid
    head_idx     positions inside the subset rows that are masked (labels > 0)   (:626-630)
    target       labels of those rows; flat_masked: their flattened positions
    """
    subset_idx: torch.Tensor
    head_idx: torch.Tensor
    target: torch.Tensor
    flat_masked: torch.Tensor

    @staticmethod
    def build(input_ids, labels, pad_token_id=PAD_TOKEN_ID):
        valid = input_ids != pad_token_id
        masked = labels > 0
        subset = masked.clone()
        subset[:, 0] = True
        subset &= valid
        flat_subset = subset.reshape(-1)
        subset_idx = torch.nonzero(flat_subset).flatten()
        head_idx = torch.nonzero(masked.reshape(-1)[flat_subset]).flatten()
        flat_masked = torch.nonzero(masked.reshape(-1)).flatten()
        target = labels.reshape(-1)[flat_masked]
        return MLMIndex(subset_idx, head_idx, target, flat_masked)

    def to(self, device, non_blocking=False):
        return MLMIndex(*(t.to(device, non_blocking=non_blocking) for t in
                          (self.subset_idx, self.head_idx, self.target, self.flat_masked)))


class BertForMaskedLM(nn.Module):
    """Registry "dnabert2" model (reference bert_layers.py:691-850)."""

    def __init__(self, config, precision: str = "bf16", **kwargs):
        super().__init__()
        config = BertConfig.from_any(config)
        if config.is_decoder:
            raise ValueError("BertForMaskedLM needs config.is_decoder=False")
        self.config = config
        self.bert = BertModel(config, add_pooling_layer=False)
        self.cls = BertOnlyMLMHead(config, self.bert.embeddings.word_embeddings.weight)
        self.hyena_framework = config.hyena_framework
        self.precision = precision
        self.dropout_rng = DF.DropoutRNG()
        self._lp_provider = None  # set by dna_amd.flat.FlatParams for a persistent bf16 copy
        self._lpt_provider = None  # ... and for the transposed bf16 projection weights
        self._init_weights()
        # projection weights: keep a W^T copy for the data gradient dx = dy . W^T^T, where the
        # MFMA kernel wants the reduction (out features) % 64 and the output (in features) % 8,
        # as dna_transpose_bf16 does; other shapes keep the library dgrad
        for m in self.modules():
            if isinstance(m, nn.Linear) and m.out_features % 64 == 0 and m.in_features % 8 == 0:
                m.weight._dna_transpose = True

    # -- reference-compatible utilities ------------------------------------------------------
    def _init_weights(self):
        """BertPreTrainedModel._init_weights semantics: N(0, initializer_range) for Linear and
        Embedding weights, zero biases, LayerNorm (1, 0), zero padding_idx row."""
        std = self.config.initializer_range
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, mean=0.0, std=std)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Embedding):
                nn.init.normal_(m.weight, mean=0.0, std=std)
                if m.padding_idx is not None:
                    with torch.no_grad():
                        m.weight[m.padding_idx].zero_()
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def get_output_embeddings(self):
        return self.cls.predictions.decoder

    def set_precision(self, precision: str):
        assert precision in ("bf16", "fp32")
        self.precision = precision
        return self

    @property
    def compute_dtype(self):
        return torch.bfloat16 if self.precision == "bf16" else torch.float32

    def _lp(self, p: torch.Tensor) -> torch.Tensor:
        """Compute-dtype view of master weight `p` (persistent shadow if a FlatParams owns it)."""
        if self.precision == "fp32":
            return p
        if self._lp_provider is not None:
            return self._lp_provider(p)
        return p.detach().to(torch.bfloat16)

    def _lp_t(self, p: torch.Tensor):
        """Transposed bf16 copy of projection weight `p` (None: the data gradient falls back)."""
        if self.precision == "fp32" or self._lpt_provider is None:
            return None
        return self._lpt_provider(p)

    def _linear(self, x, w, b=None, geglu=None):
        return DF.linear(x, w, self._lp(w), b, w_lpt=self._lp_t(w), geglu=geglu)

    # -- the hot path ------------------------------------------------------------------------
    def mlm_logits(self, input_ids: torch.Tensor, index: MLMIndex) -> torch.Tensor:
        """Compact logits [M, V] of the masked rows (row-major over (b, s)), compute dtype."""
        cfg = self.config
        b, S = input_ids.shape
        T = b * S
        H = cfg.num_attention_heads
        bf16 = self.precision == "bf16"
        train = self.training
        rng = self.dropout_rng
        p_hidden = cfg.hidden_dropout_prob if train else 0.0
        if cfg.attention_probs_dropout_prob and train:
            raise NotImplementedError("attention-probability dropout (reference default 0.0)")
        eps = cfg.layer_norm_eps
        ids = input_ids.reshape(-1)
        key_valid = (ids != cfg.pad_token_id_mask).to(torch.uint8)

        emb = self.bert.embeddings
        seed, off = rng.take(T * cfg.hidden_size) if p_hidden else (0, 0)
        x32, xb = DF.EmbeddingLN.apply(ids, emb.word_embeddings.weight,
                                       emb.token_type_embeddings.weight, emb.LayerNorm.weight,
                                       emb.LayerNorm.bias, eps, p_hidden, seed, off, True, bf16)
        xin = xb if bf16 else x32
        slopes = self.bert.encoder.alibi_slopes
        L = len(self.bert.encoder.layer)
        for i, layer in enumerate(self.bert.encoder.layer):
            att = layer.attention
            qkv = self._linear(xin, att.self.Wqkv.weight, att.self.Wqkv.bias)
            ctx = DF.alibi_attention(qkv, key_valid, slopes, b, S, H,
                                     bias_grad=att.self.Wqkv.bias is not None)
            res = x32
            if i == L - 1:  # last layer: output + MLP only on the subset rows (:480-488)
                ctx = ctx.index_select(0, index.subset_idx)
                res = x32.index_select(0, index.subset_idx)
            n = ctx.shape[0]
            out = att.output
            h = self._linear(ctx, out.dense.weight)
            seed, off = rng.take(n * cfg.hidden_size) if p_hidden else (0, 0)
            y32, yb = DF.FusedLayerNorm.apply(h, out.dense.bias, res, out.LayerNorm.weight,
                                              out.LayerNorm.bias, eps, 0, p_hidden, seed, off,
                                              True, bf16)
            mlp = layer.mlp
            seed, off = rng.take(n * cfg.intermediate_size) if p_hidden else (0, 0)
            # the GeGLU forward runs in the gated_layers GEMM's epilogue where the kernel allows
            g = self._linear(yb if bf16 else y32, mlp.gated_layers.weight,
                             geglu=(p_hidden, seed, off))
            wo_lp, wo_lpt = self._lp(mlp.wo.weight), self._lp_t(mlp.wo.weight)
            if DF.geglu_out_fused_ok(g, wo_lp, wo_lpt):
                # GeGLU + wo as one node: backward = wo's data gradient with the GeGLU backward
                # in its epilogue (da never in memory), then wo's weight gradient
                o = DF.geglu_out(g, p_hidden, seed, off, mlp.wo.weight, wo_lp, wo_lpt)
            else:
                a = DF.GeGLU.apply(g, p_hidden, seed, off)
                o = DF.linear(a, mlp.wo.weight, wo_lp, None, w_lpt=wo_lpt)
            x32, xb = DF.FusedLayerNorm.apply(o, mlp.wo.bias, y32, mlp.layernorm.weight,
                                              mlp.layernorm.bias, eps, 0, 0.0, 0, 0, True, bf16)
            xin = xb if bf16 else x32
        if L == 0:
            xin = xin.index_select(0, index.subset_idx)
        seq = xin.index_select(0, index.head_idx)
        tr = self.cls.predictions.transform
        t = self._linear(seq, tr.dense.weight)
        t32, tb = DF.FusedLayerNorm.apply(t, tr.dense.bias, None, tr.LayerNorm.weight,
                                          tr.LayerNorm.bias, 1e-12, 1, 0.0, 0, 0, not bf16, bf16)
        dec = self.cls.predictions.decoder
        return self._linear(tb if bf16 else t32, dec.weight, dec.bias)

    def mlm_loss(self, input_ids, mask, index: MLMIndex, n_mask: Optional[int] = None,
                 n_unk_masked: Optional[int] = None):
        """Task loss bert_cross_entropy (src/tasks/metrics.py:268-273) without dense logits:
        masked rows with label 0 ([UNK]) have all-zero logits in the reference (no gradient,
        loss ln V each); they are added as a constant."""
        logits = self.mlm_logits(input_ids, index)
        if n_mask is None:
            n_mask = int(mask.sum())
        if n_unk_masked is None:
            n_unk_masked = n_mask - int(index.target.numel())
        loss = DF.MaskedCrossEntropy.apply(logits, index.target, max(n_mask, 1))
        if n_unk_masked:
            loss = loss + n_unk_masked * math.log(self.config.vocab_size) / max(n_mask, 1)
        return loss, logits

    # -- reference forward protocol ----------------------------------------------------------
    def forward(self, batch=None, input_ids=None, attention_mask=None, token_type_ids=None,
                position_ids=None, head_mask=None, inputs_embeds=None, encoder_hidden_states=None,
                encoder_attention_mask=None, labels=None, output_attentions=None,
                output_hidden_states=None, return_dict=None, state=None, mlm_index=None, **kwargs):
        if self.hyena_framework:
            input_ids, labels = batch[0], batch[2]
        if input_ids is None:
            raise ValueError("Must specify input_ids (inputs_embeds is not supported)")
        if token_type_ids is not None and bool((token_type_ids != 0).any()):
            raise NotImplementedError("token_type_ids other than 0 (the MLM path never sets them)")
        if attention_mask is not None and not self.hyena_framework:
            if not torch.equal(attention_mask.bool(), input_ids != self.config.pad_token_id_mask):
                raise NotImplementedError("attention_mask must equal input_ids != [PAD]")
        if labels is None:
            raise NotImplementedError("forward without labels (encoder-only inference)")
        b, S = input_ids.shape
        index = mlm_index if mlm_index is not None else \
            MLMIndex.build(input_ids, labels, self.config.pad_token_id_mask)
        logits = self.mlm_logits(input_ids, index)
        # internal loss over labels > 0 rows (bert_layers.py:818-824)
        loss = DF.MaskedCrossEntropy.apply(logits, index.target, max(index.target.numel(), 1))
        V = logits.shape[-1]
        scores = torch.zeros(b * S, V, device=logits.device, dtype=logits.dtype)
        scores = scores.index_put((index.flat_masked,), logits).view(b, S, V)  # :828-831
        if self.hyena_framework:
            return MaskedLMOutput(loss=loss, logits=(scores, batch[1]), hidden_states=None,
                                  attentions=None), None
        return MaskedLMOutput(loss=loss, logits=scores, hidden_states=None, attentions=None)
