"""CPU fp32 restatement of the DNABERT-2 (MosaicBERT) masked-LM forward (TEST INFRASTRUCTURE).

Oracle only: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never
by the dna_amd product path. Parity pinned by tests/golden/model_{tiny,cfgA,117m}.npz, which
tests/golden/make_golden.py produced by running the reference itself.

Functional, state_dict-driven (keys of SURVEY Appendix A), autograd-capable. Follows
/root/reference/src/models/DNABERT2/bert_layers.py:
  embeddings            :62-107   LN(E_w[ids] + E_tt[0]) (+dropout)
  alibi slopes          :378-396  ; alibi[h,i,j] = -slope_h*|i-j|  :398-406
  encoder bias          :421-448  (1-mask)*-10000 + alibi, fp32
  self-attention        :160-196  softmax(q k^T / sqrt(dh) + bias) v  (PyTorch path, :167-178)
  BertSelfOutput        :209-214  LN(dropout(dense(x)) + input)
  GeGLU MLP             :283-301  LN(wo(dropout(gelu(h[:, :F]) * h[:, F:])) + x)
  last-layer subset     :469-488  masked | first-column rows after attention
  head                  :513-528,650-664  LN_1e-12(gelu(dense(x))) E_w^T + b
  BertForMaskedLM       :784-843  masked_tokens_mask = labels > 0; internal CE; zeros elsewhere
and the task loss `bert_cross_entropy` (src/tasks/metrics.py:268-273).
Padded layout is kept (no unpad): pad rows never influence non-pad rows (their keys carry a
-10000 bias, exp underflows to exactly 0 in fp32), so non-pad outputs equal the reference's.
"""
import math

import torch
import torch.nn.functional as F

PAD_ID = 3


def alibi_slopes(n_heads: int):
    """bert_layers.py:378-396 (power-of-two recipe + interleaved extension)."""
    def pow2(n):
        start = 2 ** (-2 ** -(math.log2(n) - 3))
        return [start * start ** i for i in range(n)]

    if math.log2(n_heads).is_integer():
        return pow2(n_heads)
    c = 2 ** math.floor(math.log2(n_heads))
    return pow2(c) + alibi_slopes(2 * c)[0::2][: n_heads - c]


def attention_bias(attn_mask: torch.Tensor, n_heads: int) -> torch.Tensor:
    """[b, H, S, S] fp32: (1 - keymask) * -10000 + alibi (bert_layers.py:421-448)."""
    b, S = attn_mask.shape
    pos = torch.arange(S)
    rel = (pos[None, :] - pos[:, None]).abs().to(torch.float32)
    slopes = torch.tensor(alibi_slopes(n_heads), dtype=torch.float32)
    alibi = slopes[:, None, None] * -rel[None]
    ext = (1.0 - attn_mask.to(torch.float32))[:, None, None, :] * -10000.0
    return ext + alibi[None]


def layer_norm(x, w, b, eps):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def self_attention(x, sd, pre, n_heads, bias):
    """x [b, S, d] -> context [b, S, d] (bert_layers.py:160-196)."""
    b, S, d = x.shape
    dh = d // n_heads
    qkv = F.linear(x, sd[pre + "Wqkv.weight"], sd[pre + "Wqkv.bias"])
    qkv = qkv.view(b, S, 3, n_heads, dh)
    q = qkv[:, :, 0].permute(0, 2, 1, 3)
    k = qkv[:, :, 1].permute(0, 2, 3, 1)
    v = qkv[:, :, 2].permute(0, 2, 1, 3)
    scores = torch.matmul(q, k) / math.sqrt(dh) + bias
    probs = torch.softmax(scores, dim=-1)
    return torch.matmul(probs, v).permute(0, 2, 1, 3).reshape(b, S, d)


def dnabert2_forward(sd, cfg, masked_ids, labels, dropout=None):
    """Returns (compact_logits [M, V] for rows labels>0 in row-major (b, s) order,
    internal_loss, dense_logits [b, S, V]).

    cfg: dict(num_hidden_layers, num_attention_heads, intermediate_size, layer_norm_eps).
    dropout: optional callable(tensor, site_name) applied where the reference has nn.Dropout.
    """
    drop = dropout or (lambda t, site: t)
    eps = cfg.get("layer_norm_eps", 1e-12)
    H = cfg["num_attention_heads"]
    Fdim = cfg["intermediate_size"]
    L = cfg["num_hidden_layers"]
    b, S = masked_ids.shape
    attn_mask = masked_ids != PAD_ID                       # bert_layers.py:787
    masked_tokens = labels > 0                             # :795
    subset = masked_tokens.clone()                         # :611-613
    subset[:, 0] = True
    subset &= attn_mask                                    # subset_mask[attention_mask_bool] :480

    E = sd["bert.embeddings.word_embeddings.weight"]
    # nn.Embedding(padding_idx=pad_token_id=0) (bert_layers.py:45-47): row 0 gets no lookup grad
    x = F.embedding(masked_ids, E, padding_idx=0) + sd["bert.embeddings.token_type_embeddings.weight"][0]
    x = layer_norm(x, sd["bert.embeddings.LayerNorm.weight"],
                   sd["bert.embeddings.LayerNorm.bias"], eps)
    x = drop(x, "emb")
    bias = attention_bias(attn_mask, H)
    for i in range(L):
        p = f"bert.encoder.layer.{i}."
        ctx = self_attention(x, sd, p + "attention.self.", H, bias)
        res = x
        if i == L - 1:
            # last layer: only subset rows go through output/MLP (:480-488, :249-251)
            ctx = ctx[subset]
            res = x[subset]
        h = F.linear(ctx, sd[p + "attention.output.dense.weight"],
                     sd[p + "attention.output.dense.bias"])
        h = drop(h, f"l{i}.attn")
        y = layer_norm(h + res, sd[p + "attention.output.LayerNorm.weight"],
                       sd[p + "attention.output.LayerNorm.bias"], eps)
        g = F.linear(y, sd[p + "mlp.gated_layers.weight"])
        a = F.gelu(g[..., :Fdim]) * g[..., Fdim:]
        a = drop(a, f"l{i}.mlp")
        o = F.linear(a, sd[p + "mlp.wo.weight"], sd[p + "mlp.wo.bias"])
        x = layer_norm(o + y, sd[p + "mlp.layernorm.weight"], sd[p + "mlp.layernorm.bias"], eps)
    # x: [n_subset, d] rows in (b, s) order; keep those that are masked (:626-630)
    seq_out = x[masked_tokens[subset]] if L > 0 else x[masked_tokens]
    t = F.linear(seq_out, sd["cls.predictions.transform.dense.weight"],
                 sd["cls.predictions.transform.dense.bias"])
    t = F.gelu(t)
    t = layer_norm(t, sd["cls.predictions.transform.LayerNorm.weight"],
                   sd["cls.predictions.transform.LayerNorm.bias"], 1e-12)
    logits = F.linear(t, E, sd["cls.predictions.decoder.bias"])
    flat_labels = labels.reshape(-1)
    internal = F.cross_entropy(logits, flat_labels[flat_labels > 0])   # :820-824
    dense = torch.zeros(b * S, E.shape[0], dtype=logits.dtype)
    dense = dense.index_put((torch.nonzero(flat_labels > 0).flatten(),), logits)  # :828-831
    return logits, internal, dense.view(b, S, -1)


def bert_cross_entropy(dense_logits, mask, target):
    """src/tasks/metrics.py:268-273 on flattened (b*S, V) logits and the bert_mask `mask`."""
    logits = dense_logits.reshape(-1, dense_logits.shape[-1])
    m = mask.reshape(-1)
    return F.cross_entropy(logits[m], target.reshape(-1)[m])


def state_dict_shapes(cfg):
    """(name, shape) for every parameter tensor (tied decoder excluded)."""
    V, d = cfg["vocab_size"], cfg["hidden_size"]
    Fdim = cfg["intermediate_size"]
    out = [("bert.embeddings.word_embeddings.weight", (V, d)),
           ("bert.embeddings.token_type_embeddings.weight", (cfg.get("type_vocab_size", 2), d)),
           ("bert.embeddings.LayerNorm.weight", (d,)), ("bert.embeddings.LayerNorm.bias", (d,))]
    for i in range(cfg["num_hidden_layers"]):
        p = f"bert.encoder.layer.{i}."
        out += [(p + "attention.self.Wqkv.weight", (3 * d, d)), (p + "attention.self.Wqkv.bias", (3 * d,)),
                (p + "attention.output.dense.weight", (d, d)), (p + "attention.output.dense.bias", (d,)),
                (p + "attention.output.LayerNorm.weight", (d,)), (p + "attention.output.LayerNorm.bias", (d,)),
                (p + "mlp.gated_layers.weight", (2 * Fdim, d)),
                (p + "mlp.wo.weight", (d, Fdim)), (p + "mlp.wo.bias", (d,)),
                (p + "mlp.layernorm.weight", (d,)), (p + "mlp.layernorm.bias", (d,))]
    out += [("cls.predictions.transform.dense.weight", (d, d)),
            ("cls.predictions.transform.dense.bias", (d,)),
            ("cls.predictions.transform.LayerNorm.weight", (d,)),
            ("cls.predictions.transform.LayerNorm.bias", (d,)),
            ("cls.predictions.decoder.bias", (V,))]
    return out
