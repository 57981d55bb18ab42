"""Model configuration for the DNABERT-2 MLM path.

Mirrors what the reference builds in BertForMaskedLM.__init__ (bert_layers.py:693-701:
OmegaConf.to_container(config) -> transformers.BertConfig.from_dict) plus MosaicBERT's
additions (configuration_bert.py:9-25), with the same defaults for the keys the hot path reads.
"""
import math
from dataclasses import dataclass, fields


def alibi_slopes(n_heads: int):
    """ALiBi head slopes (bert_layers.py:378-396): geometric for powers of two, interleaved
    extension otherwise (12 heads -> 2^-1..2^-8 then 2^-0.5, 2^-1.5, 2^-2.5, 2^-3.5)."""
    def pow2(n):
        start = 2 ** (-2 ** -(math.log2(n) - 3))
        return [start * start ** i for i in range(n)]

    if math.log2(n_heads).is_integer():
        return pow2(n_heads)
    c = 2 ** math.floor(math.log2(n_heads))
    return pow2(c) + alibi_slopes(2 * c)[0::2][: n_heads - c]


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = "gelu"
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.0  # MosaicBERT default (configuration_bert.py:12)
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0          # embedding padding_idx (the [UNK] row for DNABERT-2)
    alibi_starting_size: int = 512
    is_decoder: bool = False
    hyena_framework: bool = False
    # the attention mask is `input_ids != tokenizer.pad_token_id` (bert_layers.py:786-787);
    # DNABERT-2's tokenizer [PAD] is 3 -- kept separate from the embedding padding_idx above.
    pad_token_id_mask: int = 3

    @classmethod
    def from_any(cls, cfg):
        if isinstance(cfg, cls):
            return cfg
        if hasattr(cfg, "items"):
            d = dict(cfg.items())
        else:
            d = {k: getattr(cfg, k) for k in dir(cfg) if not k.startswith("_")}
        names = {f.name for f in fields(cls)}
        kw = {k: v for k, v in d.items() if k in names and v is not None}
        out = cls(**kw)
        out.extra = {k: v for k, v in d.items() if k not in names}
        return out
