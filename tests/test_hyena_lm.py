"""CPU: HyenaDNA LM ("blm") structure -- the reference config builds (7M BPE experiment
shape), flash_attn-style parameter names, tied head, vocab padding. GPU parity vs the float64
backbone oracle is in tests/test_gpu_hyena_lm.py."""
import pytest
import torch

LAYER = {"_name_": "hyena", "emb_dim": 5, "filter_order": 64, "short_filter_order": 3,
         "l_max": 1024, "modulate": True, "w": 10, "lr": 6e-4, "wd": 0.0, "lr_pos_emb": 0.0,
         "bidirectional": True}


def test_reference_7m_config_builds():
    """configs/experiment/hyena-dna/hyena_hg38_pretrain_7M_bpe.yaml model block."""
    from dna_amd.hyena_lm import BertLMHeadModel
    m = BertLMHeadModel(d_model=256, n_layer=8, d_inner=1024, vocab_size=4096, resid_dropout=0.0,
                        embed_dropout=0.1, residual_in_fp32=True, pad_vocab_size_multiple=8,
                        layer=dict(LAYER))
    assert m.lm_head.weight is m.backbone.embeddings.word_embeddings.weight
    n = sum(p.numel() for p in m.parameters())
    assert 7.0e6 < n < 8.0e6
    keys = set(m.state_dict())
    for k in ("backbone.embeddings.word_embeddings.weight", "backbone.layers.7.norm1.weight",
              "backbone.layers.0.mixer.filter_fn.implicit_filter.6.weight",
              "backbone.layers.3.mlp.fc2.bias", "backbone.ln_f.bias", "lm_head.weight"):
        assert k in keys, k
    assert m.backbone.layers[0].dropout1.p == 0.1 and m.backbone.layers[1].dropout1.p == 0.0


def test_vocab_padding_and_unsupported():
    from dna_amd.hyena_lm import BertLMHeadModel, LMBackbone
    m = BertLMHeadModel(d_model=64, n_layer=1, d_inner=128, vocab_size=12, pad_vocab_size_multiple=8,
                        layer=dict(LAYER, l_max=256))
    assert m.lm_head.weight.shape == (16, 64)
    with pytest.raises(NotImplementedError):
        LMBackbone(64, 1, 128, 16, layer=dict(LAYER), attn_layer_idx=[0])
    with pytest.raises(NotImplementedError):
        LMBackbone(64, 1, 128, 16, layer=dict(LAYER, _name_="h3"))
