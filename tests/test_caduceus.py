"""CPU: Caduceus MLM (rcps=False) structure -- reference parameter names, tied head, vocab
padding, unsupported options raise. GPU parity vs the float64 oracle: tests/test_gpu_caduceus.py."""
import pytest
import torch


def test_caduceus_structure():
    from dna_amd.caduceus import CaduceusForMaskedLM
    m = CaduceusForMaskedLM(d_model=64, n_layer=2, vocab_size=12, ssm_cfg={"d_state": 8})
    assert m.lm_head.weight is m.caduceus.backbone.embeddings.word_embeddings.weight
    assert m.lm_head.weight.shape == (16, 64)                 # padded to a multiple of 8
    keys = set(m.state_dict())
    for k in ("caduceus.backbone.embeddings.word_embeddings.weight",
              "caduceus.backbone.layers.1.mixer.mamba_fwd.A_log",
              "caduceus.backbone.layers.1.mixer.mamba_rev.conv1d.weight",
              "caduceus.backbone.layers.0.norm.weight", "caduceus.backbone.norm_f.weight",
              "lm_head.weight"):
        assert k in keys, k
    m2 = m.caduceus.backbone.layers[0].mixer
    assert m2.mamba_rev.in_proj.weight is m2.mamba_fwd.in_proj.weight
    with pytest.raises(NotImplementedError):
        CaduceusForMaskedLM(d_model=64, n_layer=1, vocab_size=12, rcps=True)
    with pytest.raises(TypeError):
        CaduceusForMaskedLM(d_model=64, n_layer=1, vocab_size=12, not_a_key=1)
    with pytest.raises(RuntimeError):  # no CPU fallback
        m(torch.zeros(1, 8, dtype=torch.long))
