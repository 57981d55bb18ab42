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


def test_caduceus_oracle_c_scan_equals_python_scan():
    """The config-E-length oracle (C scan inside the float64 Caduceus restatement) == the Python
    scan oracle on a short sequence: logits and every parameter gradient."""
    from dna_amd.caduceus import CaduceusForMaskedLM
    from oracle import caduceus_ref as CR
    from oracle.selective_scan_c import selective_scan_c
    torch.manual_seed(7)
    m = CaduceusForMaskedLM(d_model=16, n_layer=2, vocab_size=12, ssm_cfg={"d_state": 8})
    ids = torch.randint(0, 12, (2, 90), generator=torch.Generator().manual_seed(3))
    dt_rank = m.caduceus.backbone.layers[0].mixer.mamba_fwd.dt_rank
    outs = []
    for scan in (None, selective_scan_c):
        sd = {k: v.detach().double().clone().requires_grad_(True) for k, v in m.state_dict().items()}
        sd["lm_head.weight"] = sd["caduceus.backbone.embeddings.word_embeddings.weight"]
        for i in range(2):
            p = f"caduceus.backbone.layers.{i}.mixer."
            for k in ("in_proj.weight", "out_proj.weight"):
                sd[p + "mamba_rev." + k] = sd[p + "mamba_fwd." + k]
        out = CR.mlm_logits(sd, ids, 2, 8, 4, dt_rank, scan=scan)
        out.backward(torch.ones_like(out))
        outs.append((out.detach(), {k: v.grad for k, v in sd.items() if v.grad is not None}))
    (a, ga), (b, gb) = outs
    assert torch.allclose(a, b, rtol=1e-10, atol=1e-12)
    assert ga.keys() == gb.keys() and len(ga) > 10
    for k in ga:
        assert torch.allclose(ga[k], gb[k], rtol=1e-9, atol=1e-12), k
