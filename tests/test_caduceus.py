"""CPU: Caduceus MLM structure (rcps=False and the RCPS variant) -- reference parameter names,
tied head, vocab padding, unsupported options raise; the RCPS oracle's RC equivariance. GPU parity vs the float64 oracle: tests/test_gpu_caduceus.py."""
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


CM = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6, 7: 10, 8: 9, 9: 8, 10: 7, 11: 11}  # A<->T, C<->G


def _rcps_sd(m):
    """float64 leaves of the model's state_dict with the tied tensors sharing one leaf."""
    sd = {k: (v.detach().double().clone().requires_grad_(True) if v.is_floating_point() else v)
          for k, v in m.state_dict().items()}
    sd["lm_head.lm_head.weight"] = sd["caduceus.backbone.embeddings.word_embeddings.embedding.weight"]
    for i in range(m.config["n_layer"]):
        p = f"caduceus.backbone.layers.{i}.mixer.submodule."
        for k in ("in_proj.weight", "out_proj.weight"):
            sd[p + "mamba_rev." + k] = sd[p + "mamba_fwd." + k]
    return sd


def test_caduceus_rcps_structure():
    """rcps=True: reference parameter / buffer names (modeling_rcps.py), the complement map padded
    with identity ids to the padded vocabulary, head tied to the embedding, config errors."""
    from dna_amd.caduceus import CaduceusForMaskedLM
    for fused in (True, False):
        m = CaduceusForMaskedLM(d_model=16, n_layer=2, vocab_size=12, rcps=True, complement_map=CM,
                                fused_add_norm=fused, ssm_cfg={"d_state": 8})
        emb = m.caduceus.backbone.embeddings.word_embeddings
        assert m.lm_head.weight is emb.weight and emb.weight.shape == (16, 16)
        assert emb.complement_map.tolist() == [CM[i] for i in range(12)] + [12, 13, 14, 15]
        assert torch.equal(m.lm_head.complement_map, emb.complement_map)
        keys = set(m.state_dict())
        norm = "norm." if fused else "norm.submodule."
        for k in ("caduceus.backbone.embeddings.word_embeddings.embedding.weight",
                  "caduceus.backbone.embeddings.word_embeddings.complement_map",
                  "caduceus.backbone.layers.1.mixer.submodule.mamba_fwd.A_log",
                  "caduceus.backbone.layers.0.mixer.submodule.mamba_rev.conv1d.weight",
                  f"caduceus.backbone.layers.0.{norm}weight", f"caduceus.backbone.{'norm_f.' if fused else 'norm_f.submodule.'}weight",
                  "lm_head.lm_head.weight", "lm_head.complement_map"):
            assert k in keys, k
    with pytest.raises(ValueError):
        CaduceusForMaskedLM(d_model=16, n_layer=1, vocab_size=12, rcps=True)   # no complement map


@pytest.mark.parametrize("fused", [True, False])
def test_caduceus_rcps_oracle_is_rc_equivariant(fused):
    """The float64 RCPS restatement is reverse-complement equivariant:
    logits(rc(x))[t, v] == logits(x)[L-1-t, comp(v)] -- the property RCPS is built for, here
    checked on the oracle the GPU parity test compares against."""
    from dna_amd.caduceus import CaduceusForMaskedLM
    from oracle import caduceus_ref as CR
    torch.manual_seed(5)
    m = CaduceusForMaskedLM(d_model=16, n_layer=2, vocab_size=12, rcps=True, complement_map=CM,
                            fused_add_norm=fused, ssm_cfg={"d_state": 8})
    with torch.no_grad():
        for p in m.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    sd = _rcps_sd(m)
    cm = sd["lm_head.complement_map"]
    ids = torch.randint(4, 12, (2, 24), generator=torch.Generator().manual_seed(3))
    dt_rank = m.caduceus.backbone.layers[0].mixer.submodule.mamba_fwd.dt_rank
    a = CR.mlm_logits(sd, ids, 2, 8, 4, dt_rank, rcps=True, fused_add_norm=fused).detach()
    b = CR.mlm_logits(sd, cm[ids.flip(-1)], 2, 8, 4, dt_rank, rcps=True, fused_add_norm=fused).detach()
    assert torch.allclose(b, a.flip(1)[..., cm], rtol=1e-10, atol=1e-12)
    assert (a - a.flip(1)[..., cm]).abs().max() > 1e-3   # not trivially symmetric


def test_weighted_cross_entropy():
    """modeling_caduceus.py:267-275: CE weighted by loss_weights renormalised over non-ignored
    tokens; uniform weights == the plain mean CE; the caller's weights are left untouched."""
    from dna_amd.caduceus import weighted_cross_entropy
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(2, 7, 12, generator=g)
    y = torch.randint(0, 12, (2, 7), generator=g)
    y[0, :3] = -100
    w = torch.ones(2, 7)
    plain = torch.nn.functional.cross_entropy(logits.view(-1, 12), y.view(-1), ignore_index=-100)
    assert torch.allclose(weighted_cross_entropy(logits, y, w), plain)
    assert torch.equal(w, torch.ones(2, 7))
    w = torch.rand(2, 7, generator=g)
    ce = torch.nn.functional.cross_entropy(logits.view(-1, 12), y.view(-1), ignore_index=-100,
                                           reduction="none")
    keep = (y.view(-1) != -100).double()
    ref = (ce.double() * w.view(-1).double() * keep).sum() / (w.view(-1).double() * keep).sum()
    assert torch.allclose(weighted_cross_entropy(logits, y, w).double(), ref, rtol=1e-6)


def test_char_tokenizer_complement_map():
    from dna_amd.tokenizer import CharacterTokenizer
    assert CharacterTokenizer("ACGTN", 10).complement_map() == CM
    cm = CharacterTokenizer("ACGTNacgt", 10).complement_map()
    assert cm[7] == 10 and cm[11] == 11 and cm[12] == 15 and cm[13] == 14


def test_rcps_modules_equivariance_cpu():
    """Each RCPS building block on the CPU with plain torch submodules: RCPSEmbedding, RCPSWrapper
    and RCPSAddNormWrapper commute with the reverse complement (flip over length and channels),
    and RCPSLMHead maps it to the complemented, position-reversed logits -- the algebra the
    whole-model equivariance tests rest on (modeling_rcps.py)."""
    from dna_amd.caduceus import (RCPSAddNormWrapper, RCPSEmbedding, RCPSLMHead, RCPSWrapper,
                                  _complement_tensor)
    torch.manual_seed(0)
    rc = lambda h: torch.flip(h, dims=[-2, -1])  # noqa: E731
    cm = _complement_tensor(CM)
    ids = torch.randint(0, 12, (2, 9))
    emb = RCPSEmbedding(12, 6, CM)
    e = emb(ids)
    assert e.shape == (2, 9, 12)
    assert torch.allclose(emb(cm[ids.flip(-1)]), rc(e))
    h = torch.randn(2, 9, 12, dtype=torch.float64)
    wrap = RCPSWrapper(torch.nn.Linear(6, 6).double())
    assert torch.allclose(wrap(rc(h)), rc(wrap(h)))
    an = RCPSAddNormWrapper(torch.nn.LayerNorm(6).double())
    res = torch.randn_like(h)
    y0, r0 = an(h, residual=res, prenorm=True)
    y1, r1 = an(rc(h), residual=rc(res), prenorm=True)
    assert torch.allclose(y1, rc(y0)) and torch.allclose(r1, rc(r0))
    head = RCPSLMHead(6, 12, CM).double()
    lg = head(h)
    assert torch.allclose(head(rc(h)), lg.flip(1)[..., cm])
