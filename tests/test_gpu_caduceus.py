"""GPU: Caduceus MLM (rcps=False) logits and every gradient vs the float64 oracle
(oracle/caduceus_ref.py; parity unpinned: mamba_ssm absent). fp32, tolerances fwd 1e-4, grads 2e-3."""
import pytest
import torch

from oracle import caduceus_ref as CR

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.mark.parametrize("rms,strategy", [(True, "add"), (False, "ew_multiply")])
def test_caduceus_vs_oracle(rms, strategy):
    from dna_amd.caduceus import CaduceusForMaskedLM
    torch.manual_seed(7)
    m = CaduceusForMaskedLM(d_model=64, n_layer=2, vocab_size=12, rms_norm=rms,
                            bidirectional_strategy=strategy, ssm_cfg={"d_state": 16})
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.add_(torch.randn_like(p) * 0.02)
    sd = {k: v.detach().double().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    # tied tensors: one leaf for every name
    sd["lm_head.weight"] = sd["caduceus.backbone.embeddings.word_embeddings.weight"]
    for i in range(2):
        p = f"caduceus.backbone.layers.{i}.mixer."
        for k in ("in_proj.weight", "out_proj.weight"):
            sd[p + "mamba_rev." + k] = sd[p + "mamba_fwd." + k]
    m = m.to(DEV)
    ids = torch.randint(0, 12, (2, 300), generator=torch.Generator().manual_seed(3))
    ref = CR.mlm_logits(sd, ids, 2, 16, 4, m.caduceus.backbone.layers[0].mixer.mamba_fwd.dt_rank,
                        rms_norm=rms, strategy=strategy)
    _, logits = m(ids.to(DEV))
    assert _rel(logits, ref) < 1e-4
    g = torch.randn(ref.shape, generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    ref.backward(g)
    logits.backward(g.float().to(DEV))
    for n, p in m.named_parameters():
        assert _rel(p.grad, sd[n].grad) < 2e-3, n
