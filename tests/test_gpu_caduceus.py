"""GPU: Caduceus MLM (rcps=False and RCPS) logits and every gradient vs the float64 oracle
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


@pytest.mark.parametrize("d,dtype", [(256, torch.float32), (64, torch.float32), (256, torch.bfloat16)])
def test_hip_rmsnorm_module(d, dtype):
    """caduceus.RMSNorm on dna_rms_fwd/bwd vs a float64 restatement of mamba_ssm's RMSNorm:
    fp32 / bf16 inputs out of autocast (output in the input dtype), and under bf16 autocast the
    bf16 rounding of the fp32 result."""
    from dna_amd.caduceus import RMSNorm
    g = torch.Generator().manual_seed(d)
    m = RMSNorm(d).to("cuda")
    with torch.no_grad():
        m.weight.copy_(1 + 0.1 * torch.randn(d, generator=g))
    x = (torch.randn(5, 33, d, generator=g) * 2 + 0.3).to("cuda", dtype).requires_grad_(True)
    dy = torch.randn(5, 33, d, generator=g).to("cuda")
    xr = x.detach().double().requires_grad_(True)
    wr = m.weight.detach().double().requires_grad_(True)
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    y = m(x)
    assert y.dtype == dtype
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(y, yr) < tol
    y.backward(dy.to(dtype))
    yr.backward(dy.to(dtype).double())
    assert _rel(x.grad, xr.grad) < tol * 5 and _rel(m.weight.grad, wr.grad) < tol * 5
    if dtype == torch.float32:
        x.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            yb = m(x)
        assert yb.dtype == torch.bfloat16
        assert (yb.float() - yr.float().bfloat16().float()).abs().max() <= 2 ** -7 * yr.abs().max()
        yb.backward(dy.bfloat16())
        assert _rel(x.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("fused,rms", [(True, True), (False, True), (True, False)])
def test_caduceus_rcps_vs_oracle(fused, rms):
    """rcps=True (RCPSEmbedding / RCPSMambaBlock / RCPSLMHead) on the HIP mixers and norms vs the
    float64 RCPS restatement: logits, every parameter gradient, and RC equivariance of the GPU
    model itself (logits(rc(x))[t, v] == logits(x)[L-1-t, comp(v)])."""
    from dna_amd.caduceus import CaduceusForMaskedLM
    from test_caduceus import CM, _rcps_sd
    torch.manual_seed(11)
    m = CaduceusForMaskedLM(d_model=64, n_layer=2, vocab_size=12, rms_norm=rms, rcps=True,
                            complement_map=CM, fused_add_norm=fused, ssm_cfg={"d_state": 16})
    with torch.no_grad():
        for p in m.parameters():
            p.add_(torch.randn_like(p) * 0.02)
    sd = _rcps_sd(m)
    m = m.to(DEV)
    ids = torch.randint(0, 12, (2, 300), generator=torch.Generator().manual_seed(3))
    dt_rank = m.caduceus.backbone.layers[0].mixer.submodule.mamba_fwd.dt_rank
    ref = CR.mlm_logits(sd, ids, 2, 16, 4, dt_rank, rms_norm=rms, rcps=True, fused_add_norm=fused)
    _, logits = m(ids.to(DEV))
    assert _rel(logits, ref) < 1e-4
    g = torch.randn(ref.shape, generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    ref.backward(g)
    logits.backward(g.float().to(DEV))
    for n, p in m.named_parameters():
        assert _rel(p.grad, sd[n].grad) < 2e-3, n
    cm = m.lm_head.complement_map
    with torch.no_grad():
        ids_d = ids.to(DEV)
        _, a = m(ids_d)
        _, b = m(cm[ids_d.flip(-1)])
    assert _rel(b, a.flip(1)[..., cm]) < 1e-5


def test_caduceus_loss_weights():
    """forward(..., loss_weights=) == weighted_cross_entropy of the returned logits; all-ones
    weights == the unweighted loss."""
    from dna_amd.caduceus import CaduceusForMaskedLM, weighted_cross_entropy
    torch.manual_seed(2)
    m = CaduceusForMaskedLM(d_model=64, n_layer=1, vocab_size=12, ssm_cfg={"d_state": 16}).to(DEV)
    ids = torch.randint(0, 12, (2, 64), device=DEV)
    labels = ids.clone()
    labels[:, ::3] = -100
    w = torch.rand(2, 64, device=DEV)
    loss, logits = m(ids, labels, loss_weights=w)
    assert torch.allclose(loss, weighted_cross_entropy(logits, labels, w))
    l1, _ = m(ids, labels, loss_weights=torch.ones(2, 64, device=DEV))
    l0, _ = m(ids, labels)
    assert torch.allclose(l1, l0, rtol=1e-5)
