"""BASELINE config E at its own length: Caduceus / Mamba selective scan at L = 131,072 (GPU).

The checker is the float64 C restatement oracle/selective_scan_ref.c (pinned to the Python
restatement of mamba_ssm's selective_scan_ref by tests/test_selective_scan_oracle.py; parity
UNPINNED at the mamba_ssm level: mamba_ssm is absent, so no reference output exists). The
Python/autograd oracle cannot run at this length (> 15 min), the C one takes ~2 s per channel
group. Tolerances (max relative error vs the largest magnitude): fp32 forward 1e-4, gradients
1e-3; bf16 inputs (compared with the oracle on the same bf16-rounded values) 3e-2 forward.
"""
import numpy as np
import pytest
import torch

from oracle.selective_scan_c import scan_bwd, scan_fwd, selective_scan_c

pytestmark = pytest.mark.gpu
DEV = "cuda"
L = 131072


def _inputs(b, d, l, n, seed):
    g = torch.Generator().manual_seed(seed)
    u = torch.randn(b, d, l, generator=g)
    delta = torch.randn(b, d, l, generator=g) * 0.5 - 1.0
    A = -torch.exp(torch.randn(d, n, generator=g) * 0.5)
    B = torch.randn(b, n, l, generator=g)
    C = torch.randn(b, n, l, generator=g)
    D = torch.randn(d, generator=g)
    z = torch.randn(b, d, l, generator=g)
    bias = torch.randn(d, generator=g) * 0.1
    return u, delta, A, B, C, D, z, bias


def _rel(mine, ref):
    mine = np.asarray(mine, dtype=np.float64)
    return float(np.abs(mine - ref).max() / (np.abs(ref).max() + 1e-30))


@pytest.mark.parametrize("b,d,n", [(1, 16, 16), (2, 4, 16)])  # block kernels (d % 8 == 0) / per-channel path
def test_selective_scan_fp32_full_length(b, d, n):
    from dna_amd.mamba import selective_scan_fn
    u, delta, A, B, C, D, z, bias = _inputs(b, d, L, n, seed=d)
    dout = torch.randn(b, d, L, generator=torch.Generator().manual_seed(5))
    ref, ref_last = scan_fwd(u.numpy(), delta.numpy(), A.numpy(), B.numpy(), C.numpy(), D=D.numpy(),
                             z=z.numpy(), delta_bias=bias.numpy(), delta_softplus=True)
    gref = scan_bwd(u.numpy(), delta.numpy(), A.numpy(), B.numpy(), C.numpy(), dout.numpy(),
                    D=D.numpy(), z=z.numpy(), delta_bias=bias.numpy(), delta_softplus=True)
    dev = [t.to(DEV).requires_grad_(True) for t in (u, delta, A, B, C, D, z, bias)]
    out, last = selective_scan_fn(*dev[:5], D=dev[5], z=dev[6], delta_bias=dev[7],
                                  delta_softplus=True, return_last_state=True)
    assert _rel(out.detach().cpu(), ref) < 1e-4
    assert _rel(last.cpu(), ref_last) < 1e-4
    out.backward(dout.to(DEV))
    for name, t in zip(("u", "delta", "A", "B", "C", "D", "z", "delta_bias"), dev):
        assert torch.isfinite(t.grad).all(), name
        assert _rel(t.grad.cpu(), gref[name]) < 1e-3, name


def test_selective_scan_bf16_full_length():
    from dna_amd.mamba import selective_scan_fn
    b, d, n = 1, 32, 16
    u, delta, A, B, C, D, z, bias = _inputs(b, d, L, n, seed=11)
    rb = lambda t: t.bfloat16().float()
    ref, _ = scan_fwd(rb(u).numpy(), rb(delta).numpy(), A.numpy(), rb(B).numpy(), rb(C).numpy(),
                      D=D.numpy(), z=rb(z).numpy(), delta_bias=bias.numpy(), delta_softplus=True)
    dev = [t.to(DEV).bfloat16().requires_grad_(True) for t in (u, delta)]
    Bd, Cd, zd = (t.to(DEV).bfloat16().requires_grad_(True) for t in (B, C, z))
    Ad, Dd, bd = (t.to(DEV).requires_grad_(True) for t in (A, D, bias))
    out = selective_scan_fn(dev[0], dev[1], Ad, Bd, Cd, D=Dd, z=zd, delta_bias=bd,
                            delta_softplus=True)
    assert out.dtype == torch.bfloat16
    assert _rel(out.float().detach().cpu(), ref) < 3e-2
    out.float().square().mean().backward()
    for t in (*dev, Ad, Bd, Cd, zd, Dd, bd):
        assert torch.isfinite(t.grad.float()).all()


def _rel_t(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def test_caduceus_two_layers_full_length_vs_oracle():
    """2-layer Caduceus MLM (bi-directional Mamba, tied in/out projections, RMSNorm) at
    L = 131,072 in fp32, reduced width (d_model 16 -> d_inner 32, still the block-kernel path):
    logits and every parameter gradient vs the float64 oracle with the C scan."""
    from dna_amd.caduceus import CaduceusForMaskedLM
    from oracle import caduceus_ref as CR
    torch.manual_seed(7)
    m = CaduceusForMaskedLM(d_model=16, n_layer=2, vocab_size=12, ssm_cfg={"d_state": 16})
    with torch.no_grad():
        for _, p in m.named_parameters():
            p.add_(torch.randn_like(p) * 0.02)
    sd = {k: v.detach().double().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    sd["lm_head.weight"] = sd["caduceus.backbone.embeddings.word_embeddings.weight"]
    for i in range(2):
        p = f"caduceus.backbone.layers.{i}.mixer."
        for k in ("in_proj.weight", "out_proj.weight"):
            sd[p + "mamba_rev." + k] = sd[p + "mamba_fwd." + k]
    m = m.to(DEV)
    ids = torch.randint(0, 12, (1, L), generator=torch.Generator().manual_seed(3))
    dt_rank = m.caduceus.backbone.layers[0].mixer.mamba_fwd.dt_rank
    ref = CR.mlm_logits(sd, ids, 2, 16, 4, dt_rank, scan=selective_scan_c)
    _, logits = m(ids.to(DEV))
    assert _rel_t(logits, ref) < 1e-4
    g = torch.randn(ref.shape, generator=torch.Generator().manual_seed(4), dtype=torch.float64)
    ref.backward(g)
    logits.backward(g.float().to(DEV))
    for n, p in m.named_parameters():
        assert torch.isfinite(p.grad).all(), n
        assert _rel_t(p.grad, sd[n].grad) < 2e-3, n


def test_caduceus_config_e_width_bf16_step_is_finite():
    """Config E's own width (d_model 256, d_state 16, char vocab 12 -> 16) at L = 131,072 under
    bf16 autocast, two layers: masked-LM loss near ln(vocab) at init, every gradient finite."""
    import math
    from dna_amd.caduceus import CaduceusForMaskedLM
    torch.manual_seed(0)
    m = CaduceusForMaskedLM(d_model=256, n_layer=2, vocab_size=12, ssm_cfg={"d_state": 16}).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(1)
    ids = torch.randint(7, 11, (1, L), device=DEV, generator=g)
    masked = torch.rand(1, L, device=DEV, generator=g) < 0.15
    inp = torch.where(masked, torch.full_like(ids, 3), ids)
    labels = torch.where(masked, ids, torch.full_like(ids, -100))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss, _ = m(inp, labels=labels)
    loss.backward()
    assert math.isfinite(loss.item()) and abs(loss.item() - math.log(16)) < 1.0
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), n
