"""GPU: the causal depthwise conv1d kernel against torch's conv1d, and the Mamba / BiMamba mixer
(HIP conv + HIP selective scan, torch projections) against the float64 oracle
(oracle/mamba_block_ref.py; parity unpinned: mamba_ssm absent). Tolerances: conv fp32 1e-5 / bf16
1e-2 relative; block fp32 fwd 1e-4, grads 2e-3 relative (fp32 scan over L positions)."""
import pytest
import torch
import torch.nn.functional as F

from oracle import mamba_block_ref as MB

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,C,L,K,silu", [(2, 64, 1000, 4, True), (1, 3, 2500, 3, False),
                                          (3, 128, 64, 2, True), (1, 16, 4096, 4, True),
                                          (2, 8, 5128, 4, True), (1, 4, 8200, 3, False)])
def test_causal_conv1d_vs_torch(dtype, tol, B, C, L, K, silu):
    from dna_amd.mamba import CausalConv1d
    g = torch.Generator(device="cpu").manual_seed(B * C + L)
    x = torch.randn(B, C, L, generator=g).to(dtype).to(DEV)
    w = (torch.randn(C, 1, K, generator=g) * 0.5).to(DEV)
    b = (torch.randn(C, generator=g) * 0.1).to(DEV)
    dy = torch.randn(B, C, L, generator=g).to(dtype).to(DEV)
    xr, wr, br = (t.float().clone().requires_grad_(True) for t in (x, w, b))
    yr = F.conv1d(xr, wr, br, padding=K - 1, groups=C)[..., :L]
    yr = F.silu(yr) if silu else yr
    yr.backward(dy.float())
    xf, wf, bf = (t.clone().requires_grad_(True) for t in (x, w, b))
    y = CausalConv1d.apply(xf, wf, bf, silu)
    assert y.dtype == dtype
    y.backward(dy)
    for mine, ref in ((y, yr), (xf.grad, xr.grad), (wf.grad, wr.grad), (bf.grad, br.grad)):
        assert _rel(mine.float(), ref) < tol


def _sd64(module):
    return {k: v.detach().double().cpu() for k, v in module.state_dict().items()}


@pytest.mark.parametrize("b,l,d_model,d_state,bias", [(2, 300, 64, 16, False), (1, 1100, 32, 8, False),
                                                       (2, 512, 64, 16, True)])
def test_mamba_block_fwd_bwd_vs_oracle(b, l, d_model, d_state, bias):
    from dna_amd.mamba import Mamba
    torch.manual_seed(l)
    m = Mamba(d_model=d_model, d_state=d_state, bias=bias)
    if bias:
        with torch.no_grad():
            m.in_proj.bias.normal_(0, 0.1)
            m.out_proj.bias.normal_(0, 0.1)
    with torch.no_grad():
        m.D.add_(torch.randn_like(m.D) * 0.1)
        m.conv1d.weight.mul_(2.0)
    sd = {k: v.clone().requires_grad_(True) for k, v in _sd64(m).items()}
    m = m.to(DEV)
    g = torch.Generator().manual_seed(2)
    h = torch.randn(b, l, d_model, generator=g, dtype=torch.float64)
    dy = torch.randn(b, l, d_model, generator=g, dtype=torch.float64)
    hr = h.clone().requires_grad_(True)
    yr = MB.mamba_forward(sd, hr, d_state, 4, m.dt_rank)
    yr.backward(dy)
    hg = h.float().to(DEV).requires_grad_(True)
    y = m(hg)
    assert _rel(y, yr) < 1e-4
    y.backward(dy.float().to(DEV))
    assert _rel(hg.grad, hr.grad) < 2e-3
    for n, p in m.named_parameters():
        assert _rel(p.grad, sd[n].grad) < 2e-3, n


@pytest.mark.parametrize("strategy", ["add", "ew_multiply"])
def test_bimamba_fwd_bwd_vs_oracle(strategy):
    from dna_amd.mamba import BiMambaWrapper
    torch.manual_seed(5)
    w = BiMambaWrapper(d_model=64, d_state=16, bidirectional_strategy=strategy)
    sd = {k: v.clone().requires_grad_(True) for k, v in _sd64(w).items()}
    # tied parameters: the oracle must see ONE tensor for both names
    for k in ("in_proj.weight", "out_proj.weight"):
        sd["mamba_rev." + k] = sd["mamba_fwd." + k]
    w = w.to(DEV)
    g = torch.Generator().manual_seed(8)
    h = torch.randn(2, 513, 64, generator=g, dtype=torch.float64)
    dy = torch.randn(2, 513, 64, generator=g, dtype=torch.float64)
    hr = h.clone().requires_grad_(True)
    yr = MB.bimamba_forward(sd, hr, 16, 4, w.mamba_fwd.dt_rank, strategy=strategy)
    yr.backward(dy)
    hg = h.float().to(DEV).requires_grad_(True)
    y = w(hg)
    assert _rel(y, yr) < 1e-4
    y.backward(dy.float().to(DEV))
    assert _rel(hg.grad, hr.grad) < 2e-3
    for n, p in w.named_parameters():  # tied ones appear once, under the forward name
        assert _rel(p.grad, sd[n].grad) < 2e-3, n


@pytest.mark.parametrize("shape,dtype", [((1, 131072, 256), torch.bfloat16), ((3, 77, 8), torch.float32),
                                         ((2, 1000, 40), torch.bfloat16)])
def test_flip_l_equals_torch_flip(shape, dtype):
    """mamba.flip_l (dna_flip_rows, the BiMamba wrapper's sequence flip) == torch.flip(x, (1,)),
    forward and gradient, bit for bit; rows that are not whole 16-B chunks take torch's flip."""
    from dna_amd.mamba import flip_l
    g = torch.Generator(device="cpu").manual_seed(shape[1])
    x = torch.randn(*shape, generator=g).to(dtype).to("cuda").requires_grad_(True)
    y = flip_l(x)
    assert torch.equal(y, x.detach().flip(dims=(1,)))
    dy = torch.randn(*shape, generator=g).to(dtype).to("cuda")
    y.backward(dy)
    assert torch.equal(x.grad, dy.flip(dims=(1,)))


def test_mamba_block_bf16_grads_track_fp32():
    """Under bf16 autocast the x gradient is the scan's du with x_proj's data gradient summed into
    it in the strided GEMM's epilogue (GradSink, no separate add): every gradient stays within
    bf16 reach of the fp32 run of the same module (which adds the two in torch)."""
    from dna_amd.mamba import Mamba
    torch.manual_seed(11)
    m = Mamba(d_model=64, d_state=16).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(3)
    h = torch.randn(2, 1024, 64, device=DEV, generator=g)
    dy = torch.randn(2, 1024, 64, device=DEV, generator=g)
    grads = []
    for ac in (False, True):
        m.zero_grad(set_to_none=True)
        hg = h.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
            y = m(hg)
        y.float().backward(dy)
        grads.append([hg.grad.float()] + [p.grad.float() for _, p in m.named_parameters()])
    names = ["h"] + [n for n, _ in m.named_parameters()]
    for n, a, b in zip(names, *grads):
        assert _rel(b, a) < 5e-2, (n, _rel(b, a))


@pytest.mark.parametrize("b,l,bias", [(1, 2048, False), (2, 1000, True)])
def test_bimamba_fused_reverse_equals_flips(b, l, bias, monkeypatch):
    """BiMambaWrapper "add" under bf16 autocast: the fused form (reverse direction reads the
    hidden states backwards, adds its output flipped back in place, the two dh accumulate in one
    buffer) against the flip / add form of the same module -- outputs and every gradient agree
    to bf16 rounding (the fused sums round once fewer)."""
    from dna_amd.mamba import BiMambaWrapper
    torch.manual_seed(b * 100 + l)
    m = BiMambaWrapper(d_model=64, bidirectional=True, bidirectional_strategy="add",
                       d_state=16, bias=bias).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(5)
    h = torch.randn(b, l, 64, device=DEV, generator=g)
    dy = torch.randn(b, l, 64, device=DEV, generator=g)
    res = []
    for fused in ("0", "1"):
        monkeypatch.setenv("DNA_BIMAMBA_FUSED", fused)
        m.zero_grad(set_to_none=True)
        hg = h.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(hg)
        y.float().backward(dy)
        res.append([y.float()] + [hg.grad.float()] +
                   [p.grad.float() for _, p in m.named_parameters()])
    names = ["out", "h"] + [n for n, _ in m.named_parameters()]
    for n, a, c in zip(names, *res):
        assert _rel(c, a) < 2e-2, (n, _rel(c, a))
