"""GPU: the HIP FFT long convolution (dna_amd.hyena.fftconv) against the reference fixtures
(fftconv_ref outputs/grads in fp64) and the numpy oracle at HyenaDNA sizes (L = 65536).
Tolerances: fp32 in/out -- relative max error 2e-5 of the output scale (fp32 FFT of size 2L);
bf16 in/out -- 1e-2 (bf16 rounding of inputs and outputs)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import hyena_ref as H

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(__file__), "golden", "fftconv_golden.npz")


def _cases():
    z = np.load(GOLD)
    for c in range(int(z["ncases"])):
        p = f"c{c}_"
        B, D, L, bi = (int(v) for v in z[p + "shape"])
        yield c, B, D, L, bool(bi), {k[len(p):]: z[k] for k in z.files if k.startswith(p)}


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: f"c{c[0]}_B{c[1]}D{c[2]}L{c[3]}bi{int(c[4])}")
def test_fftconv_matches_reference_fixture(case):
    from dna_amd.hyena import fftconv
    _, B, D, L, bi, f = case
    u = torch.tensor(f["u"], device=DEV, requires_grad=True)          # [B,1,D,1,L] as HyenaOperator
    k = torch.tensor(f["k"], device=DEV, requires_grad=True)
    bias = torch.tensor(f["bias"], device=DEV, requires_grad=True)    # [1,D,1]
    y = fftconv(u, k, bias, bidirectional=bi)
    assert y.shape == u.shape and y.dtype == u.dtype
    assert _rel(y.detach().cpu(), f["y64"]) < 2e-5
    y.backward(torch.tensor(f["dy"], device=DEV))
    assert _rel(u.grad.cpu(), f["du"]) < 2e-5
    assert _rel(k.grad.cpu(), f["dk"]) < 2e-5
    assert _rel(bias.grad.cpu(), f["dbias"]) < 2e-5


@pytest.mark.parametrize("bi", [False, True])
def test_fftconv_hyena_size_vs_oracle(bi):
    """L = 65536 (BASELINE config D length), odd batch (an unpaired row), fp32 and bf16."""
    from dna_amd.hyena import fftconv
    B, D, L = 3, 2, 65536
    g = torch.Generator().manual_seed(3)
    u = torch.randn(B, D, L, generator=g)
    k = torch.randn(D, L, generator=g) * torch.exp(-torch.linspace(0, 6, L))[None]
    bias = torch.randn(D, 1, generator=g)
    ref = H.fftconv_fwd(u.numpy(), k.numpy(), bias.numpy(), bi)
    y = fftconv(u.to(DEV), k.to(DEV), bias.to(DEV), bidirectional=bi)
    assert _rel(y.cpu(), ref) < 2e-5
    yb = fftconv(u.to(DEV).bfloat16(), k.to(DEV), bias.to(DEV), bidirectional=bi)
    assert yb.dtype == torch.bfloat16 and _rel(yb.float().cpu(), ref) < 1e-2
    dy = torch.randn(B, D, L, generator=g)
    du, dk, db = H.fftconv_bwd(dy.numpy(), u.numpy(), k.numpy(), bias.numpy(), bi)
    ut = u.to(DEV).requires_grad_(True)
    kt = k.to(DEV).requires_grad_(True)
    bt = bias.to(DEV).requires_grad_(True)
    fftconv(ut, kt, bt, bidirectional=bi).backward(dy.to(DEV))
    assert _rel(ut.grad.cpu(), du) < 2e-5
    assert _rel(kt.grad.cpu(), dk) < 5e-5
    assert _rel(bt.grad.cpu(), db) < 2e-5


def test_fftconv_linearity_and_errors():
    from dna_amd.hyena import fftconv
    g = torch.Generator().manual_seed(5)
    u1, u2 = torch.randn(2, 4, 1024, generator=g).to(DEV), torch.randn(2, 4, 1024, generator=g).to(DEV)
    k = torch.randn(4, 1024, generator=g).to(DEV)
    b = torch.zeros(4, device=DEV)
    lhs = fftconv(2.0 * u1 - 3.0 * u2, k, b)
    rhs = 2.0 * fftconv(u1, k, b) - 3.0 * fftconv(u2, k, b)
    assert (lhs - rhs).abs().max().item() < 1e-4 * rhs.abs().max().item()
    with pytest.raises(NotImplementedError):
        fftconv(u1, k, b, gelu=True)
    with pytest.raises(NotImplementedError):  # bidirectional, L not a kernel size, 2L > 131072
        fftconv(torch.zeros(1, 4, 70000, device=DEV), torch.zeros(4, 70000, device=DEV), b,
                bidirectional=True)
    with pytest.raises(RuntimeError):
        fftconv(u1.cpu(), k.cpu(), b.cpu())       # GPU only, no fallback


def _op_state(d_model, l_max, order, seed, **kw):
    """A HyenaOperator with random (non-default) weights and its float64 state_dict."""
    from dna_amd.hyena import HyenaOperator
    torch.manual_seed(seed)
    op = HyenaOperator(d_model=d_model, l_max=l_max, order=order, **kw)
    with torch.no_grad():
        for n, p in op.named_parameters():
            if n.endswith("freq"):
                continue
            p.add_(torch.randn_like(p) * 0.05)
    return op, {k: v.detach().double().clone() for k, v in op.state_dict().items()}


@pytest.mark.parametrize("order,autocast", [(2, True), (3, False), (2, False)])
def test_filter_t_equals_filter_permuted(order, autocast, monkeypatch):
    """HyenaFilter.filter_t (ModulateT: modulation + transpose in one kernel) against the
    reference layout filter(L)[0].reshape(L, v, o).permute(2, 1, 0): forward and the gradients of
    the implicit-filter MLP parameters. (The whole-filter kernels are off here; they have their
    own test below.)"""
    from dna_amd import hyena as HY
    monkeypatch.setattr(HY, "_FILTER_FUSED", False)
    op, _ = _op_state(64, 2048, order, 5, emb_dim=5)
    f = op.filter_fn.to(DEV)
    L, O = 2048, order - 1
    g = torch.Generator(device="cpu").manual_seed(9)
    dk = torch.randn(O, 64, L, generator=g).to(DEV)
    outs = []
    for fused in (True, False):
        f.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            if fused:
                k = f.filter_t(L, O)
            else:
                k = f.filter(L)[0].reshape(L, 64, O).permute(2, 1, 0)
        (k.float() * dk).sum().backward()
        outs.append((k.detach().float().clone(),
                     {n: p.grad.detach().clone() for n, p in f.named_parameters() if p.grad is not None}))
    (k1, g1), (k2, g2) = outs
    assert k1.shape == k2.shape == (O, 64, L)
    assert (k1 - k2).abs().max().item() <= 1e-6 * k2.abs().max().item() + 1e-7
    assert g1.keys() == g2.keys() and len(g1) > 0
    for n in g1:
        sc = g2[n].abs().max().item()
        assert (g1[n] - g2[n]).abs().max().item() <= 2e-5 * max(sc, 1e-3), n


@pytest.mark.parametrize("C,O,L,lr_pos,w", [(256, 1, 65536, 0.0, 10), (256, 1, 4096, 1e-5, 10),
                                          (256, 1, 4096, 1e-5, 1), (128, 2, 2048, 1e-5, 1),
                                          (64, 1, 1024, 1e-5, 10), (512, 1, 1024, 0.0, 1)])
def test_filter_whole_kernels_vs_module_path(C, O, L, lr_pos, w, monkeypatch):
    """The implicit filter as two kernels (FilterMLP, csrc/hyena_filter.hip) against the module
    path (strided-GEMM Linears, torch Sin, ModulateT) under bf16 autocast, at the config-D shape
    (emb_dim 5, filter_order 64, Sin frequency w = 10) and others: k, and the gradients of every
    MLP parameter, the shared Sin frequency and (lr_pos_emb > 0) the positional features. Both
    run the same bf16 dtype flow and differ only in fp32 accumulation order, so a bf16 rounding
    may land one ulp apart -- and sin(w y) turns a one-ulp change of y into w times that. Relative
    Frobenius error: k < 4e-3 at w = 1 and < 2e-2 at w = 10, each gradient < 2e-2 / 5e-2."""
    from dna_amd import hyena as HY
    tk, tg = (4e-3, 2e-2) if w == 1 else (2e-2, 5e-2)
    torch.manual_seed(C + L)
    f = HY.HyenaFilter(C, emb_dim=5, order=64, seq_len=L, w=w, lr_pos_emb=lr_pos, modulate=True).to(DEV)
    with torch.no_grad():  # trained-looking weights (default init keeps the Sin arguments small)
        for n, p in f.named_parameters():
            if "implicit_filter" in n:
                p.mul_(1.5)
    g = torch.Generator(device="cpu").manual_seed(3)
    dk = torch.randn(O, C // O, L, generator=g).to(DEV)
    outs = []
    for fused in (True, False):
        monkeypatch.setattr(HY, "_FILTER_FUSED", fused)
        f.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            k = f.filter_t(L, O)
        (k * dk).sum().backward()
        outs.append((k.detach().clone(),
                     {n: p.grad.detach().clone() for n, p in f.named_parameters() if p.grad is not None}))
    (k1, g1), (k2, g2) = outs
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()
    assert k1.shape == k2.shape == (O, C // O, L)
    assert rel(k1, k2) < tk, rel(k1, k2)
    expect = {"implicit_filter.0.weight", "implicit_filter.0.bias", "implicit_filter.1.freq",
              "implicit_filter.2.weight", "implicit_filter.2.bias", "implicit_filter.4.weight",
              "implicit_filter.4.bias", "implicit_filter.6.weight"}
    assert expect <= set(g1) and set(g1) == set(g2), (set(g1), set(g2))
    if lr_pos > 0:
        assert "pos_emb.z" in g1
    for n in g1:
        assert rel(g1[n], g2[n]) < tg, (n, rel(g1[n], g2[n]))


def test_hyena_operator_matches_reference_fixture():
    """dna_amd.hyena.HyenaOperator (HIP long conv) on the reference operator's state_dict and
    input (hyena_op_golden.npz, produced by running the reference): fp32 output vs the fp64 y."""
    from dna_amd.hyena import HyenaOperator
    d = np.load(os.path.join(os.path.dirname(GOLD), "hyena_op_golden.npz"), allow_pickle=False)
    sd = {k[3:]: torch.tensor(d[k]).float() for k in d.files if k.startswith("sd/")}
    op = HyenaOperator(d_model=16, l_max=64, order=2, filter_order=16)
    op.load_state_dict(sd, strict=True)
    op = op.to(DEV)
    y = op(torch.tensor(d["x"]).float().to(DEV))
    assert _rel(y.detach().cpu().numpy(), d["y"]) < 2e-5


@pytest.mark.parametrize("d_model,L,order,bi,emb_dim", [
    (16, 64, 2, False, 3), (32, 4096, 3, True, 5), (24, 1024, 2, True, 5),   # torch ops + HIP conv
    (64, 1024, 2, True, 5), (128, 4096, 2, False, 5), (64, 512, 3, True, 3),  # fused HIP path
])
def test_hyena_operator_fwd_bwd_vs_oracle(d_model, L, order, bi, emb_dim):
    """Forward and every gradient (input, projections, short conv, implicit-filter MLP, Sin
    freq, filter bias) of the GPU operator against autograd of the float64 restatement
    (oracle/hyena_operator_ref.py, pinned to the reference operator on the CPU side)."""
    from oracle import hyena_operator_ref as HO
    op, sd64 = _op_state(d_model, L, order, seed=L + order, filter_order=16, emb_dim=emb_dim,
                         bidirectional=bi, w=10)
    op = op.to(DEV)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, L, d_model, generator=g, dtype=torch.float64)
    dy = torch.randn(2, L, d_model, generator=g, dtype=torch.float64)
    buffers = {n for n, _ in op.named_buffers()}
    ref_sd = {k: v.clone().requires_grad_(k not in buffers) for k, v in sd64.items()}
    xr = x.clone().requires_grad_(True)
    yr = HO.hyena_operator(ref_sd, xr, d_model, order=order, l_max=L, bidirectional=bi)
    yr.backward(dy)
    xg = x.float().to(DEV).requires_grad_(True)
    y = op(xg)
    assert _rel(y.detach().cpu().numpy(), yr.detach().numpy()) < 5e-5
    y.backward(dy.float().to(DEV))
    assert _rel(xg.grad.cpu().numpy(), xr.grad.numpy()) < 5e-5
    # the shared Sin freq appears under several keys; compare each parameter once
    for n, p in op.named_parameters():
        ref = ref_sd[n].grad
        if n.endswith("freq"):  # one shared parameter: the reference grads of its aliases add up
            ref = sum(ref_sd[k].grad for k in ref_sd if k.endswith("freq"))
        assert p.grad is not None, n
        assert _rel(p.grad.cpu().numpy(), ref.numpy()) < 2e-4, n


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,L,d,order,K", [(2, 1000, 64, 2, 3), (1, 4096, 128, 3, 4), (3, 64, 64, 2, 2),
                                            (1, 1003, 64, 2, 3)])
def test_hyena_fused_kernels_vs_torch(dtype, tol, B, L, d, order, K):
    """ShortConvSplit / GateOut (fused HIP kernels) fwd + bwd against the same math in torch
    fp32 (the reference's conv1d / split / gate, hyena.py:421-507) on identical inputs."""
    from dna_amd.hyena import GateOut, ShortConvSplit
    g = torch.Generator(device="cpu").manual_seed(B * L + d)
    C = (order + 1) * d
    u = torch.randn(B, L, C, generator=g).to(dtype).to(DEV)
    w = (torch.randn(C, 1, K, generator=g) * 0.5).to(DEV)
    bias = (torch.randn(C, generator=g) * 0.1).to(DEV)
    dxs = torch.randn(B, order - 1, d, L, generator=g).to(dtype).to(DEV)
    dvx = torch.randn(B, d, L, generator=g).to(dtype).to(DEV)
    # torch reference in fp32
    ur = u.float().clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), bias.clone().requires_grad_(True)
    uc = F.conv1d(ur.transpose(1, 2), wr, br, padding=K - 1, groups=C)[..., :L]
    parts = uc.split(d, dim=1)
    xs_r = torch.stack(parts[:order - 1], dim=1)
    vx_r = parts[order] * parts[order - 1]
    (xs_r * dxs.float()).sum().add((vx_r * dvx.float()).sum()).backward()
    # fused
    uf = u.clone().requires_grad_(True)
    wf, bf = w.clone().requires_grad_(True), bias.clone().requires_grad_(True)
    xs, vx = ShortConvSplit.apply(uf, wf, bf, order, d)
    assert xs.dtype == dtype and vx.dtype == dtype
    (xs.float() * dxs.float()).sum().add((vx.float() * dvx.float()).sum()).backward()
    for mine, ref in ((xs, xs_r), (vx, vx_r), (uf.grad, ur.grad), (wf.grad, wr.grad), (bf.grad, br.grad)):
        assert _rel(mine.detach().float().cpu().numpy(), ref.detach().cpu().numpy()) < tol
    # gate + transpose
    yc = torch.randn(B, d, L, generator=g).to(dtype).to(DEV).requires_grad_(True)
    xs2 = xs.detach().clone().requires_grad_(True)
    y = GateOut.apply(yc, xs2)
    ref = (yc.detach().float() * xs2.detach().float()[:, 0]).transpose(1, 2)
    assert y.shape == (B, L, d) and _rel(y.detach().float().cpu().numpy(), ref.cpu().numpy()) < tol
    dy = torch.randn(B, L, d, generator=g).to(dtype).to(DEV)
    y.backward(dy)
    dyt = dy.float().transpose(1, 2)
    assert _rel(yc.grad.float().cpu().numpy(), (dyt * xs2.detach().float()[:, 0]).cpu().numpy()) < tol
    assert _rel(xs2.grad[:, 0].float().cpu().numpy(), (dyt * yc.detach().float()).cpu().numpy()) < tol
    if order > 2:
        assert xs2.grad[:, 1:].abs().max().item() == 0.0


@pytest.mark.parametrize("bi", [False, True])
@pytest.mark.parametrize("B,D,L,five_d", [(2, 3, 130, True), (1, 4, 65, False), (3, 2, 1000, True),
                                          (2, 5, 33, False), (1, 2, 1026, True), (2, 3, 4000, False)])
def test_fftconv_any_length_vs_oracle(B, D, L, five_d, bi):
    """Lengths that are not a kernel size (BPE configs use 130, char configs 1026): causal via
    zero padding, bidirectional via the rolled causal construction; fwd and du/dk/dbias vs the
    float64 oracle (fftconv_ref semantics at the same L)."""
    from dna_amd.hyena import fftconv
    rng = np.random.default_rng(L * 7 + D + int(bi))
    shape = (B, 1, D, 1, L) if five_d else (B, D, L)
    u = rng.standard_normal(shape).astype(np.float32)
    k = (rng.standard_normal((D, L)) * np.exp(-np.linspace(0, 3, L))[None]).astype(np.float32)
    bias = rng.standard_normal((1, D, 1)).astype(np.float32)
    dy = rng.standard_normal(shape).astype(np.float32)
    ur = u.reshape(B, D, L)
    y_ref = H.fftconv_fwd(ur, k, bias, bidirectional=bi)
    du_ref, dk_ref, db_ref = H.fftconv_bwd(dy.reshape(B, D, L), ur, k, bias, bidirectional=bi)
    ut = torch.tensor(u, device=DEV, requires_grad=True)
    kt = torch.tensor(k, device=DEV, requires_grad=True)
    # the reference adds u * D.unsqueeze(-1): D is [1, D, 1] for the operator's 5-D layout and
    # per channel [D] for a 3-D input
    bt = torch.tensor(bias if five_d else bias.reshape(D), device=DEV, requires_grad=True)
    y = fftconv(ut, kt, bt, bidirectional=bi)
    assert y.shape == ut.shape and y.dtype == torch.float32
    assert _rel(y.detach().cpu().numpy().reshape(B, D, L), y_ref) < 2e-5
    y.backward(torch.tensor(dy, device=DEV))
    assert _rel(ut.grad.cpu().numpy().reshape(B, D, L), du_ref) < 2e-5
    assert _rel(kt.grad.cpu().numpy(), dk_ref) < 2e-5
    assert _rel(bt.grad.cpu().numpy().reshape(-1), np.asarray(db_ref).reshape(-1)) < 2e-5


def test_hyena_operator_bpe_length_vs_oracle():
    """HyenaDNA BPE config length (pad_max_length 130): fused operator path (d_model 64),
    bidirectional, fwd + input/parameter grads vs the float64 operator oracle."""
    from oracle import hyena_operator_ref as HO
    L, d_model = 130, 64
    op, sd64 = _op_state(d_model, L, 2, seed=21, filter_order=16, emb_dim=5, bidirectional=True, w=10)
    op = op.to(DEV)
    buffers = {n for n, _ in op.named_buffers()}
    ref_sd = {k: v.clone().requires_grad_(k not in buffers) for k, v in sd64.items()}
    g = torch.Generator().manual_seed(6)
    x = torch.randn(3, L, d_model, generator=g, dtype=torch.float64)
    dy = torch.randn(3, L, d_model, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yr = HO.hyena_operator(ref_sd, xr, d_model, order=2, l_max=L, bidirectional=True)
    yr.backward(dy)
    xg = x.float().to(DEV).requires_grad_(True)
    y = op(xg)
    assert _rel(y.detach().cpu().numpy(), yr.detach().numpy()) < 5e-5
    y.backward(dy.float().to(DEV))
    assert _rel(xg.grad.cpu().numpy(), xr.grad.numpy()) < 5e-5
    for n, p in op.named_parameters():
        ref = ref_sd[n].grad
        if n.endswith("freq"):
            ref = sum(ref_sd[kk].grad for kk in ref_sd if kk.endswith("freq"))
        assert _rel(p.grad.cpu().numpy(), ref.numpy()) < 2e-4, n


@pytest.mark.parametrize("K,N", [(3, 64), (64, 64), (64, 256)])
def test_filter_split_k_linear_matches_linear_under_autocast(K, N):
    """The implicit-filter MLP's chunked linear (hyena._split_k_linear, config D: L = 65,536)
    against the plain nn.Linear it replaces, under bf16 autocast and in fp32: same output dtype
    (bf16 under autocast, as addmm gives), output within bf16 rounding, and input / weight / bias
    gradients within the rounding of one bf16 GEMM (the chunk partials are summed in fp32 and
    rounded once). ADVICE r3; the reference path is hyena.py:197-212 (nn.Linear in
    implicit_filter)."""
    from dna_amd.hyena import _split_k_linear
    torch.manual_seed(K + N)
    L = 65536
    lin = torch.nn.Linear(K, N).to(DEV)
    with torch.no_grad():
        lin.bias.normal_()
    x0 = torch.randn(1, L, K, device=DEV)
    gy0 = torch.randn(1, L, N, device=DEV)
    for ac in (True, False):
        outs = []
        for fn in (_split_k_linear, lambda x, l: l(x)):
            lin.zero_grad()
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
                y = fn(x, lin)
            y.backward(gy0.to(y.dtype))
            outs.append((y.detach(), x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()))
        (y1, dx1, dw1, db1), (y2, dx2, dw2, db2) = outs
        assert y1.dtype == y2.dtype == (torch.bfloat16 if ac else torch.float32)
        tol = 2e-2 if ac else 1e-5
        for a, b in ((y1, y2), (dx1, dx2), (dw1, dw2), (db1, db2)):
            a, b = a.float(), b.float()
            assert (a - b).abs().max().item() <= tol * max(1.0, b.abs().max().item()), (ac, K, N)
