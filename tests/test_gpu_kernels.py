"""Per-kernel parity of the HIP path against plain PyTorch fp32 restatements (oracle/bert_ref.py
formulas), forward and backward, bf16 and fp32. GPU only."""
import math

import numpy as np
import pytest
import torch

from oracle import bert_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ref_attention(qkv, key_valid, H, b, S):
    """fp32 PyTorch attention with the reference bias (bert_layers.py:167-178, :421-448)."""
    T, three_hd = qkv.shape
    D = three_hd // (3 * H)
    x = qkv.float().view(b, S, 3, H, D)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    bias = bert_ref.attention_bias(key_valid.view(b, S).bool().cpu(), H).to(qkv.device)
    s = q @ k.transpose(-1, -2) / math.sqrt(D) + bias
    p = torch.softmax(s, -1)
    return (p @ v).transpose(1, 2).reshape(T, H * D)


def _qkv(b, S, H, dtype, pad_rows=(), seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    qkv = torch.randn(b * S, 3 * H * 64, generator=g).to(DEV)
    valid = torch.ones(b, S, dtype=torch.uint8)
    for r, n in pad_rows:
        valid[r, n:] = 0
    return qkv.to(dtype), valid.reshape(-1).to(DEV)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize("b,S,H,pads", [(2, 128, 2, [(1, 77)]), (1, 512, 12, []),
                                        (3, 64, 1, [(0, 5), (2, 63)]), (2, 256, 4, [(0, 200)]),
                                        (1, 2048, 2, [(0, 1500)])])  # 32 tiles through the ring
def test_attention_forward(dtype, tol, b, S, H, pads):
    from dna_amd import functional as DF
    from dna_amd.config import alibi_slopes
    qkv, kv = _qkv(b, S, H, dtype, pads)
    slopes = torch.tensor(alibi_slopes(H), device=DEV)
    out = DF.alibi_attention(qkv, kv, slopes, b, S, H)
    ref = _ref_attention(qkv.float(), kv, H, b, S)
    valid = kv.bool()
    err = (out.float() - ref)[valid].abs().max().item()
    assert err < tol, err


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 6e-2)])
@pytest.mark.parametrize("b,S,H,pads", [(2, 128, 2, [(1, 77)]), (1, 512, 12, [(0, 400)]),
                                        (2, 64, 1, [])])
def test_attention_backward(dtype, tol, b, S, H, pads):
    from dna_amd import functional as DF
    from dna_amd.config import alibi_slopes
    qkv, kv = _qkv(b, S, H, dtype, pads, seed=1)
    slopes = torch.tensor(alibi_slopes(H), device=DEV)
    g = torch.randn(b * S, H * 64, device=DEV) * kv[:, None].float()  # pad rows get no grad
    q1 = qkv.clone().requires_grad_(True)
    DF.alibi_attention(q1, kv, slopes, b, S, H).backward(g.to(dtype))
    q2 = qkv.float().clone().requires_grad_(True)
    _ref_attention(q2, kv, H, b, S).backward(g)
    gv = q2.grad.view(b * S, 3, H * 64)
    hv = q1.grad.float().view(b * S, 3, H * 64)
    valid = kv.bool()
    scale = gv[valid].abs().max().item()
    err = (hv - gv)[valid].abs().max().item()
    assert err < tol * max(scale, 1.0), (err, scale)
    # pad rows: gradients must be exactly zero (they never reach the loss)
    assert hv[~valid].abs().max().item() == 0.0 if (~valid).any() else True


@pytest.mark.parametrize("b,S,H,pads", [(2, 128, 2, [(1, 77)]), (3, 512, 12, [(0, 400)]),
                                        (1, 192, 3, [])])
def test_attention_backward_fused_bias_grad(b, S, H, pads):
    """bf16 backward with the fused column sums of dqkv (bias gradient of the QKV projection):
    same dqkv as without, and the fp32 column sums match dqkv's (pre-rounding values vs rounded:
    within bf16 rounding)."""
    from dna_amd import functional as DF
    from dna_amd.config import alibi_slopes
    qkv, kv = _qkv(b, S, H, torch.bfloat16, pads, seed=3)
    slopes = torch.tensor(alibi_slopes(H), device=DEV)
    g = (torch.randn(b * S, H * 64, device=DEV) * kv[:, None].float()).bfloat16()
    q1 = qkv.clone().requires_grad_(True)
    DF.alibi_attention(q1, kv, slopes, b, S, H).backward(g)
    grads = {}

    class Grab(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.view_as(x)

        @staticmethod
        def backward(ctx, d):
            grads["colsum"] = getattr(d, "_dna_colsum", None)
            grads["d"] = d
            return d

    q2 = qkv.clone().requires_grad_(True)
    DF.alibi_attention(Grab.apply(q2), kv, slopes, b, S, H, bias_grad=True).backward(g)
    assert torch.equal(q1.grad, q2.grad)
    cs = grads["colsum"]
    assert cs is not None and cs.dtype == torch.float32 and cs.shape == (3 * H * 64,)
    ref = q2.grad.float().sum(0)
    tol = 1e-2 * ref.abs().max().item() + 1e-3
    assert (cs - ref).abs().max().item() < tol


@pytest.mark.parametrize("S", [128, 256, 512])
def test_attention_backward_deterministic(S):
    """The fused backward (one workgroup per (batch, head) at S = 128/256/512) sums the two
    key-half dQ partials in a fixed order and keeps dK/dV and the bias-gradient partial rows
    per workgroup: dqkv and the partial rows are bit-identical run to run."""
    import math
    from dna_amd import _native as N
    from dna_amd.config import alibi_slopes
    b, H = 3, 4
    qkv, kv = _qkv(b, S, H, torch.bfloat16, [(1, S - 37)], seed=7)
    slopes = torch.tensor(alibi_slopes(H), device=DEV)
    T = b * S
    out = torch.empty(T, H * 64, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(b, H, S, device=DEV)
    st = N.stream_ptr()
    N.call("dna_attn_fwd", qkv.data_ptr(), kv.data_ptr(), slopes.data_ptr(), b, S, H, 64, 1,
           1 / math.sqrt(64), out.data_ptr(), lse.data_ptr(), st)
    g = torch.Generator(device="cpu").manual_seed(8)
    dout = (torch.randn(T, H * 64, generator=g) * kv.cpu()[:, None].float()).to(DEV).bfloat16()
    rows = N.lib().dna_attn_dbias_part_rows(b, S)
    res = []
    for _ in range(2):
        dqkv = torch.full_like(qkv, float("nan"))
        part = torch.full((rows, 3 * H * 64), float("nan"), device=DEV)
        delta = torch.empty(b * H * S, device=DEV)
        N.call("dna_attn_bwd_ex", qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
               kv.data_ptr(), slopes.data_ptr(), b, S, H, 64, 1, 1 / math.sqrt(64),
               dqkv.data_ptr(), delta.data_ptr(), part.data_ptr(), st)
        res.append((dqkv, part))
    (d1, p1), (d2, p2) = res
    assert torch.isfinite(d1.float()).all() and torch.isfinite(p1).all()  # every element written
    assert torch.equal(d1, d2) and torch.equal(p1, p2)
    # the partial rows sum to dqkv's column sums (pre-rounding fp32 vs rounded bf16 values)
    ref = d1.float().sum(0)
    assert (p1.sum(0) - ref).abs().max().item() < 1e-2 * ref.abs().max().item() + 1e-3


def test_colsum_f32_deterministic_and_exact():
    from dna_amd import _native as N
    g = torch.Generator(device="cpu").manual_seed(5)
    part = torch.randn(1000, 2304, generator=g, dtype=torch.float64).float().to(DEV)
    out = torch.full((2304,), 3.0, device=DEV)
    N.call("dna_colsum_f32", part.data_ptr(), 1000, 2304, out.data_ptr(), 1, N.stream_ptr())
    ref = part.double().sum(0) + 3.0
    assert (out.double() - ref).abs().max().item() < 1e-4
    out2 = torch.zeros(2304, device=DEV)
    N.call("dna_colsum_f32", part.data_ptr(), 1000, 2304, out2.data_ptr(), 0, N.stream_ptr())
    out3 = torch.zeros(2304, device=DEV)
    N.call("dna_colsum_f32", part.data_ptr(), 1000, 2304, out3.data_ptr(), 0, N.stream_ptr())
    assert torch.equal(out2, out3) and torch.allclose(out2 + 3.0, out)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols", [64, 128, 768])
@pytest.mark.parametrize("act,use_bias,use_res", [(0, True, True), (1, True, False), (0, False, True)])
def test_fused_layernorm(dtype, cols, act, use_bias, use_res):
    from dna_amd import functional as DF
    torch.manual_seed(0)
    n = 333
    x = torch.randn(n, cols, device=DEV).to(dtype)
    bias = torch.randn(cols, device=DEV) * 0.1 if use_bias else None
    res = torch.randn(n, cols, device=DEV) if use_res else None
    gm = 1 + 0.1 * torch.randn(cols, device=DEV)
    bt = 0.1 * torch.randn(cols, device=DEV)
    leaves = [t.clone().requires_grad_(True) if t is not None else None for t in (x, bias, res, gm, bt)]
    y, yb = DF.FusedLayerNorm.apply(*leaves, 1e-12, act, 0.0, 0, 0, True, True)
    refl = [t.detach().float().clone().requires_grad_(True) if t is not None else None for t in (x, bias, res, gm, bt)]
    u = refl[0] + (refl[1] if use_bias else 0)
    if act == 1:
        u = torch.nn.functional.gelu(u)
    if use_res:
        u = u + refl[2]
    yr = torch.nn.functional.layer_norm(u, (cols,), refl[3], refl[4], 1e-12)
    assert (y - yr).abs().max().item() < 1e-4
    assert (yb.float() - yr).abs().max().item() < 3e-2
    dy = torch.randn(n, cols, device=DEV)
    dyb = torch.randn(n, cols, device=DEV).to(torch.bfloat16)
    (y * dy).sum().backward(retain_graph=True)
    (yb.float() * dyb.float()).sum().backward()
    (yr * (dy + dyb.float())).sum().backward()
    tol = 2e-4 if dtype == torch.float32 else 3e-2
    for a, r in zip(leaves, refl):
        if a is None:
            continue
        sc = max(r.grad.abs().max().item(), 1.0)
        assert (a.grad.float() - r.grad).abs().max().item() < tol * sc


@pytest.mark.parametrize("cols", [128, 768])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_ln_bwd_from_y_equals_recompute_from_x(cols, p):
    """dna_ln_bwd_from_y (x_hat = (y - beta) / gamma from the forward's fp32 output) against
    dna_ln_bwd (x_hat recomputed from x + bias, the dropout mask and the residual) on the same
    forward, dropout on and off: every output within fp32 recompute noise."""
    from dna_amd import _native as N
    g = torch.Generator(device=DEV).manual_seed(cols + int(10 * p))
    n = 1000
    x = torch.randn(n, cols, device=DEV, generator=g).bfloat16()
    bias = torch.randn(cols, device=DEV, generator=g) * 0.1
    res = torch.randn(n, cols, device=DEV, generator=g)
    gm = 1 + 0.1 * torch.randn(cols, device=DEV, generator=g)
    bt = 0.1 * torch.randn(cols, device=DEV, generator=g)
    y = torch.empty(n, cols, device=DEV)
    mean, rstd = torch.empty(n, device=DEV), torch.empty(n, device=DEV)
    st = N.stream_ptr()
    N.call("dna_ln_fwd", x.data_ptr(), N.BF16, bias.data_ptr(), 0, p, 5, 7, res.data_ptr(),
           gm.data_ptr(), bt.data_ptr(), n, cols, 1e-12, y.data_ptr(), None, mean.data_ptr(),
           rstd.data_ptr(), st)
    dy = torch.randn(n, cols, device=DEV, generator=g)
    dyb = torch.randn(n, cols, device=DEV, generator=g).bfloat16()
    nws = N.lib().dna_ln_bwd_workspace(n, cols)
    ws = torch.empty(nws, device=DEV, dtype=torch.uint8)
    outs = []
    for from_y in (False, True):
        dx = torch.empty_like(x)
        dres = torch.empty(n, cols, device=DEV)
        dg, db, dbias = (torch.empty(cols, device=DEV) for _ in range(3))
        if from_y:
            N.call("dna_ln_bwd_from_y", dy.data_ptr(), dyb.data_ptr(), y.data_ptr(), N.BF16, p, 5, 7,
                   gm.data_ptr(), bt.data_ptr(), rstd.data_ptr(), n, cols, dres.data_ptr(),
                   dx.data_ptr(), dg.data_ptr(), db.data_ptr(), dbias.data_ptr(), ws.data_ptr(),
                   nws, st)
        else:
            N.call("dna_ln_bwd", dy.data_ptr(), dyb.data_ptr(), x.data_ptr(), N.BF16, bias.data_ptr(),
                   0, p, 5, 7, res.data_ptr(), gm.data_ptr(), mean.data_ptr(), rstd.data_ptr(), n,
                   cols, dres.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(),
                   dbias.data_ptr(), ws.data_ptr(), nws, st)
        outs.append((dx.float(), dres, dg, db, dbias))
    for i, (a, b) in enumerate(zip(*outs)):
        # dx is bf16: a recompute difference at fp32 noise level may flip its rounding (1 ulp)
        tol = 2 ** -7 * b.abs().max().item() if i == 0 else 2e-5 * max(b.abs().max().item(), 1.0)
        assert (a - b).abs().max().item() <= tol, i
    assert torch.equal(outs[0][0] == 0, outs[1][0] == 0)  # the same dropout mask


def _rms_ref(x, g, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * g


@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols", [128, 256, 1024])
def test_add_layernorm_vs_torch(dtype, cols, rms):
    """dna_add_ln_fwd / bwd (the HyenaDNA Block's residual add + norm): the fp32 sum is bit-equal
    to torch's `x + residual`; LN output and every gradient -- with the sum also consumed
    downstream, as the next Block's residual add does -- match the fp32 torch graph."""
    from dna_amd import functional as DF
    torch.manual_seed(1)
    n = 517
    x = torch.randn(n, cols, device=DEV).to(dtype)
    res = torch.randn(n, cols, device=DEV)
    gm = 1 + 0.1 * torch.randn(cols, device=DEV)
    bt = 0.1 * torch.randn(cols, device=DEV)
    want_bf16 = dtype == torch.bfloat16
    leaves = [t.clone().requires_grad_(True) for t in (x, res, gm, bt)]
    s, y = DF.AddLayerNorm.apply(*leaves[:3], None if rms else leaves[3], 1e-5, want_bf16)
    refl = [t.detach().clone().requires_grad_(True) for t in (x, res, gm, bt)]
    sr = refl[0] + refl[1]
    yr = (_rms_ref(sr, refl[2], 1e-5) if rms
          else torch.nn.functional.layer_norm(sr, (cols,), refl[2], refl[3], 1e-5))
    assert s.dtype == torch.float32 and torch.equal(s, sr)
    assert y.dtype == (torch.bfloat16 if want_bf16 else torch.float32)
    assert (y.float() - yr.float()).abs().max().item() < (3e-2 if want_bf16 else 1e-4)
    ds = torch.randn(n, cols, device=DEV)
    dy = torch.randn(n, cols, device=DEV).to(y.dtype)
    ((s * ds).sum() + (y.float() * dy.float()).sum()).backward()
    refl2 = [t.detach().float().clone().requires_grad_(True) for t in (x, res, gm, bt)]
    s2 = refl2[0] + refl2[1]
    y2 = (_rms_ref(s2, refl2[2], 1e-5) if rms
          else torch.nn.functional.layer_norm(s2, (cols,), refl2[2], refl2[3], 1e-5))
    ((s2 * ds).sum() + (y2 * dy.float()).sum()).backward()
    assert leaves[0].grad.dtype == dtype and leaves[1].grad.dtype == torch.float32
    tol = 2e-4 if dtype == torch.float32 else 3e-2
    for a, r in zip(leaves[:3] if rms else leaves, refl2):
        sc = max(r.grad.abs().max().item(), 1.0)
        assert (a.grad.float() - r.grad).abs().max().item() < tol * sc


@pytest.mark.parametrize("rows,cols", [(1, 64), (300, 192), (131072, 256), (5001, 768), (70000, 1024)])
def test_colsum_bf16_bias_grad(rows, cols):
    """dna_colsum_bf16 (functional.bias_grad): fp32 column sums of a bf16 gradient vs a float64
    sum, deterministic (two calls bit-equal), accumulate mode adds onto the output."""
    from dna_amd import _native as N
    from dna_amd import functional as DF
    g = torch.Generator(device="cpu").manual_seed(rows + cols)
    dy = torch.randn(rows, cols, generator=g).to(torch.bfloat16).to(DEV)
    ref = dy.double().sum(0)
    a = DF.bias_grad(dy)
    b = DF.bias_grad(dy)
    assert a.dtype == torch.float32 and torch.equal(a, b)
    assert (a.double() - ref).abs().max().item() < 1e-5 * max(rows, 1) ** 0.5 + 1e-5
    out = torch.full((cols,), 2.0, device=DEV)
    nws = N.lib().dna_colsum_bf16_workspace(rows, cols)
    ws = torch.empty(nws, device=DEV, dtype=torch.uint8)
    N.call("dna_colsum_bf16", dy.data_ptr(), rows, cols, out.data_ptr(), 1, ws.data_ptr(), nws,
           N.stream_ptr())
    assert torch.allclose(out, a + 2.0, rtol=0, atol=1e-5)


@pytest.mark.parametrize("V,d,shape,pad", [(16, 256, (2, 65536), None), (12, 128, (3, 777), 4),
                                           (4096, 64, (5000,), 0), (5, 768, (70001,), 2),
                                           (3, 64, (40960,), None), (2, 1024, (33 * 1024,), None),
                                           (1, 256, (50000,), None)])
def test_embedding_fn_grad_vs_torch(V, d, shape, pad):
    """functional.embedding (HipEmbedding): forward = F.embedding; the table gradient of the
    sorted segmented sum matches torch's embedding backward (fp32 sums in another order) and is
    bit-identical run to run; the padding row gets no gradient. Runs of thousands of chunks (the
    join's group level), runs ending with the data, one run over everything, d = 64 .. 1024."""
    from dna_amd import functional as DF
    g = torch.Generator(device="cpu").manual_seed(V + d)
    ids = torch.randint(0, V, shape, generator=g).to(DEV)
    E = torch.randn(V, d, generator=g).to(DEV)
    dy = torch.randn(*shape, d, generator=g).to(DEV)
    grads = []
    for _ in range(2):
        w = E.clone().requires_grad_(True)
        y = DF.embedding(ids, w, pad)
        assert torch.equal(y, torch.nn.functional.embedding(ids, E, pad))
        y.backward(dy)
        grads.append(w.grad)
    assert torch.equal(grads[0], grads[1])
    wr = E.clone().requires_grad_(True)
    torch.nn.functional.embedding(ids, wr, pad).backward(dy)
    sc = wr.grad.abs().max().item()
    assert (grads[0] - wr.grad).abs().max().item() < 1e-5 * max(sc, 1.0)
    if pad is not None:
        assert grads[0][pad].abs().max().item() == 0.0


def test_dropout_mask_consistent_fwd_bwd():
    """GeGLU dropout: backward regenerates the forward mask (Philox), keep rate ~0.9."""
    from dna_amd import functional as DF
    torch.manual_seed(0)
    n, F = 512, 3072
    g = torch.randn(n, 2 * F, device=DEV).abs().add(0.5).requires_grad_(True)
    a = DF.GeGLU.apply(g, 0.1, 1234, 77)
    kept = a != 0
    rate = kept.float().mean().item()
    assert abs(rate - 0.9) < 0.005, rate
    # neighbours share one 32-bit Philox word (16-bit halves): their bits must be independent,
    # also across the 8-element groups of one draw (lag 8) and down a column (next row)
    k = kept.float()
    for s in (1, 2, 3, 4, 7, 8):
        both = (k[:, :-s] * k[:, s:]).mean().item()
        assert abs(both - rate * rate) < 0.005, (s, both, rate * rate)
    both = (k[:-1] * k[1:]).mean().item()
    assert abs(both - rate * rate) < 0.005, ("row", both, rate * rate)
    for j in range(8):  # every slot of the 128-bit draw keeps at the same rate
        assert abs(k[:, j::8].mean().item() - 0.9) < 0.01, j
    da = torch.randn(n, F, device=DEV)
    a.backward(da)
    g2 = g.detach().clone().requires_grad_(True)
    x1, x2 = g2[:, :F], g2[:, F:]
    ref = torch.nn.functional.gelu(x1) * x2 * kept.float() / 0.9
    ref.backward(da)
    assert (g.grad - g2.grad).abs().max().item() < 1e-4
    # a different offset gives a different mask
    a2 = DF.GeGLU.apply(g.detach(), 0.1, 1234, 78 + n * F)
    assert ((a2 != 0) != kept).float().mean().item() > 0.1


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
def test_geglu(dtype, tol):
    from dna_amd import functional as DF
    torch.manual_seed(0)
    n, F = 100, 512
    g = torch.randn(n, 2 * F, device=DEV).to(dtype).requires_grad_(True)
    a = DF.GeGLU.apply(g, 0.0, 0, 0)
    g2 = g.detach().float().clone().requires_grad_(True)
    ref = torch.nn.functional.gelu(g2[:, :F]) * g2[:, F:]
    assert (a.float() - ref).abs().max().item() < tol * 4
    da = torch.randn(n, F, device=DEV)
    a.backward(da.to(dtype))
    ref.backward(da)
    assert (g.grad.float() - g2.grad).abs().max().item() < tol * 8


@pytest.mark.parametrize("n", [4096, 8193, 16387, 70001])
def test_geglu_row_unrolled_bf16(n):
    """bf16 kernels (U = 2 or 4 rows per thread, ragged row tails) == the fp32 U=1 kernels on the
    same bf16 inputs: identical dropout masks, values within bf16 rounding."""
    from dna_amd import _native as N
    torch.manual_seed(0)
    F = 64
    g = torch.randn(n, 2 * F, device=DEV).to(torch.bfloat16)
    da = torch.randn(n, F, device=DEV).to(torch.bfloat16)
    outs = {}
    for dt, code in ((torch.bfloat16, 1), (torch.float32, 0)):
        a = torch.empty(n, F, device=DEV, dtype=dt)
        fac = torch.empty(n, 2 * F, device=DEV, dtype=dt)
        dg = torch.empty(n, 2 * F, device=DEV, dtype=dt)
        # converted inputs held in variables: a temporary passed as `.to(dt).data_ptr()` is freed
        # before the kernel runs, and the next conversion may reuse its block (seen in the full
        # suite: the fp32 reference read a dO overwritten by g's conversion)
        gi, di = g.to(dt), da.to(dt)
        N.call("dna_geglu_fwd", gi.data_ptr(), code, n, F, 0.1, 7, 3, a.data_ptr(), fac.data_ptr(),
               N.stream_ptr())
        N.call("dna_geglu_bwd", di.data_ptr(), fac.data_ptr(), code, n, F, dg.data_ptr(),
               N.stream_ptr())
        outs[code] = (a.float(), dg.float())
    (a1, dg1), (a0, dg0) = outs[1], outs[0]
    assert torch.equal(a1 == 0, a0 == 0)
    assert (a1 - a0).abs().max().item() <= 8e-3 * a0.abs().max().item()
    assert (dg1 - dg0).abs().max().item() <= 8e-3 * dg0.abs().max().item()


@pytest.mark.parametrize("cols", [64, 128, 768])
def test_embedding_ln(cols):
    from dna_amd import functional as DF
    torch.manual_seed(0)
    V, n = 4096, 700
    ids = torch.randint(0, V, (n,), device=DEV)
    ids[:50] = 0  # padding_idx rows
    E = (torch.randn(V, cols, device=DEV) * 0.02).requires_grad_(True)
    tt = (torch.randn(2, cols, device=DEV) * 0.02).requires_grad_(True)
    gm = (1 + 0.1 * torch.randn(cols, device=DEV)).requires_grad_(True)
    bt = (0.1 * torch.randn(cols, device=DEV)).requires_grad_(True)
    y, yb = DF.EmbeddingLN.apply(ids, E, tt, gm, bt, 1e-12, 0.0, 0, 0, True, True)
    E2, tt2, gm2, bt2 = (t.detach().clone().requires_grad_(True) for t in (E, tt, gm, bt))
    yr = torch.nn.functional.layer_norm(
        torch.nn.functional.embedding(ids, E2, padding_idx=0) + tt2[0], (cols,), gm2, bt2, 1e-12)
    assert (y - yr).abs().max().item() < 1e-4
    dy = torch.randn(n, cols, device=DEV)
    (y * dy).sum().backward()
    (yr * dy).sum().backward()
    for a, r in ((E, E2), (tt, tt2), (gm, gm2), (bt, bt2)):
        assert (a.grad - r.grad).abs().max().item() < 1e-3 * max(1.0, r.grad.abs().max().item())
    assert E.grad[0].abs().max().item() == 0.0


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-4)])
def test_masked_cross_entropy(dtype, tol):
    from dna_amd import functional as DF
    torch.manual_seed(0)
    M, V = 77, 4096
    x = torch.randn(M, V, device=DEV).to(dtype).requires_grad_(True)
    t = torch.randint(0, V, (M,), device=DEV)
    loss = DF.MaskedCrossEntropy.apply(x, t, 100)
    x2 = x.detach().float().clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(x2, t, reduction="sum") / 100
    assert abs(loss.item() - ref.item()) < 1e-4
    (loss * 3).backward()
    (ref * 3).backward()
    assert (x.grad.float() - x2.grad).abs().max().item() < (tol if dtype == torch.float32 else 2e-4)


def test_fused_adamw_matches_torch():
    from dna_amd.flat import FlatParams
    from dna_amd.optim import FusedAdamW
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(37, 19), torch.nn.Linear(19, 5)).to(DEV)
    ref = [p.detach().clone().requires_grad_(True) for p in m.parameters()]
    flat = FlatParams(m, DEV)
    opt = FusedAdamW(flat, lr=5e-3, weight_decay=1e-2, max_grad_norm=1.0)
    topt = torch.optim.AdamW(ref, lr=5e-3, weight_decay=1e-2)
    for step in range(5):
        grads = [torch.randn_like(p) * 2 for p in ref]
        flat.zero_grad()
        for p, g in zip(m.parameters(), grads):
            p.grad.copy_(g)
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        topt.step()
        opt.step()
        for p, r in zip(m.parameters(), ref):
            assert (p.detach() - r.detach()).abs().max().item() < 1e-6
    assert (flat.shadow.float() - flat.flat).abs().max().item() < 1e-2


@pytest.mark.parametrize("rows,m,n", [(65536, 768, 768), (8192, 2304, 768), (1000, 768, 3072),
                                      (4096, 6144, 768)])
def test_wgrad_splitk(rows, m, n):
    from dna_amd.functional import wgrad
    torch.manual_seed(0)
    dy = torch.randn(rows, m, device=DEV).to(torch.bfloat16)
    x = torch.randn(rows, n, device=DEV).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    got = wgrad(dy, x)
    assert got.dtype == torch.float32
    assert (got - ref).abs().max().item() < 2e-3 * ref.abs().max().item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 5e-2)])
def test_attention_forward_spiked_max(dtype, tol):
    """Force late running-max jumps: the key tiles are visited diagonal-first, so a key far from
    the diagonal with a huge score makes the max grow on a late tile (rescale branch taken)."""
    from dna_amd import functional as DF
    from dna_amd.config import alibi_slopes
    b, S, H = 2, 512, 12
    qkv, kv = _qkv(b, S, H, torch.float32, [], seed=3)
    x = qkv.view(b, S, 3, H, 64)
    for (bi, qi, kj) in [(0, 3, 500), (0, 300, 10), (1, 511, 0), (1, 64, 448), (0, 128, 129)]:
        x[bi, kj, 1, :, :] = 6.0 * x[bi, qi, 0, :, :] / x[bi, qi, 0, :, :].norm(dim=-1, keepdim=True)
    qkv = qkv.to(dtype)
    slopes = torch.tensor(alibi_slopes(H), device=DEV)
    out = DF.alibi_attention(qkv, kv, slopes, b, S, H)
    ref = _ref_attention(qkv.float(), kv, H, b, S)
    err = (out.float() - ref).abs().max().item()
    assert err < tol, err


@pytest.mark.parametrize("n", [20000, 20001, 33, 1])
def test_embedding_grad_skewed_ids(n):
    """Zipf-like token ids (a few ids cover most rows, runs crossing many 32-row chunks, the
    padding id among them): sorted segmented sum == dense reference, and bit-identical run to
    run (runs crossing chunks are joined in chunk order, no atomics)."""
    from dna_amd import functional as DF
    torch.manual_seed(0)
    V, cols = 4096, 768
    ids = torch.randint(0, 8, (n,), device=DEV)
    ids[::7] = torch.randint(0, V, (len(ids[::7]),), device=DEV)
    tt = torch.zeros(2, cols, device=DEV, requires_grad=True)
    gm = torch.ones(cols, device=DEV, requires_grad=True)
    bt = torch.zeros(cols, device=DEV, requires_grad=True)
    E0 = torch.randn(V, cols, device=DEV) * 0.02
    dy = torch.randn(n, cols, device=DEV)
    grads = []
    for _ in range(2):
        E = E0.clone().requires_grad_(True)
        y, _ = DF.EmbeddingLN.apply(ids, E, tt, gm, bt, 1e-12, 0.0, 0, 0, True, False)
        (y * dy).sum().backward()
        grads.append(E.grad)
    assert torch.equal(grads[0], grads[1])
    E2 = E0.clone().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(torch.nn.functional.embedding(ids, E2, padding_idx=0),
                                        (cols,), gm.detach(), bt.detach(), 1e-12)
    (yr * dy).sum().backward()
    assert (grads[0] - E2.grad).abs().max().item() <= 1e-3 * E2.grad.abs().max().item()
    assert torch.all(grads[0][0] == 0)


# ------------------------------------------------------------------ MFMA GEMM (gemm.hip)
def _gemm_call(name, *args):
    from dna_amd import _native as N
    N.call(name, *args, N.stream_ptr())


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("M,N,K", [(4096, 2304, 768), (1000, 768, 768), (512, 768, 3072),
                                   (300, 4096, 768)])
def test_gemm_linear_fwd_dgrad_wgrad(M, N, K):
    """dna_linear_{fwd,dgrad,wgrad} vs fp32 torch on the same bf16 operands (bf16 rounding of
    the output only: rel. Frobenius error < 1e-2; fp32 wgrad partials < 1e-5)."""
    g = torch.Generator(device="cpu").manual_seed(N + K)
    x = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV).bfloat16()
    b = torch.randn(N, generator=g).to(DEV)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr(), M, N, K, y.data_ptr())
    assert _rel(y, x.float() @ w.float().t() + b) < 1e-2
    dy = torch.randn(M, N, generator=g).to(DEV).bfloat16()
    dx = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_linear_dgrad", dy.data_ptr(), w.data_ptr(), M, N, K, dx.data_ptr())
    assert _rel(dx, dy.float() @ w.float()) < 1e-2
    if M % 128 == 0:
        s = 2
        part = torch.empty(s, N, K, device=DEV)
        _gemm_call("dna_linear_wgrad", dy.data_ptr(), x.data_ptr(), M, N, K, s, part.data_ptr())
        assert _rel(part.sum(0), dy.float().t() @ x.float()) < 1e-5


def test_gemm_linear_fwd_row_blocks_past_32bit_offsets():
    """An x operand of >= 2^31 bytes (M = 2^19 + 100 rows x K = 2048) runs the persistent kernel
    in row blocks of 524,032 rows (a multiple of 256): rows on both sides of the block boundary,
    and the ragged last rows, equal fp32 torch on the same bf16 operands; the output between
    blocks is fully written."""
    M, N, K = (1 << 19) + 100, 256, 2048
    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.empty(M, K, device=DEV, dtype=torch.bfloat16).uniform_(-1, 1)
    w = (torch.randn(N, K, generator=g) * 0.05).to(DEV).bfloat16()
    b = torch.randn(N, generator=g).to(DEV)
    y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr(), M, N, K, y.data_ptr())
    torch.cuda.synchronize()
    assert not torch.isnan(y).any()
    mc = ((1 << 31) - 1) // (K * 2) // 256 * 256
    for r in (0, mc - 300, mc - 1, mc, mc + 1, M - 300):
        rows = slice(r, min(r + 300, M))
        assert _rel(y[rows], x[rows].float() @ w.float().t() + b) < 1e-2, r


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm_geglu_fused_equals_unfused(p):
    """Fused gated_layers+GeGLU fwd and wo-dgrad+GeGLU bwd give bit-identical results to the
    unfused kernels on the GEMM outputs (same Philox dropout mask)."""
    M, H, F = 1024, 768, 3072
    g0 = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(M, H, generator=g0).to(DEV).bfloat16()
    wg = (torch.randn(2 * F, H, generator=g0) * 0.05).to(DEV).bfloat16()
    bg = (torch.randn(2 * F, generator=g0) * 0.1).to(DEV)
    fac = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
    a = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_geglu_linear_fwd", x.data_ptr(), wg.data_ptr(), bg.data_ptr(), M, F, H, p, 11, 5,
               fac.data_ptr(), a.data_ptr())
    g = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_linear_fwd", x.data_ptr(), wg.data_ptr(), bg.data_ptr(), M, 2 * F, H, g.data_ptr())
    assert _rel(g, x.float() @ wg.float().t() + bg) < 1e-2
    a2, fac2 = torch.empty_like(a), torch.empty_like(fac)
    _gemm_call("dna_geglu_fwd", g.data_ptr(), 1, M, F, p, 11, 5, a2.data_ptr(), fac2.data_ptr())
    assert torch.equal(a, a2) and torch.equal(fac, fac2)
    _geglu_factors_match(g, a, fac, p)
    dy = torch.randn(M, H, generator=g0).to(DEV).bfloat16()
    wo = (torch.randn(H, F, generator=g0) * 0.05).to(DEV).bfloat16()
    dg = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_geglu_linear_dgrad", dy.data_ptr(), wo.data_ptr(), fac.data_ptr(), M, F, H,
               dg.data_ptr())
    da = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_linear_dgrad", dy.data_ptr(), wo.data_ptr(), M, H, F, da.data_ptr())
    dg2 = torch.empty_like(dg)
    _gemm_call("dna_geglu_bwd", da.data_ptr(), fac.data_ptr(), 1, M, F, dg2.data_ptr())
    assert torch.equal(dg, dg2)


def _geglu_factors_match(g, a, fac, p):
    """fac = [k s g2 gelu'(g1) | k s gelu(g1)] (k = a's keep bit, s = 1 / (1 - p)) vs fp32 torch's
    GELU and its autograd derivative on the same bf16 g, to bf16 rounding."""
    F = a.shape[1]
    h1, h2 = g[:, :F].float(), g[:, F:].float()
    kept = (a != 0).float() / (1.0 - p) if p > 0 else torch.ones_like(h1)
    x1 = h1.clone().requires_grad_(True)
    torch.nn.functional.gelu(x1).sum().backward()
    want1, want2 = h2 * x1.grad * kept, torch.nn.functional.gelu(h1) * kept
    got1, got2 = fac[:, :F].float(), fac[:, F:].float()
    assert (got1 - want1).abs().max().item() <= 8e-3 * want1.abs().max().item()
    assert (got2 - want2).abs().max().item() <= 8e-3 * want2.abs().max().item()
    wa = torch.nn.functional.gelu(h1) * h2 * kept
    assert (a.float() - wa).abs().max().item() <= 8e-3 * wa.abs().max().item()


@pytest.mark.parametrize("M", [1, 255, 257, 300, 1000])
@pytest.mark.parametrize("kind", ["fwd", "geglu"])
def test_gemm_persistent_ragged_rows_write_nothing_past_m(M, kind):
    """Canary for the persistent kernel's ragged last tile: the output is a view at the head of a
    NaN-filled buffer and the operand rows past M are NaN; every row < M equals fp32 torch, and
    not one element after the M output rows changes (rows past M fall out of the buffer
    resource's range check -- loads read zero, stores are dropped)."""
    g = torch.Generator(device="cpu").manual_seed(M)
    K, N, F = 768, 768, 3072
    xb = torch.full((M + 256, K), float("nan"), device=DEV, dtype=torch.bfloat16)
    xb[:M] = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    x = xb[:M]
    if kind == "fwd":
        w = (torch.randn(N, K, generator=g) * 0.05).to(DEV).bfloat16()
        b = torch.randn(N, generator=g).to(DEV)
        buf = torch.full((M + 512, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        _gemm_call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr(), M, N, K, buf.data_ptr())
        torch.cuda.synchronize()
        assert _rel(buf[:M], x.float() @ w.float().t() + b) < 1e-2
        assert torch.isnan(buf[M:]).all()
    else:
        wg = (torch.randn(2 * F, K, generator=g) * 0.05).to(DEV).bfloat16()
        bg = (torch.randn(2 * F, generator=g) * 0.1).to(DEV)
        gbuf = torch.full((M + 512, 2 * F), float("nan"), device=DEV, dtype=torch.bfloat16)
        abuf = torch.full((M + 512, F), float("nan"), device=DEV, dtype=torch.bfloat16)
        _gemm_call("dna_geglu_linear_fwd", x.data_ptr(), wg.data_ptr(), bg.data_ptr(), M, F, K, 0.0,
                   1, 0, gbuf.data_ptr(), abuf.data_ptr())
        torch.cuda.synchronize()
        assert torch.isnan(gbuf[M:]).all() and torch.isnan(abuf[M:]).all()
        assert not torch.isnan(abuf[:M]).any() and not torch.isnan(gbuf[:M]).any()
        g = (x.float() @ wg.float().t() + bg).bfloat16()  # the factors of fp32 torch's g
        _geglu_factors_match(g, abuf[:M], gbuf[:M], 0.0)


# ------------------------------------------------------------------ bench-shape GEMM parity
BENCH_T = 512 * 512  # per-GPU batch 512 x S 512 tokens (bench.py default)


def _sample_rows(M, n=384, seed=0):
    g = torch.Generator().manual_seed(seed)
    rows = torch.randint(0, M, (n,), generator=g)
    return torch.cat([rows, torch.tensor([0, 1, 255, 256, M // 2 - 1, M // 2, M - 2, M - 1])]).to(DEV)


def test_gemm_bench_shape_gated_fwd_and_k6144_dgrad():
    """The two row-blocked calls of the step at T = 262,144 (operands past 2^31 bytes): the
    gated_layers forward (N = 6144, K = 768) and its data gradient (K = 6144 on the transposed
    weight), on sampled rows (incl. both sides of the row-block boundary) vs fp32 torch."""
    T, F2, H = BENCH_T, 6144, 768
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(T, H, device=DEV, generator=g).bfloat16()
    w = (torch.randn(F2, H, device=DEV, generator=g) * 0.05).bfloat16()
    y = torch.empty(T, F2, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), None, T, F2, H, y.data_ptr())
    mc = ((1 << 31) - 1) // (F2 * 2) // 256 * 256
    rows = torch.cat([_sample_rows(T), torch.tensor([mc - 1, mc, mc + 1], device=DEV)])
    assert _rel(y[rows], x[rows].float() @ w.float().t()) < 1e-2
    del y
    dy = torch.randn(T, F2, device=DEV, generator=g).bfloat16()
    wt = w.t().contiguous()  # [768, 6144]: the transposed bf16 copy FlatParams keeps
    dx = torch.empty(T, H, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_linear_fwd", dy.data_ptr(), wt.data_ptr(), None, T, H, F2, dx.data_ptr())
    assert _rel(dx[rows], dy[rows].float() @ w.float()) < 1e-2


def test_gemm_geglu_fused_bench_shape_row_blocks():
    """The fused gated_layers GEMM + GeGLU forward at T = 262,144 (g is 3.2 GB: two row-block
    launches, the dropout counter advanced per block) equals the unfused pair bit for bit: g vs
    dna_linear_fwd, a vs dna_geglu_fwd on that g, incl. rows on both sides of the block seam."""
    T, F, H = BENCH_T, 3072, 768
    g0 = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(T, H, device=DEV, generator=g0).bfloat16()
    w = (torch.randn(2 * F, H, device=DEV, generator=g0) * 0.05).bfloat16()
    fac = torch.empty(T, 2 * F, device=DEV, dtype=torch.bfloat16)
    a = torch.empty(T, F, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_geglu_linear_fwd", x.data_ptr(), w.data_ptr(), None, T, F, H, 0.1, 123, 77,
               fac.data_ptr(), a.data_ptr())
    g = torch.empty_like(fac)
    _gemm_call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), None, T, 2 * F, H, g.data_ptr())
    a2 = torch.empty_like(a)
    _gemm_call("dna_geglu_fwd", g.data_ptr(), 1, T, F, 0.1, 123, 77, a2.data_ptr(), g.data_ptr())
    assert torch.equal(a, a2)
    assert torch.equal(fac, g)  # the factors, written over g in place


def _geglu_dgrad_pair(dy, wt, fac, M, F, H):
    """The unfused pair the fused kernel replaces: da = dy . wt^T (dna_linear_fwd, the dgrad
    through the transposed copy), then dg = dna_geglu_bwd(da, fac)."""
    da = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_linear_fwd", dy.data_ptr(), wt.data_ptr(), None, M, F, H, da.data_ptr())
    dg = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_geglu_bwd", da.data_ptr(), fac.data_ptr(), 1, M, F, dg.data_ptr())
    return dg


def _random_factors(M, F, gen):
    """GeGLU backward factors as a dropout-on forward leaves them: random, ~10 % exact zeros."""
    fac = torch.randn(M, 2 * F, generator=gen)
    drop = torch.rand(M, F, generator=gen) < 0.1
    fac[:, :F][drop] = 0.0
    fac[:, F:][drop] = 0.0
    return fac.to(DEV).bfloat16()


@pytest.mark.parametrize("M", [1, 257, 1000, 4096])
def test_gemm_geglu_dgrad_p_equals_pair_and_writes_nothing_past_m(M):
    """wo's data gradient with the GeGLU backward in the persistent kernel's epilogue
    (dna_geglu_linear_dgrad_p: dg = bf16(da) * fac) equals the separate pair bit for bit; the
    output is the head of a NaN-filled buffer and fac's rows past M are NaN: rows past M read as
    zero and are never written."""
    F, H = 3072, 768
    gen = torch.Generator(device="cpu").manual_seed(M)
    dy = torch.randn(M, H, generator=gen).to(DEV).bfloat16()
    wt = (torch.randn(F, H, generator=gen) * 0.05).to(DEV).bfloat16()
    gb = torch.full((M + 256, 2 * F), float("nan"), device=DEV, dtype=torch.bfloat16)
    gb[:M] = _random_factors(M, F, gen)
    g = gb[:M]
    dgb = torch.full((M + 256, 2 * F), float("nan"), device=DEV, dtype=torch.bfloat16)
    _gemm_call("dna_geglu_linear_dgrad_p", dy.data_ptr(), wt.data_ptr(), g.data_ptr(), M, F, H,
               dgb.data_ptr())
    torch.cuda.synchronize()
    ref = _geglu_dgrad_pair(dy, wt, g, M, F, H)
    assert torch.equal(dgb[:M], ref)
    assert torch.isnan(dgb[M:]).all()


def test_gemm_geglu_dgrad_p_bench_shape_row_blocks():
    """The fused wo dgrad + GeGLU backward at T = 262,144 (fac / dg are 3.2 GB: two row-block
    launches) equals the separate pair bit for bit, incl. the rows on both sides of the block
    seam, and, with the factors of a dropout-off forward on random g, matches the fp32 GeGLU
    backward (erf GELU and its derivative) on sampled rows."""
    T, F, H = BENCH_T, 3072, 768
    gen = torch.Generator(device=DEV).manual_seed(5)
    dy = torch.randn(T, H, device=DEV, generator=gen).bfloat16()
    wt = (torch.randn(F, H, device=DEV, generator=gen) * 0.05).bfloat16()
    g = torch.randn(T, 2 * F, device=DEV, generator=gen).bfloat16()
    a = torch.empty(T, F, device=DEV, dtype=torch.bfloat16)
    fac = torch.empty_like(g)
    _gemm_call("dna_geglu_fwd", g.data_ptr(), 1, T, F, 0.0, 0, 0, a.data_ptr(), fac.data_ptr())
    del a
    dg = torch.empty_like(g)
    _gemm_call("dna_geglu_linear_dgrad_p", dy.data_ptr(), wt.data_ptr(), fac.data_ptr(), T, F, H,
               dg.data_ptr())
    ref = _geglu_dgrad_pair(dy, wt, fac, T, F, H)
    assert torch.equal(dg, ref)
    del ref
    # fp32 restatement on sampled rows (bf16 da rounding as the reference's bf16 step)
    mc = ((1 << 31) - 1) // (2 * F * 2) // 256 * 256
    rows = torch.cat([_sample_rows(T), torch.tensor([mc - 1, mc, mc + 1], device=DEV)])
    da = dy[rows].float() @ wt.float().t()
    g1, g2 = g[rows, :F].float(), g[rows, F:].float()
    cdf = 0.5 * (1 + torch.erf(g1 / math.sqrt(2)))
    gelu = g1 * cdf
    dgelu = cdf + g1 * torch.exp(-0.5 * g1 * g1) / math.sqrt(2 * math.pi)
    want = torch.cat([da * g2 * dgelu, da * gelu], 1)
    assert _rel(dg[rows], want) < 1e-2


@pytest.mark.parametrize("n,k", [(2304, 768), (768, 768), (6144, 768), (768, 3072)])
def test_wgrad_p_bench_shapes(n, k):
    """dna_linear_wgrad_p (the hand-written token-major weight gradient, fp32 chunk partials +
    dna_sum_slices_accum) at the step's four projection shapes and T = 262,144 vs fp32 torch,
    and accumulating into an existing gradient; plus a ragged T."""
    from dna_amd import functional as DF
    for T in (BENCH_T, 100_003):
        g = torch.Generator(device=DEV).manual_seed(n + k + T)
        dy = torch.randn(T, n, device=DEV, generator=g).bfloat16()
        x = torch.randn(T, k, device=DEV, generator=g).bfloat16()
        ref = dy.float().t() @ x.float()
        prev = torch.randn(n, k, device=DEV, generator=g)
        grad = prev.clone()
        parts, s = DF._hip_wgrad_parts(dy, x)
        assert s >= 1 and parts.shape == (s, n, k)
        from dna_amd import _native as N
        N.call("dna_sum_slices_accum", parts.data_ptr(), s, n * k, grad.data_ptr(), N.stream_ptr())
        assert _rel(grad - prev, ref) < 1e-5, (T, s)


@pytest.mark.parametrize("M,N,K", [(1024, 2304, 768), (1000, 768, 3072), (777, 4096, 768),
                                   (129, 192, 64), (3, 5, 7), (0, 64, 64), (515, 130, 33)])
def test_gemm_f32_fwd_dgrad_wgrad_vs_fp64(M, N, K):
    """Exact-fp32 MFMA projections (csrc/gemm_f32.hip) vs float64 torch: forward with bias,
    data gradient, weight-gradient slices + dna_sum_slices_accum, at the model's shapes and at
    ragged / tiny / misaligned ones (odd leading dimensions take the scalar load path). The
    kernel is a k-ordered fp32 fma chain: error <= 1e-6 relative to sum |a.b|."""
    from dna_amd import functional as DF
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device=DEV, generator=g)
    w = torch.randn(N, K, device=DEV, generator=g)
    b = torch.randn(N, device=DEV, generator=g)
    dy = torch.randn(M, N, device=DEV, generator=g)

    def close(got, ref, a, bm):
        scale = (a.abs().double() @ bm.abs().double()).max().item() if a.numel() and bm.numel() else 1.0
        assert got.shape == ref.shape
        if got.numel():
            assert (got.double() - ref).abs().max().item() <= 1e-6 * max(scale, 1.0)
    y = DF._hip_linear_f32(x, w, b)
    close(y, x.double() @ w.double().t() + b.double(), x, w.t())
    dx = DF._hip_dgrad_f32(dy, w)
    close(dx, dy.double() @ w.double(), dy, w)
    dw = DF.wgrad(dy, x)
    close(dw, dy.double().t() @ x.double(), dy.t(), x)
    grad = torch.randn(N, K, device=DEV, generator=g)
    prev = grad.clone()
    parts, s = DF._hip_wgrad_f32_parts(dy, x)
    assert parts.shape == (s, N, K)
    from dna_amd import _native as NN
    NN.call("dna_sum_slices_accum", parts.data_ptr(), s, N * K, grad.data_ptr(), NN.stream_ptr())
    close(grad - prev, dy.double().t() @ x.double(), dy.t(), x)


@pytest.mark.parametrize("rows", [0, 1, 64, 65, 127, 128, 129])
def test_wgrad_few_rows(rows):
    """Weight gradients over a handful of rows (the MLM head's masked rows of a tiny micro-batch,
    or none): DF.wgrad / wgrad_accumulate take the torch split-K path below two 64-row K-steps
    and the hand-written kernel from 128 rows; both equal fp32 torch."""
    from dna_amd import functional as DF
    n, k = 256, 768
    g = torch.Generator(device=DEV).manual_seed(rows)
    dy = torch.randn(rows, n, device=DEV, generator=g).bfloat16()
    x = torch.randn(rows, k, device=DEV, generator=g).bfloat16()
    ref = dy.float().t() @ x.float()
    assert DF._hip_wgrad_ok(dy, x) == (rows >= 128)
    out = DF.wgrad(dy, x)
    assert out.shape == (n, k) and out.dtype == torch.float32
    assert (out - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())
    prev = torch.randn(n, k, device=DEV, generator=g)
    grad = prev.clone()
    DF.wgrad_accumulate(dy, x, grad)
    assert (grad - prev - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("V", [4096, 1000])
def test_masked_cross_entropy_fwd_bwd_vs_torch(V):
    """MaskedCrossEntropy (csrc/xent.hip; V = 4096 bf16 takes the one-read vector kernels) vs
    fp32 torch cross entropy on the same bf16 logits: loss and dlogits."""
    from dna_amd import functional as DF
    g = torch.Generator().manual_seed(V)
    M = 777
    logits = (torch.randn(M, V, generator=g) * 3).to(DEV).bfloat16().requires_grad_(True)
    tgt = torch.randint(0, V, (M,), generator=g).to(DEV)
    loss = DF.MaskedCrossEntropy.apply(logits, tgt, 500.0)
    loss.backward()
    l32 = logits.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(l32, tgt, reduction="sum") / 500.0
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    assert (logits.grad.float() - l32.grad).abs().max().item() <= 1e-2 * l32.grad.abs().max().item()


@pytest.mark.parametrize("M,F,Nn", [(5000, 1024, 256), (131072, 1024, 256), (700, 256, 256)])
def test_gelu_linear_fused_bwd_vs_separate(M, F, Nn):
    """functional.GeluLinear (fc2 of the HyenaDNA Mlp: tanh-GELU + Linear, the GELU backward in
    the data-gradient epilogue) against the separate torch GELU + HIP Linear nodes on the same
    bf16 operands: same forward (bit-equal), dh within bf16 rounding of the unfused dh (da is
    rounded to bf16 in both), weight / bias gradients equal."""
    from dna_amd import functional as DF
    from dna_amd.hyena import hip_linear
    g = torch.Generator(device="cpu").manual_seed(M + F)
    h = (torch.randn(M, F, generator=g) * 2).to(DEV).bfloat16()
    w = (torch.randn(Nn, F, generator=g) / F ** 0.5).to(DEV)
    b = torch.randn(Nn, generator=g).to(DEV) * 0.1
    do = torch.randn(M, Nn, generator=g).to(DEV).bfloat16()
    outs = []
    for fused in (True, False):
        hh = h.clone().requires_grad_(True)
        ww = w.clone().requires_grad_(True)
        bb = b.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if fused:
                assert DF.gelu_linear_ok(hh, ww)
                o = DF.gelu_linear(hh, ww, bb)
            else:
                o = hip_linear(torch.nn.functional.gelu(hh, approximate="tanh"), ww, bb)
        o.backward(do)
        outs.append((o.detach(), hh.grad, ww.grad, bb.grad))
    (o1, dh1, dw1, db1), (o2, dh2, dw2, db2) = outs
    assert torch.equal(o1, o2)
    assert dh1.dtype == torch.bfloat16 and torch.isfinite(dh1.float()).all()
    err = (dh1.float() - dh2.float()).abs().max().item()
    assert err <= 1e-2 * dh2.float().abs().max().item(), err
    assert torch.allclose(dw1, dw2, rtol=1e-5, atol=1e-5) and torch.allclose(db1, db2, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,K,Nn", [(5000, 256, 1024), (131072, 256, 1024), (700, 128, 256)])
def test_linear_gelu_fwd_vs_separate(M, K, Nn):
    """dna_linear_gelu_fwd (fc1 + tanh-GELU of the HyenaDNA Mlp in one persistent-GEMM launch):
    h bit-equal to dna_linear_fwd on the same operands; act = gelu_tanh(h) of the bf16 h within
    one bf16 rounding step of torch's GELU (the kernel evaluates x / (1 + exp(-2u)) with the
    hardware exp / rcp, so a handful of elements round the other way), plus 1e-6 |h| where
    torch's 0.5 x (1 + tanh(u)) cancels for u << 0 (it returns 0 where the kernel keeps the
    ~1e-7 tail)."""
    from dna_amd import functional as DF
    g = torch.Generator(device="cpu").manual_seed(M + K)
    x = torch.randn(M, K, generator=g).to(DEV).bfloat16()
    w = (torch.randn(Nn, K, generator=g) / K ** 0.5).to(DEV).bfloat16()
    b = (torch.randn(Nn, generator=g) * 0.1).to(DEV)
    h_ref = DF._hip_linear(x, w, b)
    h, act = DF._hip_linear_gelu(x, w, b)
    assert torch.equal(h, h_ref)
    a_ref = torch.nn.functional.gelu(h_ref, approximate="tanh")
    d = (act.float() - a_ref.float()).abs()
    tol = a_ref.float().abs() * 2.0 ** -7 + 1e-6 * h_ref.float().abs()
    assert (d <= tol).all(), (d - tol).max().item()
    assert (act != a_ref).float().mean().item() < 1e-3


def test_mlp_fc1_gelu_fused_vs_unfused(monkeypatch):
    """hyena_lm.Mlp under bf16 autocast with fc1's GELU in the GEMM epilogue
    (DNA_GELU_FC1_FUSED=1, default) against torch's separate GELU pass (=0): output and every
    parameter / input gradient within bf16 rounding of each other."""
    from dna_amd.hyena_lm import Mlp
    torch.manual_seed(0)
    m = Mlp(256, 1024).to(DEV)
    x = torch.randn(4, 2048, 256, device=DEV)
    dy = torch.randn(4, 2048, 256, device=DEV)
    res = []
    for fused in ("1", "0"):
        monkeypatch.setenv("DNA_GELU_FC1_FUSED", fused)
        m.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(xx)
        y.float().backward(dy)
        res.append((y.detach().float(), xx.grad, [p.grad.clone() for p in m.parameters()]))
    (y1, dx1, g1), (y2, dx2, g2) = res
    rel = lambda a, b: (a - b).abs().max().item() / max(b.abs().max().item(), 1e-12)
    assert rel(y1, y2) < 2e-2
    assert rel(dx1, dx2) < 2e-2
    for a, b in zip(g1, g2):
        assert rel(a, b) < 2e-2
