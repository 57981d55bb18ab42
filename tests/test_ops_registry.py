"""torch.ops.dna_amd.* -- the operator boundary of SURVEY §8(b) (dna_amd/ops.py).

CPU: every op is registered and rejects CPU tensors with a Python exception (no fallback).
GPU: the registered ops give the same results as the product path's autograd Functions
(dna_amd.functional, which call the same C ABI) and as torch references."""
import math

import pytest
import torch


def test_ops_registered_and_reject_cpu():
    from dna_amd import ops
    for name in ops.OPS:
        assert hasattr(torch.ops.dna_amd, name), name
    x = torch.zeros(4, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="GPU"):
        torch.ops.dna_amd.linear_fwd(x, torch.zeros(8, 64, dtype=torch.bfloat16), None,
                                     torch.zeros(4, 8, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError, match=r"\[b, S, 3, H, D\]"):
        ops.flash_attn_qkvpacked_func(torch.zeros(2, 8, 64), torch.ones(2))


@pytest.mark.gpu
def test_alibi_attn_op_matches_product_attention():
    """The ALiBi fast-path operator (fwd + autograd bwd) == dna_amd.functional.alibi_attention
    on the same packed inputs, bit for bit (same kernels), with pad keys."""
    from dna_amd import functional as DF
    from dna_amd import ops
    from dna_amd.config import alibi_slopes
    b, S, H, D = 2, 256, 4, 64
    g = torch.Generator().manual_seed(3)
    qkv = (torch.randn(b, S, 3, H, D, generator=g) * 0.5).cuda().bfloat16().requires_grad_(True)
    valid = torch.ones(b, S, dtype=torch.bool)
    valid[1, 200:] = False
    valid = valid.cuda()
    slopes = torch.tensor(alibi_slopes(H), dtype=torch.float32).cuda()
    out = ops.alibi_attn_qkvpacked_func(qkv, slopes, valid)
    dout = torch.randn(out.shape, generator=g).cuda().bfloat16()
    out.backward(dout)
    q2 = qkv.detach().clone().view(b * S, 3 * H * D).requires_grad_(True)
    ref = DF.alibi_attention(q2, valid.reshape(-1).to(torch.uint8), slopes, b, S, H)
    ref.backward(dout.view(b * S, H * D))
    assert torch.equal(out.reshape(b * S, H * D), ref)
    assert torch.equal(qkv.grad.reshape(b * S, -1), q2.grad)


@pytest.mark.gpu
def test_linear_geglu_xent_ops_vs_torch():
    from dna_amd import ops  # noqa: F401
    g = torch.Generator().manual_seed(5)
    x = torch.randn(512, 768, generator=g).cuda().bfloat16()
    w = (torch.randn(2304, 768, generator=g) * 0.05).cuda().bfloat16()
    bias = torch.randn(2304, generator=g).cuda()
    y = torch.empty(512, 2304, device="cuda", dtype=torch.bfloat16)
    torch.ops.dna_amd.linear_fwd(x, w, bias, y)
    ref = x.float() @ w.float().t() + bias
    assert float((y.float() - ref).norm() / ref.norm()) < 1e-2
    wt = torch.empty(768, 2304, device="cuda", dtype=torch.bfloat16)
    torch.ops.dna_amd.transpose_bf16(w, wt)
    assert torch.equal(wt, w.t().contiguous())
    gg = torch.randn(256, 2 * 512, generator=g).cuda().bfloat16()
    a = torch.empty(256, 512, device="cuda", dtype=torch.bfloat16)
    torch.ops.dna_amd.geglu_fwd(gg, 0.0, 1, 0, a, torch.empty_like(gg))
    g1, g2 = gg.float().chunk(2, dim=1)
    aref = torch.nn.functional.gelu(g1) * g2
    assert float((a.float() - aref).abs().max()) < 2e-2 * float(aref.abs().max())
    logits = torch.randn(64, 4096, generator=g).cuda().bfloat16()
    tgt = torch.randint(0, 4096, (64,), generator=g).cuda()
    loss = torch.empty(64, device="cuda")
    lse = torch.empty(64, device="cuda")
    torch.ops.dna_amd.xent_fwd(logits, tgt, loss, lse)
    lref = torch.nn.functional.cross_entropy(logits.float(), tgt, reduction="none")
    assert torch.allclose(loss, lref, atol=1e-4, rtol=1e-4)
    assert torch.allclose(lse, torch.logsumexp(logits.float(), 1), atol=1e-4, rtol=1e-5)


@pytest.mark.gpu
def test_fused_geglu_linear_ops_equal_separate_ops():
    """The fused gated_layers + GeGLU forward and wo-dgrad + GeGLU backward operators equal the
    separate linear_fwd / geglu_fwd / geglu_bwd operators bit for bit, dropout on."""
    from dna_amd import ops  # noqa: F401
    g0 = torch.Generator().manual_seed(9)
    M, H, F = 1000, 768, 3072
    x = torch.randn(M, H, generator=g0).cuda().bfloat16()
    wg = (torch.randn(2 * F, H, generator=g0) * 0.05).cuda().bfloat16()
    fac = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    a = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    torch.ops.dna_amd.geglu_linear_fwd(x, wg, None, 0.1, 5, 3, fac, a)
    g2 = torch.empty_like(fac)
    torch.ops.dna_amd.linear_fwd(x, wg, None, g2)
    a2, fac2 = torch.empty_like(a), torch.empty_like(fac)
    torch.ops.dna_amd.geglu_fwd(g2, 0.1, 5, 3, a2, fac2)
    assert torch.equal(fac, fac2) and torch.equal(a, a2)
    # the factors: [keep * s * g2 * gelu'(g1) | keep * s * gelu(g1)], s = 1 / 0.9
    h1, h2 = g2.float().chunk(2, dim=1)
    kept = (a != 0).float() / 0.9
    x1 = h1.clone().requires_grad_(True)
    torch.nn.functional.gelu(x1).sum().backward()
    ref1 = h2 * x1.grad * kept
    ref2 = torch.nn.functional.gelu(h1) * kept
    f1, f2 = fac.float().chunk(2, dim=1)
    assert float((f1 - ref1).abs().max()) <= 1e-2 * float(ref1.abs().max())
    assert float((f2 - ref2).abs().max()) <= 1e-2 * float(ref2.abs().max())
    dy = torch.randn(M, H, generator=g0).cuda().bfloat16()
    wo_t = (torch.randn(F, H, generator=g0) * 0.05).cuda().bfloat16()
    dg = torch.empty_like(fac)
    torch.ops.dna_amd.geglu_linear_dgrad(dy, wo_t, fac, dg)
    da = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    torch.ops.dna_amd.linear_fwd(dy, wo_t, None, da)
    dg2 = torch.empty_like(fac)
    torch.ops.dna_amd.geglu_bwd(da, fac, dg2)
    assert torch.equal(dg, dg2)
