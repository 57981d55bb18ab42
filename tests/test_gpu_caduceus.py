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


@pytest.mark.parametrize("d_model", [24, 40])
def test_caduceus_odd_d_inner_autocast(d_model):
    """d_inner = 2 * d_model not a multiple of 32 (48, 80): in_proj's data gradient cannot take
    the two-operand contraction (it splits K at d_inner in 32-deep steps), so it runs on the
    concatenated operand. bf16-autocast gradients vs the fp32 run of the same model."""
    from dna_amd.caduceus import CaduceusForMaskedLM
    torch.manual_seed(11)
    m = CaduceusForMaskedLM(d_model=d_model, n_layer=2, vocab_size=12,
                            ssm_cfg={"d_state": 16}).to(DEV)
    ids = torch.randint(0, 12, (2, 256), device=DEV, generator=torch.Generator(DEV).manual_seed(2))
    grads = []
    for ac in (False, True):
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
            _, logits = m(ids)
        loss = torch.nn.functional.cross_entropy(logits.float().reshape(-1, logits.shape[-1]),
                                                 ids.reshape(-1))
        loss.backward()
        grads.append({n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                      if p.grad is not None})
    assert any("in_proj" in n for n in grads[1])
    for n, g in grads[0].items():
        assert torch.isfinite(grads[1][n]).all(), n
        assert _rel(grads[1][n], g) < 6e-2, n


@pytest.mark.parametrize("autocast", [True, False])
def test_caduceus_model_has_no_library_gemm(autocast, monkeypatch):
    """Config E's model (bidirectional Mamba mixer: in_proj, x_proj, dt_proj, out_proj, the LM
    head) runs forward and backward with every torch GEMM entry point banned, under bf16 autocast
    and in fp32: the Mamba in_proj / out_proj products (forward, data and weight gradients) run on
    the strided MFMA GEMM, none on hipBLASLt / rocBLAS (VERDICT r4 missing 2)."""
    from test_gpu_model import _ban_library_gemm
    from dna_amd.caduceus import CaduceusForMaskedLM
    torch.manual_seed(5)
    m = CaduceusForMaskedLM(d_model=64, n_layer=2, vocab_size=12,
                            ssm_cfg={"d_state": 16}).to(DEV)
    ids = torch.randint(0, 12, (2, 512), device=DEV)
    with monkeypatch.context() as mp:
        _ban_library_gemm(mp)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            _, logits = m(ids)
        loss = torch.nn.functional.cross_entropy(logits.float().reshape(-1, logits.shape[-1]),
                                                 ids.reshape(-1))
        loss.backward()
    assert torch.isfinite(loss)
    grads = {n: p.grad for n, p in m.named_parameters() if p.grad is not None}
    assert any("in_proj" in n for n in grads) and any("out_proj" in n for n in grads)
    assert all(torch.isfinite(g).all() for g in grads.values())


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


# ---- RCPS layers pinned to the reference module (tests/golden/rcps_golden.npz, made from
# /root/reference/src/models/caduceus/modeling_rcps.py by tests/golden/make_rcps_golden.py):
# dna_amd.caduceus' RCPS classes over the HIP embedding / LayerNorm / MFMA-GEMM Linear, fp32
# (tolerance 1e-5 relative to the largest reference value) and under bf16 autocast (3e-2)
import os  # noqa: E402

import numpy as np  # noqa: E402

_Z = np.load(os.path.join(os.path.dirname(__file__), "golden", "rcps_golden.npz"))


def _zt(k, dtype=torch.float32, grad=False):
    return torch.tensor(_Z[k]).to(DEV, dtype).requires_grad_(grad)


def _tol(autocast):
    return 3e-2 if autocast else 1e-5


def _ctx(autocast):
    return torch.autocast("cuda", dtype=torch.bfloat16) if autocast else torch.autocast("cuda", enabled=False)


def _set_params(mod, **vals):
    with torch.no_grad():
        for name, v in vals.items():
            mod.get_parameter(name).copy_(torch.tensor(_Z[v]))


@pytest.mark.parametrize("autocast", [False, True])
def test_rcps_embedding_vs_reference(autocast):
    from dna_amd.caduceus import RCPSEmbedding
    V, D = _Z["emb_W"].shape
    m = RCPSEmbedding(V, D, {i: int(c) for i, c in enumerate(_Z["complement"])}).to(DEV)
    _set_params(m, **{"embedding.weight": "emb_W"})
    with _ctx(autocast):
        y = m(torch.tensor(_Z["emb_ids"]).to(DEV))
    assert _rel(y, torch.tensor(_Z["emb_out"])) < 1e-6  # a gather: exact in fp32
    y.float().backward(_zt("emb_gout"))
    assert _rel(m.embedding.weight.grad, torch.tensor(_Z["emb_dW"])) < 1e-5


@pytest.mark.parametrize("autocast", [False, True])
def test_rcps_wrapper_vs_reference(autocast):
    from dna_amd.caduceus import RCPSWrapper
    from dna_amd.hyena import HipLinear
    D = _Z["wrap_W"].shape[0]
    lin = HipLinear(D, D).to(DEV)
    _set_params(lin, weight="wrap_W", bias="wrap_b")
    x = _zt("wrap_x", grad=True)
    with _ctx(autocast):
        y = RCPSWrapper(lin)(x)
    tol = _tol(autocast)
    assert _rel(y, torch.tensor(_Z["wrap_out"])) < tol
    y.float().backward(_zt("wrap_gout"))
    for t, k in ((x, "wrap_dx"), (lin.weight, "wrap_dW"), (lin.bias, "wrap_db")):
        assert _rel(t.grad, torch.tensor(_Z[k])) < tol, k


@pytest.mark.parametrize("tag", ["an0", "an"])
@pytest.mark.parametrize("autocast", [False, True])
def test_rcps_add_norm_vs_reference(tag, autocast):
    from dna_amd.caduceus import RCPSAddNormWrapper
    from dna_amd.hyena_lm import LayerNorm
    D = _Z[f"{tag}_g"].shape[0]
    ln = LayerNorm(D).to(DEV)
    _set_params(ln, weight=f"{tag}_g", bias=f"{tag}_beta")
    x = _zt(f"{tag}_x", grad=True)
    res = _zt(f"{tag}_res", grad=True) if f"{tag}_res" in _Z else None
    with _ctx(autocast):
        y, r = RCPSAddNormWrapper(ln)(x, residual=res, prenorm=True)
    tol = _tol(autocast)
    assert _rel(y, torch.tensor(_Z[f"{tag}_y"])) < tol
    assert _rel(r, torch.tensor(_Z[f"{tag}_res_out"])) < 1e-6
    torch.autograd.backward([y.float(), r.float()], [_zt(f"{tag}_gy"), _zt(f"{tag}_gres")])
    checks = [(x, "dx"), (ln.weight, "dg"), (ln.bias, "dbeta")] + ([(res, "dres")] if res is not None else [])
    for t, k in checks:
        assert _rel(t.grad, torch.tensor(_Z[f"{tag}_{k}"])) < tol, k


@pytest.mark.parametrize("tag", ["blk0", "blk"])
@pytest.mark.parametrize("autocast", [False, True])
def test_rcps_block_vs_reference(tag, autocast):
    """RCPSMambaBlock(fused_add_norm=False, residual_in_fp32=True) with a Linear mixer."""
    from dna_amd.caduceus import RCPSMambaBlock
    from dna_amd.hyena import HipLinear
    from dna_amd.hyena_lm import LayerNorm
    D = _Z[f"{tag}_norm_g"].shape[0]
    ln, mix = LayerNorm(D).to(DEV), HipLinear(D, D).to(DEV)
    _set_params(ln, weight=f"{tag}_norm_g", bias=f"{tag}_norm_b")
    _set_params(mix, weight=f"{tag}_mix_W", bias=f"{tag}_mix_b")
    blk = RCPSMambaBlock(D, mix, ln, fused_add_norm=False, residual_in_fp32=True)
    h = _zt(f"{tag}_h", grad=True)
    res = _zt(f"{tag}_res", grad=True) if f"{tag}_res" in _Z else None
    with _ctx(autocast):
        hh, rr = blk(h, residual=res)
    tol = _tol(autocast)
    assert rr.dtype == torch.float32
    assert _rel(hh, torch.tensor(_Z[f"{tag}_h_out"])) < tol
    assert _rel(rr, torch.tensor(_Z[f"{tag}_res_out"])) < 1e-6
    torch.autograd.backward([hh.float(), rr], [_zt(f"{tag}_gh"), _zt(f"{tag}_gres")])
    checks = [(h, "dh"), (ln.weight, "dnorm_g"), (ln.bias, "dnorm_b"), (mix.weight, "dmix_W"),
              (mix.bias, "dmix_b")] + ([(res, "dres")] if res is not None else [])
    for t, k in checks:
        assert _rel(t.grad, torch.tensor(_Z[f"{tag}_{k}"])) < tol, k


@pytest.mark.parametrize("autocast", [False, True])
def test_rcps_lm_head_vs_reference(autocast):
    from dna_amd.caduceus import RCPSLMHead
    V, D = _Z["head_W"].shape
    head = RCPSLMHead(D, V, {i: int(c) for i, c in enumerate(_Z["complement"])}).to(DEV)
    _set_params(head, **{"lm_head.weight": "head_W"})
    x = _zt("head_x", grad=True)
    with _ctx(autocast):
        y = head(x)
    tol = _tol(autocast)
    assert _rel(y, torch.tensor(_Z["head_out"])) < tol
    y.float().backward(_zt("head_gout"))
    assert _rel(x.grad, torch.tensor(_Z["head_dx"])) < tol
    assert _rel(head.lm_head.weight.grad, torch.tensor(_Z["head_dW"])) < tol
