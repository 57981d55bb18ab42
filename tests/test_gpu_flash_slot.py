"""The flash_attn_qkvpacked_func slot with the reference's signature (flash_attn_triton.py:
1077-1130; dna_amd.ops.flash_attn_qkvpacked_func -> csrc/flash_slot.hip), called exactly as the
reference call site does (bert_layers.py:188: flash_attn_qkvpacked_func(qkv, bias) with the bias
BertEncoder.forward builds, :421-448, pads included), against the PyTorch attention path it
replaces (bert_layers.py:167-178) in fp32 on the same bf16/fp16 operands -- forward, LSE and the
dqkv backward; plus the Triton slot's other modes: causal, "vector" bias, broadcast batch/head
dims, fp16 and bf16 bias, ragged S, head_dim 32/128 and a padded 80. GPU."""
import math

import pytest
import torch

from oracle import bert_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _torch_path(qkv, bias, causal, scale):
    """bert_layers.py:167-178 (plus the Triton slot's causal mask), fp32."""
    q, k, v = qkv.float().unbind(2)                      # [b, S, H, D]
    q, k, v = (t.permute(0, 2, 1, 3) for t in (q, k, v))  # [b, H, S, D]
    s = q @ k.transpose(-1, -2) * scale
    if bias is not None:
        s = s + bias.float()
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    return (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3), lse


def _check(b, S, H, D, dtype, bias, causal, tol_o=2.5e-2, tol_g=3e-2, seed=0):
    from dna_amd.ops import flash_attn_qkvpacked_func
    g = torch.Generator().manual_seed(seed)
    qkv = (torch.randn(b, S, 3, H, D, generator=g) * 0.7).to(DEV, dtype).requires_grad_(True)
    scale = 1.0 / math.sqrt(D)
    out = flash_attn_qkvpacked_func(qkv, bias, causal)
    assert out.shape == (b, S, H, D) and out.dtype == dtype
    x32 = qkv.detach().float().requires_grad_(True)
    ref, lse_ref = _torch_path(x32, bias, causal, scale)
    err = (out.float() - ref).abs().max().item()
    assert err < tol_o, err
    _, lse = torch.ops.dna_amd.flash_attn_qkvpacked(qkv.detach(), bias, causal, None)
    assert lse.shape == (b, H, (S + 127) // 128 * 128)
    assert (lse[..., :S] - lse_ref).abs().max().item() < 1e-2
    dout = torch.randn(out.shape, generator=g).to(DEV, dtype)
    out.backward(dout)
    ref.backward(dout.float())
    rel = float((qkv.grad.float() - x32.grad).norm() / x32.grad.norm())
    assert rel < tol_g, rel
    for t in range(3):  # q, k and v gradients each (S = 1: softmax == 1, dq == dk == 0 exactly)
        ref_n = float(x32.grad[:, :, t].norm())
        diff = float((qkv.grad[:, :, t].float() - x32.grad[:, :, t]).norm())
        assert diff <= tol_g * ref_n + 1e-6, (t, diff, ref_n)


def test_reference_call_site_dnabert2_bias_with_pads():
    """flash_attn_qkvpacked_func(qkv, bias): qkv bf16 [b, S, 3, 12, 64], bias fp32 [b, 12, S, S]
    = ALiBi + (1 - mask) * -10000 from the reference construction (oracle/bert_ref.attention_bias)."""
    b, S, H = 3, 256, 12
    valid = torch.ones(b, S, dtype=torch.bool)
    valid[1, 200:] = False
    valid[2, 17:] = False
    bias = bert_ref.attention_bias(valid, H).to(DEV)
    assert bias.shape == (b, H, S, S) and bias.dtype == torch.float32
    _check(b, S, H, 64, torch.bfloat16, bias, False)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("mode", ["none", "vector", "matrix", "matrix_b1", "vector_11", "matrix_lp"])
def test_slot_modes(dtype, causal, mode):
    b, S, H, D = 2, 192, 4, 64
    g = torch.Generator().manual_seed(7)
    bias = {
        "none": None,
        "vector": torch.randn(b, H, 1, S, generator=g),
        "matrix": torch.randn(b, H, S, S, generator=g),
        "matrix_b1": torch.randn(1, H, S, S, generator=g),  # broadcast over batch
        "vector_11": torch.randn(1, 1, 1, S, generator=g),  # broadcast over batch and heads
        "matrix_lp": torch.randn(b, 1, S, S, generator=g),  # qkv-dtype bias, head broadcast
    }[mode]
    if bias is not None:
        bias = bias.to(DEV, dtype if mode == "matrix_lp" else torch.float32)
    _check(b, S, H, D, dtype, bias, causal, tol_o=1e-2 if dtype == torch.float16 else 2.5e-2)


@pytest.mark.parametrize("S,D", [(100, 64), (1, 64), (333, 32), (130, 128), (200, 80)])
def test_slot_ragged_seqlen_and_head_dims(S, D):
    g = torch.Generator().manual_seed(S + D)
    bias = torch.randn(2, 2, S, S, generator=g).to(DEV)
    _check(2, S, 2, D, torch.bfloat16, bias, S % 2 == 0)


def test_slot_rejects_what_the_reference_rejects():
    from dna_amd.ops import flash_attn_qkvpacked_func
    qkv = torch.zeros(2, 64, 3, 4, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="fp16 and bf16"):
        flash_attn_qkvpacked_func(qkv.float())
    with pytest.raises(RuntimeError, match="Last 2 dimensions"):
        flash_attn_qkvpacked_func(qkv, torch.zeros(2, 4, 2, 64, device=DEV))
    with pytest.raises(RuntimeError, match="broadcastible"):
        flash_attn_qkvpacked_func(qkv, torch.zeros(3, 4, 64, 64, device=DEV))
    with pytest.raises(RuntimeError, match="up to 128"):
        flash_attn_qkvpacked_func(torch.zeros(2, 64, 3, 4, 160, device=DEV, dtype=torch.bfloat16))
    bias = torch.zeros(2, 4, 64, 64, device=DEV, requires_grad=True)
    out = flash_attn_qkvpacked_func(qkv.clone().requires_grad_(True), bias)
    with pytest.raises(RuntimeError, match="bias gradient"):
        out.sum().backward()


def test_slot_deterministic():
    from dna_amd.ops import flash_attn_qkvpacked_func
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 256, 3, 4, 64, generator=g).to(DEV, torch.bfloat16)
    bias = torch.randn(2, 4, 256, 256, generator=g).to(DEV)
    grads = []
    for _ in range(2):
        q = x.clone().requires_grad_(True)
        flash_attn_qkvpacked_func(q, bias, True).float().square().sum().backward()
        grads.append(q.grad)
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("bias_dtype", [torch.float32, torch.bfloat16])
def test_slot_staged_bias_equals_direct_reads(bias_dtype, monkeypatch):
    """A matrix bias with 16-B aligned rows is staged through LDS one 64 x 64 tile at a time
    (16-B loads); DNA_FLASH_BIAS_DIRECT=1 reads it per score from global memory. The same fp32
    bias values enter the same arithmetic (the compiler may contract the score's multiply-adds
    differently in the two instantiations: equal to rounding); ragged S (last tile partly past S),
    causal."""
    from dna_amd.ops import flash_attn_qkvpacked_func
    g = torch.Generator().manual_seed(11)
    b, S, H, D = 2, 200, 3, 64
    x = (torch.randn(b, S, 3, H, D, generator=g) * 0.7).to(DEV, torch.bfloat16)
    bias = torch.randn(b, H, S, S, generator=g).to(DEV, bias_dtype)
    dout = torch.randn(b, S, H, D, generator=g).to(DEV, torch.bfloat16)
    res = []
    for direct in ("0", "1"):
        monkeypatch.setenv("DNA_FLASH_BIAS_DIRECT", direct)
        q = x.clone().requires_grad_(True)
        out = flash_attn_qkvpacked_func(q, bias, True)
        _, lse = torch.ops.dna_amd.flash_attn_qkvpacked(x, bias, True, None)
        out.backward(dout)
        res.append((out.detach(), lse, q.grad))
    (o0, l0, g0), (o1, l1, g1) = res
    assert (o0.float() - o1.float()).abs().max().item() <= 1e-2 * o1.float().abs().max().item()
    assert (l0[..., :S] - l1[..., :S]).abs().max().item() < 1e-4  # rows past S are padding
    assert float((g0.float() - g1.float()).norm() / g1.float().norm()) < 2e-3
