"""Whole-model parity of the HIP path against the reference golden vectors (GPU only).

fp32 mode must match the reference PyTorch forward within 1e-3 (north_star); bf16 mode is the
throughput path (MFMA bf16 GEMMs/attention, fp32 LayerNorm/residual/softmax statistics) and is
held to a bf16 tolerance stated per test.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import bert_ref
from oracle.hashinit import hash_tensor
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _golden(tag):
    z = np.load(os.path.join(GOLDEN, f"model_{tag}.npz"))
    L, d, H, Fd = json.loads(z["config"].tobytes().decode())
    cfg = dict(vocab_size=4096, hidden_size=d, num_hidden_layers=L, num_attention_heads=H,
               intermediate_size=Fd, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.0,
               layer_norm_eps=1e-12, max_position_embeddings=512, type_vocab_size=2,
               pad_token_id=0, alibi_starting_size=512, hidden_act="gelu",
               initializer_range=0.02, hyena_framework=True)
    return z, cfg


def _model(cfg, precision):
    from dna_amd.bert_layers import BertForMaskedLM
    m = BertForMaskedLM(cfg, precision=precision)
    sd = m.state_dict()
    new = {k: torch.from_numpy(hash_tensor(k if k != "cls.predictions.decoder.weight" else
                                           "bert.embeddings.word_embeddings.weight", tuple(v.shape)))
           for k, v in sd.items()}
    m.load_state_dict(new, strict=True)
    return m.to(DEV).eval()


def _ban_library_gemm(mp):
    """Any torch GEMM entry point raises: the fp32 parity mode must run every projection, its
    data gradient and its weight gradient on the hand-written kernels (csrc/gemm_f32.hip), never
    on hipBLASLt / rocBLAS."""
    def banned(name):
        def f(*a, **k):
            raise AssertionError(f"library GEMM torch.{name} called in the fp32 hot path")
        return f
    for name in ("mm", "addmm", "bmm", "baddbmm", "matmul", "einsum"):
        mp.setattr(torch, name, banned(name))
    mp.setattr(torch.nn.functional, "linear", banned("nn.functional.linear"))
    mp.setattr(torch.Tensor, "__matmul__", banned("Tensor.__matmul__"))


def _batch(z):
    return (torch.as_tensor(z["masked_ids"].astype(np.int64), device=DEV),
            torch.as_tensor(z["mask"], device=DEV),
            torch.as_tensor(z["labels"].astype(np.int64), device=DEV))


def test_state_dict_keys_match_reference():
    z, cfg = _golden("cfgA")
    from dna_amd.bert_layers import BertForMaskedLM
    m = BertForMaskedLM(cfg)
    names = {k[len("gradnorm/"):] for k in z.files if k.startswith("gradnorm/")}
    assert {n for n, _ in m.named_parameters()} == names
    assert "cls.predictions.decoder.weight" in m.state_dict()


@pytest.mark.parametrize("tag", ["tiny", "cfgA", "117m"])
def test_forward_fp32_within_1e3(tag, monkeypatch):
    z, cfg = _golden(tag)
    m = _model(cfg, "fp32")
    batch = _batch(z)
    with monkeypatch.context() as mp, torch.no_grad():
        _ban_library_gemm(mp)
        out, state = m(batch, state=None)
    assert state is None
    scores, mask = out.logits
    labels = torch.as_tensor(z["labels"].astype(np.int64))
    rows = scores.reshape(-1, 4096)[(labels.reshape(-1) > 0).to(DEV)].float().cpu().numpy()
    err = np.abs(rows - z["logits_rows"]).max()
    assert err < 1e-3, err
    assert abs(out.loss.item() - float(z["internal_loss"])) < 1e-4
    task = bert_ref.bert_cross_entropy(scores.float().cpu(), mask.cpu(),
                                       torch.as_tensor(z["target"].astype(np.int64)))
    assert abs(task.item() - float(z["task_loss"])) < 1e-4
    # rows with labels <= 0 are exactly zero (bert_layers.py:828-831)
    assert scores.reshape(-1, 4096)[(labels.reshape(-1) <= 0).to(DEV)].abs().max().item() == 0.0


@pytest.mark.parametrize("tag,tol", [("tiny", 2e-2), ("cfgA", 3e-2), ("117m", 6e-2)])
def test_forward_bf16_tolerance(tag, tol):
    z, cfg = _golden(tag)
    m = _model(cfg, "bf16")
    with torch.no_grad():
        out, _ = m(_batch(z), state=None)
    labels = torch.as_tensor(z["labels"].astype(np.int64))
    rows = out.logits[0].reshape(-1, 4096)[(labels.reshape(-1) > 0).to(DEV)].float().cpu().numpy()
    err = np.abs(rows - z["logits_rows"]).max()
    assert err < tol, err
    assert abs(out.loss.item() - float(z["internal_loss"])) < 5e-3


@pytest.mark.parametrize("tag", ["tiny", "cfgA"])
def test_grads_fp32_match_reference(tag, monkeypatch):
    from dna_amd.bert_layers import MLMIndex
    z, cfg = _golden(tag)
    m = _model(cfg, "fp32")
    ids, mask, labels = _batch(z)
    idx = MLMIndex.build(ids, labels)
    with monkeypatch.context() as mp:
        _ban_library_gemm(mp)  # forward, data and weight gradients on csrc/gemm_f32.hip
        loss, _ = m.mlm_loss(ids, mask, idx)
        loss.backward()
    assert abs(loss.item() - float(z["task_loss"])) < 1e-4
    for n, p in m.named_parameters():
        g = p.grad.detach().cpu().numpy()
        ref_norm = float(z["gradnorm/" + n])
        assert abs(np.linalg.norm(g.astype(np.float64)) - ref_norm) <= 2e-3 * max(ref_norm, 1e-3), n
        if ("grad/" + n) in z.files:
            scale = max(np.abs(z["grad/" + n]).max(), 1e-6)
            assert np.abs(g - z["grad/" + n]).max() <= 2e-3 * scale, n


def test_dense_task_loss_equals_compact():
    """bert_cross_entropy over the dense reference-style output == fused compact loss."""
    from dna_amd.bert_layers import MLMIndex
    from dna_amd.tasks import bert_cross_entropy
    z, cfg = _golden("cfgA")
    m = _model(cfg, "fp32")
    ids, mask, labels = _batch(z)
    target = torch.as_tensor(z["target"].astype(np.int64), device=DEV)
    with torch.no_grad():
        out, _ = m((ids, mask, labels))
        dense = bert_cross_entropy([out.logits[0].reshape(-1, 4096), out.logits[1]], target.reshape(-1))
        compact, _ = m.mlm_loss(ids, mask, MLMIndex.build(ids, labels))
    assert abs(dense.item() - compact.item()) < 1e-5
    assert abs(dense.item() - float(z["task_loss"])) < 1e-4


def test_bf16_training_reduces_loss():
    from dna_amd.bert_layers import BertForMaskedLM, MLMIndex
    from dna_amd.flat import FlatParams
    from dna_amd.optim import FusedAdamW
    z, cfg = _golden("cfgA")
    torch.manual_seed(0)
    m = BertForMaskedLM(cfg, precision="bf16").to(DEV).train()
    flat = FlatParams(m, DEV)
    opt = FusedAdamW(flat, lr=1e-3, weight_decay=1e-5, max_grad_norm=1.0)
    ids, mask, labels = _batch(z)
    idx = MLMIndex.build(ids, labels)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss, _ = m.mlm_loss(ids, mask, idx)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(math.isfinite(x) for x in losses)
    assert losses[-1] < losses[0] - 1.0, losses


def test_direct_grad_accumulation_matches_autograd():
    """Trainer path (weight grads written straight into the flat buffer by fused kernels) ==
    plain autograd accumulation, bf16 mode, dropout off."""
    from dna_amd.bert_layers import BertForMaskedLM, MLMIndex
    from dna_amd.flat import FlatParams
    z, cfg = _golden("cfgA")
    ids, mask, labels = _batch(z)
    idx = MLMIndex.build(ids, labels)
    grads = []
    for direct in (False, True):
        torch.manual_seed(0)
        m = BertForMaskedLM(cfg, precision="bf16").to(DEV).eval()
        flat = FlatParams(m, DEV)
        flat.enable_direct_grad(direct)
        flat.zero_grad()
        loss, _ = m.mlm_loss(ids, mask, idx)
        loss.backward()
        grads.append(flat.grad.clone())
    scale = grads[0].abs().max().item()
    assert (grads[0] - grads[1]).abs().max().item() < 1e-3 * scale


@pytest.mark.parametrize("tag", ["cfgA", "117m"])
def test_geglu_fused_into_gemm_same_step(monkeypatch, tag):
    """The GeGLU forward fused into the gated_layers GEMM epilogue (default) and the separate
    GeGLU pass (DNA_GEGLU_FUSED=0) give bit-identical loss and flat gradients, training mode with
    dropout on (same Philox masks)."""
    from dna_amd.bert_layers import BertForMaskedLM, MLMIndex
    from dna_amd.flat import FlatParams
    z, cfg = _golden(tag)
    ids, mask, labels = _batch(z)
    idx = MLMIndex.build(ids, labels)
    out = []
    for fused in ("0", "1"):
        monkeypatch.setenv("DNA_GEGLU_FUSED", fused)
        torch.manual_seed(0)
        m = BertForMaskedLM(cfg, precision="bf16").to(DEV).train()
        flat = FlatParams(m, DEV)
        flat.enable_direct_grad(True)
        flat.zero_grad()
        loss, _ = m.mlm_loss(ids, mask, idx)
        loss.backward()
        torch.cuda.synchronize()
        out.append((loss.detach().clone(), flat.grad.clone()))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("tag", ["cfgA", "117m"])
def test_geglu_bwd_fused_into_wo_dgrad_same_step(monkeypatch, tag):
    """GeGLU + wo as one autograd node whose backward runs wo's data gradient with the GeGLU
    backward in the epilogue (default) vs the separate Linear + GeGLU nodes
    (DNA_GEGLU_BWD_FUSED=0): bit-identical loss and flat gradients, training mode with dropout."""
    from dna_amd.bert_layers import BertForMaskedLM, MLMIndex
    from dna_amd.flat import FlatParams
    z, cfg = _golden(tag)
    ids, mask, labels = _batch(z)
    idx = MLMIndex.build(ids, labels)
    out = []
    for fused in ("0", "1"):
        monkeypatch.setenv("DNA_GEGLU_BWD_FUSED", fused)
        torch.manual_seed(0)
        m = BertForMaskedLM(cfg, precision="bf16").to(DEV).train()
        flat = FlatParams(m, DEV)
        flat.enable_direct_grad(True)
        flat.zero_grad()
        loss, _ = m.mlm_loss(ids, mask, idx)
        loss.backward()
        torch.cuda.synchronize()
        out.append((loss.detach().clone(), flat.grad.clone()))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


def test_wgrad_side_stream_same_gradients(monkeypatch):
    """DNA_WGRAD_STREAM=1 (weight gradients on a side stream, joined at the end of backward) gives
    bit-identical flat gradients to the single-stream path (same kernels, same split-K order)."""
    from dna_amd.bert_layers import BertForMaskedLM, MLMIndex
    from dna_amd.flat import FlatParams
    z, cfg = _golden("cfgA")
    ids, mask, labels = _batch(z)
    idx = MLMIndex.build(ids, labels)
    grads = []
    for side in ("0", "1"):
        monkeypatch.setenv("DNA_WGRAD_STREAM", side)
        torch.manual_seed(0)
        m = BertForMaskedLM(cfg, precision="bf16").to(DEV).eval()
        flat = FlatParams(m, DEV)
        flat.enable_direct_grad(True)
        for _ in range(2):  # two backwards: the join must also hold across steps
            flat.zero_grad()
            loss, _ = m.mlm_loss(ids, mask, idx)
            loss.backward()
        grads.append(flat.grad.clone())  # read right after backward(): no explicit sync
    assert torch.equal(grads[0], grads[1])


def test_bf16_train_step_vs_reference_fixture():
    """The benchmarked step itself (MLMTrainer, bf16: MFMA attention, fused LN / GeGLU / CE
    kernels, direct weight gradients, fused clip + AdamW) on the full 117M shape, S=512, against
    the reference run in fp32 and under bf16 autocast (tests/golden/model_117m_grads.npz, made
    by make_golden.py --only-grads). Tolerances are the reference's own bf16 error scaled by 2:
    whatever bf16 rounding costs the reference, ours may cost at most twice that.
      logits       max / rms |ours - ref32| <= 2x max / rms |ref_bf16 - ref32|
      gradients    per parameter, relative L2 over 1024 sampled elements
                   <= 2x (ref_bf16 vs ref32) + 5e-3; gradient norms within 1e-2
      AdamW step   sign disagreements of the step vs the reference step <= 2x the reference's
                   own bf16 sign disagreements + 0.5 % of the sampled elements."""
    from dna_amd.bert_layers import MLMIndex
    from dna_amd.trainer import DeviceBatch, MLMTrainer
    z = np.load(os.path.join(GOLDEN, "model_117m_grads.npz"))
    L, d, H, Fd = json.loads(z["config"].tobytes().decode())
    cfg = dict(vocab_size=4096, hidden_size=d, num_hidden_layers=L, num_attention_heads=H,
               intermediate_size=Fd, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.0,
               layer_norm_eps=1e-12, max_position_embeddings=512, type_vocab_size=2,
               pad_token_id=0, alibi_starting_size=512, hidden_act="gelu",
               initializer_range=0.02, hyena_framework=True)
    m = _model(cfg, "bf16")
    masked = torch.as_tensor(z["masked_ids"].astype(np.int64))
    mask = torch.as_tensor(z["mask"])
    labels = torch.as_tensor(z["labels"].astype(np.int64))
    target = torch.as_tensor(z["target"].astype(np.int64))
    # logits of the bf16 path
    with torch.no_grad():
        idx = MLMIndex.build(masked, labels).to(DEV)
        logits = m.mlm_logits(masked.to(DEV), idx).float().cpu().numpy()[:z["logits_rows32"].shape[0]]
    l32, l16 = z["logits_rows32"], z["logits_rowsbf16"]
    ref_max, ref_rms = np.abs(l16 - l32).max(), np.sqrt(((l16 - l32) ** 2).mean())
    assert np.abs(logits - l32).max() <= 2 * ref_max, (np.abs(logits - l32).max(), ref_max)
    assert np.sqrt(((logits - l32) ** 2).mean()) <= 2 * ref_rms
    tr = MLMTrainer(m, torch.device(DEV), lr=5e-4, weight_decay=1e-5, max_grad_norm=1.0)
    m.eval()  # the fixture is eval mode (no dropout)
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    loss = tr.step(DeviceBatch.from_host(masked, mask, labels, target, torch.device(DEV)))
    torch.cuda.synchronize()
    assert abs(loss.item() - float(z["task_loss32"])) <= 2 * abs(float(z["task_lossbf16"]) -
                                                                 float(z["task_loss32"])) + 1e-3
    total_sq, flips, flips_ref, count = 0.0, 0, 0, 0
    for n, p in m.named_parameters():
        gi = z["gidx/" + n]
        g = p.grad.detach().reshape(-1).cpu().numpy()
        total_sq += float((g.astype(np.float64) ** 2).sum())
        gs = g[gi]
        g32, g16 = z["gs32/" + n], z["gsbf16/" + n]
        nref = np.linalg.norm(g32)
        err = np.linalg.norm(gs - g32) / nref
        ref_err = np.linalg.norm(g16 - g32) / nref
        assert err <= 2 * ref_err + 5e-3, (n, err, ref_err)
        gn = float(np.linalg.norm(g.astype(np.float64)))
        assert abs(gn - float(z["gradnorm32/" + n])) <= 1e-2 * float(z["gradnorm32/" + n]), n
        dp = (p.detach() - before[n]).reshape(-1).cpu().numpy()[gi]
        flips += int((np.sign(dp) != np.sign(z["dp/" + n])).sum())
        flips_ref += int((np.sign(g16) != np.sign(g32)).sum())
        count += gi.size
    assert abs(math.sqrt(total_sq) - float(z["clip_total_norm"])) <= 1e-2 * float(z["clip_total_norm"])
    assert flips <= 2 * flips_ref + 0.005 * count, (flips, flips_ref, count)


def test_grads_fp32_117m_vs_reference_fixture(monkeypatch):
    """fp32 parity mode at the full 117M shape (S=512): logits, task loss and every parameter's
    gradient (norm, and 1024 sampled elements) against the reference's own fp32 run
    (model_117m_grads.npz), with every projection, data gradient and weight gradient on the
    exact-fp32 MFMA kernels (library GEMMs banned)."""
    from dna_amd.bert_layers import MLMIndex
    z = np.load(os.path.join(GOLDEN, "model_117m_grads.npz"))
    L, d, H, Fd = json.loads(z["config"].tobytes().decode())
    cfg = dict(vocab_size=4096, hidden_size=d, num_hidden_layers=L, num_attention_heads=H,
               intermediate_size=Fd, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.0,
               layer_norm_eps=1e-12, max_position_embeddings=512, type_vocab_size=2,
               pad_token_id=0, alibi_starting_size=512, hidden_act="gelu",
               initializer_range=0.02, hyena_framework=True)
    m = _model(cfg, "fp32")
    ids = torch.as_tensor(z["masked_ids"].astype(np.int64), device=DEV)
    mask = torch.as_tensor(z["mask"], device=DEV)
    labels = torch.as_tensor(z["labels"].astype(np.int64), device=DEV)
    idx = MLMIndex.build(ids, labels)
    with monkeypatch.context() as mp:
        _ban_library_gemm(mp)
        loss, logits = m.mlm_loss(ids, mask, idx)
        loss.backward()
    l32 = z["logits_rows32"]
    assert np.abs(logits.detach().float().cpu().numpy()[:l32.shape[0]] - l32).max() < 1e-3
    assert abs(loss.item() - float(z["task_loss32"])) < 1e-4
    for n, p in m.named_parameters():
        g = p.grad.detach().reshape(-1).cpu().numpy()
        g32 = z["gs32/" + n]
        assert np.linalg.norm(g[z["gidx/" + n]] - g32) <= 2e-3 * np.linalg.norm(g32) + 1e-12, n
        gn = float(np.linalg.norm(g.astype(np.float64)))
        assert abs(gn - float(z["gradnorm32/" + n])) <= 2e-3 * float(z["gradnorm32/" + n]), n


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 5e-3)])
def test_train_evaluate_equals_reference_loss(precision, tol):
    """train.evaluate (the validation / test epoch, reference train.py:339-406,442-460) on the
    config-A golden batch: val/loss == the reference's bert_cross_entropy task loss, perplexity
    == exp(loss), the model is back in training mode afterwards; a 2-batch loader weights the
    batches by size."""
    import types

    import train
    z, cfg = _golden("cfgA")
    m = _model(cfg, precision).train()
    ids, mask, labels = (t.cpu() for t in _batch(z))
    target = torch.as_tensor(z["target"].astype(np.int64))
    batch = ((ids, mask, labels), target)
    tr = types.SimpleNamespace(model=m)
    tokens = {}
    res = train.evaluate(tr, [("val", [batch]), ("test", [batch, batch])], DEV, 3, tokens=tokens)
    assert m.training
    ref = float(z["task_loss"])
    assert abs(res["val/loss"] - ref) < tol and abs(res["test/loss"] - ref) < tol
    assert abs(res["val/perplexity"] - math.exp(res["val/loss"])) < 1e-9 * res["val/perplexity"] + 1e-12
    assert res["val/num_tokens"] == target.numel() and res["test/num_tokens"] == 2 * target.numel()
    res2 = train.evaluate(tr, [("val", [batch])], DEV, 3, tokens=tokens)
    assert res2["val/num_tokens"] == 2 * target.numel()  # NumTokens is never reset
    assert res2["val/loss"] == res["val/loss"]  # eval mode: no dropout, deterministic
