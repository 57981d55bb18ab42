"""Pin the CPU oracle against the golden vectors produced by running the reference.

CPU only (no GPU marker): if these fail, no parity claim built on the oracle holds.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import bert_ref, hg38_ref, optim_ref
from oracle.bpe import BPERef
from oracle.hashinit import hash_tensor
from tests.conftest import BPE_JSON, GOLDEN


def _tok():
    return np.load(os.path.join(GOLDEN, "tok_golden.npz"))


@pytest.fixture(scope="module")
def bpe():
    return BPERef(BPE_JSON)


def _windows(z):
    data, off = z["seq_data"].tobytes(), z["seq_off"]
    return [data[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]


def test_bpe_full_encode_bit_exact(bpe):
    z = _tok()
    wins = _windows(z)
    fo, fd = z["full_off"], z["full_data"]
    # long uniform windows are slow in pure Python; all windows < 1500 bp + every 5th longer one
    for i, w in enumerate(wins):
        if len(w) > 1500 and i % 5:
            continue
        got = bpe.encode(w, add_special_tokens=True)
        exp = fd[fo[i]:fo[i + 1]].astype(np.int64).tolist()
        assert got == exp, f"window {i} (len {len(w)})"


def test_bpe_dataset_call_bit_exact(bpe):
    z = _tok()
    wins = _windows(z)
    for i, w in enumerate(wins[:120]):
        assert bpe.encode_dataset(w, 130) == z["ds130"][i].astype(np.int64).tolist()
        if len(w) < 2500:
            assert bpe.encode_dataset(w, 514) == z["ds514"][i].astype(np.int64).tolist()


def test_bpe_appendix_examples(bpe):
    # SURVEY Appendix A
    assert bpe.encode("ACGTACGTACGT", True) == [1, 5, 194, 194, 6, 1049, 2]
    assert bpe.encode("ACGTNNacgt", True) == [1, 5, 6, 1049, 0, 0, 0, 0, 0, 0, 2]


def test_bert_mask_restatement_exact():
    z = np.load(os.path.join(GOLDEN, "mask_golden.npz"))
    for s in range(12):
        out, mask, labels = hg38_ref.bert_mask_from_draws(
            z[f"s{s}_seq"], z[f"s{s}_u1"], z[f"s{s}_u2"], z[f"s{s}_rt"])
        np.testing.assert_array_equal(out, z[f"s{s}_out_seq"])
        np.testing.assert_array_equal(mask, z[f"s{s}_out_mask"])
        np.testing.assert_array_equal(labels, z[f"s{s}_out_labels"])


def test_fasta_interval_exact():
    g = json.load(open(os.path.join(GOLDEN, "fasta_golden.json")))
    for c in g["cases"]:
        got = hg38_ref.fasta_interval(g["chroms"][c["chr"]], c["start"], c["end"],
                                      c["max_length"], c["pad_interval"])
        assert got == c["out"], c
    for s, rc in g["revcomp"]:
        assert hg38_ref.reverse_complement(s) == rc


def _load_model(tag):
    z = np.load(os.path.join(GOLDEN, f"model_{tag}.npz"))
    L, d, H, Fd = json.loads(z["config"].tobytes().decode())
    cfg = dict(vocab_size=4096, hidden_size=d, num_hidden_layers=L, num_attention_heads=H,
               intermediate_size=Fd, layer_norm_eps=1e-12)
    sd = {n: torch.from_numpy(hash_tensor(n, s)) for n, s in bert_ref.state_dict_shapes(cfg)}
    return z, cfg, sd


@pytest.mark.parametrize("tag", ["tiny", "cfgA", "117m"])
def test_model_forward_matches_reference(tag):
    z, cfg, sd = _load_model(tag)
    ids = torch.as_tensor(z["masked_ids"].astype(np.int64))
    labels = torch.as_tensor(z["labels"].astype(np.int64))
    logits, internal, dense = bert_ref.dnabert2_forward(sd, cfg, ids, labels)
    np.testing.assert_allclose(logits.detach().numpy(), z["logits_rows"], atol=1e-4, rtol=0)
    assert abs(internal.item() - float(z["internal_loss"])) < 1e-5
    task = bert_ref.bert_cross_entropy(dense, torch.as_tensor(z["mask"]),
                                       torch.as_tensor(z["target"].astype(np.int64)))
    assert abs(task.item() - float(z["task_loss"])) < 1e-5
    np.testing.assert_allclose(np.asarray(bert_ref.alibi_slopes(cfg["num_attention_heads"])),
                               z["alibi_slopes"], rtol=1e-6)


@pytest.mark.parametrize("tag", ["tiny", "cfgA"])
def test_model_grads_match_reference(tag):
    z, cfg, sd = _load_model(tag)
    for v in sd.values():
        v.requires_grad_(True)
    ids = torch.as_tensor(z["masked_ids"].astype(np.int64))
    labels = torch.as_tensor(z["labels"].astype(np.int64))
    _, _, dense = bert_ref.dnabert2_forward(sd, cfg, ids, labels)
    loss = bert_ref.bert_cross_entropy(dense, torch.as_tensor(z["mask"]),
                                       torch.as_tensor(z["target"].astype(np.int64)))
    loss.backward()
    for n, p in sd.items():
        g = p.grad.numpy()
        ref_norm = float(z["gradnorm/" + n])
        assert abs(np.linalg.norm(g.astype(np.float64)) - ref_norm) <= 1e-4 * max(ref_norm, 1e-3), n
        if ("grad/" + n) in z:
            np.testing.assert_allclose(g, z["grad/" + n], atol=2e-6, rtol=1e-3, err_msg=n)


def test_adamw_clip_matches_torch():
    rng = np.random.default_rng(0)
    ps = [rng.standard_normal(s).astype(np.float32) for s in [(7, 5), (11,), (3, 3)]]
    gs = [rng.standard_normal(p.shape).astype(np.float32) * 3 for p in ps]
    tp = [torch.nn.Parameter(torch.from_numpy(p.copy())) for p in ps]
    opt = torch.optim.AdamW(tp, lr=5e-4, weight_decay=1e-5)
    m = [np.zeros_like(p, np.float64) for p in ps]
    v = [np.zeros_like(p, np.float64) for p in ps]
    cur = [p.astype(np.float64) for p in ps]
    for step in range(1, 4):
        for t, g in zip(tp, gs):
            t.grad = torch.from_numpy(g.copy())
        torch.nn.utils.clip_grad_norm_(tp, 1.0)
        opt.step()
        coef, _ = optim_ref.clip_coef(gs, 1.0)
        for i, g in enumerate(gs):
            cur[i], m[i], v[i] = optim_ref.adamw_step(cur[i], g.astype(np.float64) * coef, m[i], v[i],
                                                      step, 5e-4, weight_decay=1e-5)
    for c, t in zip(cur, tp):
        np.testing.assert_allclose(c, t.detach().numpy(), rtol=1e-5, atol=1e-6)


def test_lr_schedule_restatement():
    assert optim_ref.linear_warmup_lr(0, 5e-4, 120000, 2e6) == 0.0
    assert abs(optim_ref.linear_warmup_lr(60000, 5e-4, 120000, 2e6) - 2.5e-4) < 1e-12
    assert abs(optim_ref.linear_warmup_lr(120000, 5e-4, 120000, 2e6) - 5e-4) < 1e-12
    assert abs(optim_ref.linear_warmup_lr(1120000, 5e-4, 120000, 2e6) - 2.5e-4) < 1e-12


def test_model_117m_grads_and_step_match_reference():
    """The oracle at the benchmarked shape (117M, S=512) vs the reference's fp32 run: logits,
    sampled gradient elements, gradient norms, the clip norm and one AdamW step."""
    z, cfg, sd = _load_model("117m_grads")
    for v in sd.values():
        v.requires_grad_(True)
    ids = torch.as_tensor(z["masked_ids"].astype(np.int64))
    labels = torch.as_tensor(z["labels"].astype(np.int64))
    logits, _, dense = bert_ref.dnabert2_forward(sd, cfg, ids, labels)
    n_rows = z["logits_rows32"].shape[0]
    np.testing.assert_allclose(logits.detach().numpy()[:n_rows], z["logits_rows32"], atol=1e-4, rtol=0)
    loss = bert_ref.bert_cross_entropy(dense, torch.as_tensor(z["mask"]),
                                       torch.as_tensor(z["target"].astype(np.int64)))
    assert abs(loss.item() - float(z["task_loss32"])) < 1e-5
    loss.backward()
    gs = {n: p.grad.numpy().astype(np.float64) for n, p in sd.items()}
    coef, total = optim_ref.clip_coef(list(gs.values()), 1.0)
    assert abs(total - float(z["clip_total_norm"])) <= 1e-3 * float(z["clip_total_norm"])
    for n, g in gs.items():
        ref_norm = float(z["gradnorm32/" + n])
        assert abs(np.linalg.norm(g) - ref_norm) <= 1e-3 * max(ref_norm, 1e-3), n
        gi = z["gidx/" + n]
        gf = g.reshape(-1)[gi]
        scale = max(np.abs(z["gs32/" + n]).max(), 1e-8)
        assert np.abs(gf - z["gs32/" + n]).max() <= 2e-3 * scale, n
        p0 = sd[n].detach().numpy().astype(np.float64).reshape(-1)[gi]
        p1, _, _ = optim_ref.adamw_step(p0, gf * coef, np.zeros_like(gf), np.zeros_like(gf), 1,
                                        5e-4, weight_decay=1e-5)
        agree = np.isclose(p1 - p0, z["dp/" + n], rtol=1e-3, atol=1e-9)
        assert agree.mean() >= 0.99, (n, agree.mean())
