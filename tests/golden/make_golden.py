#!/usr/bin/env python
"""Generate the golden parity fixtures by running the REFERENCE code in this container.

Run from the repo root:  python tests/golden/make_golden.py
Needs /root/reference (read-only, imported by path, never copied) and the `tokenizers` /
`transformers` packages. Writes only small data files next to this script:

  tok_golden.npz    BPE ids from the reference tokenizer (HF tokenizers, tokenizer.json of
                    /root/reference/DNABERT-2-117M) for ~270 windows, full and dataset-style
                    (`hg38_dataset.py:369-379`: padding="max_length", truncation, then [1:-1]).
  mask_golden.npz   reference `bert_mask` (`hg38_dataset.py:238-286`) outputs together with the
                    torch random draws it consumed, so the restatement can be checked exactly.
  fasta_golden.json reference `FastaInterval.__call__` (`hg38_dataset.py:72-124`) windows.
  model_*.npz       reference `BertForMaskedLM` (`bert_layers.py:691-850`) eval-mode fp32 outputs
                    for hash-initialised weights (oracle/hashinit.py), plus gradients.

The generator is the only place that imports the reference; tests read the fixtures alone.
"""
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("DNA_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.hashinit import hash_tensor  # noqa: E402

PAD, MASK, VOCAB = 3, 4, 4096
SPECIAL = [0, 2, 3, 1, 4]


# ----------------------------------------------------------------------------- shims
def _install_shims():
    """Minimal stand-ins for packages the reference imports but this image lacks.

    omegaconf: `bert_layers.py:694-698` only calls OmegaConf.to_container(dict-like).
    pyfaidx/polars: imported at module top of hg38_dataset.py; FastaInterval receives a
    dict-backed fake instead of a real Fasta (we never touch pyfaidx behaviour beyond slicing).
    """
    om = types.ModuleType("omegaconf")

    class OmegaConf:
        @staticmethod
        def to_container(c):
            return dict(c)

    om.OmegaConf = OmegaConf
    sys.modules.setdefault("omegaconf", om)
    for name in ("pyfaidx", "polars"):
        m = types.ModuleType(name)
        m.Fasta = None
        sys.modules.setdefault(name, m)
    os.environ.setdefault("PROJECT_ROOT", REF)
    os.environ.setdefault("HF_HUB_OFFLINE", "1")


def _load_hg38_dataset():
    spec = importlib.util.spec_from_file_location(
        "ref_hg38_dataset", os.path.join(REF, "src/dataloaders/datasets/hg38_dataset.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _tokenizer():
    from transformers import PreTrainedTokenizerFast
    return PreTrainedTokenizerFast(
        tokenizer_file=os.path.join(REF, "DNABERT-2-117M/tokenizer.json"),
        unk_token="[UNK]", cls_token="[CLS]", sep_token="[SEP]", pad_token="[PAD]",
        mask_token="[MASK]")


# ----------------------------------------------------------------------------- windows
def make_windows(rng):
    wins = ["", "A", "N", "a", "ACGTACGTACGT", "ACGTNNacgt", "NNNNNNNN", "acgtacgtac",
            "AAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA", "..ACGT..", "ACGT.ACGT",
            "A" * 300, "GC" * 700, "T" * 4096]
    base = np.frombuffer(b"ACGT", dtype=np.uint8)
    lens = np.concatenate([rng.integers(1, 200, 60), rng.integers(200, 1200, 80),
                           rng.integers(1200, 4300, 60), np.full(20, 4096)])
    for n in lens:
        wins.append(base[rng.integers(0, 4, n)].tobytes().decode())
    # edge windows: N runs, lowercase runs, '.' padding (pad_interval) like hg38 soft-masking
    for _ in range(50):
        n = int(rng.integers(50, 4200))
        s = bytearray(base[rng.integers(0, 4, n)].tobytes())
        for _ in range(int(rng.integers(0, 4))):
            a = int(rng.integers(0, n)); b = min(n, a + int(rng.integers(1, 60)))
            s[a:b] = b"N" * (b - a)
        for _ in range(int(rng.integers(0, 4))):
            a = int(rng.integers(0, n)); b = min(n, a + int(rng.integers(1, 300)))
            s[a:b] = bytes(s[a:b]).lower()
        if rng.random() < 0.3:
            k = int(rng.integers(1, 40))
            s = bytearray(b"." * k) + s + bytearray(b"." * int(rng.integers(0, 40)))
        wins.append(s.decode())
    return wins


def gen_tokenizer(rng):
    tok = _tokenizer()
    wins = make_windows(rng)
    full, ds130, ds514 = [], [], []
    for w in wins:
        full.append(tok(w)["input_ids"])  # [CLS] + bpe + [SEP], untruncated
        for P, out in ((130, ds130), (514, ds514)):
            ids = tok(w, padding="max_length", max_length=P, truncation=True)["input_ids"][1:-1]
            assert len(ids) == P - 2
            out.append(ids)
    seq_bytes = [w.encode() for w in wins]
    np.savez_compressed(
        os.path.join(HERE, "tok_golden.npz"),
        seq_data=np.frombuffer(b"".join(seq_bytes), dtype=np.uint8),
        seq_off=np.cumsum([0] + [len(b) for b in seq_bytes]).astype(np.int64),
        full_data=np.concatenate([np.asarray(f, dtype=np.int16) for f in full]),
        full_off=np.cumsum([0] + [len(f) for f in full]).astype(np.int64),
        ds130=np.asarray(ds130, dtype=np.int16), ds514=np.asarray(ds514, dtype=np.int16),
        tokenizers_version=np.bytes_(__import__("tokenizers").__version__))
    print(f"tok_golden: {len(wins)} windows")
    return tok, ds514


def gen_mask(hg, ds514):
    """bert_mask consumes, in order: rand(shape), rand(shape), randint(0,V,shape), then
    re-draws for special ids. Replaying the same calls under the same seed yields the exact
    draws; we assert that the replay reproduces the reference output before saving."""
    cases = {}
    for seed in range(12):
        seq = torch.as_tensor(np.asarray(ds514[seed], dtype=np.int64))
        if seed % 3 == 2:  # make a padded sequence
            seq[200:] = PAD
        torch.manual_seed(seed)
        out_seq, out_mask, out_labels = hg.bert_mask(seq.clone(), MASK, PAD, VOCAB,
                                                     special_token_ids=SPECIAL)
        torch.manual_seed(seed)
        u1 = torch.rand(seq.shape)
        u2 = torch.rand(seq.shape)
        rt = torch.randint(0, VOCAB, seq.shape, dtype=torch.long)
        sp = torch.tensor(SPECIAL)
        while torch.isin(rt, sp).any():
            bad = torch.isin(rt, sp)
            rt[bad] = torch.randint(0, VOCAB, (int(bad.sum()),), dtype=torch.long)
        m = (seq != PAD) & (u1 < 0.15)
        lab = torch.where(m, seq, torch.full_like(seq, -100))
        s2 = seq.clone()
        s2[m & (u2 < 0.8)] = MASK
        sel = m & (u2 >= 0.8) & (u2 < 0.9)
        s2[sel] = rt[sel]
        assert torch.equal(s2, out_seq) and torch.equal(m, out_mask) and torch.equal(lab, out_labels)
        cases[f"s{seed}_seq"] = seq.numpy().astype(np.int16)
        cases[f"s{seed}_u1"] = u1.numpy()
        cases[f"s{seed}_u2"] = u2.numpy()
        cases[f"s{seed}_rt"] = rt.numpy().astype(np.int16)
        cases[f"s{seed}_out_seq"] = out_seq.numpy().astype(np.int16)
        cases[f"s{seed}_out_mask"] = out_mask.numpy()
        cases[f"s{seed}_out_labels"] = out_labels.numpy().astype(np.int16)
    np.savez_compressed(os.path.join(HERE, "mask_golden.npz"), **cases)
    print("mask_golden: 12 seeds")


class _FakeChrom(str):
    """pyfaidx-like: slicing returns a str (pyfaidx returns a Sequence whose str() is the slice)."""


def gen_fasta(hg, rng):
    base = np.frombuffer(b"ACGTacgtN", dtype=np.uint8)
    chroms = {"chr1": base[rng.integers(0, 9, 5000)].tobytes().decode(),
              "chr2": base[rng.integers(0, 9, 777)].tobytes().decode(),
              "chrM": base[rng.integers(0, 9, 60)].tobytes().decode()}

    class FakeFasta(dict):
        pass

    fi = hg.FastaInterval.__new__(hg.FastaInterval)
    fi.seqs = FakeFasta({k: _FakeChrom(v) for k, v in chroms.items()})
    fi.return_seq_indices = False
    fi.shift_augs = None
    fi.rc_aug = False
    fi.chr_lens = {k: len(v) for k, v in chroms.items()}
    cases = []
    specs = [("chr1", 0, 1024, 1024), ("chr1", 100, 200, 1024), ("chr1", 4900, 5000, 1024),
             ("chr1", 10, 3000, 1024), ("chr2", 0, 777, 1024), ("chr2", 300, 310, 64),
             ("chrM", 0, 60, 128), ("chrM", 30, 31, 16), ("chr1", 2500, 2500, 100),
             ("chr1", 4990, 5000, 4096), ("chr1", 0, 5000, 4096)]
    for _ in range(40):
        c = ["chr1", "chr2", "chrM"][int(rng.integers(0, 3))]
        L = len(chroms[c])
        s = int(rng.integers(0, L)); e = min(L, s + int(rng.integers(0, 2000)))
        specs.append((c, s, e, int(rng.choice([16, 128, 1024, 4096]))))
    for pad in (False, True):
        fi.pad_interval = pad
        for c, s, e, ml in specs:
            cases.append({"chr": c, "start": s, "end": e, "max_length": ml,
                          "pad_interval": pad, "out": fi(c, s, e, max_length=ml)})
    rc = ["ACGTNacgtn.", "", "TTTTgca"]
    json.dump({"chroms": chroms, "cases": cases,
               "revcomp": [[s, hg.string_reverse_complement(s)] for s in rc]},
              open(os.path.join(HERE, "fasta_golden.json"), "w"))
    print(f"fasta_golden: {len(cases)} cases")


# ----------------------------------------------------------------------------- model
def _model_cfg(layers, d, heads, ff):
    return dict(vocab_size=VOCAB, hidden_size=d, num_hidden_layers=layers,
                num_attention_heads=heads, intermediate_size=ff, hidden_dropout_prob=0.1,
                attention_probs_dropout_prob=0.0, layer_norm_eps=1e-12,
                max_position_embeddings=512, type_vocab_size=2, pad_token_id=0,
                alibi_starting_size=512, hidden_act="gelu", initializer_range=0.02,
                hyena_framework=True)


def _ref_model(cfg):
    import transformers
    from src.models.DNABERT2 import bert_layers as bl

    class _Tok:
        pad_token_id = PAD

    # bert_layers.py:786-787 reloads the tokenizer on every forward just to read pad id 3.
    transformers.AutoTokenizer.from_pretrained = staticmethod(lambda *a, **k: _Tok())
    m = bl.BertForMaskedLM(cfg)
    sd = m.state_dict()
    new = {}
    for k, v in sd.items():
        if k == "cls.predictions.decoder.weight":
            continue  # tied alias of bert.embeddings.word_embeddings.weight
        new[k] = torch.from_numpy(hash_tensor(k, tuple(v.shape)))
    new["cls.predictions.decoder.weight"] = new["bert.embeddings.word_embeddings.weight"]
    m.load_state_dict(new, strict=True)
    assert m.cls.predictions.decoder.weight.data_ptr() == \
        m.bert.embeddings.word_embeddings.weight.data_ptr()
    return m, bl


def _make_batch(rng, b, S, pad_rows, unk_frac=0.01):
    """(masked_ids, mask, labels), target like BertHG38Dataset.__getitem__ + collate."""
    ids = rng.integers(5, VOCAB, size=(b, S))
    ids[rng.random((b, S)) < unk_frac] = 0  # [UNK] tokens (N / lowercase windows)
    for r, n in pad_rows.items():
        ids[r, n:] = PAD
        ids[r, n - 1] = 2  # [SEP] lands inside short sequences (hg38_dataset.py:379)
    target = ids.copy()
    u1, u2 = rng.random((b, S)), rng.random((b, S))
    mask = (ids != PAD) & (u1 < 0.15)
    mask[:, 3] = ids[:, 3] != PAD  # at least one masked token per row
    # force a masked [UNK] so the zero-logit row semantics (metrics.py:270-273) are exercised
    mask[0, 5] = True
    ids[0, 5] = target[0, 5] = 0
    labels = np.where(mask, ids, -100)
    masked = ids.copy()
    masked[mask & (u2 < 0.8)] = MASK
    sel = mask & (u2 >= 0.8) & (u2 < 0.9)
    masked[sel] = rng.integers(5, VOCAB, size=int(sel.sum()))
    return masked, mask, labels, target


def _bert_cross_entropy(x, y):
    # metrics.py:268-273 (restated: importing src.tasks pulls torchmetrics/PL)
    logits, mask = x[0], x[1].reshape(y.shape)
    return torch.nn.functional.cross_entropy(logits[mask], y[mask])


def gen_model(tag, layers, d, heads, ff, b, S, pad_rows, grads, rng):
    cfg = _model_cfg(layers, d, heads, ff)
    m, bl = _ref_model(cfg)
    m.eval()
    masked, mask, labels, target = _make_batch(rng, b, S, pad_rows)
    batch = (torch.as_tensor(masked), torch.as_tensor(mask), torch.as_tensor(labels))
    out, _ = m(batch, state=None)
    scores = out.logits[0]
    x0 = scores.reshape(-1, VOCAB)
    task_loss = _bert_cross_entropy([x0, out.logits[1]], torch.as_tensor(target).reshape(-1))
    sel = torch.as_tensor(labels).reshape(-1) > 0
    res = dict(masked_ids=masked.astype(np.int16), mask=mask, labels=labels.astype(np.int16),
               target=target.astype(np.int16), logits_rows=x0[sel].detach().numpy(),
               internal_loss=np.float64(out.loss.item()), task_loss=np.float64(task_loss.item()),
               dense_zero_rows_ok=np.bool_(bool((x0[~sel] == 0).all())),
               alibi_slopes=(-m.bert.encoder.alibi[0, :, 0, 1]).numpy(),
               config=np.bytes_(json.dumps([layers, d, heads, ff])))
    if grads:
        task_loss.backward()
        for n, p in m.named_parameters():
            g = p.grad.detach().numpy()
            res["gradnorm/" + n] = np.float64(np.linalg.norm(g.astype(np.float64)))
            if grads == "full":
                res["grad/" + n] = g
    np.savez_compressed(os.path.join(HERE, f"model_{tag}.npz"), **res)
    print(f"model_{tag}: {int(sel.sum())} logit rows, task loss {task_loss.item():.6f}")


N_SAMPLE = 1024      # sampled gradient elements per parameter (model_117m_grads.npz)
N_LOGIT_ROWS = 64    # masked logit rows kept per precision


def gen_model_grads(tag, layers, d, heads, ff, b, S, pad_rows, rng):
    """The benchmarked configuration's gradients and one optimizer step, from the reference:
    the same hash-initialised BertForMaskedLM run twice on one batch -- fp32, and under CPU
    torch.autocast(bfloat16) (the reference trains with `precision: bf16`, i.e. Lightning's
    bf16 autocast; dnabert2_hg38_pretrain.yaml `trainer.precision`) -- eval mode (no dropout),
    bert_cross_entropy task loss (metrics.py:268-273). Stored: masked-row logits of both runs,
    every parameter's gradient L2 norm in both runs, N_SAMPLE seeded elements of every gradient
    in both runs, and the parameter change of one reference optimizer step on the fp32
    gradients: torch clip_grad_norm_(1.0) (gradient_clip_val) + torch.optim.AdamW(lr 5e-4,
    weight_decay 1e-5) (configs/optimizer/adamw.yaml + the experiment's overrides)."""
    cfg = _model_cfg(layers, d, heads, ff)
    masked, mask, labels, target = _make_batch(rng, b, S, pad_rows)
    batch = (torch.as_tensor(masked), torch.as_tensor(mask), torch.as_tensor(labels))
    sel = torch.as_tensor(labels).reshape(-1) > 0
    pick = np.random.default_rng(7)
    res = dict(masked_ids=masked.astype(np.int16), mask=mask, labels=labels.astype(np.int16),
               target=target.astype(np.int16), config=np.bytes_(json.dumps([layers, d, heads, ff])))
    for prec in ("32", "bf16"):
        m, bl = _ref_model(cfg)
        m.eval()
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=prec == "bf16"):
            out, _ = m(batch, state=None)
            x0 = out.logits[0].reshape(-1, VOCAB)
            task_loss = _bert_cross_entropy([x0, out.logits[1]], torch.as_tensor(target).reshape(-1))
        task_loss.backward()
        res[f"logits_rows{prec}"] = x0[sel][:N_LOGIT_ROWS].detach().float().numpy()
        res[f"task_loss{prec}"] = np.float64(task_loss.item())
        for n, p in m.named_parameters():
            g = p.grad.detach().float().reshape(-1).numpy()
            if prec == "32":
                k = min(N_SAMPLE, g.size)
                res["gidx/" + n] = np.sort(pick.choice(g.size, k, replace=False)).astype(np.int32)
            res[f"gradnorm{prec}/" + n] = np.float64(np.linalg.norm(g.astype(np.float64)))
            res[f"gs{prec}/" + n] = g[res["gidx/" + n]]
        if prec == "32":
            before = {n: p.detach().clone() for n, p in m.named_parameters()}
            res["clip_total_norm"] = np.float64(
                torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0).item())
            opt = torch.optim.AdamW(m.parameters(), lr=5e-4, weight_decay=1e-5)
            opt.step()
            for n, p in m.named_parameters():
                dp = (p.detach() - before[n]).reshape(-1).numpy()
                res["dp/" + n] = dp[res["gidx/" + n]]
        print(f"model_{tag}: precision {prec}, task loss {task_loss.item():.6f}")
    np.savez_compressed(os.path.join(HERE, f"model_{tag}.npz"), **res)


def main():
    _install_shims()
    sys.path.insert(0, REF)
    torch.set_num_threads(8)
    grads_only = "--only-grads" in sys.argv  # regenerate model_117m_grads.npz alone
    if not grads_only:
        main_round1()
    # the benchmarked step (117M, S=512): fp32 and bf16-autocast gradients + one AdamW step
    gen_model_grads("117m_grads", 12, 768, 12, 3072, 2, 512, {1: 300},
                    np.random.default_rng(2223))


def main_round1():
    rng = np.random.default_rng(2222)
    tok, ds514 = gen_tokenizer(rng)
    hg = _load_hg38_dataset()
    gen_mask(hg, ds514)
    gen_fasta(hg, rng)
    # tiny: one head of 64 -> full gradients checked elementwise
    gen_model("tiny", 2, 64, 1, 128, 2, 64, {1: 40}, "full", rng)
    # config A: 2 layers, d=128, 2 heads, ff=512, S=128, b=8 (two padded rows)
    gen_model("cfgA", 2, 128, 2, 512, 8, 128, {2: 100, 5: 17}, "norms", rng)
    # full DNABERT-2-117M shape, S=512, one padded row
    gen_model("117m", 12, 768, 12, 3072, 2, 512, {1: 300}, None, rng)


if __name__ == "__main__":
    main()
