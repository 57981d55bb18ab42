"""Character tokenizer (hg38 `char` path, HyenaDNA configs, hg38_char_tokenizer.py:15-140).
Pinned to tests/golden/char_golden.npz: the reference class's own constructor body and methods
(_tokenize, _convert_token_to_id, build_inputs_with_special_tokens, ...) run by
tests/golden/make_char_golden.py; the padding/truncation of transformers 4.28's __call__ around
them is restated (the reference class does not construct under transformers 5.x). CPU."""
import os

import numpy as np
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "char_golden.npz")


def _rows(g, name):
    d, o = g[name + "_data"], g[name + "_off"]
    return [d[o[i]:o[i + 1]].astype(np.int64).tolist() for i in range(len(o) - 1)]


def test_char_tokenizer_matches_reference_methods():
    from dna_amd.tokenizer import CharacterTokenizer
    g = np.load(GOLD)
    t = CharacterTokenizer(characters=["A", "C", "G", "T", "N"], model_max_length=int(g["model_max_length"]))
    assert t._vocab_str_to_int == dict(zip(g["vocab_keys"].tolist(), g["vocab_vals"].tolist()))
    assert t.vocab_size == int(g["vocab_size"]) and t.padding_side == str(g["padding_side"])
    sp = dict(zip(g["special_names"].tolist(), g["special_ids"].tolist()))
    assert (t.bos_token_id, t.eos_token_id, t.sep_token_id, t.cls_token_id, t.pad_token_id,
            t.mask_token_id, t.unk_token_id) == tuple(sp[k] for k in (
                "bos_token", "eos_token", "sep_token", "cls_token", "pad_token", "mask_token", "unk_token"))
    seqs = [bytes(g["seq_data"][a:b]).decode() for a, b in zip(g["seq_off"][:-1], g["seq_off"][1:])]
    ids, with_sp = _rows(g, "ids"), _rows(g, "sp")
    assert len(seqs) == len(ids) == len(with_sp) > 50
    for s, i, w in zip(seqs, ids, with_sp):
        assert t.encode_raw(s) == i, s            # _tokenize + _convert_token_to_id
        if s == "[SEP]":  # 4.28's tokenize() splits added tokens out of the text first; DNA never
            continue      # holds one (the row pins _tokenize, which the windows go through)
        assert t(s)["input_ids"] == w             # build_inputs_with_special_tokens: ids + [SEP]
        for P in (8, 64, 1026):                   # transformers 4.28 padding="max_length" (left)
            for add in (False, True):
                n_sp = 1 if add else 0
                body = (i[:max(0, P - n_sp)] + ([sp["sep_token"]] if add else []))
                want = [sp["pad_token"]] * (P - len(body)) + body
                got = t(s, add_special_tokens=add, padding="max_length", max_length=P,
                        truncation=True)["input_ids"]
                assert got == want
    back = [str(x) for x in g["back"]]
    for row, b in zip(ids[:10], back):  # _convert_id_to_token round trip
        assert "".join(t._vocab_int_to_str[x] for x in row) == b


def test_char_ids_padding_truncation():
    from dna_amd.tokenizer import CharacterTokenizer
    t = CharacterTokenizer(characters=["A", "C", "G", "T", "N"], model_max_length=14)
    assert t("ACGTNacgX", add_special_tokens=False, padding="max_length", max_length=12,
             truncation=True)["input_ids"] == [4, 4, 4, 7, 8, 9, 10, 11, 6, 6, 6, 6]
    assert t("ACGTNacgX", add_special_tokens=True, padding="max_length", max_length=12,
             truncation=True)["input_ids"] == [4, 4, 7, 8, 9, 10, 11, 6, 6, 6, 6, 1]
    assert t("ACGT" * 4, add_special_tokens=True, padding="max_length", max_length=12,
             truncation=True)["input_ids"] == [7, 8, 9, 10] * 2 + [7, 8, 9, 1]
    assert t.vocab_size == 12 and t.pad_token_id == 4 and t.mask_token_id == 3
    assert sorted(t.all_special_ids) == [0, 1, 2, 3, 4, 6]


def test_bert_hg38_char_items(tmp_path, monkeypatch):
    from dna_amd.hg38 import BertHG38
    from dna_amd.synthetic import write_hg38
    write_hg38(str(tmp_path), n_chroms=1, chrom_len=50_000, max_length=256)
    monkeypatch.setenv("DATA_PATH", str(tmp_path))
    dm = BertHG38(tokenizer_name="char", max_length=256, batch_size=2, add_eos=False,
                  replace_N_token=True, num_workers=0)
    dm.setup()
    torch.manual_seed(0)
    (masked, mask, labels), target = dm.dataset_train[0]
    assert masked.shape == (256,) and int(target.min()) >= 4 and int(target.max()) <= 10
    assert 11 not in target.tolist()  # N -> [PAD] (replace_N_token)
    assert bool((labels[~mask] == -100).all())
