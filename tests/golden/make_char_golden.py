#!/usr/bin/env python
"""Golden vectors for the hg38 `char` tokenizer (reference
src/dataloaders/datasets/hg38_char_tokenizer.py, built by genomics.py:1132-1138 with characters
ACGTN and model_max_length = max_length + 2).

The reference pins transformers 4.28 (requirements.txt:108). Under the transformers 5.x of this
container its constructor raises inside PreTrainedTokenizer.__init__ (the base class asks
get_vocab() for the vocabulary before the subclass has built it). This script therefore runs the
reference class's OWN code with the base-class constructor replaced by a recorder for the
duration of the construction: the reference __init__ body (its vocabulary, special-token
strings, padding_side) and its methods _tokenize, _convert_token_to_id, _convert_id_to_token,
build_inputs_with_special_tokens, get_special_tokens_mask, create_token_type_ids_from_sequences
all run unmodified; special-token ids are what 4.28's convert_tokens_to_ids gives for the
recorded special-token strings (the reference's own _convert_token_to_id). The __call__
padding/truncation around them is transformers' base-class logic and stays a restatement.
Run from the repo root:
    python tests/golden/make_char_golden.py      -> tests/golden/char_golden.npz
"""
import importlib.util
import os
import types

import numpy as np

REF = os.environ.get("DNA_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference_class():
    spec = importlib.util.spec_from_file_location(
        "ref_hg38_char_tokenizer", os.path.join(REF, "src/dataloaders/datasets/hg38_char_tokenizer.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.CharacterTokenizer


def construct(cls, characters, model_max_length):
    import transformers.tokenization_utils as tu
    base = tu.PreTrainedTokenizer
    recorded = {}
    orig = base.__init__

    def recorder(self, **kw):
        recorded.update(kw)

    base.__init__ = recorder
    try:
        tok = cls(characters=characters, model_max_length=model_max_length)
    finally:
        base.__init__ = orig
    return tok, recorded


def windows(rng):
    base = np.frombuffer(b"ACGT", dtype=np.uint8)
    wins = ["", "A", "ACGTN", "ACGTNacgtnX", "NNNNNNN", "..ACGT..", "AC GT", "[SEP]", "acgt" * 5]
    for n in list(rng.integers(1, 300, 20)) + list(rng.integers(1000, 1100, 10)):
        wins.append(base[rng.integers(0, 4, n)].tobytes().decode())
    for _ in range(20):  # N runs and soft-masked (lowercase) runs as in hg38
        n = int(rng.integers(20, 1200))
        s = bytearray(base[rng.integers(0, 4, n)].tobytes())
        a = int(rng.integers(0, n)); b = min(n, a + int(rng.integers(1, 60)))
        s[a:b] = b"N" * (b - a)
        a = int(rng.integers(0, n)); b = min(n, a + int(rng.integers(1, 100)))
        s[a:b] = bytes(s[a:b]).lower()
        wins.append(s.decode())
    return wins


def main():
    cls = load_reference_class()
    chars = ["A", "C", "G", "T", "N"]
    tok, kw = construct(cls, chars, 1024 + 2)
    sp = {name: tok._convert_token_to_id(str(kw[name])) for name in
          ("bos_token", "eos_token", "sep_token", "cls_token", "pad_token", "mask_token", "unk_token")}
    ids_view = types.SimpleNamespace(sep_token_id=sp["sep_token"], cls_token_id=sp["cls_token"])
    wins = windows(np.random.default_rng(12))
    toks = [tok._tokenize(w) for w in wins]
    ids = [[tok._convert_token_to_id(t) for t in ts] for ts in toks]
    with_sp = [cls.build_inputs_with_special_tokens(ids_view, i) for i in ids]
    pair = [cls.build_inputs_with_special_tokens(ids_view, ids[k], ids[k + 1]) for k in range(0, 10, 2)]
    spmask = [cls.get_special_tokens_mask(ids_view, i) for i in ids[:10]]
    ttype = [cls.create_token_type_ids_from_sequences(ids_view, ids[k], ids[k + 1]) for k in range(0, 10, 2)]
    back = ["".join(tok._convert_id_to_token(i) for i in row) for row in ids[:10]]
    cat = lambda rows: (np.concatenate([np.asarray(r, dtype=np.int16) for r in rows]) if rows else
                        np.zeros(0, np.int16), np.cumsum([0] + [len(r) for r in rows]).astype(np.int64))
    sb = [w.encode() for w in wins]
    ids_d, ids_o = cat(ids)
    sp_d, sp_o = cat(with_sp)
    pr_d, pr_o = cat(pair)
    sm_d, sm_o = cat(spmask)
    tt_d, tt_o = cat(ttype)
    np.savez_compressed(
        os.path.join(HERE, "char_golden.npz"),
        seq_data=np.frombuffer(b"".join(sb), dtype=np.uint8),
        seq_off=np.cumsum([0] + [len(b) for b in sb]).astype(np.int64),
        ids_data=ids_d, ids_off=ids_o, sp_data=sp_d, sp_off=sp_o, pair_data=pr_d, pair_off=pr_o,
        spmask_data=sm_d, spmask_off=sm_o, ttype_data=tt_d, ttype_off=tt_o,
        back=np.asarray(back, dtype=object).astype("U"),
        vocab_keys=np.asarray(list(tok._vocab_str_to_int.keys())),
        vocab_vals=np.asarray(list(tok._vocab_str_to_int.values()), dtype=np.int16),
        special_names=np.asarray(list(sp.keys())),
        special_ids=np.asarray(list(sp.values()), dtype=np.int16),
        padding_side=np.str_(kw["padding_side"]), model_max_length=np.int64(kw["model_max_length"]),
        vocab_size=np.int64(cls.vocab_size.fget(tok)))
    print(f"wrote char_golden.npz: {len(wins)} windows, specials {sp}, padding_side {kw['padding_side']}")


if __name__ == "__main__":
    main()
