#!/usr/bin/env python
"""Golden vectors for the NT-v2 6-mer tokenizer (reference genomics.py:1142-1144: bert_hg38 with
tokenizer_name=kmer loads /root/reference/nucleotide-transformer-v2-500m-multi-species).

The reference call, AutoTokenizer.from_pretrained(<dir>, trust_remote_code=True), fails in this
container before tokenising anything: the directory's special_tokens_map.json starts with a stray
"cd " and is not JSON. The tokenizer it names (tokenizer_config.json: EsmTokenizer, no eos,
model_max_length 2048; special tokens <unk> <pad> <mask> <cls>) is therefore built from the same
vocab.txt with transformers' EsmTokenizer directly. Run from the repo root:
    python tests/golden/make_kmer_golden.py      -> tests/golden/kmer_golden.npz
"""
import os

import numpy as np

REF = os.environ.get("DNA_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def windows(rng):
    base = np.frombuffer(b"ACGT", dtype=np.uint8)
    wins = ["", "A", "ACGTAC", "ACGTACGTAC", "NNNNNNN", "ACGTNNACGTAA", "acgtacgt", "ACGTACG.TT",
            "ACGTXACGTAC", "AC GT", "..ACGTACGT..", "N" * 13 + "ACGTAC", "ACGTA" * 7]
    for n in list(rng.integers(1, 200, 30)) + list(rng.integers(200, 4200, 30)):
        wins.append(base[rng.integers(0, 4, n)].tobytes().decode())
    for _ in range(30):  # N runs, lowercase (soft-masked) runs, '.' padding like hg38 windows
        n = int(rng.integers(30, 3000))
        s = bytearray(base[rng.integers(0, 4, n)].tobytes())
        for _ in range(int(rng.integers(0, 4))):
            a = int(rng.integers(0, n)); b = min(n, a + int(rng.integers(1, 50)))
            s[a:b] = b"N" * (b - a)
        for _ in range(int(rng.integers(0, 3))):
            a = int(rng.integers(0, n)); b = min(n, a + int(rng.integers(1, 200)))
            s[a:b] = bytes(s[a:b]).lower()
        if rng.random() < 0.3:
            s = bytearray(b"." * int(rng.integers(1, 20))) + s
        wins.append(s.decode())
    return wins


def main():
    from transformers import EsmTokenizer
    d = os.path.join(REF, "nucleotide-transformer-v2-500m-multi-species")
    tok = EsmTokenizer(vocab_file=os.path.join(d, "vocab.txt"), unk_token="<unk>", cls_token="<cls>",
                       pad_token="<pad>", mask_token="<mask>", eos_token=None, model_max_length=2048)
    wins = windows(np.random.default_rng(6))
    full = [tok(w)["input_ids"] for w in wins]
    P = 130
    padded = [tok(w, padding="max_length", max_length=P, truncation=True)["input_ids"] for w in wins]
    assert all(len(p) == P for p in padded)
    sb = [w.encode() for w in wins]
    np.savez_compressed(
        os.path.join(HERE, "kmer_golden.npz"),
        seq_data=np.frombuffer(b"".join(sb), dtype=np.uint8),
        seq_off=np.cumsum([0] + [len(b) for b in sb]).astype(np.int64),
        full_data=np.concatenate([np.asarray(f, dtype=np.int16) for f in full]),
        full_off=np.cumsum([0] + [len(f) for f in full]).astype(np.int64),
        padded130=np.asarray(padded, dtype=np.int16),
        vocab_size=np.int64(len(tok)), special=np.asarray(tok.all_special_ids, dtype=np.int16),
        transformers_version=np.bytes_(__import__("transformers").__version__))
    print(f"kmer_golden: {len(wins)} windows, vocab {len(tok)}")


if __name__ == "__main__":
    main()
