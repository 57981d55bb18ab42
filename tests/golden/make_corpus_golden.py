#!/usr/bin/env python
"""Golden fixtures for the DNABERT-2 text-corpus dataset, made by running the
REFERENCE `DNABERT2Dataset` (src/dataloaders/datasets/dnabert2.py:106-246) in this container.

Run from the repo root:  python tests/golden/make_corpus_golden.py
The reference module is loaded by path (read-only; pyfaidx/polars stubbed, it never uses them on
this path) and run on a synthetic corpus written to a temporary directory. Writes
corpus_golden.npz next to this script: the corpus lines, the packed .bin bytes and
padding_info the reference produced, and dataset items (masked ids, mask, labels, target) for
max_length 128 with left padding (reference default) and right padding (pad_interval=True),
each drawn after torch.manual_seed(1000 + index).
"""
import importlib.util
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = os.environ.get("DNA_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))


def _load_module():
    for name in ("pyfaidx", "polars"):
        m = types.ModuleType(name)
        m.Fasta = None
        sys.modules.setdefault(name, m)
    spec = importlib.util.spec_from_file_location(
        "ref_dnabert2_dataset", os.path.join(REF, "src/dataloaders/datasets/dnabert2.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _tokenizer():
    from transformers import PreTrainedTokenizerFast
    return PreTrainedTokenizerFast(
        tokenizer_file=os.path.join(REF, "DNABERT-2-117M/tokenizer.json"),
        unk_token="[UNK]", cls_token="[CLS]", sep_token="[SEP]", pad_token="[PAD]",
        mask_token="[MASK]")


def corpus_lines(n=60, seed=2222):
    rng = np.random.default_rng(seed)
    lines = []
    for i in range(n):
        # no empty lines: the reference packer raises on them (int("", 2), dnabert2.py:187)
        L = int(rng.choice([1, 2, 3, 4, 5, 7, 8, 50, 127, 300, 640, 1000, 2000]))
        s = "".join(rng.choice(list("ACGT"), size=L))
        if i % 7 == 3 and L > 10:  # N runs and lowercase: packed lossily as A, like the reference
            s = s[:5] + "NNNN" + s[9:].lower()
        lines.append(s)
    return lines


def main():
    mod = _load_module()
    tok = _tokenizer()
    lines = corpus_lines()
    out = {}
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "train.txt"), "w") as f:
            for s in lines:
                f.write(s + "\n")
        for tag, pad_interval in (("left", False), ("right", True)):
            ds = mod.DNABERT2Dataset(split="train", text_file=d, max_length=128, tokenizer=tok,
                                     tokenizer_name="bpe", add_eos=False, pad_interval=pad_interval)
            items = []
            for i in range(len(ds)):
                torch.manual_seed(1000 + i)
                (masked, mask, labels), target = ds[i]
                items.append(np.stack([masked.numpy(), mask.numpy().astype(np.int64),
                                       labels.numpy(), target.numpy()]))
            out[f"items_{tag}"] = np.stack(items)
        with open(os.path.join(d, "train.bin"), "rb") as f:
            out["bin"] = np.frombuffer(f.read(), dtype=np.uint8)
        with open(os.path.join(d, "train_padding_info.json")) as f:
            info = json.load(f)
        out["padding_info"] = np.array([info[str(i + 1)] for i in range(len(info))], dtype=np.int64)
    out["lines"] = np.array(lines, dtype=object).astype(str)
    np.savez_compressed(os.path.join(HERE, "corpus_golden.npz"), **out)
    print("lines", len(lines), "bin bytes", out["bin"].size, "items", out["items_left"].shape)


if __name__ == "__main__":
    main()
