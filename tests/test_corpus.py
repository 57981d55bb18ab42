"""DNABERT-2 text-corpus dataset (dna_amd/corpus.py) against the reference DNABERT2Dataset's own
outputs (tests/golden/corpus_golden.npz from tests/golden/make_corpus_golden.py): packed bytes,
padding info and items bit-for-bit for left (default) and right (pad_interval) padding. CPU."""
import json
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden", "corpus_golden.npz")


@pytest.fixture(scope="module")
def corpus_dir(tmp_path_factory):
    z = np.load(GOLD)
    d = tmp_path_factory.mktemp("corpus")
    with open(d / "train.txt", "w") as f:
        for s in z["lines"]:
            f.write(str(s) + "\n")
    return d, z


def test_packing_matches_reference(corpus_dir):
    from dna_amd.corpus import PackedCorpus, pack_text_corpus
    d, z = corpus_dir
    pack_text_corpus(str(d / "train.txt"))
    assert np.array_equal(np.fromfile(d / "train.bin", dtype=np.uint8), z["bin"])
    info = json.load(open(d / "train_padding_info.json"))
    assert np.array_equal(np.array([info[str(i + 1)] for i in range(len(info))]), z["padding_info"])
    pc = PackedCorpus(str(d / "train.bin"), str(d / "train_padding_info.json"))
    for i, s in enumerate(z["lines"]):
        s = str(s)
        lossy = "".join(c if c in "ACGT" else "A" for c in s)  # N / lowercase pack as 00
        assert pc.line(i) == lossy


@pytest.mark.parametrize("tag,pad_interval", [("left", False), ("right", True)])
def test_items_match_reference(corpus_dir, tag, pad_interval):
    from dna_amd.corpus import DNABERT2Dataset
    from dna_amd.tokenizer import DNABertTokenizer
    d, z = corpus_dir
    ds = DNABERT2Dataset(split="train", text_file=str(d), max_length=128,
                         tokenizer=DNABertTokenizer(), tokenizer_name="bpe", add_eos=False,
                         pad_interval=pad_interval)
    ref = z[f"items_{tag}"]
    assert len(ds) == ref.shape[0]
    for i in range(len(ds)):
        torch.manual_seed(1000 + i)
        (masked, mask, labels), target = ds[i]
        got = np.stack([masked.numpy(), mask.numpy().astype(np.int64), labels.numpy(), target.numpy()])
        assert np.array_equal(got, ref[i]), f"item {i}"


def test_empty_line_rejected_like_reference(tmp_path):
    from dna_amd.corpus import pack_text_corpus
    (tmp_path / "train.txt").write_text("ACGT\n\nTTGA\n")
    with pytest.raises(ValueError):
        pack_text_corpus(str(tmp_path / "train.txt"))


def test_data_module_registry(corpus_dir):
    from dna_amd.hg38 import SequenceDataset
    import dna_amd.corpus  # noqa: F401  (registers "dnabert2_pretrain")
    d, _ = corpus_dir
    import shutil
    for split in ("dev",):
        shutil.copy(d / "train.txt", d / f"{split}.txt")
    dm = SequenceDataset.registry["dnabert2_pretrain"](text_file=str(d), tokenizer_name="bpe",
                                                       max_length=128, batch_size=4, add_eos=False)
    dm.setup()
    (masked, mask, labels), target = next(iter(dm.train_dataloader()))
    assert masked.shape == (4, 128) and mask.dtype == torch.bool and target.shape == (4, 128)
    assert len(dm.dataset_val) == len(dm.dataset_test) == len(dm.dataset_train)
