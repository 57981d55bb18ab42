"""NT-v2 6-mer tokenizer (bert_hg38 tokenizer_name=kmer, reference genomics.py:1142-1144) vs the
EsmTokenizer golden vectors (tests/golden/kmer_golden.npz, make_kmer_golden.py): full ids and
the dataset-style padded/truncated form at 130."""
import os

import numpy as np

from tests.conftest import GOLDEN


def test_kmer_tokenizer_matches_golden():
    from dna_amd.tokenizer import KmerTokenizer
    z = np.load(os.path.join(GOLDEN, "kmer_golden.npz"))
    tok = KmerTokenizer()
    assert len(tok) == int(z["vocab_size"]) == 4107
    assert sorted(tok.all_special_ids) == sorted(z["special"].tolist())
    seqs = z["seq_data"].tobytes()
    so, fo = z["seq_off"], z["full_off"]
    n = len(so) - 1
    assert n > 100
    for i in range(n):
        s = seqs[so[i]:so[i + 1]].decode()
        want = z["full_data"][fo[i]:fo[i + 1]].tolist()
        assert tok(s)["input_ids"] == want, (i, s[:40])
        assert tok(s, padding="max_length", max_length=130, truncation=True)["input_ids"] == \
            z["padded130"][i].tolist(), i


def test_bert_hg38_kmer_setup(tmp_path, monkeypatch):
    """tokenizer_name=kmer builds the data module with this tokenizer; items raise like the
    reference, whose BertHG38Dataset has no kmer branch (hg38_dataset.py:357-380)."""
    import pytest
    from dna_amd.hg38 import BertHG38
    from dna_amd.synthetic import write_hg38
    write_hg38(str(tmp_path), n_chroms=1, chrom_len=100_000, max_length=1024)
    monkeypatch.setenv("DATA_PATH", str(tmp_path))
    dm = BertHG38(tokenizer_name="kmer", max_length=1024)
    dm.setup()
    assert dm.vocab_size == 4107 and dm.tokenizer.cls_token_id == 3
    with pytest.raises(NotImplementedError, match="kmer"):
        dm.dataset_train[0]
