"""Character tokenizer (hg38 `char` path, HyenaDNA configs): semantics restated from
hg38_char_tokenizer.py:15-140 (the reference class does not construct under transformers 5.x, so
expected values are derived from its source: ids 7.. for ACGTN, [SEP] appended with specials,
left padding). CPU."""
import torch


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
