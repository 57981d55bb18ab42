"""CPU tests of the native library's host side and the data path (no GPU needed).

The C-ABI library must load and export every symbol declared in include/dna_amd.h; the C++ BPE,
masking and FASTA windowing must reproduce the reference golden vectors bit-exactly.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from oracle import hg38_ref
from oracle.bpe import BPERef
from tests.conftest import BPE_JSON, GOLDEN


def _windows():
    z = np.load(os.path.join(GOLDEN, "tok_golden.npz"))
    data, off = z["seq_data"].tobytes(), z["seq_off"]
    return z, [data[off[i]:off[i + 1]] for i in range(len(off) - 1)]


def test_library_exports_every_declared_symbol():
    from dna_amd import _native as N
    L = N.lib()
    syms = N.declared_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert L.dna_abi_version() == 1


def test_error_reporting():
    from dna_amd import _native as N
    L = N.lib()
    assert not L.dna_bpe_create(b"/nonexistent/tokenizer.json")
    assert "cannot open" in N.last_error()
    with pytest.raises(N.NativeError):
        N.call("dna_fasta_interval", None, b"chr1", 0, 10, 10, 0, 0, None, 0, None)


def test_cpp_bpe_full_encode_bit_exact():
    from dna_amd.tokenizer import DNABertTokenizer
    tok = DNABertTokenizer()
    z, wins = _windows()
    fo, fd = z["full_off"], z["full_data"]
    for i, w in enumerate(wins):
        got = tok(w.decode())["input_ids"]
        assert got == fd[fo[i]:fo[i + 1]].astype(np.int64).tolist(), i


@pytest.mark.parametrize("P,key", [(130, "ds130"), (514, "ds514")])
def test_cpp_bpe_dataset_batch_bit_exact(P, key):
    from dna_amd.tokenizer import DNABertTokenizer
    tok = DNABertTokenizer()
    z, wins = _windows()
    out = tok.encode_windows(wins, P, nthreads=4)
    np.testing.assert_array_equal(out, z[key].astype(np.int64))
    # single-sample HF-style call path, as BertHG38Dataset uses it
    for i in range(0, len(wins), 17):
        ids = tok(wins[i].decode(), padding="max_length", max_length=P, truncation=True)["input_ids"]
        assert ids[1:-1] == z[key][i].astype(np.int64).tolist()


def test_cpp_bpe_reads_hf_tokenizer_json(tmp_path):
    """The reference's own tokenizer.json layout is accepted too (vocab dict + 'a b' merges)."""
    from dna_amd.tokenizer import DNABertTokenizer
    c = json.load(open(BPE_JSON))
    hf = {"version": "1.0", "added_tokens": [{"id": i, "content": t, "special": True}
                                             for t, i in c["special_tokens"].items()],
          "normalizer": None, "pre_tokenizer": {"type": "Whitespace"},
          "model": {"type": "BPE", "unk_token": c["unk_token"], "fuse_unk": False,
                    "vocab": {t: i for i, t in enumerate(c["tokens"])},
                    "merges": [" ".join(m) for m in c["merges"]]}}
    p = tmp_path / "tokenizer.json"
    p.write_text(json.dumps(hf))
    a, b = DNABertTokenizer(str(tmp_path)), DNABertTokenizer()
    z, wins = _windows()
    for w in wins[:60]:
        assert a.encode_raw(w) == b.encode_raw(w)


def test_cpp_bpe_matches_python_oracle_random_edge_text():
    from dna_amd.tokenizer import DNABertTokenizer
    tok, ref = DNABertTokenizer(), BPERef(BPE_JSON)
    rng = np.random.default_rng(5)
    alphabet = list("ACGTNacgtn.-_ [MASK][PAD]xyz09\t\n")
    for _ in range(200):
        s = "".join(rng.choice(alphabet, size=int(rng.integers(0, 120))))
        assert tok.encode_raw(s) == ref.encode(s), repr(s)


def test_native_bert_mask_from_draws_exact():
    from dna_amd.hg38 import bert_mask_from_draws
    z = np.load(os.path.join(GOLDEN, "mask_golden.npz"))
    for s in range(12):
        out, mask, labels = bert_mask_from_draws(
            z[f"s{s}_seq"].astype(np.int64), z[f"s{s}_u1"], z[f"s{s}_u2"],
            z[f"s{s}_rt"].astype(np.int64))
        np.testing.assert_array_equal(out.numpy(), z[f"s{s}_out_seq"])
        np.testing.assert_array_equal(mask.numpy(), z[f"s{s}_out_mask"])
        np.testing.assert_array_equal(labels.numpy(), z[f"s{s}_out_labels"])


def test_bert_mask_reproduces_reference_torch_draws():
    """Same torch seed -> identical output to the reference bert_mask (same draw order)."""
    from dna_amd.hg38 import bert_mask
    z = np.load(os.path.join(GOLDEN, "mask_golden.npz"))
    for s in range(12):
        torch.manual_seed(s)
        out, mask, labels = bert_mask(torch.as_tensor(z[f"s{s}_seq"].astype(np.int64)), 4, 3, 4096,
                                      special_token_ids=[0, 2, 3, 1, 4])
        np.testing.assert_array_equal(out.numpy(), z[f"s{s}_out_seq"])
        np.testing.assert_array_equal(labels.numpy(), z[f"s{s}_out_labels"])


def test_bert_mask_fast_statistics():
    from dna_amd.hg38 import bert_mask_fast
    seq = torch.randint(5, 4096, (200_000,))
    seq[-1000:] = 3
    out, mask, labels = bert_mask_fast(seq, 4, 3, 4096, [0, 2, 3, 1, 4], seed=7, sample_id=11)
    assert not mask[-1000:].any()                     # pads never masked
    rate = mask[:-1000].float().mean().item()
    assert abs(rate - 0.15) < 0.005
    m = mask
    frac_mask = (out[m] == 4).float().mean().item()
    frac_same = (out[m] == seq[m]).float().mean().item()
    assert abs(frac_mask - 0.8) < 0.01 and abs(frac_same - 0.1) < 0.01
    rnd = out[m & (out != 4) & (out != seq)]
    assert not torch.isin(rnd, torch.tensor([0, 1, 2, 3, 4])).any()
    np.testing.assert_array_equal(labels[m].numpy(), seq[m].numpy())
    assert (labels[~m] == -100).all()
    out2, _, _ = bert_mask_fast(seq, 4, 3, 4096, [0, 2, 3, 1, 4], seed=7, sample_id=11)
    assert torch.equal(out, out2)
    out3, _, _ = bert_mask_fast(seq, 4, 3, 4096, [0, 2, 3, 1, 4], seed=7, sample_id=12)
    assert not torch.equal(out, out3)


def _write_fasta(path, chroms, width, with_fai):
    fai = []
    with open(path, "wb") as f:
        for name, seq in chroms.items():
            f.write(f">{name} description text\n".encode())
            off = f.tell()
            for i in range(0, len(seq), width):
                f.write(seq[i:i + width].encode() + b"\n")
            fai.append(f"{name}\t{len(seq)}\t{off}\t{width}\t{width + 1}\n")
    if with_fai:
        open(str(path) + ".fai", "w").writelines(fai)


@pytest.mark.parametrize("width,with_fai", [(60, True), (60, False), (17, False), (5000, True)])
def test_fasta_interval_matches_reference(tmp_path, width, with_fai):
    from dna_amd.hg38 import FastaInterval
    g = json.load(open(os.path.join(GOLDEN, "fasta_golden.json")))
    fa = tmp_path / "g.fa"
    _write_fasta(fa, g["chroms"], width, with_fai)
    for pad in (False, True):
        fi = FastaInterval(fasta_file=str(fa), pad_interval=pad)
        assert fi.chr_lens == {k: len(v) for k, v in g["chroms"].items()}
        for c in g["cases"]:
            if c["pad_interval"] != pad:
                continue
            assert fi(c["chr"], c["start"], c["end"], c["max_length"]) == c["out"], c
    fi = FastaInterval(fasta_file=str(fa), rc_aug=True)
    seen = set()
    for _ in range(40):  # coin flip: both orientations appear, each exact
        s = fi("chr2", 100, 300, 200)
        fwd = hg38_ref.fasta_interval(g["chroms"]["chr2"], 100, 300, 200)
        assert s in (fwd, hg38_ref.reverse_complement(fwd))
        seen.add(s == fwd)
    assert seen == {True, False}


def test_bert_hg38_dataset_item(tmp_path):
    from dna_amd.hg38 import BertHG38
    from dna_amd.synthetic import write_hg38
    write_hg38(str(tmp_path), n_chroms=2, chrom_len=50_000, max_length=1024)
    dm = BertHG38(bed_file=str(tmp_path / "bert_hg38/human-sequences.bed"),
                  fasta_file=str(tmp_path / "bert_hg38/hg38.ml.fa"), tokenizer_name="bpe",
                  max_length=1024, pad_max_length=130, add_eos=False, batch_size=4,
                  num_workers=0)
    dm.setup()
    assert len(dm.dataset_train) > 0 and len(dm.dataset_val) > 0
    torch.manual_seed(3)
    (masked, mask, labels), target = dm.dataset_train[0]
    assert masked.shape == mask.shape == labels.shape == target.shape == (128,)
    # the same window through the oracle pipeline
    chr_name, start, end = dm.dataset_train.rows[0]
    chrom = dm.dataset_train.fasta(chr_name, 0, dm.dataset_train.fasta.chr_lens[chr_name],
                                   max_length=dm.dataset_train.fasta.chr_lens[chr_name])
    window = hg38_ref.fasta_interval(chrom, start, end, 1024)
    ref_ids = BPERef(BPE_JSON).encode_dataset(window, 130)
    assert target.tolist() == ref_ids
    batch = next(iter(dm.train_dataloader()))
    assert batch[0][0].shape == (4, 128) and batch[1].shape == (4, 128)


def test_bert_hg38_masks_change_per_epoch(tmp_path):
    """Batched path (Philox masks): the same window gets a fresh mask every epoch (the
    reference draws torch RNG per __getitem__, hg38_dataset.py:258-279) and the same mask when
    an epoch is replayed (mid-epoch resume); the DistributedSampler permutation is
    randperm(seed + epoch) on one rank too."""
    from dna_amd.hg38 import BertHG38
    from dna_amd.synthetic import write_hg38
    write_hg38(str(tmp_path), n_chroms=1, chrom_len=60_000, max_length=1024)
    dm = BertHG38(bed_file=str(tmp_path / "bert_hg38/human-sequences.bed"),
                  fasta_file=str(tmp_path / "bert_hg38/hg38.ml.fa"), tokenizer_name="bpe",
                  max_length=1024, pad_max_length=130, add_eos=False, batch_size=4,
                  num_workers=0)
    dm.setup()
    ds = dm.dataset_train
    smp = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=1, rank=0, shuffle=True,
                                                          seed=7)
    loader = dm.train_dataloader(sampler=smp)

    def epoch_masks(e):
        loader.sampler.set_epoch(e)
        order = list(smp)
        out = {}
        for (masked, mask, labels), target in loader:
            for j in range(target.shape[0]):
                out[len(out)] = (mask[j].clone(), target[j].clone())
        # window id -> mask, via the epoch's permutation
        return {order[k]: v for k, v in out.items()}

    e0, e0b, e1 = epoch_masks(0), epoch_masks(0), epoch_masks(1)
    assert set(e0) == set(e1) == set(range(len(ds)))
    same = sum(torch.equal(e0[i][0], e1[i][0]) for i in e0)
    assert same == 0, f"{same} windows kept their epoch-0 mask in epoch 1"
    for i in e0:
        assert torch.equal(e0[i][0], e0b[i][0]) and torch.equal(e0[i][1], e1[i][1])
    loader.sampler.set_epoch(0)
    p0 = list(smp)
    loader.sampler.set_epoch(1)
    assert p0 != list(smp)
