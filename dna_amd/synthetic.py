"""Synthetic hg38-shaped inputs (no network, no genome download) -- SURVEY §8(d).

FASTA chr1..chr8, 4,194,304 bp each, i.i.d. uniform {A,C,G,T} (numpy PCG64, seed 2222), 60 bp
lines, with a samtools-style .fai; BED `chr_name start end split` tiling each chromosome with
non-overlapping windows of `max_length` bp: window i -> valid if i%200==0, test if i%200==1,
train otherwise. Written as $DATA_PATH/bert_hg38/{human-sequences.bed,hg38.ml.fa(.fai)}, the
default paths of BertHG38 (genomics.py:1112-1115).
"""
import os

import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def random_windows(n, length, seed):
    """n uniform-ACGT windows (bytes) of `length` bp."""
    rng = np.random.default_rng(seed)
    codes = rng.integers(0, 4, size=(n, length), dtype=np.uint8)
    arr = ACGT[codes]
    return [arr[i].tobytes() for i in range(n)]


def write_hg38(root, n_chroms=8, chrom_len=4_194_304, max_length=4096, seed=2222, line=60):
    d = os.path.join(root, "bert_hg38")
    os.makedirs(d, exist_ok=True)
    fa = os.path.join(d, "hg38.ml.fa")
    bed = os.path.join(d, "human-sequences.bed")
    rng = np.random.default_rng(seed)
    fai = []
    with open(fa, "wb") as f:
        for c in range(1, n_chroms + 1):
            name = f"chr{c}"
            seq = ACGT[rng.integers(0, 4, size=chrom_len, dtype=np.uint8)]
            hdr = f">{name}\n".encode()
            f.write(hdr)
            off = f.tell()
            full = chrom_len // line
            body = seq[: full * line].reshape(full, line)
            nl = np.full((full, 1), ord("\n"), dtype=np.uint8)
            f.write(np.concatenate([body, nl], axis=1).tobytes())
            rest = seq[full * line:]
            if rest.size:
                f.write(rest.tobytes() + b"\n")
            fai.append(f"{name}\t{chrom_len}\t{off}\t{line}\t{line + 1}\n")
    with open(fa + ".fai", "w") as f:
        f.writelines(fai)
    with open(bed, "w") as f:
        i = 0
        for c in range(1, n_chroms + 1):
            for s in range(0, chrom_len - max_length + 1, max_length):
                split = "valid" if i % 200 == 0 else ("test" if i % 200 == 1 else "train")
                f.write(f"chr{c}\t{s}\t{s + max_length}\t{split}\n")
                i += 1
    return fa, bed
