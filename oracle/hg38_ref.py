"""Restatement of the hg38 window extraction and BERT masking (TEST INFRASTRUCTURE).

Oracle only (tests/, smoke(), bench cpu_baseline). Follows
/root/reference/src/dataloaders/datasets/hg38_dataset.py:
  string_reverse_complement  :28-37
  FastaInterval.__call__     :72-124  (shift_augs unused by the hot-path configs)
  bert_mask                  :238-286
Pinned by tests/golden/fasta_golden.json and tests/golden/mask_golden.npz.
"""
import numpy as np

_COMP = {"A": "T", "C": "G", "G": "C", "T": "A", "a": "t", "c": "g", "g": "c", "t": "a"}


def reverse_complement(seq: str) -> str:
    return "".join(_COMP.get(ch, ch) for ch in reversed(seq))


def fasta_interval(chrom: str, start: int, end: int, max_length: int, pad_interval=False) -> str:
    """Window of `chrom` for BED interval [start, end) (hg38_dataset.py:72-124).

    Shorter intervals grow by extra//2 on the left and the rest on the right; the result is
    clamped to the chromosome WITHOUT re-shifting (so edge windows come out shorter); longer
    intervals keep their first max_length bp. '.' padding only with pad_interval.
    """
    L = len(chrom)
    interval_length = end - start
    left_pad = right_pad = 0
    if interval_length < max_length:
        extra = max_length - interval_length
        start -= extra // 2
        end += extra - extra // 2
    if start < 0:
        left_pad, start = -start, 0
    if end > L:
        right_pad, end = end - L, L
    if interval_length > max_length:
        end = start + max_length
    seq = chrom[start:end]
    if pad_interval:
        seq = "." * left_pad + seq + "." * right_pad
    return seq


def bert_mask_from_draws(seq, u1, u2, rand_tok, mask_id=4, pad_id=3, mask_prob=0.15,
                         random_token_prob=0.1, unchanged_token_prob=0.1):
    """bert_mask with its random draws made explicit.

    u1, u2: uniforms in [0,1) per position; rand_tok: a non-special token id per position.
    Returns (masked_seq, mask, labels) exactly as the reference does for the same draws.
    """
    seq = np.asarray(seq, dtype=np.int64)
    mask = (seq != pad_id) & (u1 < mask_prob)
    labels = np.where(mask, seq, -100)
    keep_mask_tok = 1.0 - random_token_prob - unchanged_token_prob
    out = seq.copy()
    out[mask & (u2 < keep_mask_tok)] = mask_id
    sel = mask & (u2 >= keep_mask_tok) & (u2 < 1.0 - unchanged_token_prob)
    out[sel] = np.asarray(rand_tok, dtype=np.int64)[sel]
    return out, mask, labels
