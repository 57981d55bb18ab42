"""DNABERT-2 BPE tokenizer over the native C++ implementation (libdna_amd.so, bpe.cpp).

Drop-in for what BertHG38.setup builds with AutoTokenizer.from_pretrained(root+"/DNABERT-2-117M")
(src/dataloaders/genomics.py:1141) as far as the MLM data path uses it
(src/dataloaders/datasets/hg38_dataset.py:369-379, :393-397): __call__ with
padding="max_length"/max_length/truncation, special ids, vocab size. Bit-exact with HF tokenizers
on the golden windows (tests/test_native_data.py).
"""
import ctypes
import os

import numpy as np

from . import _native as N

DEFAULT_VOCAB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "dnabert2_bpe.json")


class DNABertTokenizer:
    unk_token, cls_token, sep_token, pad_token, mask_token = "[UNK]", "[CLS]", "[SEP]", "[PAD]", "[MASK]"

    def __init__(self, path=None):
        path = path or DEFAULT_VOCAB
        if os.path.isdir(path):  # a HF model dir like DNABERT-2-117M/
            path = os.path.join(path, "tokenizer.json")
        self.path = path
        self._open()

    def _open(self):
        L = N.lib()
        self._h = L.dna_bpe_create(self.path.encode())
        if not self._h:
            raise N.NativeError(f"dna_bpe_create: {N.last_error()}")
        self.vocab_size = L.dna_bpe_vocab_size(self._h)
        self.unk_token_id, self.cls_token_id, self.sep_token_id = 0, 1, 2
        self.pad_token_id, self.mask_token_id = 3, 4

    # the ctypes handle does not pickle: re-open in spawned DataLoader workers (fork shares it)
    def __getstate__(self):
        return {"path": self.path}

    def __setstate__(self, st):
        self.path = st["path"]
        self._open()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                N.lib().dna_bpe_destroy(h)
            except Exception:
                pass
            self._h = None

    def __len__(self):
        return self.vocab_size

    @property
    def all_special_ids(self):
        return [self.unk_token_id, self.sep_token_id, self.pad_token_id, self.cls_token_id,
                self.mask_token_id]

    def encode_raw(self, text):
        b = text.encode() if isinstance(text, str) else bytes(text)
        cap = max(16, len(b) + 8)
        buf = np.empty(cap, dtype=np.int32)
        n = N.lib().dna_bpe_encode(self._h, b, len(b), buf.ctypes.data, cap)
        if n < 0:
            raise N.NativeError(f"dna_bpe_encode: {N.last_error()}")
        return buf[:n].tolist()

    def __call__(self, text, padding=False, max_length=None, truncation=False,
                 add_special_tokens=True):
        ids = self.encode_raw(text)
        n_sp = 2 if add_special_tokens else 0
        if truncation and max_length is not None:
            ids = ids[: max(0, max_length - n_sp)]
        if add_special_tokens:
            ids = [self.cls_token_id] + ids + [self.sep_token_id]
        if padding == "max_length" and max_length is not None and len(ids) < max_length:
            ids = ids + [self.pad_token_id] * (max_length - len(ids))
        return {"input_ids": ids}

    def encode_windows(self, seqs, pad_max_length, add_eos=False, nthreads=0):
        """Dataset-style batch encode (hg38_dataset.py:369-379): int64 [n, P-2(+1 if add_eos)]."""
        bs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
        n = len(bs)
        W = pad_max_length - 2 + (1 if add_eos else 0)
        out = np.empty((n, W), dtype=np.int32)
        if n == 0:
            return out.astype(np.int64)
        arr = (ctypes.c_char_p * n)(*bs)
        lens = np.array([len(b) for b in bs], dtype=np.int32)
        N.call("dna_bpe_encode_batch", self._h, ctypes.cast(arr, ctypes.c_void_p),
               lens.ctypes.data, n, pad_max_length, int(add_eos), out.ctypes.data, None,
               int(nthreads))
        return out.astype(np.int64)


def from_pretrained(path=None):
    return DNABertTokenizer(path)
