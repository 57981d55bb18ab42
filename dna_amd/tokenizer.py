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


class CharacterTokenizer:
    """Character-level tokenizer of the hg38 `char` path and the HyenaDNA configs
    (reference src/dataloaders/datasets/hg38_char_tokenizer.py:15-140, built in
    genomics.py:1132-1138 with characters ACGTN and model_max_length = max_length + 2).

    ids: [CLS]=0 [SEP]=1 [BOS]=2 [MASK]=3 [PAD]=4 [RESERVED]=5 [UNK]=6, characters from 7;
    any other character (lowercase, space) -> [UNK]. With special tokens the sequence is
    `ids + [SEP]` (build_inputs_with_special_tokens, :88-96); truncation keeps room for it;
    padding with [PAD] on the LEFT (padding_side default 'left').
    Parity: tests/golden/char_golden.npz -- the reference class's constructor body and methods
    run unmodified by tests/golden/make_char_golden.py (its base-class constructor, which fails
    under the transformers 5.x here, replaced by a recorder); the 4.28 padding / truncation of
    __call__ around them is restated (tests/test_char_tokenizer.py)."""
    special = {"[CLS]": 0, "[SEP]": 1, "[BOS]": 2, "[MASK]": 3, "[PAD]": 4, "[RESERVED]": 5,
               "[UNK]": 6}

    def __init__(self, characters, model_max_length, padding_side="left", **kwargs):
        self.characters = list(characters)
        self.model_max_length = model_max_length
        self.padding_side = padding_side
        self._vocab_str_to_int = dict(self.special)
        self._vocab_str_to_int.update({ch: i + 7 for i, ch in enumerate(self.characters)})
        self._vocab_int_to_str = {v: k for k, v in self._vocab_str_to_int.items()}
        self._lut = np.full(256, 6, dtype=np.int64)
        for ch, i in self._vocab_str_to_int.items():
            if len(ch) == 1 and ord(ch) < 256:
                self._lut[ord(ch)] = i
        self.cls_token_id, self.sep_token_id, self.bos_token_id = 0, 1, 2
        self.mask_token_id, self.pad_token_id, self.unk_token_id = 3, 4, 6
        self.eos_token_id = self.sep_token_id

    @property
    def vocab_size(self):
        return len(self._vocab_str_to_int)

    def __len__(self):
        return self.vocab_size

    @property
    def all_special_ids(self):
        return [self.bos_token_id, self.eos_token_id, self.unk_token_id, self.pad_token_id,
                self.cls_token_id, self.mask_token_id]

    def complement_map(self):
        """{id: id of the complementary base} over the whole vocabulary (A<->T, C<->G, either
        case when both are characters; every other id maps to itself) -- the `complement_map` a
        Caduceus rcps=True model takes (RCPSEmbedding / RCPSLMHead, reference
        src/models/caduceus/modeling_rcps.py:18-64, :206-243)."""
        pairs = {"A": "T", "T": "A", "C": "G", "G": "C", "a": "t", "t": "a", "c": "g", "g": "c"}
        v = self._vocab_str_to_int
        return {i: v.get(pairs.get(s, s), i) if s in pairs else i
                for s, i in sorted(v.items(), key=lambda kv: kv[1])}

    def encode_raw(self, text):
        b = np.frombuffer(text.encode("latin-1", errors="replace"), dtype=np.uint8)
        return self._lut[b].tolist()

    def __call__(self, text, padding=False, max_length=None, truncation=False,
                 add_special_tokens=True):
        ids = self.encode_raw(text)
        n_sp = 1 if add_special_tokens else 0
        if truncation and max_length is not None:
            ids = ids[: max(0, max_length - n_sp)]
        if add_special_tokens:
            ids = ids + [self.sep_token_id]
        if padding == "max_length" and max_length is not None and len(ids) < max_length:
            pad = [self.pad_token_id] * (max_length - len(ids))
            ids = pad + ids if self.padding_side == "left" else ids + pad
        return {"input_ids": ids}


class KmerTokenizer:
    """The NT-v2 6-mer tokenizer of `bert_hg38` with tokenizer_name=kmer (reference
    genomics.py:1142-1144 -> AutoTokenizer.from_pretrained("nucleotide-transformer-v2-500m-
    multi-species") = transformers' EsmTokenizer over its vocab.txt, no eos).

    Vocabulary (identical to that vocab.txt, generated rather than shipped): <unk> <pad> <mask>
    <cls> <eos> <bos>, the 4096 6-mers in A,T,C,G order (AAAAAA, AAAAAT, ...), then A T C G N.
    Tokenisation is EsmTokenizer's: every vocabulary entry is a no-split token, matched greedily
    left to right, longest first (a 6-mer where one fits, else a single nucleotide); characters
    no entry matches (lowercase, '.', other letters) form runs that are split on whitespace, each
    piece -> <unk>; then <cls> in front. padding="max_length" pads with <pad> on the right,
    truncation cuts at max_length (the <cls> included). Parity: tests/golden/kmer_golden.npz
    (make_kmer_golden.py: EsmTokenizer on the reference vocab -- the reference's own
    from_pretrained call fails on a corrupt special_tokens_map.json, see that script)."""

    SPECIALS = ["<unk>", "<pad>", "<mask>", "<cls>", "<eos>", "<bos>"]

    def __init__(self, k=6, model_max_length=2048):
        import itertools
        self.k = k
        toks = self.SPECIALS + ["".join(p) for p in itertools.product("ATCG", repeat=k)] + list("ATCGN")
        self.vocab = {t: i for i, t in enumerate(toks)}
        self.ids_to_tokens = toks
        self.unk_token_id, self.pad_token_id, self.mask_token_id, self.cls_token_id = 0, 1, 2, 3
        self.eos_token_id = None
        self.model_max_length = model_max_length

    def __len__(self):
        return len(self.ids_to_tokens)

    @property
    def vocab_size(self):
        return len(self.ids_to_tokens)

    @property
    def all_special_ids(self):
        # transformers' order for these special tokens: unk, pad, cls, mask
        return [self.unk_token_id, self.pad_token_id, self.cls_token_id, self.mask_token_id]

    def encode_raw(self, text):
        v, k = self.vocab, self.k
        n = len(text)
        out, i, run = [], 0, []
        while i < n:
            tok = text[i:i + k] if i + k <= n else None
            if tok is not None and tok in v:
                hit, step = v[tok], k
            elif text[i] in v and len(text[i]) == 1 and text[i] in "ATCGN":
                hit, step = v[text[i]], 1
            else:
                run.append(text[i])
                i += 1
                continue
            if run:
                out.extend(self.unk_token_id for _ in "".join(run).split())
                run = []
            out.append(hit)
            i += step
        if run:
            out.extend(self.unk_token_id for _ in "".join(run).split())
        return out

    def __call__(self, text, padding=False, max_length=None, truncation=False,
                 add_special_tokens=True):
        ids = ([self.cls_token_id] if add_special_tokens else []) + self.encode_raw(text)
        if truncation and max_length is not None:
            ids = ids[:max_length]
        if padding == "max_length" and max_length is not None and len(ids) < max_length:
            ids = ids + [self.pad_token_id] * (max_length - len(ids))
        return {"input_ids": ids}

    def convert_ids_to_tokens(self, ids):
        return [self.ids_to_tokens[i] for i in ids]
