"""DNABERT-2 text-corpus MLM dataset (registry dataset "dnabert2_pretrain").

Same on-disk format, item structure and error behaviour as the reference
(src/dataloaders/datasets/dnabert2.py:106-246, data module src/dataloaders/genomics.py:1326-1500):

* `<text_file>/<split>.txt` (val/test read `dev`), one sequence per line, is packed once into
  `<split>.bin`: 2 bits per base, most significant bits first, A=00 T=01 C=10 G=11 and every
  other character (N, lowercase) -> 00 (lossy, :163-171); each line padded with zero bits to a
  whole byte. `<split>_padding_info.json` maps the 1-based line number to
  [bytes in the line, pad bits] (:173-189). An empty line makes the reference packer raise
  (int("", 2)); so does this one.
* Items: decode the line, BPE-encode without special tokens truncated to `max_length`, optional
  eos, pad to `pad_max_length` (= max_length; the data module never passes it) with [PAD] on the
  LEFT unless `pad_interval` (:205-222), then `bert_mask` (the hg38 one: same torch draw order)
  -> `((masked, mask, labels), target)`; objective != "stdmlm" -> `(random_mask(...), target)`.

Unlike the reference, which reads the whole .bin into a list of per-line bytes objects, the
packed corpus is memory-mapped and addressed through a byte-offset table (fork-friendly for
DataLoader workers); decoding is a 256-entry byte -> 4-base lookup.
"""
import json
import math
import os

import numpy as np
import torch

from .hg38 import FaultTolerantMixin, SequenceDataset, bert_mask, random_mask
from .tokenizer import DNABertTokenizer

_CODE = np.zeros(256, dtype=np.uint8)  # char -> 2-bit code (unknown -> 0 = 'A')
for _c, _v in (("A", 0), ("T", 1), ("C", 2), ("G", 3)):
    _CODE[ord(_c)] = _v
_BASES = np.frombuffer(b"ATCG", dtype=np.uint8)
# byte -> its 4 bases, most significant pair first
_LUT4 = np.stack([_BASES[(np.arange(256) >> s) & 3] for s in (6, 4, 2, 0)], axis=1).astype(np.uint8)


def pack_line(line: str) -> bytes:
    """One stripped line -> its packed bytes (dnabert2.py:180-187)."""
    if not line:
        raise ValueError("invalid literal for int() with base 2: '' (empty corpus line; the "
                         "reference packer rejects it too, dnabert2.py:187)")
    codes = _CODE[np.frombuffer(line.encode("latin-1"), dtype=np.uint8)]
    n = len(codes)
    nb = math.ceil(n / 4)
    padded = np.zeros(nb * 4, dtype=np.uint8)
    padded[:n] = codes
    q = padded.reshape(nb, 4).astype(np.uint16)
    return ((q[:, 0] << 6) | (q[:, 1] << 4) | (q[:, 2] << 2) | q[:, 3]).astype(np.uint8).tobytes()


def pack_text_corpus(txt_path, bin_path=None):
    """Write `<split>.bin` and `<split>_padding_info.json` next to `<split>.txt` exactly as the
    reference's convert_dna_to_binary does (its json name: txt path minus ".txt" + "_padding_info.json")."""
    txt_path = str(txt_path)
    bin_path = str(bin_path) if bin_path else txt_path[:-4] + ".bin"
    info = {}
    with open(txt_path) as fin, open(bin_path, "wb") as fout:
        for ln, line in enumerate(fin, 1):
            s = line.strip()
            b = pack_line(s)
            bits = 2 * len(s)
            info[ln] = [math.ceil(len(s) / 4), (8 - bits % 8) % 8]
            fout.write(b)
    with open(txt_path[:-4] + "_padding_info.json", "w") as f:
        json.dump(info, f)
    return bin_path


class PackedCorpus:
    """Memory-mapped packed corpus: line i -> decoded string."""

    def __init__(self, bin_path, info_path):
        with open(info_path) as f:
            info = json.load(f)
        n = len(info)
        arr = np.array([info[str(i + 1)] for i in range(n)], dtype=np.int64).reshape(n, 2)
        self.nbytes = arr[:, 0]
        self.padbits = arr[:, 1]
        self.offsets = np.concatenate([[0], np.cumsum(self.nbytes)])
        size = os.path.getsize(bin_path)
        if size < self.offsets[-1]:
            raise ValueError(f"{bin_path}: {size} bytes < {self.offsets[-1]} listed in the padding info")
        self.data = np.memmap(bin_path, dtype=np.uint8, mode="r") if size else np.zeros(0, np.uint8)

    def __len__(self):
        return len(self.nbytes)

    def line(self, i):
        o, nb = int(self.offsets[i]), int(self.nbytes[i])
        if nb == 0:  # format(0, '00b') -> '0' -> one unmapped 1-bit "pair" -> 'N' (dnabert2.py:199-207)
            return "N"
        nbases = (8 * nb - int(self.padbits[i])) // 2
        return _LUT4[np.asarray(self.data[o:o + nb])].reshape(-1)[:nbases].tobytes().decode("ascii")


class DNABERT2Dataset(torch.utils.data.Dataset):
    """Reference `DNABERT2Dataset` (dnabert2.py:106-246), same constructor."""

    def __init__(self, split, text_file, max_length, pad_max_length=None, tokenizer_name=None,
                 add_eos=False, replace_N_token=False, pad_interval=False, use_tokenizer=True,
                 tokenizer=None, return_augs=False, objective="stdmlm"):
        self.max_length = max_length
        self.pad_max_length = pad_max_length if pad_max_length is not None else max_length
        self.tokenizer_name = tokenizer_name
        self.add_eos = add_eos
        self.replace_N_token = replace_N_token
        self.pad_interval = pad_interval
        self.use_tokenizer = use_tokenizer
        self.tokenizer = tokenizer
        self.return_augs = return_augs
        self.objective = objective
        if not use_tokenizer:
            raise NotImplementedError("use_tokenizer=False (char-level ids, SURVEY §8f row 4)")
        if replace_N_token:
            raise NotImplementedError("replace_N_token needs the char tokenizer's vocab (SURVEY §8f row 4)")
        self.split = split if split not in ("val", "test") else "dev"
        base = os.path.join(str(text_file), self.split)
        self.bin_path = base + ".bin"
        if not os.path.exists(self.bin_path):
            pack_text_corpus(base + ".txt", self.bin_path)
        self.corpus = PackedCorpus(self.bin_path, base + "_padding_info.json")
        self.length = len(self.corpus)

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        tok = self.tokenizer
        line = self.corpus.line(idx)
        tokens = tok.encode_raw(line)[: self.max_length]
        if self.add_eos:
            eos = getattr(tok, "eos_token_id", None)
            if eos is None:
                raise TypeError("add_eos=True but the tokenizer has no eos token (the reference "
                                "fails the same way building the LongTensor)")
            tokens.append(eos)
        if len(tokens) > self.max_length:
            tokens = tokens[: self.max_length]
        if len(tokens) < self.pad_max_length:
            pad = [tok.pad_token_id] * (self.pad_max_length - len(tokens))
            tokens = tokens + pad if self.pad_interval else pad + tokens
        seq = torch.LongTensor(tokens)
        data = seq.clone()
        target = seq.clone()
        if self.objective == "stdmlm":
            return bert_mask(data, tok.mask_token_id, tok.pad_token_id, tok.vocab_size,
                             special_token_ids=tok.all_special_ids), target
        return random_mask(data, tok.mask_token_id), target


class DNABERT2Pretrain(FaultTolerantMixin, SequenceDataset):
    """Data module "dnabert2_pretrain" (genomics.py:1326-1500)."""
    _name_ = "dnabert2_pretrain"

    def __init__(self, text_file=None, tokenizer_name=None, dataset_config_name=None, max_length=1024,
                 d_output=2, rc_aug=False, max_length_val=None, max_length_test=None,
                 val_ratio=0.0005, val_split_seed=2357, use_fixed_len_val=False, add_eos=True,
                 detokenize=False, val_only=False, batch_size=32, batch_size_eval=None,
                 num_workers=1, shuffle=False, pin_memory=False, drop_last=False,
                 fault_tolerant=False, ddp=False, fast_forward_epochs=None,
                 fast_forward_batches=None, replace_N_token=False, pad_interval=False,
                 use_tokenizer=True, objective="stdmlm", tokenizer_path=None, **kwargs):
        if text_file is None:  # like bert_hg38's default paths: $DATA_PATH/<dataset name>
            text_file = os.path.join(os.environ.get("DATA_PATH", os.path.join(os.getcwd(), "data")),
                                     "dnabert2")
        if use_fixed_len_val:
            raise NotImplementedError("use_fixed_len_val (BertHG38FixedDataset) is out of scope")
        self.text_file = text_file
        self.tokenizer_name = tokenizer_name
        self.tokenizer_path = tokenizer_path
        self.max_length = max_length
        self.max_length_val = max_length_val if max_length_val is not None else max_length
        self.max_length_test = max_length_test if max_length_test is not None else max_length
        self.add_eos = add_eos
        self.batch_size = batch_size
        self.batch_size_eval = batch_size_eval if batch_size_eval is not None else batch_size
        self.num_workers = num_workers
        self.shuffle = shuffle
        self.pin_memory = pin_memory
        self.drop_last = drop_last
        self.replace_N_token = replace_N_token
        self.pad_interval = pad_interval
        self.use_tokenizer = use_tokenizer
        self.objective = objective
        self._init_fault_tolerant(shuffle, fault_tolerant, ddp, fast_forward_epochs,
                                  fast_forward_batches)

    def setup(self, stage=None):
        if self.tokenizer_name != "bpe":
            raise NotImplementedError(f"tokenizer_name={self.tokenizer_name!r}: bpe only (SURVEY §8f row 4)")
        self.tokenizer = DNABertTokenizer(self.tokenizer_path)
        self.vocab_size = len(self.tokenizer)
        self.dataset_train, self.dataset_val, self.dataset_test = [
            DNABERT2Dataset(split=split, text_file=self.text_file, max_length=ml,
                            tokenizer=self.tokenizer, tokenizer_name=self.tokenizer_name,
                            add_eos=self.add_eos, replace_N_token=self.replace_N_token,
                            pad_interval=self.pad_interval, use_tokenizer=self.use_tokenizer,
                            objective=self.objective)
            for split, ml in zip(["train", "val", "test"],
                                 [self.max_length, self.max_length_val, self.max_length_test])]

    def _data_loader(self, dataset, batch_size, shuffle=False, sampler=None):
        from .hg38 import worker_context
        return torch.utils.data.DataLoader(dataset, batch_size=batch_size,
                                           num_workers=self.num_workers, shuffle=shuffle,
                                           sampler=sampler, drop_last=self.drop_last,
                                           pin_memory=self.pin_memory,
                                           multiprocessing_context=worker_context(self.num_workers))

    def train_dataloader(self, sampler=None, **kwargs):
        return self._data_loader(self.dataset_train, self.batch_size,
                                 shuffle=self.shuffle and sampler is None, sampler=sampler)

    def val_dataloader(self, sampler=None, **kwargs):
        return self._data_loader(self.dataset_val, self.batch_size_eval, sampler=sampler)

    def test_dataloader(self, sampler=None, **kwargs):
        return self._data_loader(self.dataset_test, self.batch_size_eval, sampler=sampler)
